// corr_pt.hip — correlation forward, stride-2 displacements, on 24-row parity tiles (gfx950).
//
// Semantics: correlation_cuda_kernel.cu:34-106 of daigo0927/PWC-Net_pytorch with
// kernel_size 1, stride1 1, max_displacement / stride2 = 4, stride2 = 2 (model.py:24 builds
// Correlation(9, 1, 9, 1, 2)):
//   out[n, tc, oy, ox] = sum_c f1[n,c,oy+off,ox+off] * f2[n,c,oy+off+2tj,ox+off+2ti] / divisor
// zeros outside the image (the reference's zero-filled padded scratch, cu:10-32),
// off = max_displacement - pad_size, channels summed in order c = 0, 1, ... (one fp32 fma
// chain per output, as the reference's per-thread partial sums are not reproduced bit for bit
// anyway: parity is to 1e-5 against the fp64 oracle).
//
// Decomposition (measured on MI355X, tools/cbench.hip):
//   * Row parity: an output row oy only meets f2 rows of its own parity (oy + off + 2tj), so
//     the image splits into two disjoint half-height problems.  A tile = 24 output rows of one
//     parity x 16 columns of one image: it stages 24 + 8 f2 rows (parity rows) instead of the
//     24 + 16 a consecutive-row tile needs.
//   * One tile per workgroup, one workgroup per CU (the ring takes ~154 KiB of LDS): at
//     384x448 / B = 8 this is 224 tiles for 256 CUs, so every CU that works does the same
//     amount of work (16x16 tiles gave 336 tiles: 80 CUs doing two while the rest did one).
//   * Deep prefetch: NS-1 = 6 stages of CC = 4 channels (24 of l4's 32 channels) are in flight
//     from the first cycle; HBM latency under full load is several microseconds, and the
//     shallow rings of the 16x16 kernels were latency-bound on the DMA.
//   * 432 lanes = 9 displacement rows tj x 24 rows x 2 eight-pixel segments; a lane keeps
//     8 px x 9 ti = 72 fp32 sums and per channel reads 2 f1 quads + 6 f2 quads (8 x
//     ds_read_b128 for 72 FMAs).  Reads of channel c+1 are issued before the FMAs of channel c
//     (double-buffered registers), so LDS latency hides under the lane's own FMAs.
//   * Bank conflicts: every ds_read_b128 lane group (16 lanes: {0-3,12-15,20-27}, ...) must hit
//     16 distinct 16-B slots.  Lanes 0..287 are (tj, r < 16, s) in the order of corr_par.hip
//     (each half-wave = one tj, 16 rows: 8 distinct rows mod 8 per group).  Rows 16..23 pair
//     two displacement rows per half-wave: the second tj's lanes take rows rotated by 7, which
//     makes the f2 rows of every group again 8 distinct residues mod 8.  With the per-row XOR
//     swizzle of quad slots (par_f2_swz / par_f1_swz, applied on the DMA source) that gives 16
//     distinct slots for every group and every window quad.
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace pt {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// f2 LDS row rho holds logical quad q at slot q ^ f2_swz(rho) (8 rows of distinct residues
// mod 8, both 8-pixel segments: 16 distinct 16-B slots); f1 rows are 4 quads, XOR by row bit 2.
__host__ __device__ __forceinline__ int f2_swz(int rho) {
  return ((rho >> 1) & 1) | (((rho >> 2) & 1) << 2);
}
__host__ __device__ __forceinline__ int f1_swz(int r) { return (r >> 2) & 1; }

// K channel groups share a workgroup of 8 waves: group g = waves g*8/K .. (g+1)*8/K - 1, each
// wave three tile rows, so a tile is TR = 24/K parity rows.  Every stage carries CC = K*CPG
// channels; group g accumulates channels g*CPG .. g*CPG+CPG-1 of each stage and the K partial
// sums meet in LDS at the end (fixed order: deterministic).  K = 1 is the l4 shape; K > 1
// trades tile rows for channel parallelism on the coarse levels (fewer, deeper pixels).
template <int K_, int CPG_, int NS_>
struct PtTile {
  static constexpr int DR = 4, S = 2, D = 9;
  static constexpr int K = K_, CPG = CPG_, NS = NS_, PD = 1;
  static constexpr int NWAVES = 8, THREADS = 64 * NWAVES;
  static constexpr int WPG = NWAVES / K;  // waves per channel group
  static constexpr int TR = 3 * WPG;      // parity rows per tile
  static constexpr int TX = 16;           // columns per tile: two 8-pixel segments
  static constexpr int R2 = TR + 2 * DR;  // f2 rows
  static constexpr int X2 = 32;           // f2 row: columns x0-8 .. x0+23
  static constexpr int CC = K * CPG;      // channels per stage
  static constexpr int F2_FLOATS = R2 * X2;
  static constexpr int F1_FLOATS = TR * TX;
  static constexpr int CH_FLOATS = F2_FLOATS + F1_FLOATS;
  static constexpr int CH_BYTES = CH_FLOATS * 4;
  static constexpr int STAGE_BYTES = CC * CH_BYTES;
  static constexpr int RED_BYTES = K > 1 ? 18 * THREADS * 16 : 0;  // partial sums, K > 1
  static constexpr int RING_BYTES = NS * STAGE_BYTES;
  static constexpr int LDS_BYTES = RING_BYTES > RED_BYTES ? RING_BYTES : RED_BYTES;
  // DMA pieces per channel (1 KiB wave-instructions, partial EXEC on the last of each kind)
  static constexpr int F2P = (R2 + 7) / 8;   // 8 rows x 8 quads
  static constexpr int F1P = (TR + 15) / 16; // 16 rows x 4 quads
  static constexpr int PPC = F2P + F1P;
  static constexpr int PIECES = CC * PPC;
  static constexpr int ISSUERS = NWAVES;
  static constexpr int PPW = PIECES / ISSUERS;
  static_assert(K == 1 || K == 2 || K == 4 || K == 8, "channel groups");
  static_assert(CPG % 2 == 0, "register buffers alternate by channel parity within a stage");
  static_assert(PIECES % ISSUERS == 0, "uniform DMA pieces per issuing wave");
  static_assert((NS - 3) * PPW <= 63, "vmcnt range");
  static_assert(NS >= 3, "ring depth: stage st+1 must be resident while st is consumed");
  static_assert(8 * PD <= 15, "lgkmcnt is 4 bits: one channel of reads ahead");
  static_assert(LDS_BYTES <= 163840, "LDS");
};

// Eight ds_read_b128 into r (no wait: the caller waits with rd_wait before using r).
template <int OFF>
__device__ __forceinline__ void rd8(const uint32_t (&a)[8], f32x4 (&r)[8]) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  asm volatile(
      "ds_read_b128 %0, %8 offset:%16\n\t"
      "ds_read_b128 %1, %9 offset:%16\n\t"
      "ds_read_b128 %2, %10 offset:%16\n\t"
      "ds_read_b128 %3, %11 offset:%16\n\t"
      "ds_read_b128 %4, %12 offset:%16\n\t"
      "ds_read_b128 %5, %13 offset:%16\n\t"
      "ds_read_b128 %6, %14 offset:%16\n\t"
      "ds_read_b128 %7, %15 offset:%16"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
        "=&v"(r[6]), "=&v"(r[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "n"(OFF)
      : "memory");
}

// Wait until at most N LDS operations are outstanding.  r is tied through the wait, so its
// uses (the FMAs) cannot move above it and its registers cannot be reused before it.
template <int N>
__device__ __forceinline__ void rd_wait(f32x4 (&r)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),
                 "+v"(r[6]), "+v"(r[7])
               : "n"(N));
}

template <int D>
__device__ __forceinline__ void fma8(const f32x4 (&v)[8], float (&lo)[D][4], float (&hi)[D][4]) {
  const f32x4 wl[5] = {v[2], v[3], v[4], v[5], v[6]};
  const f32x4 wh[5] = {v[3], v[4], v[5], v[6], v[7]};
  corr_fma_pairs_s2<D, 5>(lo, v[0], wl);
  corr_fma_pairs_s2<D, 5>(hi, v[1], wh);
  __builtin_amdgcn_sched_barrier(0);
}

// Channel CI (of the group's CPG per stage) of the current stage; register buffer CI & 1.
// The reads of the next channel (in the next stage's slot after the last) are issued before
// the FMAs of this one, so one channel of LDS latency hides under the lane's own FMAs;
// lgkmcnt(8) then waits for this channel's eight reads only.
template <class G, int CI>
__device__ __forceinline__ void pt_chan(const uint32_t (&a)[8], const uint32_t (&an)[8],
                                        f32x4 (&buf)[2][8], float (&lo)[G::D][4],
                                        float (&hi)[G::D][4]) {
  if constexpr (CI < G::CPG) {
    if constexpr (CI + 1 < G::CPG)
      rd8<(CI + 1) * G::CH_BYTES>(a, buf[(CI + 1) & 1]);
    else
      rd8<0>(an, buf[(CI + 1) & 1]);
    rd_wait<8>(buf[CI & 1]);
    fma8<G::D>(buf[CI & 1], lo, hi);
    pt_chan<G, CI + 1>(a, an, buf, lo, hi);
  }
}

// DMA of one stage: issuer wave w owns pieces w*PPW .. w*PPW+PPW-1 (channel p / PPC, piece
// p % PPC: f2 pieces first, then f1).  The buffer resource's base moves to the stage's first
// channel (scalar work only) so the per-lane voffsets are stage-invariant; channels past C
// read zeros because num_records shrinks with the base.  Lanes past a partial piece's rows
// are masked off (their linear LDS destination would spill into the next region).
template <class G>
__device__ __forceinline__ void pt_issue(int stage, int wave, uint32_t plane, uint32_t lds0,
                                         const float* img1, const float* img2,
                                         uint32_t img_bytes, const uint32_t (&src_off)[G::PPW],
                                         const uint32_t (&dst_off)[G::PPW], uint32_t act) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t cbytes = (uint32_t)(stage * G::CC) * plane * 4u;
  const int nrec = cbytes < img_bytes ? (int)(img_bytes - cbytes) : 0;
  const uint32_t sbase = lds0 + (uint32_t)(stage % G::NS) * (uint32_t)G::STAGE_BYTES;
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    const int k = (wave * G::PPW + i) % G::PPC;  // wave-uniform
    const uint64_t b = (uint64_t)(uintptr_t)(k < G::F2P ? img2 : img1) + (uint64_t)cbytes;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
        __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
    if ((act >> i) & 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(uintptr_t)(sbase + dst_off[i]), 16,
          src_off[i], 0, 0, 0);
  }
#endif
}

#ifdef PWC_PT_ABLATION  // diagnostic build, bits: 1 = no FMA work, 2 = no DMA, 4 = no stores
__constant__ int g_pt_abl;
#endif

template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_fwd_pt(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    int C, int H, int W, int Ho, int Wo, int off, int layout, float divisor, float inv_divisor,
    int n_tr, int n_tx, OutEpi epi) {
  extern __shared__ __attribute__((aligned(16))) float lds[];

  // tile order: image-major, then parity, tile row, tile column; the XCD remap keeps an
  // image's tiles (which share f2 halo rows and columns) on one XCD's L2
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % n_tx;
  const int tr = (t / n_tx) % n_tr;
  const int p = (t / (n_tx * n_tr)) & 1;
  const int n = t / (n_tx * n_tr * 2);
  const int R0 = tr * G::TR;
  const int x0 = tx * G::TX;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave / G::WPG;  // channel group
  const int wj = wave % G::WPG;   // wave inside the group: tile rows 3wj .. 3wj+2
  // lane -> (tj, r, s): 54 lanes = 9 tj x 3 rows x 2 eight-pixel segments (s fastest, then
  // row, then tj).  Lanes 54..63 mirror lanes 44..53 (identical addresses: LDS broadcasts)
  // and store nothing.  Every ds_read_b128 lane group then hits 16 distinct 16-B slots or
  // repeats an address (checked exhaustively for the swizzles above, all window quads and
  // both f1 quads).  Eight waves = two per SIMD: with an odd count one SIMD holds a lone
  // wave, which issues VALU at half rate.
  const bool valid = lane < 54;
  const int ll = valid ? lane : lane - 10;
  const int tj = ll / 6;
  const int r = 3 * wj + (ll % 6) / 2;
  const int s = ll & 1;

  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t img_bytes = (uint32_t)C * plane * 4u;  // < 2^31, checked by the launcher
  const float* img1 = in1 + (size_t)n * C * plane;
  const float* img2 = in2 + (size_t)n * C * plane;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA plan: source byte offset for channel 0 (or OOB), LDS offset, active lanes ----
  uint32_t src_off[G::PPW];
  uint32_t dst_off[G::PPW];
  uint32_t act = 0;
  constexpr uint32_t kOOB = 0x80000000u;  // >= num_records: the buffer unit returns zeros
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    const int pc = wave * G::PPW + i;
    const int cc = pc / G::PPC;
    const int k = pc % G::PPC;
    uint32_t dst = (uint32_t)(cc * G::CH_BYTES);
    int gy, gx;
    bool on;
    if (k < G::F2P) {
      const int rho = 8 * k + (lane >> 3);
      const int q = (lane & 7) ^ f2_swz(rho);
      on = rho < G::R2;
      gy = 2 * (R0 + rho - G::DR) + p + off;
      gx = x0 + off - 2 * G::DR + 4 * q;
      dst += (uint32_t)(8 * k * G::X2) * 4u;
    } else {
      const int rr = 16 * (k - G::F2P) + (lane >> 2);
      const int q = (lane & 3) ^ f1_swz(rr);
      on = rr < G::TR;
      gy = 2 * (R0 + rr) + p + off;
      gx = x0 + off + 4 * q;
      dst += (uint32_t)(G::F2_FLOATS + 16 * (k - G::F2P) * G::TX) * 4u;
    }
    const bool ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
    src_off[i] = ok ? ((uint32_t)cc * plane + (uint32_t)(gy * W + gx)) * 4u : kOOB;
    dst_off[i] = dst;
    act |= (on ? 1u : 0u) << i;
  }

  // ---- lane-constant LDS read offsets (bytes from the stage slot; group's channel block) ----
  const int rho = r + tj;
  const uint32_t gbase = (uint32_t)(grp * G::CPG * G::CH_BYTES);
  uint32_t off8[8];
  off8[0] = gbase + (uint32_t)(G::F2_FLOATS + r * G::TX + (((2 * s) ^ f1_swz(r)) << 2)) * 4u;
  off8[1] = gbase + (uint32_t)(G::F2_FLOATS + r * G::TX + (((2 * s + 1) ^ f1_swz(r)) << 2)) * 4u;
#pragma unroll
  for (int u = 0; u < 6; ++u)
    off8[2 + u] = gbase + (uint32_t)(rho * G::X2 + (((2 * s + u) ^ f2_swz(rho)) << 2)) * 4u;

  float lo[G::D][4], hi[G::D][4];
#pragma unroll
  for (int a = 0; a < G::D; ++a)
#pragma unroll
    for (int k = 0; k < 4; ++k) lo[a][k] = hi[a][k] = 0.f;

  const int nst = (C + G::CC - 1) / G::CC;
#pragma unroll
  for (int st = 0; st < G::NS - 1; ++st)
    if (st < nst)
      pt_issue<G>(st, wave, plane, lds0, img1, img2, img_bytes, src_off, dst_off, act);

  // Stage st is consumed with stage st+1 already resident (the reads run into it), so the
  // barrier at the top of stage st waits for stage st+1's DMA; it also releases the slot of
  // stage st-1, which all waves have finished reading, to the DMA of stage st+NS-1.
  f32x4 buf[2][8];
  for (int st = 0; st < nst; ++st) {
    {
      // issued so far: stages 0 .. min(nst, st+NS-1)-1; keep all but stages <= st+1 in flight
      const int issued = min(nst, st + G::NS - 1);
      if (issued - (st + 2) >= G::NS - 3)
        wait_vmcnt<(G::NS - 3) * G::PPW>();
      else
        wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
#ifdef PWC_PT_ABLATION
    if (!(g_pt_abl & 2))
#endif
    if (st + G::NS - 1 < nst)
      pt_issue<G>(st + G::NS - 1, wave, plane, lds0, img1, img2, img_bytes, src_off, dst_off,
                  act);
#ifdef PWC_PT_ABLATION
    if (g_pt_abl & 1) continue;
#endif
    const uint32_t sb = lds0 + (uint32_t)(st % G::NS) * (uint32_t)G::STAGE_BYTES;
    const uint32_t sn = lds0 + (uint32_t)((st + 1) % G::NS) * (uint32_t)G::STAGE_BYTES;
    uint32_t a[8], an[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = sb + off8[u];
      an[u] = sn + off8[u];
    }
    if (st == 0) rd8<0>(a, buf[0]);
    pt_chan<G, 0>(a, an, buf, lo, hi);
  }
  // the last prefetch read a slot past the data (discarded): drain it
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- epilogue: out = acc / divisor (cu:100); a power-of-two divisor is an exact scale ----
  const int oy = 2 * (R0 + r) + p;
  const int ox = x0 + 8 * s;
  const bool st_ok = valid && oy < Ho && ox < Wo;
#ifdef PWC_PT_ABLATION
  if (g_pt_abl & 4) {
    float z = 0.f;
#pragma unroll
    for (int a = 0; a < G::D; ++a)
#pragma unroll
      for (int k = 0; k < 4; ++k) z += lo[a][k] + hi[a][k];
    if (z != z) out[0] = z;
    return;
  }
#endif
  const int OC = G::D * G::D;
  const bool pow2 = inv_divisor != 0.f;
  const bool has_hi = ox + 4 < Wo;
  float* obase = out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * OC * Ho * Wo) +
                 (size_t)oy * Wo + ox;
  auto emit = [&](int v, f32x4 q) {  // v = 2*ti + h
    const int ti = v >> 1, h = v & 1;
    if (!st_ok || (h && !has_hi)) return;
    const int oc = out_channel(layout, tj - G::DR, ti - G::DR, G::DR, G::D, G::S);
    if (pow2)
      q *= inv_divisor;
    else
      q /= divisor;
    q = f32x4{epi_act(q.x, epi.slope), epi_act(q.y, epi.slope), epi_act(q.z, epi.slope),
              epi_act(q.w, epi.slope)};
    st_out4(obase + (size_t)oc * Ho * Wo + 4 * h, q);
  };
  if constexpr (G::K == 1) {
#pragma unroll
    for (int ti = 0; ti < G::D; ++ti) {
      emit(2 * ti, f32x4{lo[ti][0], lo[ti][1], lo[ti][2], lo[ti][3]});
      emit(2 * ti + 1, f32x4{hi[ti][0], hi[ti][1], hi[ti][2], hi[ti][3]});
    }
  } else {
    // K partial sums per output: every lane parks its 18 float4 in LDS ([v][group][slot],
    // 16-B consecutive per lane: conflict-free), then group g finalises slots v == g mod K as
    // ((p_0 + p_1) + p_2) + ... in group order and stores them.
    __builtin_amdgcn_s_barrier();  // every wave is past its last ring read
    f32x4* red = reinterpret_cast<f32x4*>(lds);
    const int slot = wj * 64 + lane;  // the same output item in every group
#pragma unroll
    for (int v = 0; v < 18; ++v) {
      const int ti = v >> 1;
      const f32x4 q = (v & 1) ? f32x4{hi[ti][0], hi[ti][1], hi[ti][2], hi[ti][3]}
                              : f32x4{lo[ti][0], lo[ti][1], lo[ti][2], lo[ti][3]};
      red[(v * G::K + grp) * (G::WPG * 64) + slot] = q;
    }
    __syncthreads();
    for (int v = grp; v < 18; v += G::K) {
      f32x4 q = red[(v * G::K) * (G::WPG * 64) + slot];
#pragma unroll
      for (int g = 1; g < G::K; ++g) q += red[(v * G::K + g) * (G::WPG * 64) + slot];
      emit(v, q);
    }
  }
}

template <class G>
static hipError_t launch_pt(const void* in1, const void* in2, void* out, int B, int C, int H,
                            int W, int Ho, int Wo, int off, int layout, float divisor,
                            hipStream_t stream) {
  const int n_tr = ((Ho + 1) / 2 + G::TR - 1) / G::TR;  // parity-0 rows: ceil(Ho / 2)
  const int n_tx = (Wo + G::TX - 1) / G::TX;
  const long long nblk = (long long)B * 2 * n_tr * n_tx;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e = lds_limit(reinterpret_cast<const void*>(&corr_fwd_pt<G>), G::LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL((corr_fwd_pt<G>), dim3((unsigned)nblk), dim3(G::THREADS), G::LDS_BYTES,
                        stream, ev0, ev1, 0, (const float*)in1, (const float*)in2, (float*)out,
                        C, H, W, Ho, Wo, off, layout, divisor, inv, n_tr, n_tx, current_epi());
  return hipGetLastError();
}

//                   K  CPG NS    tile rows  stage    ring
using Pt1 = PtTile<1, 4, 5>;   // 24       22 KiB   110 KiB: stages st+1 .. st+3 in flight
using Pt2 = PtTile<2, 2, 12>;  // 12       13 KiB   156 KiB
using Pt4 = PtTile<4, 2, 9>;   //  6       17 KiB   153 KiB
using Pt8 = PtTile<8, 2, 6>;   //  3       25 KiB   150 KiB

}  // namespace pt

// Parity-tile correlation (stride-2 displacements, dr = 4) with `groups` channel groups per
// workgroup (1, 2, 4 or 8; 0 = pick by grid size).  hipErrorNotSupported: shape / alignment
// outside what the kernel handles.
hipError_t corr_forward_pt_f32(const void* in1, const void* in2, void* out, int B, int C, int H,
                               int W, int Ho, int Wo, int off, int dr, int s2, int layout,
                               float divisor, int groups, hipStream_t stream) {
  if (!(dr == 4 && s2 == 2)) return hipErrorNotSupported;
  if (W % 4 || Wo % 4 || off % 4) return hipErrorNotSupported;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16)
    return hipErrorNotSupported;
  if ((size_t)C * H * W * 4 >= 0x7ffffff0ull) return hipErrorNotSupported;
  if (const int k = debug_knob("pt_k", 0)) groups = k;
  if (groups <= 0) {
    // the largest tile (fewest halo bytes per output) that still gives ~one tile per CU;
    // grids that fill the chip with single-group tiles (l4-sized, when the stream and row-band
    // kernels decline the shape) take Pt1
    const int hp = (Ho + 1) / 2, ntx = (Wo + 15) / 16;
    groups = 8;
    for (int k : {1, 2, 4}) {
      const long long tiles = (long long)B * 2 * ((hp + 24 / k - 1) / (24 / k)) * ntx;
      if (tiles >= 192) { groups = k; break; }
    }
  }
  switch (groups) {
    case 1: return pt::launch_pt<pt::Pt1>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    case 2: return pt::launch_pt<pt::Pt2>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    case 4: return pt::launch_pt<pt::Pt4>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    case 8: return pt::launch_pt<pt::Pt8>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    default: return hipErrorNotSupported;
  }
}

}  // namespace pwc
