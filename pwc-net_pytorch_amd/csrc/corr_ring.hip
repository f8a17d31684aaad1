// corr_ring.hip — correlation forward, LDS-DMA ring kernel for gfx950 (the l4 / "level 2" path).
//
// Semantics: correlation_cuda_kernel.cu:34-106 of daigo0927/PWC-Net_pytorch with
// kernel_size 1, stride1 1 (model.py:24 builds Correlation(9, 1, 9, 1, 2)):
//   out[n, tc, oy, ox] = sum_c f1[n,c,oy+off,ox+off] * f2[n,c,oy+off+tj*S,ox+off+ti*S] / divisor
// with zeros outside the image (the reference's zero-filled padded scratch), off = md - pad.
//
// Structure (one workgroup = one 16x16 output tile of one image, 9 waves = one displacement row
// tj each; lane = (output row ty, 4-pixel group q)):
//   * the f1 tile (16x16) and the f2 tile (16+2*HALO rows x 32 columns) of CC channels form a
//     stage; stages are streamed HBM/L2 -> LDS by buffer_load_dwordx4 ... lds (LDS-DMA, 1 KiB
//     per wave-instruction, no VGPR staging) into an NS-deep ring, so NS-1 stages are in flight
//     while one is consumed;
//   * out-of-image quads get a voffset past the buffer's num_records, which the buffer unit
//     turns into zeros (the reference's zero padding) -- no branches, no zero page;
//   * f2 rows are stored unpadded with the quad index XOR-swizzled by bit 1 of the row
//     (swizzle applied to the DMA source, LDS destination linear), so the four rows a
//     ds_read_b128 lane group touches hit disjoint 16-bank slices (measured 0 conflicts);
//   * each lane reads its f1 quad + 5 f2 quads per channel (6 x ds_read_b128, in one asm
//     statement: compiler-visible LDS loads would each get an s_waitcnt vmcnt(0) because hipcc
//     cannot prove they miss the in-flight DMA) and runs 36 FMAs (4 pixels x 9 ti);
//   * waves wait on their own DMA with a counted vmcnt and meet at a raw s_barrier (a
//     __syncthreads() would drain every in-flight stage);
//   * tiles are remapped XCD-aware so neighbouring tiles (shared halo rows) share an L2.
#include <hip/hip_ext.h>

#include <cstdlib>
#include <cstring>

#include "pwc_common.cuh"

namespace pwc {

// capi.hip: one-shot start/stop events for the next main correlation dispatch of this thread.
void take_launch_events(hipEvent_t* start, hipEvent_t* stop);

// corr_fwd.hip: out[i] = (sum_k partial[k][i]) / divisor, k in order (deterministic).
hipError_t corr_reduce_splits_f32(const void* partial, void* out, size_t n, int nsplit,
                                  float divisor, float inv_divisor, hipStream_t stream);

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Six ds_read_b128 + lgkmcnt(0) in one statement (see file header).  OFF is the channel's
// byte offset inside the stage, folded into the instructions' 16-bit offset field so the
// per-channel address arithmetic disappears.
template <int OFF>
__device__ __forceinline__ void lds_read6(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                          uint32_t a4, uint32_t a5, f32x4& r0, f32x4& r1,
                                          f32x4& r2, f32x4& r3, f32x4& r4, f32x4& r5) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  asm volatile(
      "ds_read_b128 %0, %6 offset:%12\n\t"
      "ds_read_b128 %1, %7 offset:%12\n\t"
      "ds_read_b128 %2, %8 offset:%12\n\t"
      "ds_read_b128 %3, %9 offset:%12\n\t"
      "ds_read_b128 %4, %10 offset:%12\n\t"
      "ds_read_b128 %5, %11 offset:%12\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "n"(OFF)
      : "memory");
}

// One channel of one stage: 6 LDS quads in, 36 FMAs (4 pixels x 9 ti) out.
template <class G, int CC_I>
__device__ __forceinline__ void ring_channel(const uint32_t (&addr)[6], float (&acc)[G::D][G::PX]) {
  f32x4 a4, b[G::NWQ];
#if defined(PWC_RING_ABL_MODE) && PWC_RING_ABL_MODE == 5  // diagnostic: FMAs without LDS reads
  a4 = f32x4{acc[0][0], 1.f, 2.f, 3.f};
  for (int u = 0; u < G::NWQ; ++u) b[u] = f32x4{acc[1][u & 3], 0.5f, 0.25f, 0.125f};
#else
  lds_read6<CC_I * G::CH_FLOATS * 4>(addr[0], addr[1], addr[2], addr[3], addr[4], addr[5], a4,
                                     b[0], b[1], b[2], b[3], b[4]);
#endif
#if defined(PWC_RING_ABL_MODE) && PWC_RING_ABL_MODE == 4  // diagnostic: LDS reads, no FMAs
  asm volatile("" ::"v"(a4), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]));
  return;
#endif
  static_assert(G::S == 2 && G::PX == 4, "packed pixel pairs need stride-2 displacements");
  corr_fma_pairs_s2<G::D, G::NWQ>(acc, a4, b);
}

template <class G, int CC_I>
__device__ __forceinline__ void ring_stage(const uint32_t (&addr)[6], float (&acc)[G::D][G::PX]) {
  if constexpr (CC_I < G::CC) {
    ring_channel<G, CC_I>(addr, acc);
    ring_stage<G, CC_I + 1>(addr, acc);
  }
}

// JG: displacement rows tj per workgroup (one wave each); a tile's D rows are spread over
// D / JG workgroups, each staging only the f2 rows its tj need (TY + S*(JG-1), padded to whole
// 8-row DMA pieces): more, smaller workgroups for grids with few tiles per CU.
template <int DR_, int S_, int TY_, int CC_, int NS_, int PPW_, int JG_ = 2 * DR_ + 1>
struct RingTile {
  static constexpr int DR = DR_, S = S_, TY = TY_, CC = CC_, NS = NS_, PPW = PPW_, JG = JG_;
  static constexpr int D = 2 * DR + 1;
  static constexpr int NTJG = D / JG;
  static constexpr int HALO = DR * S;
  static constexpr int TX = 16, NQ = 4, PX = 4;
  static constexpr int X2 = 32;  // f2 tile row: 8 quads
  static constexpr int R2 = ((TY + S * (JG - 1) + 7) / 8) * 8;
  static constexpr int NWQ = (PX + 2 * DR * S) / 4;  // f2 window quads per lane
  static constexpr int THREADS = TY * NQ * JG;
  static constexpr int F2_FLOATS = R2 * X2;
  static constexpr int F1_FLOATS = TY * TX;
  static constexpr int CH_FLOATS = F2_FLOATS + F1_FLOATS;
  static constexpr int STAGE_FLOATS = CC * CH_FLOATS;
  static constexpr int LDS_BYTES = NS * STAGE_FLOATS * 4;
  static constexpr int F2P = R2 / 8;   // 1 KiB pieces per channel (8 rows of 8 quads)
  static constexpr int F1P = TY / 16;  // 16 rows of 4 quads
  static constexpr int PIECES = CC * (F2P + F1P);
  static constexpr int ISSUERS = PIECES / PPW;
  static_assert(TX + 2 * HALO == X2, "ring tile needs a 32-float f2 row");
  static_assert(R2 % 8 == 0 && TY % 16 == 0, "whole 1 KiB pieces");
  static_assert(PIECES % PPW == 0, "uniform pieces per issuing wave");
  static_assert(ISSUERS <= THREADS / 64, "enough waves to issue");
  static_assert(NWQ == 5, "lds_read6: one f1 quad + five f2 quads");
  static_assert((NWQ - 1) + (NQ - 1) < 8, "window inside the row");
  static_assert(THREADS % 64 == 0 && THREADS <= 1024, "workgroup");
  static_assert(NS >= 2, "ring depth");
  static_assert(D % JG == 0, "tj groups");
};

#ifdef PWC_RING_ABLATION
__constant__ int g_ablation;
#endif

// DMA of one stage.  The buffer resource is rebuilt per stage with its base at the stage's first
// channel (scalar work only), so the per-lane voffsets stay the lane constants src_off and the
// vector registers carry nothing stage-dependent; num_records shrinks with the base, so channels
// past C still read zeros.  (The body is device-only: hipcc's host pass rejects the buffer
// resource builtins in some template instantiation chains.)
template <class G>
__device__ __forceinline__ void ring_issue(int stage, int c_begin, int wave, uint32_t plane,
                                           uint32_t lds0, const float* img1, const float* img2,
                                           uint32_t img_bytes,
                                           const uint32_t (&src_off)[G::PPW],
                                           const uint32_t (&dst_off)[G::PPW],
                                           const bool (&from_f2)[G::PPW]) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (wave >= G::ISSUERS) return;
  const uint32_t c0 = (uint32_t)(c_begin + stage * G::CC);
  const uint32_t cbytes = c0 * plane * 4u;
  const int nrec = cbytes < img_bytes ? (int)(img_bytes - cbytes) : 0;
  const uint32_t sbase = lds0 + (uint32_t)((stage % G::NS) * G::STAGE_FLOATS) * 4u;
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    // wave-uniform by construction; readfirstlane lets the compiler see it (else it wraps the
    // DMA in a waterfall loop over "divergent" resource descriptors)
    const uint64_t b = (uint64_t)(uintptr_t)(from_f2[i] ? img2 : img1) + (uint64_t)cbytes;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
        __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(uintptr_t)(sbase + dst_off[i]), 16,
        src_off[i], 0, 0, 0);
  }
#endif
}

// Channel split (blockIdx.y = split k of nsplit): split k sums channels
// [k*cps, min(C, (k+1)*cps)) and, when nsplit > 1, stores its raw sums to
// partial[k][n][oc][oy][ox] for corr_reduce_splits (fixed-order, deterministic).
template <class G>
__global__ __launch_bounds__(G::THREADS, 6) void corr_fwd_ring(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    int C, int H, int W, int Ho, int Wo, int off, int layout, float divisor, float inv_divisor,
    int n_ty, int n_tx, int cps, float* __restrict__ partial, OutEpi epi
#ifdef PWC_RING_CENSUS
    , unsigned* census
#endif
    ) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
#ifdef PWC_RING_CENSUS  // diagnostic build only (tools/occupancy.hip): residency census
  unsigned long long census_t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long census_c0 = __builtin_amdgcn_s_memtime();
  unsigned long long census_c1 = 0, census_r1 = 0;
#endif

  const int t0 = xcd_remap(blockIdx.x, gridDim.x);
  const int tjg = t0 % G::NTJG;  // the tj groups of a tile are neighbours: same XCD
  const int t = t0 / G::NTJG;
  const int tx_tile = t % n_tx;
  const int ty_tile = (t / n_tx) % n_ty;
  const int n = t / (n_tx * n_ty);
  const int oy0 = ty_tile * G::TY, ox0 = tx_tile * G::TX;
  const int y1 = oy0 + off, x1 = ox0 + off;  // f1 tile origin, unpadded image coordinates
  const int tj0 = tjg * G::JG;
  const int f2y0 = y1 - G::HALO + G::S * tj0;  // image row of f2 tile row 0

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = threadIdx.x % G::NQ;
  const int ty = (threadIdx.x / G::NQ) % G::TY;
  const int tjx = threadIdx.x / (G::NQ * G::TY);

  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t img_bytes = (uint32_t)C * plane * 4u;  // checked < 2^31 by the launcher
  const float* img1 = in1 + (size_t)n * C * plane;
  const float* img2 = in2 + (size_t)n * C * plane;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA issue plan: issuer wave w owns pieces w*PPW .. w*PPW+PPW-1 of every stage ----
  // per piece: source byte offset of this lane for channel 0 (or OOB), LDS byte offset.
  uint32_t src_off[G::PPW];
  uint32_t dst_off[G::PPW];
  bool from_f2[G::PPW];
  constexpr uint32_t kOOB = 0x80000000u;  // >= num_records: the buffer unit returns zeros
  if (wave < G::ISSUERS) {
#pragma unroll
    for (int i = 0; i < G::PPW; ++i) {
      const int p = wave * G::PPW + i;
      const int cc = p / (G::F2P + G::F1P);
      const int k = p % (G::F2P + G::F1P);
      int gy, gx;
      uint32_t dst = (uint32_t)(cc * G::CH_FLOATS) * 4u;
      if (k < G::F2P) {
        const int r = 8 * k + (lane >> 3);
        const int srcq = (lane & 7) ^ (((r >> 1) & 1) << 2);
        gy = f2y0 + r;
        gx = x1 - G::HALO + 4 * srcq;
        dst += (uint32_t)(8 * k * G::X2) * 4u;
      } else {
        gy = y1 + (lane >> 2);
        gx = x1 + 4 * (lane & 3);
        dst += (uint32_t)G::F2_FLOATS * 4u;
      }
      const bool ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
      src_off[i] = ok ? ((uint32_t)cc * plane + (uint32_t)(gy * W + gx)) * 4u : kOOB;
      dst_off[i] = dst;
      from_f2[i] = k < G::F2P;
    }
  }
  // ---- lane-constant LDS read offsets (bytes, relative to a channel block) ----
  const int r2 = ty + G::S * tjx;
  const int sw = ((r2 >> 1) & 1) << 2;
  uint32_t woff[G::NWQ];
#pragma unroll
  for (int u = 0; u < G::NWQ; ++u) woff[u] = (uint32_t)(r2 * G::X2 + (((q + u) ^ sw) << 2)) * 4u;
  const uint32_t aoff = (uint32_t)(G::F2_FLOATS + ty * G::TX + (q << 2)) * 4u;

  float acc[G::D][G::PX];
#pragma unroll
  for (int a = 0; a < G::D; ++a)
#pragma unroll
    for (int k = 0; k < G::PX; ++k) acc[a][k] = 0.f;

  const int c_begin = blockIdx.y * cps;
  const int c_end = min(C, c_begin + cps);
  const int nst = (c_end - c_begin + G::CC - 1) / G::CC;  // cps is a multiple of CC
#pragma unroll
  for (int s = 0; s < G::NS - 1; ++s)
    if (s < nst)
      ring_issue<G>(s, c_begin, wave, plane, lds0, img1, img2, img_bytes, src_off, dst_off,
                    from_f2);

#ifdef PWC_RING_CENSUS
  census_c1 = __builtin_amdgcn_s_memtime();
  census_r1 = __builtin_amdgcn_s_memrealtime();
#endif
  for (int st = 0; st < nst; ++st) {
#if !(defined(PWC_RING_ABL_MODE) && PWC_RING_ABL_MODE == 3)  // 3: no DMA, no barriers
    if (wave < G::ISSUERS) {
      if (nst - 1 - st >= G::NS - 2)
        wait_vmcnt<(G::NS - 2) * G::PPW>();
      else
        wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
#endif
#ifdef PWC_RING_ABLATION  // diagnostic build: g_ablation bits 1 = no FMA work, 2 = no DMA
    if (!(g_ablation & 2))
#endif
    if (st + G::NS - 1 < nst)
      ring_issue<G>(st + G::NS - 1, c_begin, wave, plane, lds0, img1, img2, img_bytes, src_off,
                    dst_off, from_f2);
    const uint32_t sb = lds0 + (uint32_t)((st % G::NS) * G::STAGE_FLOATS) * 4u;
#ifdef PWC_RING_ABLATION
    if (g_ablation & 1) continue;
#endif
    const uint32_t addr[6] = {sb + aoff, sb + woff[0], sb + woff[1], sb + woff[2], sb + woff[3],
                              sb + woff[4]};
    ring_stage<G, 0>(addr, acc);
  }

#ifdef PWC_RING_CENSUS
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned cb = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned long long c2 = __builtin_amdgcn_s_memtime();
    const unsigned long long r2 = __builtin_amdgcn_s_memrealtime();
    census[cb * 8 + 0] = hw;
    census[cb * 8 + 1] = xcc;
    census[cb * 8 + 2] = (unsigned)census_t0;
    census[cb * 8 + 3] = (unsigned)r2;
    census[cb * 8 + 4] = (unsigned)(census_c1 - census_c0);  // prologue, shader cycles
    census[cb * 8 + 5] = (unsigned)(c2 - census_c1);         // stage loop, shader cycles
    census[cb * 8 + 6] = (unsigned)(r2 - census_r1);         // stage loop, 100 MHz ticks
  }
#endif
  // ---- epilogue: out = acc / divisor (cu:100); a power-of-two divisor is an exact scale ----
  const int oy = oy0 + ty;
  const int ox = ox0 + 4 * q;
  if (oy >= Ho || ox >= Wo) return;
#ifdef PWC_RING_ABLATION  // bit 4 = no output stores (results kept live through a NaN test)
  if (g_ablation & 4) {
    float z = 0.f;
#pragma unroll
    for (int a = 0; a < G::D; ++a)
#pragma unroll
      for (int k = 0; k < G::PX; ++k) z += acc[a][k];
    if (z != z) out[0] = z;
    return;
  }
#endif
  const int OC = G::D * G::D;
  const int tj = tj0 + tjx - G::DR;
  if (gridDim.y > 1) {  // split: raw partial sums, reduced by corr_reduce_splits
    float* pk = partial + (size_t)blockIdx.y * ((size_t)gridDim.x / (n_tx * n_ty * G::NTJG)) *
                              OC * Ho * Wo;
#pragma unroll
    for (int ti = 0; ti < G::D; ++ti) {
      const int oc = out_channel(layout, tj, ti - G::DR, G::DR, G::D, G::S);
      float* orow = pk + (((size_t)n * OC + oc) * Ho + oy) * Wo;
      *reinterpret_cast<float4*>(orow + ox) =
          make_float4(acc[ti][0], acc[ti][1], acc[ti][2], acc[ti][3]);
    }
    return;
  }
  const bool pow2 = inv_divisor != 0.f;
  float* oimg = out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * OC * Ho * Wo);
#pragma unroll
  for (int ti = 0; ti < G::D; ++ti) {
    const int oc = out_channel(layout, tj, ti - G::DR, G::DR, G::D, G::S);
    float* orow = oimg + ((size_t)oc * Ho + oy) * Wo;
    st_f32x4 v;
    if (pow2)
      v = st_f32x4{acc[ti][0] * inv_divisor, acc[ti][1] * inv_divisor,
                   acc[ti][2] * inv_divisor, acc[ti][3] * inv_divisor};
    else
      v = st_f32x4{acc[ti][0] / divisor, acc[ti][1] / divisor, acc[ti][2] / divisor,
                   acc[ti][3] / divisor};
    v = st_f32x4{epi_act(v.x, epi.slope), epi_act(v.y, epi.slope), epi_act(v.z, epi.slope),
                 epi_act(v.w, epi.slope)};
    st_out4(orow + ox, v);
  }
}

// ------------------------------------------------------------------------------------
// configuration: three workgroups per 16x16 tile (3 tj rows each, 24-row f2 tiles), 2 channels
// per stage, 5-deep ring (4 stages in flight), 40 KiB of LDS.  Round 2 measured 17 other ring
// shapes, a software-pipelined and a de-interleaved variant (profiles/r02d_stream_ring_sweep.txt,
// r02d_bench_ring_ab.txt); none beat this one and they were removed from the library (round 3).
// ------------------------------------------------------------------------------------
using RingN = RingTile<4, 2, 16, 2, 5, 4, 3>;

#ifdef PWC_RING_CENSUS
unsigned* g_census = nullptr;
#endif

template <class G>
static hipError_t launch_ring(const void* in1, const void* in2, void* out, int B, int C, int H,
                              int W, int Ho, int Wo, int off, int layout, float divisor,
                              int nsplit, void* partial, hipStream_t stream) {
  const int n_ty = (Ho + G::TY - 1) / G::TY;
  const int n_tx = (Wo + G::TX - 1) / G::TX;
  const long long nblk = (long long)B * n_ty * n_tx * G::NTJG;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_fwd_ring<G>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int nchunks = (C + G::CC - 1) / G::CC;
  if (nsplit > nchunks) nsplit = nchunks;
  if (nsplit < 1) nsplit = 1;
  const int cps = ((nchunks + nsplit - 1) / nsplit) * G::CC;
  nsplit = (C + cps - 1) / cps;
  const OutEpi epi = current_epi();
  if (nsplit > 1 && !epi_is_default(epi)) return hipErrorNotSupported;  // dense partials only
  // exact reciprocal when the divisor is a power of two (then x * inv == x / divisor)
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  // Optional kernel-start/-end events armed by pwc_time_next_corr (bench.py's live roofline
  // timing: the events bracket exactly this dispatch on `stream`).
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL((corr_fwd_ring<G>), dim3((unsigned)nblk, (unsigned)nsplit),
                        dim3(G::THREADS), G::LDS_BYTES, stream, ev0, ev1, 0, (const float*)in1,
                        (const float*)in2, (float*)out, C, H, W, Ho, Wo, off, layout, divisor,
                        inv, n_ty, n_tx, cps, (float*)partial, epi
#ifdef PWC_RING_CENSUS
                        , g_census
#endif
                        );
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nsplit == 1) return e;
  return corr_reduce_splits_f32(partial, out, (size_t)B * G::D * G::D * Ho * Wo, nsplit,
                                divisor, inv, stream);
}

// Number of channel splits for a grid of `base_blocks` tiles: none once the tiles alone give
// every CU a workgroup; otherwise aim at two workgroups per CU (512), at most one split per
// channel chunk and at most `max_splits` (the caller sizes max_splits so that the partial
// volumes stay within the workspace budget, corr_workspace_bytes).
int corr_pick_splits(long long base_blocks, int nchunks, int max_splits) {
  if (base_blocks <= 0 || base_blocks >= 256) return 1;
  long long k = (512 + base_blocks - 1) / base_blocks;
  if (k > nchunks) k = nchunks;
  if (k > max_splits) k = max_splits;
  return k < 1 ? 1 : (int)k;
}

// hipErrorNotSupported: shape / alignment outside what the ring kernel handles.
// `partial` (nsplit * B*81*Ho*Wo floats) may be null when nsplit == 1.
hipError_t corr_forward_ring_f32(const void* in1, const void* in2, void* out, int B, int C,
                                 int H, int W, int Ho, int Wo, int off, int dr, int s2,
                                 int layout, float divisor, int max_splits, void* partial,
                                 hipStream_t stream) {
  if (!(dr == 4 && s2 == 2)) return hipErrorNotSupported;
  if (W % 4 || Wo % 4 || off % 4) return hipErrorNotSupported;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16)
    return hipErrorNotSupported;
  if ((size_t)C * H * W * 4 >= 0x7ffffff0ull) return hipErrorNotSupported;
  const long long tiles = (long long)B * ((Ho + 15) / 16) * ((Wo + 15) / 16);
  const int ns = partial ? corr_pick_splits(tiles, (C + 3) / 4, max_splits) : 1;
  return launch_ring<RingN>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, ns, partial,
                           stream);
}

}  // namespace pwc
