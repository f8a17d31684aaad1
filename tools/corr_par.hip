// corr_par.hip — correlation forward for stride-2 displacements on row-parity tiles (gfx950).
//
// Semantics: correlation_cuda_kernel.cu:34-106 of daigo0927/PWC-Net_pytorch with
// kernel_size 1, stride1 1, max_displacement/stride2 = 4, stride2 = 2 (model.py:24 builds
// Correlation(9, 1, 9, 1, 2)):
//   out[n, tc, oy, ox] = sum_c f1[n,c,oy+off,ox+off] * f2[n,c,oy+off+2tj,ox+off+2ti] / divisor
// with tc = (tj+4)*9 + (ti+4) (raster) or the CostVolumeLayer order, zeros outside the image
// (the reference's zero-filled padded scratch, cu:10-32), off = max_displacement - pad_size.
//
// Why row parity: with stride-2 displacements an output row oy only ever meets f2 rows of its
// own parity (oy + off + 2tj).  A tile of 16 output rows of ONE parity (32 image rows) needs
// 16 + 8 f2 rows instead of the 32 a 16x16 tile of consecutive rows needs, and the two parity
// halves of the image are disjoint problems (no f1/f2 row is staged by both).
//
// Structure: one workgroup = one tile = 16 parity rows x 16 columns of one image, all 81
// displacements.  288 lanes = 9 displacement rows tj x 16 rows x 2 eight-pixel segments; lane
// (tj, r, s) accumulates 8 pixels x 9 ti = 72 fp32 sums.  Per channel a lane reads its two f1
// quads and the six f2 quads of its window (8 x ds_read_b128 for 72 FMAs: 0.44 LDS floats per
// FMA against 0.67 for 4-pixel lanes).  Channels stream through an NS-deep LDS ring filled by
// LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction): per channel three f2
// pieces (24 rows x 32 columns) and one f1 piece (16 x 16); out-of-image quads get an
// out-of-range voffset, which the buffer unit turns into zeros.  Quad slots are XOR-swizzled
// per row on the DMA source (destination linear) so every ds_read_b128 lane group reads 16
// distinct 16-byte bank slots (derivation at par_f2_swz / par_f1_swz).
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>

#include "../pwc-net_pytorch_amd/csrc/pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace par {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// f2 LDS row rho holds logical quad q at slot q ^ par_f2_swz(rho).  A ds_read_b128 lane group
// ({0-3,12-15,20-27} and the like) of lanes (r, s) = (lane/2 % 16, lane % 2) spans 8 rows whose
// residues mod 8 are all distinct and both segments; rows 128 B apart alternate 256-B halves
// by rho & 1, and within a half the four rows (rho >> 1) & 3 XOR the quads {u, u+2} of the two
// segments with {0, 1, 4, 5}: 8 distinct slots, so 16 distinct 16-B slots = all 64 banks.
__host__ __device__ __forceinline__ int par_f2_swz(int rho) {
  return ((rho >> 1) & 1) | (((rho >> 2) & 1) << 2);
}
// f1 rows are 64 B (4 quads): a lane group's 8 rows pair up by rho & 3, the pairs differ in
// bit 2, and the group reads quads {h, 2+h}: XOR bit 0 by row bit 2 separates the pairs.
__host__ __device__ __forceinline__ int par_f1_swz(int r) { return (r >> 2) & 1; }

template <int CC_, int NS_>
struct ParTile {
  static constexpr int DR = 4, S = 2, D = 9;
  static constexpr int TR = 16;            // parity rows per tile
  static constexpr int TX = 16, PX = 8, NSEG = 2;
  static constexpr int R2 = TR + 2 * DR;   // 24 f2 rows (halo DR parity rows each side)
  static constexpr int X2 = 32;            // f2 row: columns x0-8 .. x0+23
  static constexpr int CC = CC_, NS = NS_;
  static constexpr int F2_FLOATS = R2 * X2;
  static constexpr int F1_FLOATS = TR * TX;
  static constexpr int CH_FLOATS = F2_FLOATS + F1_FLOATS;
  static constexpr int STAGE_FLOATS = CC * CH_FLOATS;
  static constexpr int LDS_BYTES = NS * STAGE_FLOATS * 4;
  static constexpr int THREADS = D * TR * NSEG;  // 288: four full waves + one half wave
  static constexpr int F2P = R2 / 8;             // 1 KiB pieces (8 rows x 8 quads)
  static constexpr int PPC = F2P + 1;            // + one f1 piece (16 rows x 4 quads)
  static constexpr int PIECES = CC * PPC;
  static constexpr int ISSUERS = 4;
  static constexpr int PPW = PIECES / ISSUERS;
  static_assert(PIECES % ISSUERS == 0, "uniform DMA pieces per issuing wave");
  static_assert((NS - 2) * PPW <= 63, "vmcnt range");
  static_assert(NS >= 2, "ring depth");
  static_assert((NS - 1) * STAGE_FLOATS * 4 + (CC - 1) * CH_FLOATS * 4 < 65536,
                "slot + channel offsets fit the ds offset field");
};

// Eight ds_read_b128 (two f1 quads, six window quads) + lgkmcnt(0) in one statement: a
// compiler-visible LDS load would get an s_waitcnt vmcnt(0) (hipcc cannot prove it misses the
// in-flight LDS-DMA), which would drain the ring every channel.
template <int OFF>
__device__ __forceinline__ void lds_read8(const uint32_t (&a)[8], f32x4 (&r)[8]) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  asm volatile(
      "ds_read_b128 %0, %8 offset:%16\n\t"
      "ds_read_b128 %1, %9 offset:%16\n\t"
      "ds_read_b128 %2, %10 offset:%16\n\t"
      "ds_read_b128 %3, %11 offset:%16\n\t"
      "ds_read_b128 %4, %12 offset:%16\n\t"
      "ds_read_b128 %5, %13 offset:%16\n\t"
      "ds_read_b128 %6, %14 offset:%16\n\t"
      "ds_read_b128 %7, %15 offset:%16\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
        "=&v"(r[6]), "=&v"(r[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "n"(OFF)
      : "memory");
}

template <class G, int CI>
__device__ __forceinline__ void par_stage(const uint32_t (&a)[8], float (&lo)[G::D][4],
                                          float (&hi)[G::D][4]) {
  if constexpr (CI < G::CC) {
    f32x4 v[8];
    lds_read8<CI * G::CH_FLOATS * 4>(a, v);
    const f32x4 wl[5] = {v[2], v[3], v[4], v[5], v[6]};
    const f32x4 wh[5] = {v[3], v[4], v[5], v[6], v[7]};
    corr_fma_pairs_s2<G::D, 5>(lo, v[0], wl);
    corr_fma_pairs_s2<G::D, 5>(hi, v[1], wh);
    par_stage<G, CI + 1>(a, lo, hi);
  }
}

// DMA of one stage: issuer wave w owns pieces w*PPW .. w*PPW+PPW-1 (channel p / PPC, piece
// p % PPC of it).  The buffer resource's base moves to the stage's first channel (scalar work
// only) so the per-lane voffsets are stage-invariant; channels past C read zeros because
// num_records shrinks with the base.
template <class G>
__device__ __forceinline__ void par_issue(int stage, int c_begin, int wave, uint32_t plane,
                                          uint32_t lds0, const float* img1, const float* img2,
                                          uint32_t img_bytes, const uint32_t (&src_off)[G::PPW],
                                          const uint32_t (&dst_off)[G::PPW],
                                          const bool (&from_f2)[G::PPW]) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (wave >= G::ISSUERS) return;
  const uint32_t cbytes = (uint32_t)(c_begin + stage * G::CC) * plane * 4u;
  const int nrec = cbytes < img_bytes ? (int)(img_bytes - cbytes) : 0;
  const uint32_t sbase = lds0 + (uint32_t)((stage % G::NS) * G::STAGE_FLOATS) * 4u;
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
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

#ifdef PWC_PAR_ABLATION  // diagnostic build, bits: 1 = no FMA work, 2 = no DMA, 4 = no stores
__constant__ int g_par_abl;
#endif

template <class G>
__global__ __launch_bounds__(G::THREADS, 4) void corr_fwd_par(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    int C, int H, int W, int Ho, int Wo, int off, int layout, float divisor, float inv_divisor,
    int n_tr, int n_tx) {
  extern __shared__ __attribute__((aligned(16))) float lds[];

  // tile order: image-major, then parity, then tile row, then tile column; the XCD remap puts
  // consecutive tiles (which share f2 halo rows and columns) on one XCD's L2
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % n_tx;
  const int tr = (t / n_tx) % n_tr;
  const int p = (t / (n_tx * n_tr)) & 1;
  const int n = t / (n_tx * n_tr * 2);
  const int R0 = tr * G::TR;  // first parity row of the tile: output row 2*R0 + p
  const int x0 = tx * G::TX;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tj = threadIdx.x >> 5;         // 0..8 (displacement tj - 4)
  const int r = (threadIdx.x >> 1) & 15;   // parity row in the tile
  const int s = threadIdx.x & 1;           // 8-pixel segment

  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t img_bytes = (uint32_t)C * plane * 4u;  // < 2^31, checked by the launcher
  const float* img1 = in1 + (size_t)n * C * plane;
  const float* img2 = in2 + (size_t)n * C * plane;
  const uint32_t lds0 = lds_addr(lds);

  // ---- DMA plan (issuer waves): source byte offset for channel 0 (or OOB) and LDS offset ----
  uint32_t src_off[G::PPW];
  uint32_t dst_off[G::PPW];
  bool from_f2[G::PPW];
  constexpr uint32_t kOOB = 0x80000000u;  // >= num_records: the buffer unit returns zeros
  if (wave < G::ISSUERS) {
#pragma unroll
    for (int i = 0; i < G::PPW; ++i) {
      const int pc = wave * G::PPW + i;
      const int cc = pc / G::PPC;
      const int k = pc % G::PPC;
      uint32_t dst = (uint32_t)(cc * G::CH_FLOATS) * 4u;
      int gy, gx;
      if (k < G::F2P) {
        const int rho = 8 * k + (lane >> 3);
        const int q = (lane & 7) ^ par_f2_swz(rho);
        gy = 2 * (R0 + rho - G::DR) + p + off;
        gx = x0 + off - 2 * G::DR + 4 * q;
        dst += (uint32_t)(8 * k * G::X2) * 4u;
      } else {
        const int rr = lane >> 2;
        const int q = (lane & 3) ^ par_f1_swz(rr);
        gy = 2 * (R0 + rr) + p + off;
        gx = x0 + off + 4 * q;
        dst += (uint32_t)G::F2_FLOATS * 4u;
      }
      const bool ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
      src_off[i] = ok ? ((uint32_t)cc * plane + (uint32_t)(gy * W + gx)) * 4u : kOOB;
      dst_off[i] = dst;
      from_f2[i] = k < G::F2P;
    }
  }

  // ---- lane-constant LDS read offsets (bytes inside a channel block) ----
  const int rho = r + tj;
  uint32_t off8[8];
  off8[0] = (uint32_t)(G::F2_FLOATS + r * G::TX + (((2 * s) ^ par_f1_swz(r)) << 2)) * 4u;
  off8[1] = (uint32_t)(G::F2_FLOATS + r * G::TX + (((2 * s + 1) ^ par_f1_swz(r)) << 2)) * 4u;
#pragma unroll
  for (int u = 0; u < 6; ++u)
    off8[2 + u] = (uint32_t)(rho * G::X2 + (((2 * s + u) ^ par_f2_swz(rho)) << 2)) * 4u;

  float lo[G::D][4], hi[G::D][4];
#pragma unroll
  for (int a = 0; a < G::D; ++a)
#pragma unroll
    for (int k = 0; k < 4; ++k) lo[a][k] = hi[a][k] = 0.f;

  const int nst = (C + G::CC - 1) / G::CC;
#pragma unroll
  for (int st = 0; st < G::NS - 1; ++st)
    if (st < nst)
      par_issue<G>(st, 0, wave, plane, lds0, img1, img2, img_bytes, src_off, dst_off, from_f2);

  for (int st = 0; st < nst; ++st) {
    if (wave < G::ISSUERS) {
      if (nst - 1 - st >= G::NS - 2)
        wait_vmcnt<(G::NS - 2) * G::PPW>();
      else
        wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
#ifdef PWC_PAR_ABLATION
    if (!(g_par_abl & 2))
#endif
    if (st + G::NS - 1 < nst)
      par_issue<G>(st + G::NS - 1, 0, wave, plane, lds0, img1, img2, img_bytes, src_off,
                   dst_off, from_f2);
#ifdef PWC_PAR_ABLATION
    if (g_par_abl & 1) continue;
#endif
    const uint32_t sb = lds0 + (uint32_t)((st % G::NS) * G::STAGE_FLOATS) * 4u;
    uint32_t a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = sb + off8[u];
    par_stage<G, 0>(a, lo, hi);
  }

  // ---- epilogue: out = acc / divisor (cu:100); a power-of-two divisor is an exact scale ----
  const int oy = 2 * (R0 + r) + p;
  const int ox = x0 + 8 * s;
  if (oy >= Ho || ox >= Wo) return;
#ifdef PWC_PAR_ABLATION
  if (g_par_abl & 4) {
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
#pragma unroll
  for (int ti = 0; ti < G::D; ++ti) {
    const int oc = out_channel(layout, tj - G::DR, ti - G::DR, G::DR, G::D, G::S);
    float* orow = out + (((size_t)n * OC + oc) * Ho + oy) * Wo + ox;
    float4 v0, v1;
    if (pow2) {
      v0 = make_float4(lo[ti][0] * inv_divisor, lo[ti][1] * inv_divisor,
                       lo[ti][2] * inv_divisor, lo[ti][3] * inv_divisor);
      v1 = make_float4(hi[ti][0] * inv_divisor, hi[ti][1] * inv_divisor,
                       hi[ti][2] * inv_divisor, hi[ti][3] * inv_divisor);
    } else {
      v0 = make_float4(lo[ti][0] / divisor, lo[ti][1] / divisor, lo[ti][2] / divisor,
                       lo[ti][3] / divisor);
      v1 = make_float4(hi[ti][0] / divisor, hi[ti][1] / divisor, hi[ti][2] / divisor,
                       hi[ti][3] / divisor);
    }
    *reinterpret_cast<float4*>(orow) = v0;
    if (has_hi) *reinterpret_cast<float4*>(orow + 4) = v1;
  }
}

template <class G>
static hipError_t launch_par(const void* in1, const void* in2, void* out, int B, int C, int H,
                             int W, int Ho, int Wo, int off, int layout, float divisor,
                             hipStream_t stream) {
  const int n_tr = ((Ho + 1) / 2 + G::TR - 1) / G::TR;  // parity-0 rows: ceil(Ho / 2)
  const int n_tx = (Wo + G::TX - 1) / G::TX;
  const long long nblk = (long long)B * 2 * n_tr * n_tx;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_fwd_par<G>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL((corr_fwd_par<G>), dim3((unsigned)nblk), dim3(G::THREADS), G::LDS_BYTES,
                        stream, ev0, ev1, 0, (const float*)in1, (const float*)in2, (float*)out,
                        C, H, W, Ho, Wo, off, layout, divisor, inv, n_tr, n_tx);
  return hipGetLastError();
}

using ParA = ParTile<2, 6>;  // 48 KiB: 3 workgroups per CU, 4 stages (8 channels) in flight
using ParB = ParTile<2, 4>;  // 32 KiB: 5 per CU (LDS), 2 stages in flight
using ParC = ParTile<4, 4>;  // 64 KiB: 2 per CU, 2 stages (8 channels) in flight
using ParD = ParTile<1, 10>; // 40 KiB: 8 single-channel stages in flight

static int par_cfg() {
  static int v = -1;
  if (v < 0) {
    const char* s = std::getenv("PWC_PAR_CFG");
    v = 0;
    if (s && s[0] >= 'A' && s[0] <= 'D' && s[1] == 0) v = s[0] - 'A';
  }
  return v;
}

}  // namespace par

// hipErrorNotSupported: shape / alignment outside what the parity-tile kernel handles.
hipError_t corr_forward_par_f32(const void* in1, const void* in2, void* out, int B, int C,
                                int H, int W, int Ho, int Wo, int off, int dr, int s2,
                                int layout, float divisor, hipStream_t stream) {
  if (!(dr == 4 && s2 == 2)) return hipErrorNotSupported;
  if (W % 4 || Wo % 4 || off % 4) return hipErrorNotSupported;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16)
    return hipErrorNotSupported;
  if ((size_t)C * H * W * 4 >= 0x7ffffff0ull) return hipErrorNotSupported;
  switch (par::par_cfg()) {
    case 1: return par::launch_par<par::ParB>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    case 2: return par::launch_par<par::ParC>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    case 3: return par::launch_par<par::ParD>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
    default: return par::launch_par<par::ParA>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream);
  }
}

}  // namespace pwc
