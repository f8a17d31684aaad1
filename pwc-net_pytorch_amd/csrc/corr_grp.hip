// corr_grp.hip — correlation forward for the coarse pyramid levels (k 1, s1 1, d = 4, s2 = 2).
//
// Semantics as corr_ring.hip (correlation_cuda_kernel.cu:34-106): out[n, tc, oy, ox] =
// sum_c f1[n,c,oy+off,ox+off] * f2[n,c,oy+off+tj*2,ox+off+ti*2] / divisor, zeros outside.
//
// The coarse levels (l0..l3 of PWC-Net: 6x7 .. 48x56 pixels, 192 .. 64 channels, B = 8) have
// too few 16x16 tiles to fill 256 CUs, and their output volumes are LARGER than their inputs,
// so splitting channels across workgroups through a global partial-sum volume plus a reduce
// launch costs more than the correlation itself.  Here the channel split stays inside the
// workgroup:
//   * one workgroup = one 16x16 output tile x JG displacement rows tj x K channel groups,
//     one wave per (group, tj); a tile's 9 rows spread over 9/JG workgroups;
//   * the f1 tile and the f2 rows those JG displacement rows need (16 + 2(JG-1) rows x 32
//     columns) of K*CC channels form a stage, streamed into an NS-deep LDS ring by LDS-DMA:
//     16-byte pieces when rows are 16-B aligned (W % 4 == 0), else dword pieces whose per-lane
//     source addresses absorb the misalignment; out-of-image elements read zeros through the
//     buffer range check; the f2 quad slots are XOR-swizzled as in corr_ring.hip;
//   * group k's wave accumulates 4 pixels x 9 ti over its CC channels of every stage
//     (6 x ds_read_b128 + 36 FMA per channel, the corr_ring inner loop);
//   * the K partial accumulators are summed through LDS in a fixed binary tree (deterministic)
//     and group 0 writes the 81-channel output.
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace grp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Six ds_read_b128 + lgkmcnt(0) in one statement: compiler-visible LDS loads would each get a
// vmcnt(0) (hipcc cannot prove they miss the in-flight LDS-DMA).
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

template <int JG_, int K_, int CC_, int NS_, bool DW_>
struct GrpTile {
  static constexpr int JG = JG_, K = K_, CC = CC_, NS = NS_;
  static constexpr bool DW = DW_;
  static constexpr int DR = 4, S = 2, D = 9, TY = 16, TX = 16, NQ = 4, PX = 4, X2 = 32;
  static constexpr int NW = JG * K, THREADS = 64 * NW;
  static constexpr int R2N = TY + S * (JG - 1);                   // f2 rows the waves read
  static constexpr int R2 = DW ? R2N : ((R2N + 7) / 8) * 8;       // rows staged
  static constexpr int F2_FLOATS = R2 * X2, F1_FLOATS = TY * TX;
  static constexpr int CH_FLOATS = F2_FLOATS + F1_FLOATS;
  static constexpr int NCH = K * CC;                              // channels per stage
  static constexpr int STAGE_FLOATS = NCH * CH_FLOATS;
  static constexpr int PIECE_FLOATS = DW ? 64 : 256;              // one wave-instruction
  static constexpr int F2P = F2_FLOATS / PIECE_FLOATS, F1P = F1_FLOATS / PIECE_FLOATS;
  static constexpr int PPC = F2P + F1P;                           // pieces per channel
  static constexpr int PPW = NCH * PPC / NW;                      // pieces per wave per stage
  static constexpr int RING_BYTES = NS * STAGE_FLOATS * 4;
  static constexpr int RED_BYTES = (K / 2) * JG * D * 64 * 16;
  static constexpr int LDS_BYTES = RING_BYTES > RED_BYTES ? RING_BYTES : RED_BYTES;
  static_assert(D % JG == 0, "tj groups");
  static_assert(K >= 1 && (K & (K - 1)) == 0, "binary-tree reduction over K groups");
  static_assert(F2_FLOATS % PIECE_FLOATS == 0 && F1_FLOATS % PIECE_FLOATS == 0, "pieces");
  static_assert((NCH * PPC) % NW == 0, "uniform DMA pieces per wave");
  static_assert((NS - 2) * PPW <= 63, "vmcnt range");
  static_assert(NS >= 2 && THREADS <= 1024, "ring / workgroup");
  static_assert((CC - 1) * CH_FLOATS * 4 < 65536, "channel offset immediate");
};

// DMA of stage `stage`: wave w owns pieces p = w + i*NW of every stage (channel kc = p / PPC,
// piece pc = p % PPC of that channel); src_off[i] is the lane's byte offset inside the channel
// plane (or past num_records: zeros).  The resource base sits at the piece's channel, so the
// vector offsets are stage-invariant and channels past C fall outside num_records.
template <class G>
__device__ __forceinline__ void grp_issue(int stage, int c_begin, int wave, uint32_t plane,
                                          uint32_t lds0, const float* img1, const float* img2,
                                          uint32_t img_bytes, const uint32_t (&src_off)[G::PPW]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t sbase = lds0 + (uint32_t)((stage % G::NS) * G::STAGE_FLOATS) * 4u;
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    const int p = wave + i * G::NW;
    const int kc = p / G::PPC, pc = p % G::PPC;
    const bool f2 = pc < G::F2P;
    const uint32_t c = (uint32_t)(c_begin + stage * G::NCH + kc);
    const uint32_t cbytes = c * plane * 4u;
    const int nrec = cbytes < img_bytes ? (int)(img_bytes - cbytes) : 0;
    const uint64_t b = (uint64_t)(uintptr_t)(f2 ? img2 : img1) + (uint64_t)cbytes;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
        __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
    const uint32_t dst = sbase + (uint32_t)(kc * G::CH_FLOATS * 4) +
                         (f2 ? (uint32_t)(pc * G::PIECE_FLOATS * 4)
                             : (uint32_t)((G::F2_FLOATS + (pc - G::F2P) * G::PIECE_FLOATS) * 4));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(uintptr_t)dst, G::DW ? 4 : 16, src_off[i],
        0, 0, 0);
  }
#endif
}

// CC channels of one stage: per channel 6 LDS quads (f1 + 5 window quads) and 36 FMAs.
template <class G, int I>
__device__ __forceinline__ void grp_stage(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                          uint32_t a4, uint32_t a5, float (&acc)[G::D][G::PX]) {
  if constexpr (I < G::CC) {
    f32x4 fa, b0, b1, b2, b3, b4;
    lds_read6<I * G::CH_FLOATS * 4>(a0, a1, a2, a3, a4, a5, fa, b0, b1, b2, b3, b4);
    const f32x4 b[5] = {b0, b1, b2, b3, b4};
    corr_fma_pairs_s2<G::D, 5>(acc, fa, b);
    grp_stage<G, I + 1>(a0, a1, a2, a3, a4, a5, acc);
  }
}

template <class G>
__global__ __launch_bounds__(G::THREADS) void corr_fwd_grp(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    int C, int H, int W, int Ho, int Wo, int off, int layout, float divisor, float inv_divisor,
    int n_ty, int n_tx, int vec_out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NTJG = G::D / G::JG;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tjg = t % NTJG;
  const int tile = t / NTJG;
  const int tx_tile = tile % n_tx;
  const int ty_tile = (tile / n_tx) % n_ty;
  const int n = tile / (n_tx * n_ty);
  const int oy0 = ty_tile * G::TY, ox0 = tx_tile * G::TX;
  const int y1 = oy0 + off, x1 = ox0 + off;         // f1 tile origin
  const int tj0 = tjg * G::JG;
  const int f2y0 = y1 + (tj0 - G::DR) * G::S;        // image row of f2 tile row 0
  const int f2x0 = x1 - G::DR * G::S;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kgrp = wave / G::JG, jj = wave % G::JG;
  const int ty = lane >> 2, q = lane & 3;

  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t img_bytes = (uint32_t)C * plane * 4u;  // < 2^31, checked by the launcher
  const float* img1 = in1 + (size_t)n * C * plane;
  const float* img2 = in2 + (size_t)n * C * plane;
  const uint32_t lds0 = lds_addr(lds);

  // ---- per-lane DMA source offsets of this wave's pieces ----
  constexpr uint32_t kOOB = 0x80000000u;
  uint32_t src_off[G::PPW];
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    const int p = wave + i * G::NW;
    const int pc = p % G::PPC;
    int gy, gx;
    bool ok;
    if (G::DW) {
      if (pc < G::F2P) {
        const int F = pc * 64 + lane;
        const int r = F / G::X2, pos = F % G::X2;
        const int srcq = (pos >> 2) ^ (((r >> 1) & 1) << 2);
        gy = f2y0 + r;
        gx = f2x0 + 4 * srcq + (pos & 3);
      } else {
        const int F = (pc - G::F2P) * 64 + lane;
        gy = y1 + F / G::TX;
        gx = x1 + F % G::TX;
      }
      ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
    } else {
      if (pc < G::F2P) {
        const int r = pc * 8 + (lane >> 3);
        const int srcq = (lane & 7) ^ (((r >> 1) & 1) << 2);
        gy = f2y0 + r;
        gx = f2x0 + 4 * srcq;
      } else {
        gy = y1 + (lane >> 2);
        gx = x1 + 4 * (lane & 3);
      }
      ok = gy >= 0 && gy < H && gx >= 0 && gx + 3 < W;  // W % 4 == 0: whole quads
    }
    src_off[i] = ok ? (uint32_t)(gy * W + gx) * 4u : kOOB;
  }

  // ---- lane LDS read addresses (channel kgrp*CC of slot 0) ----
  const uint32_t cbase = lds0 + (uint32_t)(kgrp * G::CC * G::CH_FLOATS) * 4u;
  const int r2 = ty + G::S * jj;
  const int sw = ((r2 >> 1) & 1) << 2;
  uint32_t woff[5];
#pragma unroll
  for (int u = 0; u < 5; ++u) woff[u] = cbase + (uint32_t)(r2 * G::X2 + (((q + u) ^ sw) << 2)) * 4u;
  const uint32_t aoff = cbase + (uint32_t)(G::F2_FLOATS + ty * G::TX + (q << 2)) * 4u;

  float acc[G::D][G::PX];
#pragma unroll
  for (int a = 0; a < G::D; ++a)
#pragma unroll
    for (int k = 0; k < G::PX; ++k) acc[a][k] = 0.f;

  const int nst = (C + G::NCH - 1) / G::NCH;
#pragma unroll
  for (int s = 0; s < G::NS - 1; ++s)
    if (s < nst) grp_issue<G>(s, 0, wave, plane, lds0, img1, img2, img_bytes, src_off);

  // (PWC_GRP_ABL: diagnostic builds only -- bit 1 drops the compute, 2 the DMA, 4 the K
  // reduction, 8 the stage loop)
#if defined(PWC_GRP_ABL) && (PWC_GRP_ABL & 8)
  for (int st = 0; st < 0; ++st) {
#else
  for (int st = 0; st < nst; ++st) {
#endif
#if !defined(PWC_GRP_ABL) || (PWC_GRP_ABL & 2) == 0
    if (nst - 1 - st >= G::NS - 2)
      wait_vmcnt<(G::NS - 2) * G::PPW>();
    else
      wait_vmcnt<0>();
#endif
    __builtin_amdgcn_s_barrier();
#if !defined(PWC_GRP_ABL) || (PWC_GRP_ABL & 2) == 0
    if (st + G::NS - 1 < nst)
      grp_issue<G>(st + G::NS - 1, 0, wave, plane, lds0, img1, img2, img_bytes, src_off);
#endif
#if defined(PWC_GRP_ABL) && (PWC_GRP_ABL & 1)
    continue;
#endif
    const uint32_t sb = (uint32_t)((st % G::NS) * G::STAGE_FLOATS) * 4u;
    const uint32_t a0 = aoff + sb, a1 = woff[0] + sb, a2 = woff[1] + sb, a3 = woff[2] + sb,
                   a4 = woff[3] + sb, a5 = woff[4] + sb;
    grp_stage<G, 0>(a0, a1, a2, a3, a4, a5, acc);
  }

  // ---- K-group reduction through LDS (fixed tree: deterministic) ----
  f32x4* red = reinterpret_cast<f32x4*>(lds);
#if defined(PWC_GRP_ABL) && (PWC_GRP_ABL & 4)
  if constexpr (false) {
#else
  if constexpr (G::K > 1) {
#endif
    __syncthreads();  // ring reads done (all DMA was waited for in the last stages)
#pragma unroll
    for (int h = G::K / 2; h >= 1; h /= 2) {
      if (kgrp >= h && kgrp < 2 * h) {
        f32x4* dst = red + ((kgrp - h) * G::JG + jj) * G::D * 64 + lane;
#pragma unroll
        for (int ti = 0; ti < G::D; ++ti)
          dst[ti * 64] = f32x4{acc[ti][0], acc[ti][1], acc[ti][2], acc[ti][3]};
      }
      __syncthreads();
      if (kgrp < h) {
        const f32x4* src = red + (kgrp * G::JG + jj) * G::D * 64 + lane;
#pragma unroll
        for (int ti = 0; ti < G::D; ++ti) {
          const f32x4 v = src[ti * 64];
          acc[ti][0] += v.x;
          acc[ti][1] += v.y;
          acc[ti][2] += v.z;
          acc[ti][3] += v.w;
        }
      }
      if (h > 1) __syncthreads();
    }
  }
  if (kgrp != 0) return;

  // ---- epilogue: out = acc / divisor (cu:100); a power-of-two divisor is an exact scale ----
  const int oy = oy0 + ty;
  const int ox = ox0 + 4 * q;
  if (oy >= Ho || ox >= Wo) return;
  const int OC = G::D * G::D;
  const int tj = tj0 + jj - G::DR;
  const bool pow2 = inv_divisor != 0.f;
#pragma unroll
  for (int ti = 0; ti < G::D; ++ti) {
    const int oc = out_channel(layout, tj, ti - G::DR, G::DR, G::D, G::S);
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = pow2 ? acc[ti][k] * inv_divisor : acc[ti][k] / divisor;
    float* orow = out + (((size_t)n * OC + oc) * Ho + oy) * Wo;
    if (vec_out) {
      *reinterpret_cast<float4*>(orow + ox) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (ox + k < Wo) orow[ox + k] = v[k];
    }
  }
}

template <class G>
hipError_t launch(const void* in1, const void* in2, void* out, int B, int C, int H, int W,
                  int Ho, int Wo, int off, int layout, float divisor, hipStream_t stream) {
  const int n_ty = (Ho + G::TY - 1) / G::TY;
  const int n_tx = (Wo + G::TX - 1) / G::TX;
  const long long nblk = (long long)B * n_ty * n_tx * (G::D / G::JG);
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_fwd_grp<G>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  const int vec_out = (Wo % 4 == 0) && ((uintptr_t)out % 16 == 0);
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL((corr_fwd_grp<G>), dim3((unsigned)nblk), dim3(G::THREADS), G::LDS_BYTES,
                        stream, ev0, ev1, 0, (const float*)in1, (const float*)in2, (float*)out, C,
                        H, W, Ho, Wo, off, layout, divisor, inv, n_ty, n_tx, vec_out);
  return hipGetLastError();
}

// Configurations (JG, K, CC, NS, dword DMA): round 2 measured eight ring shapes (A..H); the two
// the dispatcher picks stayed in the library.
using GC = GrpTile<1, 8, 1, 2, false>;  // 48 KiB, 8 waves
using GD = GrpTile<3, 2, 3, 3, false>;  // 6 waves, 3 tj rows per workgroup, 72 KiB
using GCd = GrpTile<1, 8, 1, 2, true>;
using GDd = GrpTile<3, 2, 3, 3, true>;

}  // namespace grp

// hipErrorNotSupported outside the shapes this kernel handles (then the caller falls back).
hipError_t corr_forward_grp_f32(const void* in1, const void* in2, void* out, int B, int C, int H,
                                int W, int Ho, int Wo, int off, int dr, int s2, int layout,
                                float divisor, hipStream_t stream) {
  using namespace grp;
  if (!(dr == 4 && s2 == 2)) return hipErrorNotSupported;
  if ((size_t)C * H * W * 4 >= 0x7ffffff0ull) return hipErrorNotSupported;
  const bool dw = !(W % 4 == 0 && off % 4 == 0 && (uintptr_t)in1 % 16 == 0 &&
                    (uintptr_t)in2 % 16 == 0);
  // one tj row per workgroup (9 workgroups per tile) and 8 channel groups in a 2-deep ring (3
  // workgroups per CU); 3 rows per workgroup once that fills the chip (measured: D at 48x56
  // (B 8), C at 24x28)
  const long long tiles = (long long)B * ((Ho + 15) / 16) * ((Wo + 15) / 16);
  const bool d = tiles * 3 >= 256;
#define PWC_GRP_LAUNCH(T) \
  launch<T>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor, stream)
  if (d) return dw ? PWC_GRP_LAUNCH(GDd) : PWC_GRP_LAUNCH(GD);
  return dw ? PWC_GRP_LAUNCH(GCd) : PWC_GRP_LAUNCH(GC);
#undef PWC_GRP_LAUNCH
}

}  // namespace pwc
