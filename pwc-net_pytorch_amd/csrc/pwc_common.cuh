// pwc_common.cuh — shared device helpers for the gfx950 hot-path kernels.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pwc {

// ---- element conversion (fp32 accumulate for every storage type) ----
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(__half v) { return __half2float(v); }
__device__ __forceinline__ float to_f32(__hip_bfloat16 v) { return __bfloat162float(v); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ __half from_f32<__half>(float v) { return __float2half(v); }
template <> __device__ __forceinline__ __hip_bfloat16 from_f32<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}

// Correlation channel layouts.
//   RASTER: correlation_cuda_kernel.cu:98  tc = (tj+dr)*D + (ti+dr)
//   CVL:    modules.py:58-72 CostVolumeLayer order, displacement (dy,dx) = (tj*s2, ti*s2)
enum Layout : int { kRaster = 0, kCvl = 1 };

// The correlation forward's first dispatch stages (corr_fwd.hip, corr_forward_path).
enum CorrPath : int { kPathOther = 0, kPathStream = 1, kPathBand = 2, kPathRows = 3 };
int corr_forward_path(const void* in1, const void* in2, const void* out, int B, int C, int H,
                      int W, int pad, int k, int md, int s1, int s2, int layout, int dtype);

// CostVolumeLayer channel of displacement (dy, dx) for search range sr (modules.py:58-72):
// 0 -> (0,0); for i = 1..sr the block of 4+4*sr channels starting at 1+(i-1)*(4+4sr) holds
// (-i,0),(+i,0),(0,-i),(0,+i) then for j = 1..sr (-i,-j),(+i,+j),(-i,+j),(+i,-j).
// Note (dy, dx) = (0, ±i) belongs to the block of i = |dx|, and (±i, ±j) to block i = |dy|.
__host__ __device__ __forceinline__ int cvl_channel(int dy, int dx, int sr) {
  if (dy == 0 && dx == 0) return 0;
  if (dx == 0) {
    int i = dy < 0 ? -dy : dy;
    return 1 + (i - 1) * (4 + 4 * sr) + (dy < 0 ? 0 : 1);
  }
  if (dy == 0) {
    int i = dx < 0 ? -dx : dx;
    return 1 + (i - 1) * (4 + 4 * sr) + (dx < 0 ? 2 : 3);
  }
  int i = dy < 0 ? -dy : dy;
  int j = dx < 0 ? -dx : dx;
  int base = 1 + (i - 1) * (4 + 4 * sr) + 4 + (j - 1) * 4;
  if (dy < 0 && dx < 0) return base + 0;
  if (dy > 0 && dx > 0) return base + 1;
  if (dy < 0) return base + 2;  // (-i, +j)
  return base + 3;              // (+i, -j)
}

__host__ __device__ __forceinline__ int out_channel(int layout, int tj, int ti, int dr, int D,
                                                    int s2) {
  return layout == kCvl ? cvl_channel(tj * s2, ti * s2, dr)
                        : (tj + dr) * D + (ti + dr);
}

// ---- correlation inner product, stride-2 displacements ----
// One channel of a lane's 4 pixels x D displacements: acc[ti][k] += a[k] * w[k + 2*ti] with w the
// lane's f2 window (quads b[0..]).  Both operands of every pixel PAIR (k, k+1) sit in aligned
// register pairs (a.xy/a.zw, and w[2ti..2ti+1] / w[2ti+2..2ti+3] are halves of window quads),
// so the 4*D FMAs issue as 2*D v_pk_fma_f32.  Same per-element fp32 fma as the scalar form
// (bitwise), half the instructions -- and measured 2.1x the scalar loop's throughput under
// full load, where the chip is power-limited and fewer instructions hold a higher clock.
typedef float pk_f32x4 __attribute__((ext_vector_type(4)));
typedef float pk_f32x2 __attribute__((ext_vector_type(2)));

template <int D, int NQ>
__device__ __forceinline__ void corr_fma_pairs_s2(float (&acc)[D][4], const pk_f32x4& a,
                                                  const pk_f32x4 (&b)[NQ]) {
  static_assert(NQ * 4 >= 4 + 2 * (D - 1), "window covers all displacements");
#pragma unroll
  for (int ti = 0; ti < D; ++ti) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * h + 2 * ti;  // even: a register pair inside quad j / 4
      const pk_f32x4 q = b[j >> 2];
      const pk_f32x2 w2 = (j & 2) ? pk_f32x2{q.z, q.w} : pk_f32x2{q.x, q.y};
      const pk_f32x2 a2 = h ? pk_f32x2{a.z, a.w} : pk_f32x2{a.x, a.y};
      pk_f32x2 c2 = {acc[ti][2 * h], acc[ti][2 * h + 1]};
      c2 = __builtin_elementwise_fma(a2, w2, c2);
      acc[ti][2 * h] = c2.x;
      acc[ti][2 * h + 1] = c2.y;
    }
  }
}

// Output stores of the big result volumes.  PWC_STORE_POLICY (build-time, for measurement):
// 0 = plain, 1 = nontemporal (nt, default: the l4 correlation 19.1 -> 17.1 us at an unchanged
// bench step), 2 = write-through (sc1: the line is not kept dirty in the
// XCD's L2, so the kernel boundary has less to write back).
#ifndef PWC_STORE_POLICY
#define PWC_STORE_POLICY 1
#endif
typedef float st_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_out4(float* p, st_f32x4 v) {
#if PWC_STORE_POLICY == 1
  __builtin_nontemporal_store(v, reinterpret_cast<st_f32x4*>(p));
#elif PWC_STORE_POLICY == 2
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#else
  *reinterpret_cast<st_f32x4*>(p) = v;
#endif
}
__device__ __forceinline__ void st_out1(float* p, float v) {
#if PWC_STORE_POLICY == 1
  __builtin_nontemporal_store(v, p);
#elif PWC_STORE_POLICY == 2
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#else
  *p = v;
#endif
}

// Output epilogue of the model-path correlation kernels: image n's
// 81-channel block starts at out + n * ostride elements (ostride 0: dense, n * 81 * H * W) --
// so a kernel can write straight into the corr slice of model.py:89/91's cat([x1, corr, flow])
// buffer -- and every value goes through leaky_relu with `slope` (model.py:84's in-place
// F.leaky_relu_, slope 0.01; slope 1 is the identity, bit for bit).
struct OutEpi {
  long long ostride;
  float slope;
};

__device__ __forceinline__ float epi_act(float v, float slope) { return v > 0.f ? v : v * slope; }

// Host side: the descriptor the next launch of this thread uses (capi.hip sets it around a
// pwc_corr_forward_into call; default dense / identity).
OutEpi current_epi();
inline bool epi_is_default(const OutEpi& e) { return e.ostride == 0 && e.slope == 1.f; }

// One warp -> correlation problem of a grouped launch (capi.hip's pwc_warp_corr_problem).
struct BandProblem {
  const void* f1;
  const void* x2;
  const void* flow;
  void* x2w;
  void* out;
  int B, C, H, W;
};

// One warp problem of a grouped launch (capi.hip's pwc_warp_problem).
struct WarpProblem {
  const void* x;
  const void* flow;
  void* out;
  int B, C, H, W;
};

// Debug / measurement knobs: ONE environment variable, PWC_DEBUG="name=value,name=value",
// parsed once per process (capi.hip).  Unset knobs return `def`; production runs set nothing.
// Kernels never read it -- launchers turn a knob into a template choice or an argument.
int debug_knob(const char* name, int def);

// Opt `kernel` in to `bytes` of dynamic LDS (more than 64 KiB needs hipFuncSetAttribute) on the
// CURRENT device.  The attribute is per device, so the launchers' one-time opt-in is cached per
// (kernel, device): a process that launches on several devices sets it on each (capi.hip).
hipError_t lds_limit(const void* kernel, int bytes);

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): consecutive logical tiles land on the same XCD (and L2), so neighbouring
// tiles that re-read each other's halo rows hit the same L2.  Pure speed choice.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

}  // namespace pwc
