// warp_sample.cuh — the WarpingLayer sample chain (modules.py:31-42, utils.py:3-8, torch-0.4
// grid_sample: bilinear, zeros, align_corners=True), shared by the warp kernels (warp.hip) and
// the fused warp -> correlation kernel (warp_corr.hip) so both produce bit-identical samples.
#pragma once

#include "pwc_common.cuh"

namespace pwc {

// torch.linspace(-1, 1, n)[i] in fp32 (ATen RangeFactories: step = (end-start)/(n-1),
// lower half start + step*i, upper half end - step*(n-1-i)).
// Contraction is disabled in this scope with plain operators: hipcc's __fmul_rn/__fadd_rn are
// plain operators defined in a header (outside this pragma), so they would still be fused,
// and an fma here rounds differently from the reference's separate fp32 ops.
__device__ __forceinline__ float linspace_m1p1(int i, int n) {
#pragma clang fp contract(off)
  if (n == 1) return -1.f;
  const float step = 2.f / (float)(n - 1);
  return (i < n / 2) ? -1.f + step * (float)i : 1.f - step * (float)(n - 1 - i);
}

// Source coordinate of the reference chain for one axis.  `half` = (size-1.0)/2.0 computed in
// double on the host (Python float), divided in fp32 like tensor / python-float.
__device__ __forceinline__ float src_coord(float disp, int i, int n, float half) {
#pragma clang fp contract(off)
  const float g = linspace_m1p1(i, n) + disp / half;
  return ((g + 1.f) / 2.f) * (float)(n - 1);
}

struct Bilinear {
  int x0, y0;
  float wx0, wx1, wy0, wy1;
  bool vx0, vx1, vy0, vy1;
};

__device__ __forceinline__ Bilinear bilinear(float ix, float iy, int H, int W) {
#pragma clang fp contract(off)
  Bilinear b;
  const float fx = floorf(ix), fy = floorf(iy);
  b.x0 = (int)fx;
  b.y0 = (int)fy;
  // ATen: nw = (ix_se - ix) * (iy_se - iy) etc.
  b.wx1 = ix - fx;
  b.wx0 = (fx + 1.f) - ix;
  b.wy1 = iy - fy;
  b.wy0 = (fy + 1.f) - iy;
  b.vx0 = b.x0 >= 0 && b.x0 < W;
  b.vx1 = b.x0 + 1 >= 0 && b.x0 + 1 < W;
  b.vy0 = b.y0 >= 0 && b.y0 < H;
  b.vy1 = b.y0 + 1 >= 0 && b.y0 + 1 < H;
  return b;
}

// Corner addresses clamped into the image plus validity masks: every gather is issued
// unconditionally (one batch of loads per thread, no per-corner branches), invalid corners are
// zeroed after the load -- the reference's "skip out-of-bounds corners" (zeros padding).
struct Corners {
  unsigned i00, i01, i10, i11;
  float m00, m01, m10, m11;  // 1 where the corner is inside the image
};

__device__ __forceinline__ Corners corners(const Bilinear& b, int H, int W) {
  const int x0 = min(max(b.x0, 0), W - 1), x1 = min(max(b.x0 + 1, 0), W - 1);
  const int y0 = min(max(b.y0, 0), H - 1), y1 = min(max(b.y0 + 1, 0), H - 1);
  Corners k;
  k.i00 = (unsigned)(y0 * W + x0);
  k.i01 = (unsigned)(y0 * W + x1);
  k.i10 = (unsigned)(y1 * W + x0);
  k.i11 = (unsigned)(y1 * W + x1);
  k.m00 = (b.vy0 && b.vx0) ? 1.f : 0.f;
  k.m01 = (b.vy0 && b.vx1) ? 1.f : 0.f;
  k.m10 = (b.vy1 && b.vx0) ? 1.f : 0.f;
  k.m11 = (b.vy1 && b.vx1) ? 1.f : 0.f;
  return k;
}

__device__ __forceinline__ float masked(float v, float m) { return m != 0.f ? v : 0.f; }

// Horizontal corner pairs: both corners of a sample row come from ONE 8-byte load at
// xs = clamp(x0, 0, W-2) (dword-aligned, which global loads accept), halving the gather
// instructions -- the texture-address unit, not HBM, bounds this kernel.  Corner x0 is
// element x0 - xs of the pair, corner x0+1 element x0 + 1 - xs; out-of-image corners are
// masked as before.  (W == 1 keeps single loads.)
typedef float f32x2u __attribute__((ext_vector_type(2), aligned(4)));

struct Pairs {
  unsigned i0, i1;       // row starts of the two sample rows + xs (element index in the plane)
  bool l_lo, r_lo;       // left / right corner is the pair's low element
  float m00, m01, m10, m11;
};

__device__ __forceinline__ Pairs pairs(const Bilinear& b, int H, int W) {
  Pairs p;
  const int xs = min(max(b.x0, 0), W - 2);
  const int y0 = min(max(b.y0, 0), H - 1), y1 = min(max(b.y0 + 1, 0), H - 1);
  p.i0 = (unsigned)(y0 * W + xs);
  p.i1 = (unsigned)(y1 * W + xs);
  p.l_lo = b.x0 == xs;
  p.r_lo = b.x0 + 1 == xs;
  p.m00 = (b.vy0 && b.vx0) ? 1.f : 0.f;
  p.m01 = (b.vy0 && b.vx1) ? 1.f : 0.f;
  p.m10 = (b.vy1 && b.vx0) ? 1.f : 0.f;
  p.m11 = (b.vy1 && b.vx1) ? 1.f : 0.f;
  return p;
}

template <typename T>
__device__ __forceinline__ void load_pair(const T* p, float& lo, float& hi) {
  if constexpr (sizeof(T) == 4) {
    const f32x2u v = *reinterpret_cast<const f32x2u*>(p);
    lo = v.x;
    hi = v.y;
  } else {
    lo = to_f32(p[0]);
    hi = to_f32(p[1]);
  }
}

}  // namespace pwc
