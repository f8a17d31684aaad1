// warp.hip — bilinear flow warp (WarpingLayer) forward / backward for gfx950.
//
// Semantics: WarpingLayer.forward, modules.py:31-42 of daigo0927/PWC-Net_pytorch:
//   flow_n = flow / ((size-1)/2);  grid = get_grid(x) + flow_n  (utils.py:3-8: linspace(-1,1))
//   out = F.grid_sample(x, grid)   with torch==0.4.0 semantics (requirements.txt:62):
//   bilinear, zeros padding, align_corners=True: ix = ((gx + 1) / 2) * (W - 1).
// The reference builds the base grid on the host and copies it to the device on every call
// (modules.py:40) and runs ~5 elementwise kernels + a permute before grid_sampler_2d; here the
// whole normalisation chain is recomputed in registers, in the same fp32 operation order
// (no FMA contraction), so sample coordinates match the reference chain.
// Backward follows ATen grid_sampler_2d_backward: grad_x by fp32 atomics (scatter), grad of
// the sample point by the bilinear derivative; d(ix)/d(u) = ((W-1)/2) / ((W-1)/2) = 1.
#include <cstdlib>

#include "warp_sample.cuh"

namespace pwc {

// One thread per output pixel and CB channels (grid.y splits the channels).  32-bit indexing
// (the launcher checks B*C*H*W < 2^31).
template <typename T, int CB>
struct WarpGroup {  // one channel group's raw corner values
  float r[CB][4];
};

template <typename T, int CB>
__device__ __forceinline__ void warp_load(WarpGroup<T, CB>& g, const T* __restrict__ x,
                                          unsigned n, int C, unsigned plane, int c0, int W,
                                          const Pairs& kp, const Corners& kc) {
  if (W >= 2) {
    float lo[CB][2], hi[CB][2];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = min(c0 + i, C - 1);
      const T* p = x + ((unsigned)(n * C + c)) * plane;
      load_pair(p + kp.i0, lo[i][0], hi[i][0]);
      load_pair(p + kp.i1, lo[i][1], hi[i][1]);
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      g.r[i][0] = kp.l_lo ? lo[i][0] : hi[i][0];
      g.r[i][1] = kp.r_lo ? lo[i][0] : hi[i][0];
      g.r[i][2] = kp.l_lo ? lo[i][1] : hi[i][1];
      g.r[i][3] = kp.r_lo ? lo[i][1] : hi[i][1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = min(c0 + i, C - 1);
      const T* p = x + ((unsigned)(n * C + c)) * plane;
      g.r[i][0] = to_f32(p[kc.i00]);
      g.r[i][1] = to_f32(p[kc.i01]);
      g.r[i][2] = to_f32(p[kc.i10]);
      g.r[i][3] = to_f32(p[kc.i11]);
    }
  }
}

// One thread per output pixel; grid.y splits the channels into slices of NG groups of CB
// channels, and a thread walks its slice's groups with the next group's gathers in flight
// while the current one is blended and stored.  32-bit indexing (the launcher checks
// B*C*H*W < 2^31).
template <typename T, int CB, int NG, bool XCD>
__global__ __launch_bounds__(256) void warp_fwd_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ flow,
                                                       T* __restrict__ out, int B, int C, int H,
                                                       int W, float halfx, float halfy) {
  const unsigned plane = (unsigned)(H * W);
  // XCD: consecutive pixel blocks (which gather overlapping source rows) share an L2
  const unsigned bx = XCD ? (unsigned)xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const unsigned idx = bx * 256u + threadIdx.x;
  if (idx >= (unsigned)B * plane) return;
  const unsigned n = idx / plane;
  const unsigned pix = idx - n * plane;
  const int py = (int)(pix / (unsigned)W);
  const int px = (int)pix - py * W;
  const float u = to_f32(flow[(2 * n + 0) * plane + pix]);
  const float v = to_f32(flow[(2 * n + 1) * plane + pix]);
  const float ix = src_coord(u, px, W, halfx);
  const float iy = src_coord(v, py, H, halfy);
  const Bilinear b = bilinear(ix, iy, H, W);
  const float w00 = b.wx0 * b.wy0, w01 = b.wx1 * b.wy0;  // feed fma operands: not fusable
  const float w10 = b.wx0 * b.wy1, w11 = b.wx1 * b.wy1;
  const Pairs kp = pairs(b, H, W);
  const Corners kc = corners(b, H, W);
  const float m00 = kc.m00, m01 = kc.m01, m10 = kc.m10, m11 = kc.m11;
  const int cs = blockIdx.y * CB * NG;
  WarpGroup<T, CB> g[2];
  warp_load(g[0], x, n, C, plane, cs, W, kp, kc);
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    const int c0 = cs + gi * CB;
    if (gi + 1 < NG) warp_load(g[(gi + 1) & 1], x, n, C, plane, c0 + CB, W, kp, kc);
    const WarpGroup<T, CB>& cur = g[gi & 1];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      float acc = 0.f;
      acc = fmaf(masked(cur.r[i][0], m00), w00, acc);
      acc = fmaf(masked(cur.r[i][1], m01), w01, acc);
      acc = fmaf(masked(cur.r[i][2], m10), w10, acc);
      acc = fmaf(masked(cur.r[i][3], m11), w11, acc);
      if (c0 + i < C) {
        T* o = out + ((unsigned)(n * C + c0 + i)) * plane + pix;
        if constexpr (sizeof(T) == 4)
          st_out1(reinterpret_cast<float*>(o), acc);
        else
          *o = from_f32<T>(acc);
      }
    }
  }
}

// fp32 only: grad_x accumulated with atomics (zeroed by the launcher), grad_flow per pixel.
// Channels are processed CB at a time with all loads of a group issued together.
template <int CB>
__global__ __launch_bounds__(256) void warp_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ gx,
                                                       float* __restrict__ gflow, int B, int C,
                                                       int H, int W, float halfx, float halfy) {
  const unsigned plane = (unsigned)(H * W);
  const unsigned idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= (unsigned)B * plane) return;
  const unsigned n = idx / plane;
  const unsigned pix = idx - n * plane;
  const int py = (int)(pix / (unsigned)W);
  const int px = (int)pix - py * W;
  const float u = flow[(2 * n + 0) * plane + pix];
  const float v = flow[(2 * n + 1) * plane + pix];
  const float ix = src_coord(u, px, W, halfx);
  const float iy = src_coord(v, py, H, halfy);
  const Bilinear b = bilinear(ix, iy, H, W);
  const Corners k = corners(b, H, W);
  const float w00 = b.wx0 * b.wy0, w01 = b.wx1 * b.wy0;
  const float w10 = b.wx0 * b.wy1, w11 = b.wx1 * b.wy1;
  float gix = 0.f, giy = 0.f;
  for (int c0 = 0; c0 < C; c0 += CB) {
    float r[CB][4], go[CB];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = min(c0 + i, C - 1);
      const float* p = x + ((unsigned)(n * C + c)) * plane;
      r[i][0] = masked(p[k.i00], k.m00);
      r[i][1] = masked(p[k.i01], k.m01);
      r[i][2] = masked(p[k.i10], k.m10);
      r[i][3] = masked(p[k.i11], k.m11);
      go[i] = (c0 + i < C) ? gout[((unsigned)(n * C + c)) * plane + pix] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      if (c0 + i >= C) break;
      float* q = gx + ((unsigned)(n * C + c0 + i)) * plane;
      if (k.m00 != 0.f) atomicAdd(q + k.i00, go[i] * w00);
      if (k.m01 != 0.f) atomicAdd(q + k.i01, go[i] * w01);
      if (k.m10 != 0.f) atomicAdd(q + k.i10, go[i] * w10);
      if (k.m11 != 0.f) atomicAdd(q + k.i11, go[i] * w11);
      gix += go[i] * ((r[i][1] - r[i][0]) * b.wy0 + (r[i][3] - r[i][2]) * b.wy1);
      giy += go[i] * ((r[i][2] - r[i][0]) * b.wx0 + (r[i][3] - r[i][1]) * b.wx1);
    }
  }
  // grid grad (ATen: * (size-1)/2) then through flow / ((size-1)/2): net factor 1 in exact
  // arithmetic; keep the two fp32 roundings of the reference chain.
  const float mx = (float)(W - 1) / 2.f, my = (float)(H - 1) / 2.f;
  gflow[(2 * n + 0) * plane + pix] = (gix * mx) / halfx;
  gflow[(2 * n + 1) * plane + pix] = (giy * my) / halfy;
}

// PWC_WARP_CFG=<digit> selects a (channels per group, groups per thread) variant for
// measurement: 0 = 4 channels per thread, XCD-grouped pixel blocks (default), 1 = 8, 2 = 2,
// 3 = 4 without XCD grouping, 4 = 2 grouped, 5 = 8 grouped.
static int warp_cfg() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("PWC_WARP_CFG");
    v = (e && e[0] >= '0' && e[0] <= '9' && e[1] == 0) ? e[0] - '0' : 0;
  }
  return v;
}

template <typename T>
hipError_t warp_forward_t(const void* x, const void* flow, void* out, int B, int C, int H,
                          int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0 || C == 0) return hipSuccess;
  if (npix * (size_t)(C > 2 ? C : 2) >= (1ull << 31)) return hipErrorInvalidValue;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  const unsigned gx = (unsigned)((npix + 255) / 256);
#define PWC_WARP_LAUNCH(CB, NG, XCD)                                                          \
  hipLaunchKernelGGL((warp_fwd_kernel<T, CB, NG, XCD>),                                       \
                     dim3(gx, (unsigned)((C + CB * NG - 1) / (CB * NG))), dim3(256), 0, stream, \
                     (const T*)x, (const T*)flow, (T*)out, B, C, H, W, halfx, halfy)
  switch (warp_cfg()) {
    case 1: PWC_WARP_LAUNCH(8, 1, false); break;
    case 2: PWC_WARP_LAUNCH(2, 1, false); break;
    case 3: PWC_WARP_LAUNCH(4, 1, false); break;
    case 4: PWC_WARP_LAUNCH(2, 1, true); break;
    case 5: PWC_WARP_LAUNCH(8, 1, true); break;
    case 6: PWC_WARP_LAUNCH(4, 2, true); break;
    case 7: PWC_WARP_LAUNCH(4, 4, true); break;
    case 8: PWC_WARP_LAUNCH(4, 8, true); break;
    case 9: PWC_WARP_LAUNCH(2, 4, true); break;
    default: PWC_WARP_LAUNCH(4, 1, true); break;
  }
#undef PWC_WARP_LAUNCH
  return hipGetLastError();
}

hipError_t warp_backward_f32(const void* x, const void* flow, const void* gout, void* gx,
                             void* gflow, int B, int C, int H, int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0) return hipSuccess;
  if (npix * (size_t)(C > 2 ? C : 2) >= (1ull << 31)) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(gx, 0, sizeof(float) * npix * C, stream);
  if (e != hipSuccess) return e;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  hipLaunchKernelGGL(warp_bwd_kernel<8>, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0,
                     stream, (const float*)x, (const float*)flow, (const float*)gout,
                     (float*)gx, (float*)gflow, B, C, H, W, halfx, halfy);
  return hipGetLastError();
}

template hipError_t warp_forward_t<float>(const void*, const void*, void*, int, int, int, int,
                                          hipStream_t);
template hipError_t warp_forward_t<__half>(const void*, const void*, void*, int, int, int, int,
                                           hipStream_t);
template hipError_t warp_forward_t<__hip_bfloat16>(const void*, const void*, void*, int, int,
                                                   int, int, hipStream_t);

}  // namespace pwc
