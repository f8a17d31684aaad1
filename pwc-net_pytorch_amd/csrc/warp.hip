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
#include "pwc_common.cuh"

namespace pwc {

// torch.linspace(-1, 1, n)[i] in fp32 (ATen RangeFactories: step = (end-start)/(n-1),
// lower half start + step*i, upper half end - step*(n-1-i)).
__device__ __forceinline__ float linspace_m1p1(int i, int n) {
  if (n == 1) return -1.f;
  const float step = __fdiv_rn(2.f, (float)(n - 1));
  return (i < n / 2) ? __fadd_rn(-1.f, __fmul_rn(step, (float)i))
                     : __fsub_rn(1.f, __fmul_rn(step, (float)(n - 1 - i)));
}

// Source coordinate of the reference chain for one axis.  `half` = (size-1.0)/2.0 computed in
// double on the host (Python float), divided in fp32 like tensor / python-float.
__device__ __forceinline__ float src_coord(float disp, int i, int n, float half) {
  const float g = __fadd_rn(linspace_m1p1(i, n), __fdiv_rn(disp, half));
  return __fmul_rn(__fdiv_rn(__fadd_rn(g, 1.f), 2.f), (float)(n - 1));
}

struct Bilinear {
  int x0, y0;
  float wx0, wx1, wy0, wy1;
  bool vx0, vx1, vy0, vy1;
};

__device__ __forceinline__ Bilinear bilinear(float ix, float iy, int H, int W) {
  Bilinear b;
  const float fx = floorf(ix), fy = floorf(iy);
  b.x0 = (int)fx;
  b.y0 = (int)fy;
  // ATen: nw = (ix_se - ix) * (iy_se - iy) etc.
  b.wx1 = __fsub_rn(ix, fx);
  b.wx0 = __fsub_rn(fx + 1.f, ix);
  b.wy1 = __fsub_rn(iy, fy);
  b.wy0 = __fsub_rn(fy + 1.f, iy);
  b.vx0 = b.x0 >= 0 && b.x0 < W;
  b.vx1 = b.x0 + 1 >= 0 && b.x0 + 1 < W;
  b.vy0 = b.y0 >= 0 && b.y0 < H;
  b.vy1 = b.y0 + 1 >= 0 && b.y0 + 1 < H;
  return b;
}

// One thread per output pixel and CB channels (grid.y splits the channels).
template <typename T, int CB>
__global__ __launch_bounds__(256) void warp_fwd_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ flow,
                                                       T* __restrict__ out, int B, int C, int H,
                                                       int W, float halfx, float halfy) {
  const size_t plane = (size_t)H * W;
  const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * plane) return;
  const int px = idx % W;
  const int py = (idx / W) % H;
  const int n = idx / plane;
  const size_t pix = (size_t)py * W + px;
  const float u = to_f32(flow[((size_t)n * 2 + 0) * plane + pix]);
  const float v = to_f32(flow[((size_t)n * 2 + 1) * plane + pix]);
  const float ix = src_coord(u, px, W, halfx);
  const float iy = src_coord(v, py, H, halfy);
  const Bilinear b = bilinear(ix, iy, H, W);
  const float w00 = __fmul_rn(b.wx0, b.wy0), w01 = __fmul_rn(b.wx1, b.wy0);
  const float w10 = __fmul_rn(b.wx0, b.wy1), w11 = __fmul_rn(b.wx1, b.wy1);
  const size_t i00 = (size_t)b.y0 * W + b.x0;
  const int c0 = blockIdx.y * CB;
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int c = c0 + i;
    if (c >= C) break;
    const T* p = x + ((size_t)n * C + c) * plane;
    float acc = 0.f;
    if (b.vy0 && b.vx0) acc = fmaf(to_f32(p[i00]), w00, acc);
    if (b.vy0 && b.vx1) acc = fmaf(to_f32(p[i00 + 1]), w01, acc);
    if (b.vy1 && b.vx0) acc = fmaf(to_f32(p[i00 + W]), w10, acc);
    if (b.vy1 && b.vx1) acc = fmaf(to_f32(p[i00 + W + 1]), w11, acc);
    out[((size_t)n * C + c) * plane + pix] = from_f32<T>(acc);
  }
}

// fp32 only: grad_x accumulated with atomics (zeroed by the launcher), grad_flow per pixel.
__global__ __launch_bounds__(256) void warp_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ gx,
                                                       float* __restrict__ gflow, int B, int C,
                                                       int H, int W, float halfx, float halfy) {
  const size_t plane = (size_t)H * W;
  const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (idx >= (size_t)B * plane) return;
  const int px = idx % W;
  const int py = (idx / W) % H;
  const int n = idx / plane;
  const size_t pix = (size_t)py * W + px;
  const float u = flow[((size_t)n * 2 + 0) * plane + pix];
  const float v = flow[((size_t)n * 2 + 1) * plane + pix];
  const float ix = src_coord(u, px, W, halfx);
  const float iy = src_coord(v, py, H, halfy);
  const Bilinear b = bilinear(ix, iy, H, W);
  const float w00 = b.wx0 * b.wy0, w01 = b.wx1 * b.wy0;
  const float w10 = b.wx0 * b.wy1, w11 = b.wx1 * b.wy1;
  const size_t i00 = (size_t)b.y0 * W + b.x0;
  float gix = 0.f, giy = 0.f;
  for (int c = 0; c < C; ++c) {
    const float* p = x + ((size_t)n * C + c) * plane;
    float* q = gx + ((size_t)n * C + c) * plane;
    const float go = gout[((size_t)n * C + c) * plane + pix];
    const float v00 = (b.vy0 && b.vx0) ? p[i00] : 0.f;
    const float v01 = (b.vy0 && b.vx1) ? p[i00 + 1] : 0.f;
    const float v10 = (b.vy1 && b.vx0) ? p[i00 + W] : 0.f;
    const float v11 = (b.vy1 && b.vx1) ? p[i00 + W + 1] : 0.f;
    if (b.vy0 && b.vx0) atomicAdd(q + i00, go * w00);
    if (b.vy0 && b.vx1) atomicAdd(q + i00 + 1, go * w01);
    if (b.vy1 && b.vx0) atomicAdd(q + i00 + W, go * w10);
    if (b.vy1 && b.vx1) atomicAdd(q + i00 + W + 1, go * w11);
    gix += go * ((v01 - v00) * b.wy0 + (v11 - v10) * b.wy1);
    giy += go * ((v10 - v00) * b.wx0 + (v11 - v01) * b.wx1);
  }
  // grid grad (ATen: * (size-1)/2) then through flow / ((size-1)/2): net factor 1 in exact
  // arithmetic; keep the two fp32 roundings of the reference chain.
  const float mx = (float)(W - 1) / 2.f, my = (float)(H - 1) / 2.f;
  gflow[((size_t)n * 2 + 0) * plane + pix] = (gix * mx) / halfx;
  gflow[((size_t)n * 2 + 1) * plane + pix] = (giy * my) / halfy;
}

template <typename T>
hipError_t warp_forward_t(const void* x, const void* flow, void* out, int B, int C, int H,
                          int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0 || C == 0) return hipSuccess;
  constexpr int CB = 8;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  dim3 grid((unsigned)((npix + 255) / 256), (unsigned)((C + CB - 1) / CB));
  hipLaunchKernelGGL((warp_fwd_kernel<T, CB>), grid, dim3(256), 0, stream, (const T*)x,
                     (const T*)flow, (T*)out, B, C, H, W, halfx, halfy);
  return hipGetLastError();
}

hipError_t warp_backward_f32(const void* x, const void* flow, const void* gout, void* gx,
                             void* gflow, int B, int C, int H, int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(gx, 0, sizeof(float) * npix * C, stream);
  if (e != hipSuccess) return e;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  hipLaunchKernelGGL(warp_bwd_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0,
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
