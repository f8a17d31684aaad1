// warp_layout_probe.hip -- is a channel-interleaved (NHWC) gather cheaper for the fp16 warp?
// Config-4 l4 shape (B=16, C=32, 112x256, fp16), flows N(0, 2^2) px.  Times, back to back over
// rotating buffer sets:
//   nchw   : one thread per pixel x 8 channels, two 2-byte gathers per sample row and channel
//            (the access pattern of warp.hip's fp16 kernel)
//   tr     : NCHW -> NHWC transpose (fp16)
//   nhwc   : one thread per pixel, one 16-byte gather per corner and 8 channels, NCHW stores
// Timing only: bilinear weights from fp32 flow, no reference coordinate chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/warp_layout_probe tools/warp_layout_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

struct Tap {
  int i00, i01, i10, i11;
  float w00, w01, w10, w11;
};

__device__ __forceinline__ Tap tap(const float* fl, int n, int y, int x, int H, int W) {
  const size_t plane = (size_t)H * W;
  const float u = fl[(2 * n) * plane + y * W + x], v = fl[(2 * n + 1) * plane + y * W + x];
  const float ix = x + u, iy = y + v;
  const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  const float ax = ix - x0, ay = iy - y0;
  const int xa = min(max(x0, 0), W - 1), xb = min(max(x0 + 1, 0), W - 1);
  const int ya = min(max(y0, 0), H - 1), yb = min(max(y0 + 1, 0), H - 1);
  Tap t;
  t.i00 = ya * W + xa, t.i01 = ya * W + xb, t.i10 = yb * W + xa, t.i11 = yb * W + xb;
  t.w00 = (1 - ax) * (1 - ay), t.w01 = ax * (1 - ay), t.w10 = (1 - ax) * ay, t.w11 = ax * ay;
  return t;
}

__global__ __launch_bounds__(256) void warp_nchw(const _Float16* x, const float* fl, _Float16* o,
                                                 int B, int C, int H, int W) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int plane = H * W;
  if (idx >= B * plane) return;
  const int n = idx / plane, p = idx % plane, y = p / W, xx = p % W;
  const Tap t = tap(fl, n, y, xx, H, W);
  const int c0 = blockIdx.y * 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const _Float16* s = x + (size_t)(n * C + c0 + k) * plane;
    const float v = t.w00 * (float)s[t.i00] + t.w01 * (float)s[t.i01] + t.w10 * (float)s[t.i10] +
                    t.w11 * (float)s[t.i11];
    o[(size_t)(n * C + c0 + k) * plane + p] = (_Float16)v;
  }
}

// NCHW -> NHWC: one thread per (pixel, 8-channel group), 8 strided 2-byte reads, one 16-B write
__global__ __launch_bounds__(256) void transpose8(const _Float16* x, _Float16* t, int B, int C,
                                                  int H, int W) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int plane = H * W;
  if (idx >= B * plane) return;
  const int n = idx / plane, p = idx % plane;
  const int g = blockIdx.y;
  h8 v;
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = x[(size_t)(n * C + 8 * g + k) * plane + p];
  *reinterpret_cast<h8*>(t + ((size_t)n * plane + p) * C + 8 * g) = v;
}

__global__ __launch_bounds__(256) void warp_nhwc(const _Float16* t, const float* fl, _Float16* o,
                                                 int B, int C, int H, int W) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int plane = H * W;
  if (idx >= B * plane) return;
  const int n = idx / plane, p = idx % plane, y = p / W, xx = p % W;
  const Tap tp = tap(fl, n, y, xx, H, W);
  const int g = blockIdx.y;
  const _Float16* base = t + (size_t)n * plane * C + 8 * g;
  const h8 a = *reinterpret_cast<const h8*>(base + (size_t)tp.i00 * C);
  const h8 b = *reinterpret_cast<const h8*>(base + (size_t)tp.i01 * C);
  const h8 c = *reinterpret_cast<const h8*>(base + (size_t)tp.i10 * C);
  const h8 d = *reinterpret_cast<const h8*>(base + (size_t)tp.i11 * C);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float v = tp.w00 * (float)a[k] + tp.w01 * (float)b[k] + tp.w10 * (float)c[k] +
                    tp.w11 * (float)d[k];
    o[(size_t)(n * C + 8 * g + k) * plane + p] = (_Float16)v;
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 16, C = argc > 2 ? std::atoi(argv[2]) : 32;
  const int H = argc > 3 ? std::atoi(argv[3]) : 112, W = argc > 4 ? std::atoi(argv[4]) : 256;
  const size_t nx = (size_t)B * C * H * W, nf = (size_t)B * 2 * H * W;
  const int NS = 8;
  std::vector<_Float16*> xs(NS), ts(NS), os(NS);
  std::vector<float*> fs(NS);
  std::vector<_Float16> hx(nx);
  std::vector<float> hf(nf);
  unsigned s = 7;
  auto rnd = [&] {
    s = s * 1664525u + 1013904223u;
    return (float)((s >> 8) & 0xffff) / 32768.f - 1.f;
  };
  for (auto& v : hx) v = (_Float16)rnd();
  for (auto& v : hf) v = 2.f * (rnd() + rnd() + rnd());  // ~N(0, 2^2)-ish
  for (int i = 0; i < NS; ++i) {
    CK(hipMalloc(&xs[i], nx * 2));
    CK(hipMalloc(&ts[i], nx * 2));
    CK(hipMalloc(&os[i], nx * 2));
    CK(hipMalloc(&fs[i], nf * 4));
    CK(hipMemcpy(xs[i], hx.data(), nx * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(fs[i], hf.data(), nf * 4, hipMemcpyHostToDevice));
  }
  const dim3 grid((unsigned)((B * H * W + 255) / 256), (unsigned)(C / 8));
  auto time = [&](auto launch, const char* name) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) launch(i % NS);
    CK(hipDeviceSynchronize());
    const int it = 200;
    CK(hipEventRecord(a));
    for (int i = 0; i < it; ++i) launch(i % NS);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"kernel\": \"%s\", \"us\": %.2f}\n", name, ms * 1e3f / it);
  };
  time([&](int i) { warp_nchw<<<grid, 256>>>(xs[i], fs[i], os[i], B, C, H, W); }, "nchw");
  time([&](int i) { transpose8<<<grid, 256>>>(xs[i], ts[i], B, C, H, W); }, "tr");
  time([&](int i) { warp_nhwc<<<grid, 256>>>(ts[i], fs[i], os[i], B, C, H, W); }, "nhwc");
  time([&](int i) {
    transpose8<<<grid, 256>>>(xs[i], ts[i], B, C, H, W);
    warp_nhwc<<<grid, 256>>>(ts[i], fs[i], os[i], B, C, H, W);
  }, "tr+nhwc");
  return 0;
}
