// floor_probe.hip -- what a pure streaming kernel achieves for the l4 correlation's traffic
// (read 2 x 11.0 MB, write 27.9 MB: B=8, 32x96x112 in, 81x96x112 out, fp32), on rotating
// buffer sets past the 256 MiB Infinity Cache.  Variants: grid-stride vs one float4 per
// thread, plain vs nontemporal stores, read-only and write-only halves, and a plain 50 MB
// copy.  Each line: average of per-launch hipEvent durations over 200 launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/floor_probe tools/floor_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// one float4 of output per thread; inputs read where i < n_in
template <bool NT>
__global__ __launch_bounds__(256) void flat(const f4* __restrict__ a, const f4* __restrict__ b,
                                            f4* __restrict__ o, long n_in, long n_out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_out) return;
  f4 v = {0.f, 0.f, 0.f, 0.f};
  if (i < n_in) v = a[i] + b[i];
  st<NT>(o + i, v);
}

template <bool NT>
__global__ __launch_bounds__(256) void gstride(const f4* __restrict__ a, const f4* __restrict__ b,
                                               f4* __restrict__ o, long n_in, long n_out) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n_out; i += stride) {
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (i < n_in) v = a[i] + b[i];
    st<NT>(o + i, v);
  }
}

// each thread: 4 consecutive float4 per pass (more bytes in flight per wave)
template <bool NT>
__global__ __launch_bounds__(256) void flat4(const f4* __restrict__ a, const f4* __restrict__ b,
                                             f4* __restrict__ o, long n_in, long n_out) {
  const long base = (long)blockIdx.x * 1024 + threadIdx.x;
  f4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long i = base + 256 * k;
    v[k] = f4{0.f, 0.f, 0.f, 0.f};
    if (i < n_in) v[k] = a[i] + b[i];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long i = base + 256 * k;
    if (i < n_out) st<NT>(o + i, v[k]);
  }
}

__global__ __launch_bounds__(256) void rd(const f4* __restrict__ a, const f4* __restrict__ b,
                                          f4* __restrict__ o, long n_in) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_in) return;
  const f4 v = a[i] + b[i];
  if (v.x == 1234.5f) o[0] = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void wr(f4* __restrict__ o, long n_out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_out) return;
  st<NT>(o + i, f4{1.f, 2.f, 3.f, (float)i});
}

__global__ __launch_bounds__(256) void cp(const f4* __restrict__ a, f4* __restrict__ o, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) o[i] = a[i];
}

int main() {
  const long B = 8, C = 32, H = 96, W = 112;
  const long n_in = B * C * H * W / 4, n_out = B * 81 * H * W / 4;  // float4 counts
  const int NSETS = 8;  // 8 x 50 MB = 400 MB > 256 MiB MALL
  std::vector<f4*> A(NSETS), Bv(NSETS), O(NSETS);
  for (int s = 0; s < NSETS; ++s) {
    CK(hipMalloc(&A[s], n_in * 16));
    CK(hipMalloc(&Bv[s], n_in * 16));
    CK(hipMalloc(&O[s], n_out * 16));
    CK(hipMemset(A[s], 0, n_in * 16));
    CK(hipMemset(Bv[s], 0, n_in * 16));
  }
  hipEvent_t e0[200], e1[200];
  for (int i = 0; i < 200; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  const double bytes = (2.0 * n_in + n_out) * 16;
  auto run = [&](const char* name, double nbytes, auto launch) -> int {
    for (int i = 0; i < 20; ++i) launch(i % NSETS, nullptr, nullptr);
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 200; ++i) launch(i % NSETS, e0[i], e1[i]);
    CK(hipDeviceSynchronize());
    double sum = 0, mn = 1e9;
    for (int i = 0; i < 200; ++i) {
      float ms;
      CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      sum += ms;
      mn = ms < mn ? ms : mn;
    }
    const double us = sum / 200 * 1e3;
    std::printf("{\"probe\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"MB\": %.1f, \"TBs\": %.3f}\n",
                name, us, mn * 1e3, nbytes / 1e6, nbytes / (us * 1e-6) / 1e12);
    return 0;
  };
  const unsigned g_flat = (unsigned)((n_out + 255) / 256);
  const unsigned g_flat4 = (unsigned)((n_out + 1023) / 1024);
#define L(K, G, ...)                                                                         \
  [&](int s, hipEvent_t a, hipEvent_t b) {                                                 \
    hipExtLaunchKernelGGL(K, dim3(G), dim3(256), 0, 0, a, b, 0, __VA_ARGS__);              \
  }
  if (run("corr_traffic_flat", bytes, L(flat<false>, g_flat, A[s], Bv[s], O[s], n_in, n_out))) return 1;
  if (run("corr_traffic_flat_nt", bytes, L(flat<true>, g_flat, A[s], Bv[s], O[s], n_in, n_out))) return 1;
  if (run("corr_traffic_flat4", bytes, L(flat4<false>, g_flat4, A[s], Bv[s], O[s], n_in, n_out))) return 1;
  if (run("corr_traffic_flat4_nt", bytes, L(flat4<true>, g_flat4, A[s], Bv[s], O[s], n_in, n_out))) return 1;
  for (unsigned g : {1024u, 2048u, 4096u})
    if (run(g == 1024 ? "corr_traffic_gstride1024" : g == 2048 ? "corr_traffic_gstride2048"
                                                               : "corr_traffic_gstride4096",
            bytes, L(gstride<false>, g, A[s], Bv[s], O[s], n_in, n_out)))
      return 1;
  if (run("read_only_22MB", 2.0 * n_in * 16, L(rd, (unsigned)((n_in + 255) / 256), A[s], Bv[s], O[s], n_in))) return 1;
  if (run("write_only_28MB", n_out * 16.0, L(wr<false>, g_flat, O[s], n_out))) return 1;
  if (run("write_only_28MB_nt", n_out * 16.0, L(wr<true>, g_flat, O[s], n_out))) return 1;
  // a plain copy of 25 MB -> 25 MB (50 MB of traffic, the output buffer read and rewritten)
  if (run("copy_25MB_to_25MB", 2.0 * (n_out - n_out / 10) * 16,
          L(cp, (unsigned)((n_out - n_out / 10 + 255) / 256), O[(s + 1) % NSETS], O[s],
            n_out - n_out / 10)))
    return 1;
  return 0;
}
