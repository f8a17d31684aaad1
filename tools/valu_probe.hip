// Diagnostic: sustained v_fmac_f32 rate on gfx950 for the correlation inner-loop shape
// (36 independent accumulators, 4 + 20 operands reloaded per iteration) at several
// waves-per-SIMD counts.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ITERS>
__global__ void fma_loop(float* out, float seed) {
  float acc[36];
  float a[4], w[20];
#pragma unroll
  for (int i = 0; i < 36; ++i) acc[i] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = seed + threadIdx.x + i;
#pragma unroll
  for (int i = 0; i < 20; ++i) w[i] = seed * i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int ti = 0; ti < 9; ++ti)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[ti * 4 + k] = fmaf(a[k], w[k + 2 * ti], acc[ti * 4 + k]);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = __shfl_xor(a[i], 1) + 1.f;  // keep operands live
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 36; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 1024 * 8 * sizeof(float));
  constexpr int IT = 2048;
  for (int threads : {64, 256, 576, 1024}) {
    for (int blocks_per_cu : {1, 2, 4}) {
      int nb = 256 * blocks_per_cu;
      if (threads * blocks_per_cu > 2048) continue;
      hipLaunchKernelGGL(fma_loop<IT>, dim3(nb), dim3(threads), 0, 0, d, 1.0f);
      (void)hipDeviceSynchronize();
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, 0);
      for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(fma_loop<IT>, dim3(nb), dim3(threads), 0, 0, d, 1.0f);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double fma = 5.0 * nb * threads * (double)IT * 36;
      const double waves_per_simd = threads / 64.0 * blocks_per_cu / 4.0;
      printf("threads %4d x %d/CU (%.2f waves/SIMD): %.1f TFMA/s = %.1f%% of 78.6 (2 cyc/v_fma "
             "@2.4GHz)\n", threads, blocks_per_cu, waves_per_simd, fma / (ms * 1e-3) / 1e12,
             100.0 * fma / (ms * 1e-3) / 78.6e12);
    }
  }
  return 0;
}
