// Diagnostic: dispatch cost of an empty 512-thread kernel vs its dynamic LDS allocation.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
__global__ __launch_bounds__(512) void empty_k(float* out, int touch) {
  extern __shared__ float lds[];
  if (touch) { lds[threadIdx.x] = threadIdx.x; __syncthreads(); if (lds[511 - threadIdx.x] == -1.f) out[0] = 1; }
}
int main() {
  float* d; (void)hipMalloc(&d, 4096);
  (void)hipFuncSetAttribute((const void*)empty_k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int blocks : {128, 256, 1024})
    for (int kb : {0, 16, 32, 64, 65, 96, 128, 147, 160}) {
      const size_t lds = (size_t)kb * 1024;
      float sum = 0; int n = 0;
      for (int r = 0; r < 60; ++r) {
        hipExtLaunchKernelGGL(empty_k, dim3(blocks), dim3(512), lds, 0, e0, e1, 0, d, 1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 10) { sum += ms; ++n; }
      }
      std::printf("blocks %4d lds %3d KB: %.2f us\n", blocks, kb, sum / n * 1e3);
    }
  return 0;
}
