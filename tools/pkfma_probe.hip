// Diagnostic: issue cost of v_pk_fma_f32 vs v_fma_f32 on gfx950 (independent accumulators,
// operands in registers), at 1..4 waves per SIMD on every CU.  Prints cycles per instruction
// per SIMD from s_memtime and wall time.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int PK>
__global__ void loop(float* out, int iters, unsigned long long* cyc) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a0 = {1.f + threadIdx.x, 2.f}, b0 = {0.5f, 0.25f};
  f2 c[16];
  for (int i = 0; i < 16; ++i) c[i] = f2{(float)i, (float)-i};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (PK)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[i]) : "v"(a0), "v"(b0));
      else
        asm volatile("v_fma_f32 %0, %1, %2, %0\n\tv_fma_f32 %3, %4, %5, %3"
                     : "+v"(c[i].x), "+v"(c[i].y) : "v"(a0.x), "v"(b0.x), "v"(a0.y), "v"(b0.y));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c[i].x + c[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* d;
  unsigned long long* cyc;
  (void)hipMalloc(&d, 256 * 2048 * sizeof(float));
  (void)hipMalloc(&cyc, 4096 * sizeof(unsigned long long));
  const int iters = 4096;
  for (int pk = 0; pk < 2; ++pk)
    for (int wps : {1, 2, 4}) {
      const int threads = 256 * wps;  // 4*wps waves per block, 1 block per CU
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        if (pk)
          hipLaunchKernelGGL(loop<1>, dim3(256), dim3(threads), 0, 0, d, iters, cyc);
        else
          hipLaunchKernelGGL(loop<0>, dim3(256), dim3(threads), 0, 0, d, iters, cyc);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
      }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[256];
      (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < 256; ++i) avg += h[i];
      avg /= 256;
      // per SIMD: wps waves x iters x 16 instructions (pk) or 32 (scalar)
      const double ninst = (double)wps * iters * (pk ? 16 : 32);
      const double fmas = (double)threads * 256 * iters * 32;
      std::printf("%s waves/SIMD=%d  memtime cyc/inst/SIMD=%.2f  wall %.3f ms  %.1f TFLOP/s\n",
                  pk ? "v_pk_fma_f32" : "v_fma_f32   ", wps, avg / ninst, ms,
                  2 * fmas / (ms * 1e-3) / 1e12);
    }
  return 0;
}
