// chain_probe.hip -- gfx950 dependent-issue cost of v_pk_fma_f32 / v_fma_f32: a loop of K
// independent accumulator chains (each instruction depends on the one K earlier), at 1 / 2 / 4
// waves per SIMD, one workgroup per CU, wall time per instruction per SIMD.  Decides how many
// independent accumulators the correlation lanes need.
//   hipcc --offload-arch=gfx950 -O3 -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int K, bool PK>
__global__ void chain(float* out, int iters) {
  f2 a = {1.f + threadIdx.x * 1e-7f, 0.5f}, b = {0.999f, 1.0001f};
  f2 c[K];
#pragma unroll
  for (int i = 0; i < K; ++i) c[i] = f2{(float)i, (float)-i};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 72 / K; ++r)
#pragma unroll
      for (int i = 0; i < K; ++i) {
        if constexpr (PK)
          asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[i]) : "v"(a), "v"(b));
        else
          asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c[i].x) : "v"(a.x), "v"(b.x));
      }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) s += c[i].x + c[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int K, bool PK>
static void run(float* d, int wps) {
  const int iters = 4096, threads = 256 * wps;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((chain<K, PK>), dim3(256), dim3(threads), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  const double inst_per_simd = (double)wps * iters * (72 / K) * K;
  std::printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ns_per_inst_per_simd\": %.3f, "
              "\"ns_per_inst_per_wave\": %.3f}\n",
              PK ? "v_pk_fma_f32" : "v_fma_f32", K, wps, best * 1e6 / inst_per_simd,
              best * 1e6 / inst_per_simd * wps);
}

template <bool PK>
static void sweep(float* d) {
  for (int w : {1, 2, 4}) {
    run<1, PK>(d, w);
    run<2, PK>(d, w);
    run<4, PK>(d, w);
    run<6, PK>(d, w);
    run<8, PK>(d, w);
    run<12, PK>(d, w);
    run<18, PK>(d, w);
    run<36, PK>(d, w);
  }
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 1024 * sizeof(float));
  sweep<true>(d);
  sweep<false>(d);
  return 0;
}
