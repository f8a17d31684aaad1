// bank_probe.hip -- v_pk_fma_f32 issue rate by VGPR bank pattern (gfx950): three 64-bit
// operands in one bank pair (0-1) vs two, at 2 waves per SIMD; explicit registers (clobbered).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bank_probe tools/bank_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

// MODE 0: dst/src2 v[32+4i:], src0 v[0:1], src1 v[4:5]   -> all in bank pair 0 (3-way)
// MODE 1: dst/src2 v[34+4i:], src0 v[0:1], src1 v[4:5]   -> src2 in pair 2 (src0/src1 2-way)
// MODE 2: dst/src2 v[34+4i:], src0 v[0:1], src1 v[6:7]   -> src1, src2 pair 2 (2-way)
template <int MODE>
__global__ void loop(float* out, int iters, unsigned long long* cyc) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  asm volatile("v_mov_b32 v0, 1.0\n\tv_mov_b32 v1, 1.0\n\tv_mov_b32 v4, 1.0\n\tv_mov_b32 v5, 1.0\n\t"
               "v_mov_b32 v6, 1.0\n\tv_mov_b32 v7, 1.0" ::: "v0", "v1", "v4", "v5", "v6", "v7");
  for (int it = 0; it < iters; ++it) {
#define F(d) \
    if constexpr (MODE == 0) asm volatile("v_pk_fma_f32 v[" #d ":" #d "+1], v[0:1], v[4:5], v[" #d ":" #d "+1]" ::: "v" #d); \
    else if constexpr (MODE == 1) asm volatile("v_pk_fma_f32 v[" #d "+2:" #d "+3], v[0:1], v[4:5], v[" #d "+2:" #d "+3]" ::: "v" #d); \
    else asm volatile("v_pk_fma_f32 v[" #d "+2:" #d "+3], v[0:1], v[6:7], v[" #d "+2:" #d "+3]" ::: "v" #d);
    F(32) F(36) F(40) F(44) F(48) F(52) F(56) F(60) F(64) F(68) F(72) F(76) F(80) F(84) F(88) F(92)
#undef F
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = 0.f;
}

template <int MODE>
static void run(float* d, unsigned long long* cyc, int wps) {
  const int iters = 4096, threads = 256 * wps;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(loop<MODE>, dim3(256), dim3(threads), 0, 0, d, iters, cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
  }
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double inst = (double)wps * iters * 16;  // per SIMD
  std::printf("{\"mode\": %d, \"waves_per_simd\": %d, \"wall_ms\": %.3f, \"ns_per_pk_per_simd\": %.3f}\n",
              MODE, wps, ms, ms * 1e6 / inst);
}

int main() {
  float* d;
  unsigned long long* cyc;
  (void)hipMalloc(&d, 256 * 1024 * sizeof(float));
  (void)hipMalloc(&cyc, 4096 * sizeof(unsigned long long));
  for (int i = 0; i < 3; ++i) run<0>(d, cyc, 2);  // warm the clock
  for (int w : {1, 2, 4}) {
    run<0>(d, cyc, w);
    run<1>(d, cyc, w);
    run<2>(d, cyc, w);
  }
  return 0;
}
