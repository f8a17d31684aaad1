// issue_probe.hip -- gfx950 issue rates that decide the l4 correlation's lane design
// (DESIGN.md §4): cycles per instruction per SIMD for v_pk_fma_f32, v_fma_f32 and
// v_fmac_f32 with a DPP row_shr:1 operand, at 1 and 2 waves per SIMD; and the same
// pk_fma stream with 8 ds_read_b128 per 36 pk_fma interleaved (the correlation's inner
// ratio) at 1 wave per SIMD.  One workgroup per CU, s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 -o tools/issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// The correlation's channel step (csrc/corr_stream.hip fma_ti<2, 0, 9>): acc[9][8] += f1[p] *
// win[p + 2 ti] as 36 v_pk_fma_f32 over 6 window quads and 2 f1 quads held in registers.
__device__ __forceinline__ void corr_step(float (&acc)[9][8], const f4 (&w)[6], const f4 (&f)[2]) {
#pragma unroll
  for (int ti = 0; ti < 9; ++ti)
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int p = 2 * h, j = p + 2 * ti;
      const f4 a = f[h >> 1];
      const f2 a2 = (h & 1) ? f2{a.z, a.w} : f2{a.x, a.y};
      const f4 q = w[j >> 2];
      const f2 w2 = (j & 2) ? f2{q.z, q.w} : f2{q.x, q.y};
      f2 c2 = {acc[ti][p], acc[ti][p + 1]};
      c2 = __builtin_elementwise_fma(a2, w2, c2);
      acc[ti][p] = c2.x;
      acc[ti][p + 1] = c2.y;
    }
}

// MODE 4: corr_step with operands in registers (opaque per iteration, no instruction)
__global__ void corr_loop(float* out, int iters, unsigned long long* cyc) {
  float acc[9][8];
  for (int a = 0; a < 9; ++a)
    for (int k = 0; k < 8; ++k) acc[a][k] = 0.f;
  f4 w[6], f[2];
  for (int k = 0; k < 6; ++k) w[k] = f4{1.f * k, 2.f, 3.f, (float)threadIdx.x};
  for (int k = 0; k < 2; ++k) f[k] = f4{0.5f * k, 2.f, 1.f, (float)threadIdx.x};
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    asm volatile("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]),
                 "+v"(f[0]), "+v"(f[1]));
    corr_step(acc, w, f);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) cyc[512 + blockIdx.x] = r1 - r0;
  float s = 0;
  for (int a = 0; a < 9; ++a)
    for (int k = 0; k < 8; ++k) s += acc[a][k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// MODE 0: pk_fma x16   1: v_fma x32   2: v_fmac_dpp x32   3: pk_fma x36 + ds_read_b128 x8
template <int MODE>
__global__ void loop(float* out, int iters, unsigned long long* cyc) {
  extern __shared__ f4 lds[];
  f2 a0 = {1.f + threadIdx.x, 2.f}, b0 = {0.5f, 0.25f};
  f2 c[36];
  for (int i = 0; i < 36; ++i) c[i] = f2{(float)i, (float)-i};
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = f4{1.f, 2.f, 3.f, (float)i};
  __syncthreads();
  const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds +
                        (threadIdx.x & 255) * 16;
  f4 r[8];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[i]) : "v"(a0), "v"(b0));
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        asm volatile("v_fma_f32 %0, %1, %2, %0\n\tv_fma_f32 %3, %4, %5, %3"
                     : "+v"(c[i].x), "+v"(c[i].y)
                     : "v"(a0.x), "v"(b0.x), "v"(a0.y), "v"(b0.y));
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        asm volatile(
            "v_fmac_f32_dpp %0, %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_fmac_f32_dpp %1, %4, %5 row_shr:1 row_mask:0xf bank_mask:0xf"
            : "+v"(c[i].x), "+v"(c[i].y)
            : "v"(a0.x), "v"(b0.x), "v"(a0.y), "v"(b0.y));
    } else {
      asm volatile(
          "ds_read_b128 %0, %8 offset:0\n\tds_read_b128 %1, %8 offset:4096\n\t"
          "ds_read_b128 %2, %8 offset:8192\n\tds_read_b128 %3, %8 offset:12288\n\t"
          "ds_read_b128 %4, %8 offset:16384\n\tds_read_b128 %5, %8 offset:20480\n\t"
          "ds_read_b128 %6, %8 offset:24576\n\tds_read_b128 %7, %8 offset:28672"
          : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]),
            "=v"(r[7])
          : "v"(base)
          : "memory");
#pragma unroll
      for (int i = 0; i < 36; ++i)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[i]) : "v"(a0), "v"(b0));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      a0.x += r[0].x + r[1].y + r[2].z + r[3].w;
      b0.y += r[4].x + r[5].y + r[6].z + r[7].w;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 36; ++i) s += c[i].x + c[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(float* d, unsigned long long* cyc, int wps) {
  const int iters = 2048, threads = 256 * wps;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    if constexpr (MODE == 4)
      hipLaunchKernelGGL(corr_loop, dim3(256), dim3(threads), 0, 0, d, iters, cyc);
    else
      hipLaunchKernelGGL(loop<MODE>, dim3(256), dim3(threads), 65536, 0, d, iters, cyc);
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
  const int per = MODE == 0 ? 16 : MODE >= 3 ? 36 : 32;   // VALU instructions per iteration
  const int fma = MODE == 1 || MODE == 2 ? 1 : 2;          // FMAs per lane per instruction
  const double ninst = (double)wps * iters * per;
  const double flops = 2.0 * threads * 256 * (double)iters * per * fma;
  const char* nm[] = {"v_pk_fma_f32", "v_fma_f32", "v_fmac_f32_dpp", "pk_fma36+ds_read_b128x8",
                      "corr_step (36 pk_fma, register operands)"};
  double ghz = 0;
  if constexpr (MODE == 4) {  // s_memtime ticks per s_memrealtime tick (100 MHz)
    unsigned long long rt[256];
    (void)hipMemcpy(rt, cyc + 512, sizeof(rt), hipMemcpyDeviceToHost);
    double r = 0;
    for (int i = 0; i < 256; ++i) r += rt[i];
    ghz = avg / (r / 256) * 0.1;
  }
  std::printf("{\"probe\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_valu_inst_per_simd\": %.2f, "
              "\"wall_ms\": %.3f, \"tflops\": %.1f, \"memtime_ghz\": %.3f}\n",
              nm[MODE], wps, avg / ninst, ms, flops / (ms * 1e-3) / 1e12, ghz);
}

int main() {
  float* d;
  unsigned long long* cyc;
  (void)hipMalloc(&d, 256 * 2048 * sizeof(float));
  (void)hipMalloc(&cyc, 4096 * sizeof(unsigned long long));
  for (int w : {1, 2, 3, 4}) {
    run<4>(d, cyc, w);
    run<0>(d, cyc, w);
    run<1>(d, cyc, w);
    run<2>(d, cyc, w);
    run<3>(d, cyc, w);
  }
  return 0;
}
