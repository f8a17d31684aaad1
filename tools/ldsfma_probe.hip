// Diagnostic (not part of the library): throughput of the correlation inner loop on one CU,
// without DMA.  Per "channel" each lane reads LDS quads and runs 36 FMAs (4 pixels x 9 ti),
// exactly as corr_ring's consumer; varied: waves per workgroup, workgroups per CU, barrier
// period, read scheme.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize
//                                  -o tools/ldsfma_probe tools/ldsfma_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int OFF>
__device__ __forceinline__ void rd6(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                    uint32_t a4, uint32_t a5, f32x4& r0, f32x4& r1, f32x4& r2,
                                    f32x4& r3, f32x4& r4, f32x4& r5) {
  asm volatile(
      "ds_read_b128 %0, %6 offset:%12\n\t"
      "ds_read_b128 %1, %7 offset:%12\n\t"
      "ds_read_b128 %2, %8 offset:%12\n\t"
      "ds_read_b128 %3, %9 offset:%12\n\t"
      "ds_read_b128 %4, %10 offset:%12\n\t"
      "ds_read_b128 %5, %11 offset:%12\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "n"(OFF)
      : "memory");
}
template <int OFF>
__device__ __forceinline__ void rd4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                    f32x4& r0, f32x4& r1, f32x4& r2, f32x4& r3) {
  asm volatile(
      "ds_read_b128 %0, %4 offset:%8\n\t"
      "ds_read_b128 %1, %5 offset:%8\n\t"
      "ds_read_b128 %2, %6 offset:%8\n\t"
      "ds_read_b128 %3, %7 offset:%8\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "n"(OFF)
      : "memory");
}

constexpr int CH_B = 5120;  // bytes per channel block (as RingC)
constexpr int NCHB = 8;     // channel blocks cycled through (40 KiB)

// MODE 0: 6 reads / wait / 36 FMA.  MODE 1: 4 reads (de-interleaved window) / 36 FMA.
// MODE 2: reads only.  MODE 3: FMA only (operands from registers).
template <int MODE, int CI>
__device__ __forceinline__ void chan(const uint32_t (&ad)[6], float (&acc)[9][4], f32x4 (&keep)[6]) {
  constexpr int OFF = (CI % NCHB) * CH_B;
  f32x4 a, b[5];
  if constexpr (MODE == 0 || MODE == 2) {
    rd6<OFF>(ad[0], ad[1], ad[2], ad[3], ad[4], ad[5], a, b[0], b[1], b[2], b[3], b[4]);
  } else if constexpr (MODE == 1) {
    rd4<OFF>(ad[0], ad[1], ad[2], ad[3], a, b[0], b[1], b[2]);
    b[3] = b[0];
    b[4] = b[1];
  } else {
    a = keep[0];
    for (int u = 0; u < 5; ++u) b[u] = keep[u + 1];
  }
  if constexpr (MODE == 2) {
    asm volatile("" ::"v"(a), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]));
    return;
  }
  if constexpr (MODE == 4 || MODE == 5) {  // packed: acc pairs += a pairs * w pairs
    if constexpr (MODE == 5) {
      a = keep[0];
      for (int u = 0; u < 5; ++u) b[u] = keep[u + 1];
    }
#pragma unroll
    for (int ti = 0; ti < 9; ++ti) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * h + 2 * ti;  // even
        const f32x4 q = b[j >> 2];
        const f32x2 w2 = (j & 2) ? f32x2{q.z, q.w} : f32x2{q.x, q.y};
        const f32x2 a2 = h ? f32x2{a.z, a.w} : f32x2{a.x, a.y};
        f32x2 c2 = {acc[ti][2 * h], acc[ti][2 * h + 1]};
        c2 = __builtin_elementwise_fma(a2, w2, c2);
        acc[ti][2 * h] = c2.x;
        acc[ti][2 * h + 1] = c2.y;
      }
    }
    return;
  }
  const float av[4] = {a.x, a.y, a.z, a.w};
  float w[20];
  for (int u = 0; u < 5; ++u) {
    w[4 * u] = b[u].x; w[4 * u + 1] = b[u].y; w[4 * u + 2] = b[u].z; w[4 * u + 3] = b[u].w;
  }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int ti = 0; ti < 9; ++ti)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[ti][k] = fmaf(av[k], w[k + ti], acc[ti][k]);
  } else {
#pragma unroll
    for (int ti = 0; ti < 9; ++ti)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[ti][k] = fmaf(av[k], w[k + 2 * ti], acc[ti][k]);
  }
}

template <int MODE, int BAR, int CI>
__device__ __forceinline__ void period(const uint32_t (&ad)[6], float (&acc)[9][4], f32x4 (&keep)[6]) {
  if constexpr (CI < BAR) {
    chan<MODE, CI>(ad, acc, keep);
    period<MODE, BAR, CI + 1>(ad, acc, keep);
  }
}

template <int MODE, int BAR>
__global__ __launch_bounds__(1024) void probe(float* out, int periods, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) float lds[NCHB * CH_B / 4];
  for (int i = threadIdx.x; i < NCHB * CH_B / 4; i += blockDim.x) lds[i] = (float)(i & 255) * 0.001f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane & 3, ty = lane >> 2, tjx = wave % 9;
  const int r2 = ty + 2 * tjx, sw = ((r2 >> 1) & 1) << 2;
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds;
  uint32_t ad[6];
  ad[0] = base + (uint32_t)(1024 + ty * 16 + 4 * q) * 4u;
  for (int u = 0; u < 5; ++u) ad[u + 1] = base + (uint32_t)(r2 * 32 + (((q + u) ^ sw) << 2)) * 4u;
  float acc[9][4];
  for (int a = 0; a < 9; ++a)
    for (int k = 0; k < 4; ++k) acc[a][k] = 0.f;
  f32x4 keep[6];
  for (int u = 0; u < 6; ++u) keep[u] = f32x4{0.1f * u, 0.2f, 0.3f, 0.4f + lane};
  for (int p = 0; p < periods; ++p) {
    period<MODE, BAR, 0>(ad, acc, keep);
    __builtin_amdgcn_s_barrier();
  }
  float s = 0.f;
  for (int a = 0; a < 9; ++a)
    for (int k = 0; k < 4; ++k) s += acc[a][k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    clk[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int MODE, int BAR>
void run(const char* name, int waves, int bpc, int chans) {
  const int periods = chans / BAR;
  const int nblk = 256 * bpc;
  float* out;
  unsigned long long* clk;
  (void)hipMalloc(&out, (size_t)nblk * waves * 64 * 4);
  (void)hipMalloc(&clk, (size_t)nblk * 16);
  hipLaunchKernelGGL((probe<MODE, BAR>), dim3(nblk), dim3(waves * 64), 0, 0, out, periods, clk);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((probe<MODE, BAR>), dim3(nblk), dim3(waves * 64), 0, 0, out, periods, clk);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2];
  (void)hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double us = ms * 1e3 / reps;
  const double ghz = (double)h[0] / ((double)h[1] / 100.0) / 1e3;  // memtime ticks per us
  const double cyc_per_ch = (double)h[0] / (periods * BAR);
  const double reads = waves * (MODE == 1 ? 4 : 6) * bpc;  // per channel per CU
  printf("%-10s waves %2d x %d/CU bar %2d: %7.2f us, block0 %.0f cyc/ch (clk %.2f GHz) -> "
         "%.1f cyc per ds_read_b128/CU, %.2f cyc per FMA/SIMD\n",
         name, waves, bpc, BAR, us, cyc_per_ch, ghz, cyc_per_ch / reads,
         cyc_per_ch / (waves * bpc * 36.0 / 4.0));
  (void)hipFree(out);
  (void)hipFree(clk);
}

int main() {
  const int CH = 512;
  run<4, 2>("rd6+pkfma", 9, 1, CH);
  run<4, 2>("rd6+pkfma", 9, 2, CH);
  run<4, 8>("rd6+pkfma", 9, 1, CH);
  run<4, 8>("rd6+pkfma", 9, 2, CH);
  run<4, 32>("rd6+pkfma", 9, 1, CH);
  run<4, 32>("rd6+pkfma", 9, 2, CH);
  run<4, 2>("rd6+pkfma", 3, 4, CH);
  run<4, 2>("rd6+pkfma", 3, 6, CH);
  return 0;
}
