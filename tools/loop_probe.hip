// loop_probe.hip -- the l4 correlation's inner loop in isolation (no DMA, no stores, no barrier):
// per "step" a lane runs 16 channels of (window reads from LDS + v_pk_fma_f32 into its
// accumulators), one workgroup per CU, WPC waves per CU; wall time per step.  Variants:
//   MODE 0: 4 ds_read_b64 + 6 pk per channel, read-ahead LA channels, a wait per channel
//   MODE 1: 2 ds_read_b128 + 6 pk per channel (quad-aligned windows), read-ahead LA
//   MODE 2: as 0 with the waits batched (3 channels per wait)
//   MODE 3: 5 ds_read_b128 + 18 pk per channel (corr_strip.hip's inner loop), LA
//   MODE 4: pk only (window regs opaque), MODE 5: reads only (b64, waits as MODE 0)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/loop_probe tools/loop_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void lgk() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void rd64(f2& d, uint32_t a, int o) {
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(o) : "memory");
}
__device__ __forceinline__ void rd128(f4& d, uint32_t a, int o) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(o) : "memory");
}
__device__ __forceinline__ void pk(f2& c, f2 a, f2 b) {
  asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

template <int MODE, int LA>
__global__ void probe(float* out, int steps) {
  extern __shared__ f4 lds[];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = f4{1.f, 0.5f, 0.25f, (float)i};
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // conflict-free lane addresses: 8 B per lane for the b64 modes, 16 B for the b128 ones
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds +
                     (uint32_t)((lane & 31) * (MODE == 0 || MODE == 2 || MODE == 5 ? 8 : 16) +
                                (lane >> 5) * 7680);
  f4 f1[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) f1[i] = f4{1.f + i, 0.5f, 0.25f, (float)lane};
  f2 acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f2{0.f, 0.f};
  for (int st = 0; st < steps; ++st) {
    if constexpr (MODE == 0 || MODE == 5) {
      f2 w[LA + 1][4];
#pragma unroll
      for (int k = 0; k < LA; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) rd64(w[k][j], a, k * 480 + 8 * j);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i + LA < 16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) rd64(w[(i + LA) % (LA + 1)][j], a, (i + LA) * 480 + 8 * j);
          lgk<4 * LA>();
        } else {
          lgk<0>();
        }
        if constexpr (MODE == 0) {
          f2(&q)[4] = w[i % (LA + 1)];
          const f2 lo = {f1[i].x, f1[i].y}, hi = {f1[i].z, f1[i].w};
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            pk(acc[t][0], lo, q[t]);
            pk(acc[t][1], hi, q[t + 1]);
          }
        } else {
          asm volatile("" ::"v"(w[i % (LA + 1)][0]), "v"(w[i % (LA + 1)][3]));
        }
      }
    } else if constexpr (MODE == 1) {
      f4 w[LA + 1][2];
#pragma unroll
      for (int k = 0; k < LA; ++k)
#pragma unroll
        for (int j = 0; j < 2; ++j) rd128(w[k][j], a, k * 480 + 16 * j);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i + LA < 16) {
#pragma unroll
          for (int j = 0; j < 2; ++j) rd128(w[(i + LA) % (LA + 1)][j], a, (i + LA) * 480 + 16 * j);
          lgk<2 * LA>();
        } else {
          lgk<0>();
        }
        f4(&q)[2] = w[i % (LA + 1)];
        const f2 p[4] = {{q[0].x, q[0].y}, {q[0].z, q[0].w}, {q[1].x, q[1].y}, {q[1].z, q[1].w}};
        const f2 lo = {f1[i].x, f1[i].y}, hi = {f1[i].z, f1[i].w};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          pk(acc[t][0], lo, p[t]);
          pk(acc[t][1], hi, p[t + 1]);
        }
      }
    } else if constexpr (MODE == 2) {
      // batches of 3 channels (12 reads) per wait; the 16th channel alone
      f2 w[2][3][4];
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) rd64(w[0][c][j], a, c * 480 + 8 * j);
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const int nb = b + 1;
        if (nb < 6) {
#pragma unroll
          for (int c = 0; c < 3; ++c)
            if (3 * nb + c < 16)
#pragma unroll
              for (int j = 0; j < 4; ++j) rd64(w[nb & 1][c][j], a, (3 * nb + c) * 480 + 8 * j);
          if (3 * nb + 2 < 16) lgk<12>(); else lgk<4>();
        } else {
          lgk<0>();
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int i = 3 * b + c;
          if (i >= 16) break;
          f2(&q)[4] = w[b & 1][c];
          const f2 lo = {f1[i].x, f1[i].y}, hi = {f1[i].z, f1[i].w};
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            pk(acc[t][0], lo, q[t]);
            pk(acc[t][1], hi, q[t + 1]);
          }
        }
      }
    } else if constexpr (MODE == 3) {
      f4 w[LA + 1][5];
#pragma unroll
      for (int k = 0; k < LA; ++k)
#pragma unroll
        for (int j = 0; j < 5; ++j) rd128(w[k][j], a, k * 480 + 16 * j);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (i + LA < 16) {
#pragma unroll
          for (int j = 0; j < 5; ++j) rd128(w[(i + LA) % (LA + 1)][j], a, (i + LA) * 480 + 16 * j);
          lgk<5 * LA>();
        } else {
          lgk<0>();
        }
        f4(&q)[5] = w[i % (LA + 1)];
        const f2 lo = {f1[i].x, f1[i].y}, hi = {f1[i].z, f1[i].w};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int j0 = 2 * t, j1 = 2 * t + 2;
          const f2 w0 = (j0 & 2) ? f2{q[j0 >> 2].z, q[j0 >> 2].w} : f2{q[j0 >> 2].x, q[j0 >> 2].y};
          const f2 w1 = (j1 & 2) ? f2{q[j1 >> 2].z, q[j1 >> 2].w} : f2{q[j1 >> 2].x, q[j1 >> 2].y};
          pk(acc[t][0], lo, w0);
          pk(acc[t][1], hi, w1);
        }
      }
    } else {  // MODE 4: pk only
      f2 q[4] = {{1.f, 2.f}, {3.f, 4.f}, {5.f, 6.f}, {7.f, 8.f}};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        asm volatile("" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]));
        const f2 lo = {f1[i].x, f1[i].y}, hi = {f1[i].z, f1[i].w};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          pk(acc[t][0], lo, q[t]);
          pk(acc[t][1], hi, q[t + 1]);
        }
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) s += acc[t][0].x + acc[t][1].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int LA>
static void run(float* d, int wpc, const char* name) {
  const int steps = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&probe<MODE, LA>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((probe<MODE, LA>), dim3(256), dim3(64 * wpc), 131072, 0, d, steps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  std::printf("{\"variant\": \"%s\", \"mode\": %d, \"la\": %d, \"waves_per_cu\": %d, "
              "\"us_per_step\": %.3f}\n",
              name, MODE, LA, wpc, best * 1e3 / steps);
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 1024 * sizeof(float));
  for (int w : {8, 12, 16}) {
    run<0, 2>(d, w, "b64 x4 + 6 pk, LA2");
    run<0, 3>(d, w, "b64 x4 + 6 pk, LA3");
    run<1, 2>(d, w, "b128 x2 + 6 pk, LA2");
    run<1, 4>(d, w, "b128 x2 + 6 pk, LA4");
    run<1, 7>(d, w, "b128 x2 + 6 pk, LA7");
    run<2, 0>(d, w, "b64 x4 + 6 pk, 3-channel batches");
    run<3, 1>(d, w, "b128 x5 + 18 pk (strip), LA1");
    run<3, 2>(d, w, "b128 x5 + 18 pk (strip), LA2");
    run<4, 0>(d, w, "6 pk only");
    run<5, 2>(d, w, "b64 x4 reads only, LA2");
  }
  return 0;
}
