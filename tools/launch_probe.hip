// Diagnostic (not part of the library): the per-launch floor of dependent back-to-back kernels
// on one stream, plain and replayed from a hipGraph, for trivial kernels of several grid sizes.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void touch(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

template <bool USE_LDS, bool BAR>
__global__ void touch_v(float* p, int n) {
  extern __shared__ float l[];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = (float)i;
  if (USE_LDS) {
    l[threadIdx.x] = v;
    v = l[(threadIdx.x + 1) % blockDim.x];
  }
  if (BAR) __syncthreads();
  if (i < n) p[i] = v;
}

__global__ void touch_lds(float* p, int n) {
  extern __shared__ float l[];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  l[threadIdx.x] = (float)i;
  __syncthreads();
  if (i < n) p[i] = l[(threadIdx.x + 1) % blockDim.x];
}

template <class F>
float time_it(hipStream_t s, int reps, F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int r = 0; r < 20; ++r) f();
  (void)hipStreamSynchronize(s);
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  float* p;
  const int nmax = 1 << 24;
  (void)hipMalloc(&p, nmax * 4);
  (void)hipMemset(p, 0, nmax * 4);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int sizes[] = {64, 4096, 65536, 1 << 20, 1 << 22};
  for (int n : sizes) {
    const int blocks = (n + 255) / 256;
    const int reps = 200;
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(touch, dim3(blocks), dim3(256), 0, s, p, n);
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(touch, dim3(blocks), dim3(256), 0, s, p, n);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // graph of 10 dependent launches
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(touch, dim3(blocks), dim3(256), 0, s, p, n);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps / 10; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float msg = 0;
    (void)hipEventElapsedTime(&msg, e0, e1);
    printf("n=%8d blocks=%6d: stream %.2f us/launch, graph %.2f us/launch (%.1f GB/s at graph)\n",
           n, blocks, ms * 1e3 / reps, msg * 1e3 / reps, 8.0 * n / (msg * 1e-3 / reps) / 1e9);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  hipFuncSetAttribute(reinterpret_cast<const void*>(&touch_v<true, true>), hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  // floor of a trivial kernel vs grid size, LDS use and a workgroup barrier
  for (int nb : {256, 288, 512, 1024}) {
    const int n = nb * 256;
    const float a = time_it(s, 200, [&] { hipLaunchKernelGGL((touch_v<false, false>), dim3(nb), dim3(256), 0, s, p, n); });
    const float b = time_it(s, 200, [&] { hipLaunchKernelGGL((touch_v<false, true>), dim3(nb), dim3(256), 0, s, p, n); });
    const float c = time_it(s, 200, [&] { hipLaunchKernelGGL((touch_v<true, false>), dim3(nb), dim3(256), 4096, s, p, n); });
    const float d = time_it(s, 200, [&] { hipLaunchKernelGGL((touch_v<true, true>), dim3(nb), dim3(256), 4096, s, p, n); });
    const float e = time_it(s, 200, [&] { hipLaunchKernelGGL((touch_v<true, true>), dim3(nb), dim3(256), 65536, s, p, n); });
    printf("%4d blocks: plain %.2f | barrier %.2f | lds %.2f | lds+barrier %.2f | 64K lds+barrier %.2f us\n",
           nb, a, b, c, d, e);
  }
  return 0;
}
