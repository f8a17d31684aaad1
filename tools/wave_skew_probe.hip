// Diagnostic (not part of the library): how far apart the waves of ONE workgroup start, and
// what the first barrier costs, against threads per workgroup, VGPR footprint and dynamic LDS.
// Every wave's first lane stamps s_memrealtime (100 MHz) at entry and after an s_barrier.
// Launches run back to back (the stamped launch is the last of 20), as in the bench.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/wave_skew_probe tools/wave_skew_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int VG, int NT>
__global__ __launch_bounds__(NT) void skew_k(unsigned long long* st, float* sink, int nw) {
  extern __shared__ float lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float acc[VG];
#pragma unroll
  for (int i = 0; i < VG; ++i) acc[i] = (float)(threadIdx.x + i);
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int i = 0; i < VG; ++i) acc[i] = acc[i] * acc[(i + 1) % VG] + 1.f;
  lds[threadIdx.x] = acc[0];
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  float s = lds[(threadIdx.x + 1) % blockDim.x];
#pragma unroll
  for (int i = 0; i < VG; ++i) s += acc[i];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    st[(blockIdx.x * nw + w) * 2] = t0;
    st[(blockIdx.x * nw + w) * 2 + 1] = t1;
  }
  if (s == -1.f) sink[threadIdx.x] = s;
}

template <int VG, int NT>
void run(int nblk, int lds) {
  const int nt = NT;
  const int nw = nt / 64;
  unsigned long long* st;
  float* sink;
  hipMalloc(&st, sizeof(unsigned long long) * nblk * nw * 2);
  hipMalloc(&sink, 4096);
  hipFuncSetAttribute(reinterpret_cast<const void*>(&skew_k<VG, NT>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int i = 0; i < 20; ++i)
    hipLaunchKernelGGL((skew_k<VG, NT>), dim3(nblk), dim3(nt), lds, 0, st, sink, nw);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(nblk * nw * 2);
  hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> skew, bar;
  unsigned long long tmin = ~0ull;
  for (int b = 0; b < nblk; ++b) tmin = std::min(tmin, h[(b * nw) * 2]);
  for (int b = 0; b < nblk; ++b) {
    unsigned long long e0 = ~0ull, e1 = 0;
    for (int w = 0; w < nw; ++w) {
      e0 = std::min(e0, h[(b * nw + w) * 2]);
      e1 = std::max(e1, h[(b * nw + w) * 2]);
    }
    skew.push_back((e1 - e0) / 100.0);
    bar.push_back((h[(b * nw) * 2 + 1] - e0) / 100.0);
  }
  std::sort(skew.begin(), skew.end());
  std::sort(bar.begin(), bar.end());
  printf("{\"blocks\": %d, \"threads\": %d, \"vgprs_req\": %d, \"lds\": %d, "
         "\"wave_skew_us\": [%.2f, %.2f], \"barrier_after_entry_us\": [%.2f, %.2f]}\n",
         nblk, nt, VG, lds, skew[skew.size() / 2], skew.back(), bar[bar.size() / 2], bar.back());
  hipFree(st);
  hipFree(sink);
}

int main() {
  run<16, 256>(144, 0);
  run<160, 256>(144, 0);
  run<16, 512>(144, 0);
  run<160, 512>(144, 0);
  run<160, 512>(144, 80 * 1024);
  run<16, 1024>(144, 0);
  run<96, 1024>(144, 0);
  run<16, 512>(256, 128 * 1024);
  return 0;
}
