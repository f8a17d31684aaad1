// Diagnostic (not part of the library): workgroup entry-time spread of one launch vs. grid
// size, threads per workgroup, dynamic LDS and VGPR footprint, from s_memrealtime (100 MHz)
// stamps written by every workgroup's thread 0.  Also the round trip of one dependent global
// load (HBM-resident and L2-resident lines) measured inside a workgroup.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/entry_probe tools/entry_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int VG>
__global__ void entry_k(unsigned long long* stamps, float* sink, int touch) {
  extern __shared__ float lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float acc[VG];
#pragma unroll
  for (int i = 0; i < VG; ++i) acc[i] = (float)(threadIdx.x + i);
  if (touch) lds[threadIdx.x] = acc[0];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < VG; ++i) acc[i] = acc[i] * acc[(i + 1) % VG] + 1.f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VG; ++i) s += acc[i];
  if (threadIdx.x == 0) stamps[blockIdx.x] = t0;
  if (s == -1.f) sink[threadIdx.x] = s;
}

// dependent-load chain: p[i] holds the index of the next element (stride `step` floats)
__global__ void chase_k(const int* __restrict__ p, unsigned long long* out, int hops, int start) {
  if (threadIdx.x != 0) return;
  int i = start + blockIdx.x * 4096;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int h = 0; h < hops; ++h) i = __builtin_nontemporal_load(p + i);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x] = (t1 - t0) * 1000ull / (unsigned)hops + (i == -7 ? 1 : 0);  // 10*ns/hop
}

template <int VG>
static void run(int grid, int threads, int lds_kb) {
  unsigned long long* st;
  float* sink;
  (void)hipMalloc(&st, sizeof(unsigned long long) * grid);
  (void)hipMalloc(&sink, 4096);
  (void)hipFuncSetAttribute((const void*)entry_k<VG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  std::vector<unsigned long long> h(grid);
  double spread = 0;
  for (int r = 0; r < 8; ++r) {
    hipLaunchKernelGGL(entry_k<VG>, dim3(grid), dim3(threads), (size_t)lds_kb * 1024, 0, st,
                       sink, 1);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h.data(), st, sizeof(unsigned long long) * grid, hipMemcpyDeviceToHost);
    auto mm = std::minmax_element(h.begin(), h.end());
    if (r >= 3) spread += (double)(*mm.second - *mm.first) / 100.0;
  }
  std::printf("{\"probe\": \"entry\", \"grid\": %d, \"threads\": %d, \"lds_kb\": %d, \"vgpr_arr\": %d, "
              "\"spread_us\": %.2f}\n", grid, threads, lds_kb, VG, spread / 5);
  (void)hipFree(st);
  (void)hipFree(sink);
}

int main() {
  for (int grid : {144, 256, 512})
    for (int threads : {256, 512})
      for (int lds : {0, 74, 150}) {
        run<8>(grid, threads, lds);
        run<200>(grid, threads, lds);
      }
  // dependent-load round trip: 1 GB buffer (HBM, lines never reused), 1 MB (L2)
  for (size_t bytes : {(size_t)1 << 30, (size_t)1 << 20}) {
    const int n = (int)(bytes / 4);
    std::vector<int> h(n);
    const int step = 64 * 1024 + 32;  // new line, new page region each hop
    for (int i = 0; i < n; ++i) h[i] = (int)(((long long)i + step) % n);
    int* d;
    unsigned long long* o;
    (void)hipMalloc(&d, bytes);
    (void)hipMalloc(&o, 256 * 8);
    (void)hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
    std::vector<unsigned long long> ho(256);
    for (int r = 0; r < 3; ++r) {
      hipLaunchKernelGGL(chase_k, dim3(256), dim3(64), 0, 0, d, o, 64, r * 977);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(ho.data(), o, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(ho.begin(), ho.end());
    std::printf("{\"probe\": \"chase\", \"bytes\": %zu, \"ns_per_hop_median\": %.1f, \"max\": %.1f}\n",
                bytes, ho[128] / 100.0, ho[255] / 100.0);
    (void)hipFree(d);
    (void)hipFree(o);
  }
  return 0;
}
