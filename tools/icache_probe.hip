// Diagnostic (not part of the library): is a kernel's instruction stream re-fetched from L2
// on every launch?  A wave runs a straight block of N 4-byte `s_nop 0` (1 cycle each when the
// instruction cache hits) between two s_memrealtime stamps; launches repeat back to back.
// If each launch starts with a cold instruction cache the block runs at the fetch latency per
// 64-B line instead of ~1 instruction per cycle.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/icache_probe tools/icache_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define NOPS(n) asm volatile(".rept " #n "\n\ts_nop 0\n\t.endr" ::: "memory")

template <int K>
__global__ void nop_k(unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (K == 1) NOPS(256);
  if constexpr (K == 2) NOPS(4096);
  if constexpr (K == 3) NOPS(16384);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char* name, int grid, unsigned long long* d) {
  std::vector<unsigned long long> h(grid);
  for (int r = 0; r < 6; ++r) {
    hipLaunchKernelGGL(nop_k<K>, dim3(grid), dim3(256), 0, 0, d);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h.data(), d, 8 * grid, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    std::printf("{\"probe\": \"icache\", \"block\": \"%s\", \"grid\": %d, \"launch\": %d, "
                "\"median_us\": %.2f, \"max_us\": %.2f}\n",
                name, grid, r, h[grid / 2] / 100.0, h[grid - 1] / 100.0);
  }
}

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 8 * 4096);
  run<1>("256 nops (1 KB)", 256, d);
  run<2>("4096 nops (16 KB)", 256, d);
  run<3>("16384 nops (64 KB)", 256, d);
  return 0;
}
