// Diagnostic: per-CU LDS-DMA fill rate on gfx950.  One 512-thread workgroup per CU streams
// `chunk` bytes of a large buffer into a ring of NS 16-KiB slots (buffer_load_dwordx4 ... lds,
// 1 KiB per wave-instruction, 2 pieces per wave per slot), waiting with a counted vmcnt and a
// barrier per slot.  Modes: 0 = contiguous source, 1 = 8 rows x 128 B per piece at a 448-B row
// pitch (the correlation tile rows, misaligned to 64 B), 2 = like 0 but every pair of
// workgroups reads the same chunk (half the unique bytes: L2 reuse), 3 = register path
// (global_load_dwordx4 + ds_write_b128) on the contiguous source.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

template <int N>
__device__ __forceinline__ void vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int NS>
__global__ __launch_bounds__(512) void dma(const float* src, size_t chunk, int mode, float* out) {
#if defined(__HIP_DEVICE_COMPILE__)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = mode & 7;
  const int wg = m == 2 ? blockIdx.x / 2 : m == 4 ? 0 : blockIdx.x;
  const char* base = (const char*)src + (size_t)wg * (1u << 20);
  const int slots = (int)(chunk / 16384);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 1 << 20, 0x00020000);
  auto voff = [&](int slot, int piece) -> uint32_t {
    const uint32_t pb = (uint32_t)slot * 16384u + (uint32_t)piece * 1024u;
    if (m == 1)  // piece = 8 rows of 128 B at pitch 448, starting 64 B into a line
      return (pb / 1024) * 8 * 448 + (lane >> 3) * 448 + 64 + (lane & 7) * 16;  // < 1 MiB
    if (m == 5)  // 8 rows of 128 B at pitch 512: line-aligned segments
      return (pb / 1024) * 8 * 512 + (lane >> 3) * 512 + (lane & 7) * 16;
    if (m == 6)  // 16 rows of 64 B at pitch 448 (f1-like half lines)
      return (pb / 1024) * 16 * 448 + (lane >> 2) * 448 + (lane & 3) * 16;
    if (m == 7)  // 8 rows of 128 B at pitch 448, 32 B into the row (the f2 window shape)
      return (pb / 1024) * 8 * 448 + (lane >> 3) * 448 + 32 + (lane & 7) * 16;
    if (m == 4) return (pb + lane * 16) & ((1u << 18) - 1);  // every WG: the same 256 KiB
    return pb + lane * 16;
  };
  auto issue = [&](int slot) {
    for (int i = 0; i < 2; ++i) {
      const int piece = wave * 2 + i;
      const uint32_t dst = lds0 + (uint32_t)(slot % NS) * 16384u + piece * 1024u;
      if (m == 3) {
        const uint32_t o = voff(slot, piece);
        const float4 v = o < (1u << 20) ? *(const float4*)(base + o) : make_float4(0, 0, 0, 0);
        *(float4*)((char*)lds + (dst - lds0) + lane * 16) = v;
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(uintptr_t)dst, 16, voff(slot, piece), 0, 0, 0);
      }
    }
  };
  for (int s = 0; s < NS - 1 && s < slots; ++s) issue(s);
  float acc = 0.f;
  for (int s = 0; s < slots; ++s) {
    if (m != 3) {
      if (slots - 1 - s >= NS - 2) vm<(NS - 2) * 2>(); else vm<0>();
    }
    if (!(mode & 8)) __syncthreads();
    if (s + NS - 1 < slots) issue(s + NS - 1);
    acc += lds[(s % NS) * 4096 + threadIdx.x];
  }
  if (acc == 1234.5f) out[blockIdx.x] = acc;
#endif
}

int main() {
  const size_t chunk = 256 * 1024;  // per workgroup
  const int nwg = 256;
  float *src, *out;
  (void)hipMalloc(&src, (size_t)nwg * (1u << 20) * 4);  // 1 MiB per workgroup, 4 copies
  (void)hipMalloc(&out, 4096);
  (void)hipMemset(src, 0, (size_t)nwg * (1u << 20) * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int mode : {0, 4, 8, 12, 7, 15}) {
    if (hipGetLastError() != hipSuccess) return 1;
    for (int ns : {4, 8}) {
      (void)hipFuncSetAttribute((const void*)dma<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 16384);
      (void)hipFuncSetAttribute((const void*)dma<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 16384);
      float best = 1e9, sum = 0;
      const int reps = 40;
      for (int r = 0; r < reps + 5; ++r) {
        const float* s = src + (size_t)(r % 4) * nwg * (1u << 20) / 4;
        if (ns == 4)
          hipExtLaunchKernelGGL(dma<4>, dim3(nwg), dim3(512), ns * 16384, 0, e0, e1, 0, s, chunk, mode, out);
        else
          hipExtLaunchKernelGGL(dma<8>, dim3(nwg), dim3(512), ns * 16384, 0, e0, e1, 0, s, chunk, mode, out);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 5) { sum += ms; if (ms < best) best = ms; }
      }
      const double avg = sum / reps;
      const double bytes = (double)chunk * nwg;
      std::printf("mode %d NS %d: avg %.2f us  per-CU %.1f GB/s  chip %.2f TB/s (min %.2f us)\n", mode, ns,
                  avg * 1e3, chunk / (avg * 1e-3) / 1e9, bytes / (avg * 1e-3) / 1e12, best * 1e3);
    }
  }
  return 0;
}
