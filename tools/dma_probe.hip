// Diagnostic (not part of the library): L2 -> LDS fill rate per CU for LDS-DMA
// (buffer_load_dwordx4 ... lds) vs register staging (global_load_dwordx4 + ds_write_b128) vs
// plain loads to registers, on an L2-resident source.  Each wave moves 1 KiB per
// instruction into a private 16 KiB LDS slice, `depth` instructions in flight.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/dma_probe tools/dma_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE, int DEPTH>
__global__ __launch_bounds__(1024) void fill(const float* __restrict__ src, float* out,
                                             unsigned src_bytes, int iters) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds;
  const unsigned my_lds = lds_base + wave * 16384u;  // 16 KiB per wave
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)src_bytes, 0x00020000);
  // each block walks its own region of the source (wraps): 1 KiB per wave-instruction
  unsigned off = (blockIdx.x * 64u + wave * 4u) * 1024u % src_bytes;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const unsigned o = (off + d * 1024u) % src_bytes;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(uintptr_t)(my_lds + (d % 16) * 1024u),
            16, o + lane * 16u, 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      float4 v[DEPTH];
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const unsigned o = (off + d * 1024u) % src_bytes;
        v[d] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rs, o + lane * 16u, 0, 0));
      }
      if constexpr (MODE == 1) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
          *reinterpret_cast<float4*>(&lds[wave * 4096 + (d % 16) * 256 + lane * 4]) = v[d];
      } else {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) acc += v[d].x + v[d].y + v[d].z + v[d].w;
      }
    }
    off = (off + DEPTH * 1024u * 4u) % src_bytes;
  }
  if (MODE == 2) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  else out[blockIdx.x * blockDim.x + threadIdx.x] = lds[threadIdx.x];
}

template <int MODE, int DEPTH>
void run(const char* name, const float* src, float* out, unsigned src_bytes, int waves, int bpc) {
  const int nblk = 256 * bpc, iters = 200;
  const size_t lds = (size_t)waves * 16384;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&fill<MODE, DEPTH>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((fill<MODE, DEPTH>), dim3(nblk), dim3(waves * 64), lds, 0, src, out,
                     src_bytes, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((fill<MODE, DEPTH>), dim3(nblk), dim3(waves * 64), lds, 0, src, out,
                     src_bytes, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)nblk * waves * iters * DEPTH * 1024.0;
  printf("%-14s src %5u KiB waves %2d x %d/CU depth %2d: %7.1f GB/s chip, %6.1f GB/s per CU\n",
         name, src_bytes >> 10, waves, bpc, DEPTH, bytes / (ms * 1e-3) / 1e9,
         bytes / (ms * 1e-3) / 1e9 / 256);
}

int main() {
  float *src, *out;
  const unsigned big = 64u << 20;
  (void)hipMalloc(&src, big);
  (void)hipMalloc(&out, 1 << 24);
  (void)hipMemset(src, 0, big);
  for (unsigned sb : {1u << 20, 64u << 20}) {
    run<0, 4>("lds-dma", src, out, sb, 4, 1);
    run<0, 8>("lds-dma", src, out, sb, 4, 1);
    run<0, 8>("lds-dma", src, out, sb, 8, 1);
    run<0, 8>("lds-dma", src, out, sb, 4, 2);
    run<0, 16>("lds-dma", src, out, sb, 8, 1);
    run<1, 4>("reg+ds_write", src, out, sb, 4, 1);
    run<1, 8>("reg+ds_write", src, out, sb, 8, 1);
    run<1, 8>("reg+ds_write", src, out, sb, 4, 2);
    run<2, 8>("reg only", src, out, sb, 8, 1);
    run<2, 8>("reg only", src, out, sb, 4, 2);
  }
  return 0;
}
