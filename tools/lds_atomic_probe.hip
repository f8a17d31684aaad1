// lds_atomic_probe.hip -- gfx950 cost of LDS atomics per wave instruction: ds_add_f32 (no
// return), ds_add_u32 (no return), ds_add_rtn_u32, and a plain ds_write_b32 for reference,
// with lane addresses (a) distinct consecutive dwords, (b) random within 256 dwords (the warp
// backward's 16 x 16 grad_x tile), (c) all lanes on one dword.  One workgroup per CU, 8 waves;
// wall time per wave instruction per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/lds_atomic_probe tools/lds_atomic_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int OP, int PAT>
__global__ __launch_bounds__(512) void probe(unsigned* out, int iters) {
  __shared__ float f[4096];
  __shared__ unsigned u[4096];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int i = t; i < 4096; i += 512) f[i] = 0.f, u[i] = 0u;
  __syncthreads();
  unsigned h = (unsigned)(lane * 2654435761u + wave * 40503u);
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int a;
      if (PAT == 0) a = wave * 64 + lane;
      else if (PAT == 1) { h = h * 1664525u + 1013904223u; a = wave * 256 + (h >> 24); }
      else a = wave * 64;
      if (OP == 0) __hip_atomic_fetch_add(&f[a & 4095], 1.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else if (OP == 1) __hip_atomic_fetch_add(&u[a & 4095], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else if (OP == 2) acc += __hip_atomic_fetch_add(&u[a & 4095], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else f[a & 4095] = (float)it;
    }
  }
  __syncthreads();
  out[blockIdx.x * 512 + t] = acc + u[t] + __float_as_uint(f[t]);
}

template <int OP, int PAT>
static void run(unsigned* d, const char* op, const char* pat) {
  const int iters = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((probe<OP, PAT>), dim3(256), dim3(512), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  const double winst = 8.0 * iters * 16;  // wave instructions per CU
  std::printf("{\"op\": \"%s\", \"addresses\": \"%s\", \"ns_per_wave_inst_per_cu\": %.3f, "
              "\"cycles_at_2.4GHz\": %.1f}\n",
              op, pat, best * 1e6 / winst, best * 1e6 / winst * 2.4);
}

template <int OP>
static void sweep(unsigned* d, const char* op) {
  run<OP, 0>(d, op, "distinct");
  run<OP, 1>(d, op, "random in 256");
  run<OP, 2>(d, op, "one dword");
}

int main() {
  unsigned* d;
  (void)hipMalloc(&d, 256 * 512 * sizeof(unsigned));
  sweep<0>(d, "ds_add_f32");
  sweep<1>(d, "ds_add_u32");
  sweep<2>(d, "ds_add_rtn_u32");
  sweep<3>(d, "ds_write_b32");
  return 0;
}
