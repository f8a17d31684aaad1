// store_probe.hip -- write-only timing of the l4 correlation volume (B=8, 81 x 96 x 112 fp32,
// 27.9 MB) under different store address patterns, 256 workgroups x 512 threads, 15 16-B
// nontemporal stores per lane (what corr_fwd_strip issues), rotating over 8 volumes:
//   strip      -- corr_fwd_strip's pattern: workgroup = (n, parity, 6-row group, 56-px strip),
//                 lane = (tj, 4-px segment, half), 5 planes x 3 steps; a row segment is 224 B
//                 and consecutive rows of a workgroup are 2 image rows apart
//   rows       -- workgroup = (n, 12 consecutive image rows): every store instruction writes
//                 one plane's rows as whole contiguous runs (896-B pieces)
//   flat       -- workgroup w writes the w-th 1/256 of the volume, lane-contiguous
// Each line: mean per-launch hipEvent time over 200 launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int B = 8, H = 96, W = 112;
constexpr unsigned PLANE = H * W * 4, IMG = 81 * PLANE;
constexpr unsigned kOOB = 0x80000000u;

__device__ int g_aux = 2;  // store cache policy bits (aux): 0 plain, 2 nt, 8 sc1 (set per run)
template <int AUX>
__device__ __forceinline__ void st16a(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, AUX);
}
template <int AUX = 2>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  st16a<AUX>(r, off, v);
}
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// corr_fwd_strip's stores (Geo<32,6,56>: 8 compute waves of 64 lanes, 3 steps)
template <int AUX, bool REMAP>
__global__ __launch_bounds__(512) void strip_pattern(float* out, int gap) {
  // (n, py, grp, tx), tx fastest; REMAP: the kernel's XCD-aware order (one image per XCD)
  const int t = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int tx = t % 2, grp = (t / 2) % 8, py = (t / 16) & 1, n = t / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qd = wave / 4, wq = wave % 4, slot = lane & 31, chalf = lane >> 5;
  const int task = 32 * wq + slot;
  const bool active = task < 126;
  const int tj = (active ? task : 125) / 14, seg = (active ? task : 125) % 14;
  const int px = tx * 56 + 4 * seg;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(out + (size_t)n * 81 * H * W, (short)0, (int)IMG, 0x00020000);
  for (int st = 0; st < 3; ++st) {
    const int yrow = 2 * (grp * 6 + 2 * st + qd) + py;
    const unsigned o0 = (unsigned)(((tj * 9 + 5 * chalf) * H + yrow) * W + px) * 4u;
    for (int q = 0; q < 5; ++q) {
      const bool ok = active && (q < 4 || chalf == 0);
      st16<AUX>(r, ok ? o0 + q * PLANE : kOOB, u32x4{1u, 2u, 3u, (unsigned)q});
    }
    if (gap) __builtin_amdgcn_s_sleep(127);  // a compute step's worth of spacing (optional)
  }
}

// whole rows: workgroup = (n, 12 consecutive image rows, plane group); lane = 16 B of a row
template <int AUX>
__global__ __launch_bounds__(512) void rows_pattern(float* out, int gap) {
  const int t = blockIdx.x;  // 8 images x 8 row groups x 4 plane groups = 256
  const int pg = t % 4, rg = (t / 4) % 8, n = t / 32;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(out + (size_t)n * 81 * H * W, (short)0, (int)IMG, 0x00020000);
  // the workgroup's block: planes [pg*21, pg*21+21) (last group 18) x rows [rg*12, +12) x 112 px
  // = up to 21 x 12 x 28 quads; 512 lanes, 15 stores each = 7680 quads >= 7056
  const int np = pg < 3 ? 21 : 18;
  const int nq = np * 12 * 28;
  for (int st = 0; st < 3; ++st) {
    for (int q = 0; q < 5; ++q) {
      const int k = (st * 5 + q) * 512 + threadIdx.x;
      const int p = k / (12 * 28), rem = k % (12 * 28);
      const unsigned off = (unsigned)(((pg * 21 + p) * H + rg * 12) * W) * 4u + rem * 16u;
      st16<AUX>(r, k < nq ? off : kOOB, u32x4{1u, 2u, 3u, (unsigned)q});
    }
    if (gap) __builtin_amdgcn_s_sleep(127);
  }
}

// full-width parity rows: workgroup = (n, parity, 6 parity rows, tj half): planes 0-44 or 45-80,
// each row a whole 448-B image row (every other row of the plane); remapped like the kernel
template <int AUX>
__global__ __launch_bounds__(512) void parity_full_pattern(float* out, int gap) {
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tg = t % 2, rg = (t / 2) % 8, py = (t / 16) & 1, n = t / 32;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(out + (size_t)n * 81 * H * W, (short)0, (int)IMG, 0x00020000);
  const int p0 = tg ? 45 : 0, np = tg ? 36 : 45;
  const int nq = np * 6 * 28;  // <= 7680
  for (int st = 0; st < 3; ++st) {
    for (int q = 0; q < 5; ++q) {
      const int k = (st * 5 + q) * 512 + threadIdx.x;
      const int p = k / (6 * 28), rem = k % (6 * 28), rr = rem / 28, xq = rem % 28;
      const int y = 2 * (rg * 6 + rr) + py;
      const unsigned off = (unsigned)(((p0 + p) * H + y) * W) * 4u + xq * 16u;
      st16<AUX>(r, k < nq ? off : kOOB, u32x4{1u, 2u, 3u, (unsigned)q});
    }
  }
}

// generic shapes (the coarse levels): nwg workgroups each write a block of 81 planes x rows;
// PAR: a workgroup's rows are one row parity (rows 2r + p), else consecutive image rows
template <bool PAR>
__global__ __launch_bounds__(512) void level_pattern(float* out, int Hh, int Ww, int rows_per) {
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bands = (PAR ? (Hh / 2) : Hh) / rows_per;
  const int b = t % bands, rest = t / bands;
  const int p = PAR ? rest % 2 : 0, n = PAR ? rest / 2 : rest;
  const unsigned plane = (unsigned)(Hh * Ww) * 4u, img = 81u * plane;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(out + (size_t)n * img / 4, (short)0, (int)img, 0x00020000);
  const int qpr = Ww / 4, nq = 81 * rows_per * qpr;
  for (int k = threadIdx.x; k < nq; k += 512) {
    const int pl = k / (rows_per * qpr), rem = k % (rows_per * qpr), rr = rem / qpr, xq = rem % qpr;
    const int y = PAR ? 2 * (b * rows_per + rr) + p : b * rows_per + rr;
    st16<2>(r, (unsigned)((pl * Hh + y) * Ww) * 4u + xq * 16u, u32x4{1u, 2u, 3u, (unsigned)k});
  }
}

__global__ __launch_bounds__(512) void flat_pattern(float* out, int gap) {
  const unsigned total_q = (unsigned)B * IMG / 16;
  const unsigned per = (total_q + 255) / 256;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(B * IMG), 0x00020000);
  for (int st = 0; st < 3; ++st) {
    for (int q = 0; q < 5; ++q) {
      const unsigned k = (st * 5 + q) * 512 + threadIdx.x;
      const unsigned gq = blockIdx.x * per + k;
      st16(r, k < per && gq < total_q ? gq * 16u : kOOB, u32x4{1u, 2u, 3u, (unsigned)q});
    }
    if (gap) __builtin_amdgcn_s_sleep(127);
  }
}

int main() {
  const int NS = 8;
  std::vector<float*> O(NS);
  for (int s = 0; s < NS; ++s) CK(hipMalloc(&O[s], (size_t)B * IMG));
  hipEvent_t e0[200], e1[200];
  for (int i = 0; i < 200; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  auto run = [&](const char* name, auto kern, int gap) -> int {
    for (int i = 0; i < 20; ++i)
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, O[i % NS], gap);
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 200; ++i)
      hipExtLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, e0[i], e1[i], 0, O[i % NS], gap);
    CK(hipDeviceSynchronize());
    double sum = 0;
    for (int i = 0; i < 200; ++i) {
      float ms;
      CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      sum += ms;
    }
    const double us = sum / 200 * 1e3, mb = (double)B * IMG / 1e6;
    std::printf("{\"pattern\": \"%s\", \"gap\": %d, \"us\": %.2f, \"MB\": %.1f, \"TBs\": %.3f}\n", name,
                gap, us, mb, mb / us);
    return 0;
  };
  if (run("strip_nt", strip_pattern<2, false>, 0)) return 1;
  if (run("strip_remap_nt", strip_pattern<2, true>, 0)) return 1;
  if (run("strip_remap_plain", strip_pattern<0, true>, 0)) return 1;
  if (run("strip_remap_sc1", strip_pattern<8, true>, 0)) return 1;
  if (run("rows_nt", rows_pattern<2>, 0)) return 1;
  if (run("rows_plain", rows_pattern<0>, 0)) return 1;
  if (run("parity_full_nt", parity_full_pattern<2>, 0)) return 1;
  if (run("parity_full_plain", parity_full_pattern<0>, 0)) return 1;
  if (run("flat_nt", flat_pattern, 0)) return 1;
  // coarse levels, B = 8: l3 (48 x 56), l2 (24 x 28); parity bands vs consecutive rows
  auto runl = [&](const char* name, auto kern, int Hh, int Ww, int rows_per, int nwg) -> int {
    const double mb = 8.0 * 81 * Hh * Ww * 4 / 1e6;
    for (int i = 0; i < 20; ++i)
      hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), 0, 0, O[i % NS], Hh, Ww, rows_per);
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 200; ++i)
      hipExtLaunchKernelGGL(kern, dim3(nwg), dim3(512), 0, 0, e0[i], e1[i], 0, O[i % NS], Hh, Ww,
                            rows_per);
    CK(hipDeviceSynchronize());
    double sum = 0;
    for (int i = 0; i < 200; ++i) {
      float ms;
      CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      sum += ms;
    }
    const double us = sum / 200 * 1e3;
    std::printf("{\"pattern\": \"%s\", \"us\": %.2f, \"MB\": %.1f, \"TBs\": %.3f}\n", name, us, mb,
                mb / us);
    return 0;
  };
  if (runl("l3_parity_bands_3", level_pattern<true>, 48, 56, 3, 8 * 2 * 8)) return 1;
  if (runl("l3_rows_6", level_pattern<false>, 48, 56, 6, 8 * 8)) return 1;
  if (runl("l3_rows_3", level_pattern<false>, 48, 56, 3, 8 * 16)) return 1;
  if (runl("l2_parity_bands_1", level_pattern<true>, 24, 28, 1, 8 * 2 * 12)) return 1;
  if (runl("l2_rows_2", level_pattern<false>, 24, 28, 2, 8 * 12)) return 1;
  if (runl("l2_rows_1", level_pattern<false>, 24, 28, 1, 8 * 24)) return 1;
  return 0;
}
