// warp_corr.hip — one pyramid level of PWC-Net's hot path in ONE launch: the flow warp of the
// second image's features followed by the correlation against the first (model.py:80-83):
//   x2_warp = WarpingLayer(x2, flow)                     (modules.py:31-42, utils.py:3-8)
//   out     = Correlation(pad 9, k 1, md 9, s1 1, s2 2)(x1, x2_warp)   (model.py:24;
//             correlation_cuda_kernel.cu:34-106)
// out[n, tj*9+ti, y, x] = sum_c x1[n,c,y,x] * x2_warp[n,c,y+2tj-8,x+2ti-8] / C, zeros outside.
// x2_warp (returned by the reference Net in summaries['x2_warps'], model.py:107,113) is
// optionally written too, bit-identical to warp.hip's.  WARP = false correlates x2 directly.
//
// Decomposition (coarse levels: a few hundred to a few thousand pixels per image, 96-192
// channels).  An output row only meets f2 rows of its own parity and an output column only f2
// columns of its own parity (2tj, 2ti are even), so one workgroup takes
//   one image n  x  one row parity p  x  one band of R parity rows  x  T displacement rows tj
// with EVERY channel staged in LDS at once (one batch of loads, no channel ring, no partial
// volumes in HBM and no second launch): f1 = the band's R rows, f2 = the R + T - 1 parity rows
// the band meets at those tj, full width.  In LDS each row is split into its even and odd
// columns (parity-column space, where the displacement step 2ti becomes 1) with 4 zero slots
// on each side of the f2 rows -- the reference's zero padding, and the warp's "zeros" mode for
// rows outside the image -- so the inner loop has no bounds checks.  The warped f2 values are
// computed while staging (bilinear gathers from x2 on the reference's fp32 coordinate chain,
// warp_sample.cuh); the workgroup whose tj range holds tj = 4 (dy = 0) stages exactly its
// band's rows and writes them to x2_warp, so every x2_warp element is written once.
// Compute: item = (tj, row, column parity, 4-pixel segment), G channel groups per workgroup;
// per channel one item reads 1 f1 quad + 3 f2 quads for 36 FMAs.  The G partial sums meet in
// LDS in a fixed order (deterministic) and the result is written row by row (lane = x).
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "warp_sample.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace band {

constexpr int NT = 512;   // threads per workgroup (8 waves, 2 per SIMD)
constexpr int D = 9;      // displacements per axis (md / s2 = 4)
constexpr int MAXJ = 32;  // channels per staging batch per thread (loads in flight)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct Geo {
  int Wq4;    // parity-column slots of an f1 row half (ceil(W/2) rounded up to 4)
  int Wf;     // slots of an f2 row half: Wq4 + 8 (4 zero slots each side)
  int S;      // 4-pixel segments per row half
  int I;      // compute items: T * R * 2 * S
  int G;      // channel groups (G * I <= NT)
  int nb;     // bands per parity half
  int units;  // B * 2 * nb
  int f1f;    // floats of the f1 image: C * R * 2 * Wq4
  int clr4;   // float4s of staging to clear
  float inv_np1, inv_np2, inv_W, inv_I, inv_S;  // 1/d for qdiv
  int abl;    // measurement only (PWC_BAND_ABL): 1 no f1 staging, 2 no f2 staging,
              // 4 no FMA loop, 8 no epilogue, 16 no clear
};

// x / d for 0 <= x < 2^22 from a host-computed float 1/d: (x + 0.5) / d lies at least 0.5/d
// from an integer and the float error is below that, so the truncation is exact (3 VALU
// instead of a ~30-instruction integer division; issue slots bound these small kernels).
__device__ __forceinline__ int qdiv(int x, float inv) {
  return (int)(((float)x + 0.5f) * inv);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads (__syncthreads() also drains vmcnt, which put a full memory round trip (~2 us
// measured) in front of every barrier while the staging loads were in flight).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Phase timestamps (measurement only, PWC_BAND_ABL & 256): s_memrealtime (100 MHz) of
// workgroup b's thread 0 at kernel entry and after each barrier -> g_band_dbg[b * 8 + k].
__device__ unsigned long long g_band_dbg[4096 * 8];
#define BAND_MARK(k)                                                                   \
  do {                                                                                 \
    if ((g.abl & 256) && threadIdx.x == 0 && blockIdx.x < 4096)                        \
      g_band_dbg[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();             \
  } while (0)

// One problem of a (possibly grouped) launch: the tensors and geometry of one level.
struct Prob {  // element pointers of the problem's storage type (fp32 or fp16)
  const void* f1;
  const void* x2;
  const void* flow;
  void* x2w;
  void* out;
  int C, H, W;
  float divisor, inv_divisor, halfx, halfy;
  Geo g;
};

// Storage-type loads and stores of the band kernel (fp32, or fp16 with fp32 arithmetic: each
// element widened on the way into LDS, each result rounded on the way out).
template <typename E>
__device__ __forceinline__ float ld_elem(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t so) {
  if constexpr (sizeof(E) == 4)
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, (int)so, 0));
  else
    return to_f32(__builtin_bit_cast(__half, __builtin_amdgcn_raw_buffer_load_b16(rs, (int)off,
                                                                                   (int)so, 0)));
}
// two horizontally adjacent elements (a bilinear corner pair)
template <typename E>
__device__ __forceinline__ void ld_pair(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t so,
                                        float& lo, float& hi) {
  if constexpr (sizeof(E) == 4) {
    const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, (int)so, 0);
    lo = __uint_as_float(a.x);
    hi = __uint_as_float(a.y);
  } else {
    const uint32_t a = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, (int)so, 0);
    lo = to_f32(__builtin_bit_cast(__half, (unsigned short)(a & 0xffffu)));
    hi = to_f32(__builtin_bit_cast(__half, (unsigned short)(a >> 16)));
  }
}
template <typename E>
__device__ __forceinline__ void st_elem_nt(float v, __amdgpu_buffer_rsrc_t rs, uint32_t off,
                                           uint32_t so) {
  if constexpr (sizeof(E) == 4)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)off, (int)so, 2 /* nt */);
  else
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, from_f32<__half>(v)),
                                          rs, (int)off, (int)so, 2 /* nt */);
}

// The workgroup body; `bid` is the workgroup's index inside its problem's grid.  MJ: channels
// per staging batch per thread (loads in flight; MAXJ for the single-level kernel, 16 under
// the two-workgroups-per-CU register cap of the grouped kernel).
template <typename E, int R, int T, bool WARP, int MJ>
__device__ __forceinline__ void band_body(const int bid, float* __restrict__ lds, const Prob& P,
                                          const OutEpi& epi) {
  constexpr uint32_t ES = (uint32_t)sizeof(E);
  const E* __restrict__ f1 = (const E*)P.f1;
  const E* __restrict__ x2 = (const E*)P.x2;
  const E* __restrict__ flow = (const E*)P.flow;
  E* __restrict__ x2w = (E*)P.x2w;
  E* __restrict__ out = (E*)P.out;
  const int C = P.C, H = P.H, W = P.W;
  const float divisor = P.divisor, inv_divisor = P.inv_divisor, halfx = P.halfx,
              halfy = P.halfy;
  const Geo& g = P.g;
  constexpr int NR2 = R + T - 1;  // f2 parity rows staged
  BAND_MARK(0);
  const int t = threadIdx.x;
  // bid = tg * units + unit: the T-groups of one band are units apart (same XCD when
  // units % 8 == 0), so they meet the same x1 / x2 rows in one L2 -- speed only
  const int unit = bid % g.units, tg = bid / g.units;
  const int b = unit % g.nb, np = unit / g.nb;
  const int p = np & 1, n = np >> 1;
  const int hp = (H - p + 1) >> 1;  // image rows of parity p
  const int r0 = b * R, tj0 = tg * T;
  const unsigned plane = (unsigned)(H * W);
  float* f1s = lds;
  float* f2s = lds + g.f1f;
  const int ch1 = R * 2 * g.Wq4;     // f1 floats per channel
  const int ch2 = NR2 * 2 * g.Wf;    // f2 floats per channel

  // ---- staging.  f1 thread map: (band pixel, channel group); f2 thread map: (f2 pixel,
  // channel group).  All global traffic is buffer loads/stores over image n of each tensor:
  // the per-lane VGPR offset is fixed for the whole staging and the channel step is a scalar
  // offset, so no per-load address arithmetic and no register reuse (re-writing a register an
  // in-flight store still reads costs a vmcnt wait per store); offsets past the image -- the
  // channels beyond C, idle lanes -- read 0 / drop the store in the buffer range check.  Every
  // load of a thread is issued before anything waits: flow and f1 first, the LDS clear runs
  // under them, then the bilinear gathers. ----
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t img_bytes = (uint32_t)C * plane * ES;
  const int np1 = R * W, ncg1 = NT / np1;
  const int cg1 = qdiv(t, g.inv_np1), pix1 = t - cg1 * np1;
  const int r1 = qdiv(pix1, g.inv_W), x1 = pix1 - r1 * W;
  const bool ok1 = cg1 < ncg1 && r0 + r1 < hp && !(g.abl & 1);
  const uint32_t vo1 =
      ok1 ? ((uint32_t)cg1 * plane + (uint32_t)(2 * (r0 + r1) + p) * W + x1) * ES : kOOB;
  const int dst1 = (r1 * 2 + (x1 & 1)) * g.Wq4 + (x1 >> 1);

  const int np2 = NR2 * W, ncg2 = NT / np2;
  const int cg2 = qdiv(t, g.inv_np2), pix2 = t - cg2 * np2;
  const int k2 = qdiv(pix2, g.inv_W), x2i = pix2 - k2 * W;
  const int rr = r0 + tj0 - 4 + k2;  // parity row of f2
  const bool ok2 = cg2 < ncg2 && rr >= 0 && rr < hp && !(g.abl & 2);
  const int y2 = 2 * rr + p;
  const unsigned src2 = (unsigned)(ok2 ? y2 : 0) * W + x2i;
  const int dst2 = (k2 * 2 + (x2i & 1)) * g.Wf + (x2i >> 1) + 4;
  // the dy = 0 workgroup of the band writes x2_warp (each element once in the grid)
  const bool emit = WARP && ok2 && x2w != nullptr && tj0 <= 4 && 4 < tj0 + T &&
                    k2 >= 4 - tj0 && k2 < 4 - tj0 + R;
  const uint32_t cbase2 = (uint32_t)cg2 * plane;
  const uint32_t vow = emit ? (cbase2 + src2) * ES : kOOB;
  const size_t img = (size_t)n * C * plane;
  const __amdgpu_buffer_rsrc_t rs1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(f1 + img), (short)0, (int)img_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(x2 + img), (short)0, (int)img_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x2w ? x2w + img : x2w), (short)0, x2w ? (int)img_bytes : 0, 0x00020000);
  const uint32_t cs1 = (uint32_t)ncg1 * plane * ES;  // bytes between a thread's channels
  const uint32_t cs2 = (uint32_t)ncg2 * plane * ES;

  float fu = 0.f, fv = 0.f;
  if constexpr (WARP) {
    fu = to_f32(flow[(unsigned)(2 * n + 0) * plane + src2]);
    fv = to_f32(flow[(unsigned)(2 * n + 1) * plane + src2]);
  }
  // channels per thread (uniform): iterations past it are skipped by a scalar branch
  const int nj1 = (C + ncg1 - 1) / ncg1, nj2 = (C + ncg2 - 1) / ncg2;
  int jb1 = 0, jb2 = 0;  // channel slot of the batch's first j
  float v1[MJ];
  auto f1_issue = [&]() {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (jb1 + j >= nj1) break;
      v1[j] = ld_elem<E>(rs1, vo1, (uint32_t)((jb1 + j) * cs1));
    }
  };
  auto f1_store = [&]() {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (jb1 + j >= nj1) break;
      const int c = cg1 + (jb1 + j) * ncg1;
      if (ok1 && c < C) f1s[c * ch1 + dst1] = v1[j];
    }
  };
  f1_issue();

  {  // zeros: padding slots, rows outside the image, columns past W
    f32x4* z = reinterpret_cast<f32x4*>(lds);
    for (int i = t; i < ((g.abl & 16) ? 0 : g.clr4); i += NT) z[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  lds_barrier();
  BAND_MARK(1);

  // bilinear setup of this thread's f2 pixel (warp.hip's chain, bit-identical samples)
  Pairs kp{};
  float w00 = 0.f, w01 = 0.f, w10 = 0.f, w11 = 0.f;
  if (WARP) {
    const float ix = src_coord(fu, x2i, W, halfx);
    const float iy = src_coord(fv, y2, H, halfy);
    const Bilinear bl = bilinear(ix, iy, H, W);
    w00 = bl.wx0 * bl.wy0;
    w01 = bl.wx1 * bl.wy0;
    w10 = bl.wx0 * bl.wy1;
    w11 = bl.wx1 * bl.wy1;
    kp = pairs(bl, H, W);  // W >= 2 (launcher)
  }
  const uint32_t voA = ok2 ? (cbase2 + (WARP ? kp.i0 : src2)) * ES : kOOB;
  const uint32_t voB = ok2 ? (cbase2 + kp.i1) * ES : kOOB;
  float lo[MJ][2], hi[MJ][2];
  auto f2_issue = [&]() {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (jb2 + j >= nj2) break;
      const uint32_t so = (uint32_t)((jb2 + j) * cs2);
      if constexpr (WARP) {
        ld_pair<E>(rs2, voA, so, lo[j][0], hi[j][0]);
        ld_pair<E>(rs2, voB, so, lo[j][1], hi[j][1]);
      } else {
        lo[j][0] = ld_elem<E>(rs2, voA, so);
      }
    }
  };
  // blend + LDS write of every channel first; the x2_warp stores go out after the batch's last
  // load was consumed (vmcnt retires in issue order: a store between loads delays them)
  auto f2_store = [&]() {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      if (jb2 + j >= nj2) break;
      const int c = cg2 + (jb2 + j) * ncg2;
      float val;
      if constexpr (WARP) {
        // warp.hip's blend, same operation order (bit-identical x2_warp)
        const float c00 = kp.l_lo ? lo[j][0] : hi[j][0];
        const float c01 = kp.r_lo ? lo[j][0] : hi[j][0];
        const float c10 = kp.l_lo ? lo[j][1] : hi[j][1];
        const float c11 = kp.r_lo ? lo[j][1] : hi[j][1];
        float acc = 0.f;
        acc = fmaf(masked(c00, kp.m00), w00, acc);
        acc = fmaf(masked(c01, kp.m01), w01, acc);
        acc = fmaf(masked(c10, kp.m10), w10, acc);
        acc = fmaf(masked(c11, kp.m11), w11, acc);
        // fp16 storage: the correlation reads x2_warp as stored (rounded), as the two-launch
        // path does
        if constexpr (ES == 2) acc = to_f32(from_f32<__half>(acc));
        val = acc;
        lo[j][0] = acc;
      } else {
        val = lo[j][0];
      }
      if (ok2 && c < C) f2s[c * ch2 + dst2] = val;
    }
    if constexpr (WARP) {
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        if (jb2 + j >= nj2) break;
        st_elem_nt<E>(lo[j][0], rsw, vow, (uint32_t)((jb2 + j) * cs2));
      }
    }
  };
  f2_issue();
  f1_store();
  f2_store();
  // further batches when a thread has more than MJ channels (uniform trip count)
  const int nbat1 = (nj1 + MJ - 1) / MJ;
  const int nbat2 = (nj2 + MJ - 1) / MJ;
  for (int b = 1; b < max(nbat1, nbat2); ++b) {
    jb1 = b * MJ;
    jb2 = b * MJ;
    const bool m1 = b < nbat1, m2 = b < nbat2;
    if (m1) f1_issue();
    if (m2) f2_issue();
    if (m1) f1_store();
    if (m2) f2_store();
  }
  lds_barrier();
  BAND_MARK(2);

  // ---- correlation: item (tt, r, q, s) of channel group grp ----
  const int grp = qdiv(t, g.inv_I), it = t - grp * g.I;
  float acc[D][4];
#pragma unroll
  for (int ti = 0; ti < D; ++ti)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc[ti][kk] = 0.f;
  if (grp < g.G && !(g.abl & 4)) {
    int rest = qdiv(it, g.inv_S);
    const int s = it - rest * g.S;
    const int q = rest & 1;
    rest >>= 1;
    const int r = rest % R, tt = rest / R;
    const f32x4* pa = reinterpret_cast<const f32x4*>(f1s + (r * 2 + q) * g.Wq4 + 4 * s);
    const f32x4* pb = reinterpret_cast<const f32x4*>(f2s + ((r + tt) * 2 + q) * g.Wf + 4 * s);
    const int s1 = ch1 >> 2, s2 = ch2 >> 2;
    // one channel's quads in flight while the previous channel's 36 FMAs issue
    int c = grp;
    f32x4 a = pa[c * s1], q0 = pb[c * s2], q1 = pb[c * s2 + 1], q2 = pb[c * s2 + 2];
    for (; c < C; c += g.G) {
      const int cn = c + g.G < C ? c + g.G : c;
      const f32x4 an = pa[cn * s1], n0 = pb[cn * s2], n1 = pb[cn * s2 + 1],
                  n2 = pb[cn * s2 + 2];
      const float w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                           q2.x, q2.y, q2.z, q2.w};
      const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int ti = 0; ti < D; ++ti)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) acc[ti][kk] = fmaf(av[kk], w[kk + ti], acc[ti][kk]);
      a = an;
      q0 = n0;
      q1 = n1;
      q2 = n2;
    }
  }
  lds_barrier();  // staging dead: the partial sums reuse it
  BAND_MARK(3);
  if (grp < g.G) {
    f32x4* rp = reinterpret_cast<f32x4*>(lds) + (grp * g.I + it) * D;
#pragma unroll
    for (int ti = 0; ti < D; ++ti)
      rp[ti] = f32x4{acc[ti][0], acc[ti][1], acc[ti][2], acc[ti][3]};
  }
  lds_barrier();
  BAND_MARK(4);

  // ---- epilogue: fixed-order sum of the G groups, / divisor (cu:100), rows of W (lane = x) --
  const int nout = (g.abl & 8) ? 0 : T * D * R * W;
  for (int o = t; o < nout; o += NT) {
    int rest = qdiv(o, g.inv_W);
    const int x = o - rest * W;
    const int r = rest % R;
    rest /= R;
    const int ti = rest % D, tt = rest / D;
    const int tj = tj0 + tt, row = r0 + r;
    if (tj >= D || row >= hp) continue;
    const int i = x >> 1;
    const int it2 = ((tt * R + r) * 2 + (x & 1)) * g.S + (i >> 2);
    const float* sp = lds + (it2 * D + ti) * 4 + (i & 3);
    const int gstride = g.I * D * 4;
    // fixed order: four interleaved partial sums (independent LDS reads in flight)
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int gg = 0;
    for (; gg + 4 <= g.G; gg += 4) {
      s0 += sp[gg * gstride];
      s1 += sp[(gg + 1) * gstride];
      s2 += sp[(gg + 2) * gstride];
      s3 += sp[(gg + 3) * gstride];
    }
    for (; gg < g.G; ++gg) s0 += sp[gg * gstride];
    float sum = (s0 + s1) + (s2 + s3);
    sum = inv_divisor != 0.f ? sum * inv_divisor : sum / divisor;
    const size_t ib = epi.ostride ? (size_t)n * epi.ostride : (size_t)n * (D * D) * H * W;
    E* dst = out + ib + ((size_t)(tj * D + ti) * H + (2 * row + p)) * W + x;
    if constexpr (ES == 4)
      st_out1(reinterpret_cast<float*>(dst), epi_act(sum, epi.slope));
    else
      *dst = from_f32<E>(epi_act(sum, epi.slope));
  }
  if (g.abl & 256) {
    __syncthreads();
    BAND_MARK(5);
  }
}

template <typename E, int R, int T, bool WARP>
__global__ __launch_bounds__(NT, 1) void warp_corr_band(Prob P, OutEpi epi) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  band_body<E, R, T, WARP, MAXJ>((int)blockIdx.x, lds, P, epi);
}

// Two independent problems in one launch (e.g. two coarse levels, or two requests): blocks
// [0, nblk0) run problem 0's grid, the rest problem 1's.  Each workgroup of these latency-bound
// grids holds its CU for a few microseconds at two waves per SIMD, so the two grids co-reside
// (<= 128 VGPRs: two 512-thread workgroups per CU; the launcher checks that the two LDS
// footprints fit one CU together) instead of running one after the other.
template <typename E, int R0, int T0, int R1, int T1>
__global__ __launch_bounds__(NT, 2) void warp_corr_band_pair(Prob P0, Prob P1, int nblk0,
                                                             OutEpi epi) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if ((int)blockIdx.x < nblk0)
    band_body<E, R0, T0, true, 16>((int)blockIdx.x, lds, P0, epi);
  else
    band_body<E, R1, T1, true, 16>((int)blockIdx.x - nblk0, lds, P1, epi);
}

struct Cfg {
  int R, T;
};

// knobs band_r, band_t [, band_g] override the per-level choice (measurement, tests).
static bool env_cfg(int* R, int* T, int* G) {
  const int r = debug_knob("band_r", 0), tt = debug_knob("band_t", 0);
  if (r <= 0 || tt <= 0) return false;
  *R = r;
  *T = tt;
  const int gg = debug_knob("band_g", 0);
  if (gg > 0) *G = gg;
  return true;
}

template <typename E, int R, int T, bool WARP>
static hipError_t launch(const Prob& P, size_t lds, hipStream_t stream) {
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e =
        lds_limit(reinterpret_cast<const void*>(&warp_corr_band<E, R, T, WARP>), 160 * 1024);
    if (e != hipSuccess) return e;
  }
  const int ntg = (D + T - 1) / T;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL((warp_corr_band<E, R, T, WARP>), dim3((unsigned)(P.g.units * ntg)),
                        dim3(NT), lds, stream, ev0, ev1, 0, P, current_epi());
  return hipGetLastError();
}

// Geometry for (R, T); false if it does not fit one workgroup.
static bool make_geo(int B, int C, int H, int W, int R, int T, int Greq, Geo* g, size_t* lds) {
  const int Wq = (W + 1) / 2;
  g->Wq4 = (Wq + 3) & ~3;
  g->Wf = g->Wq4 + 8;
  g->S = g->Wq4 / 4;
  g->I = T * R * 2 * g->S;
  if (g->I > NT || R * W > NT || (R + T - 1) * W > NT) return false;
  int G = NT / g->I;
  // channel groups: at least 4 channels per group and at most 32 groups (the epilogue sums G
  // partials per output)
  int gc = C / 4;
  if (gc > 32) gc = 32;
  if (gc < 1) gc = 1;
  if (G > gc) G = gc;
  if (Greq > 0 && Greq <= NT / g->I) G = Greq;
  g->G = G;
  const int hp = (H + 1) / 2;
  g->nb = (hp + R - 1) / R;
  g->units = B * 2 * g->nb;
  g->f1f = C * R * 2 * g->Wq4;
  const size_t stage = (size_t)(g->f1f + C * (R + T - 1) * 2 * g->Wf) * 4;
  const size_t red = (size_t)G * g->I * D * 16;
  g->clr4 = (int)(stage / 16);
  g->inv_np1 = 1.f / (float)(R * W);
  g->inv_np2 = 1.f / (float)((R + T - 1) * W);
  g->inv_W = 1.f / (float)W;
  g->inv_I = 1.f / (float)g->I;
  g->inv_S = 1.f / (float)g->S;
  g->abl = debug_knob("band_abl", 0);
  *lds = stage > red ? stage : red;
  return *lds <= 160 * 1024;
}

}  // namespace band

// measurement only: copy the phase timestamps of the last PWC_BAND_ABL & 256 launch
extern "C" __attribute__((visibility("default"))) int pwc_debug_band_times(void* dst, int n) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(band::g_band_dbg),
                             sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}

extern "C" __attribute__((visibility("default"))) int pwc_debug_band_reset(void) {
  static unsigned long long zeros[4096 * 8];
  return hipMemcpyToSymbol(HIP_SYMBOL(band::g_band_dbg), zeros, sizeof(zeros)) == hipSuccess;
}

namespace band {

// The per-level (R, T) choice (measured at 384x448, B = 8, tools/kbench.py), the geometry and
// the kernel arguments of one problem; false when it does not take a band workgroup.
static bool make_prob(const void* f1, const void* x2, const void* flow, void* x2w, void* out,
                      int B, int C, int H, int W, float divisor, int warp, int* R, int* T,
                      Prob* P, size_t* lds) {
  if (W < 2 || (size_t)B * C * H * W >= (1ull << 31) || (size_t)B * 81 * H * W >= (1ull << 31))
    return false;
  // the whole parity half in one band where it fits, one tj per workgroup
  int Greq = 0;
  const int hp = (H + 1) / 2;
  *T = 1;
  if (!env_cfg(R, T, &Greq)) {
    if (hp <= 3) {
      *R = 3;  // l0: 7.7 us (warp 3.1 + correlation 10.9 unfused)
      *T = 1;
    } else if (hp <= 6) {
      *R = 2;  // l1: fused 10.7 us (3.4 + 13.4 unfused); plain correlation 7.8 us with T = 1
      *T = warp ? 3 : 1;
    } else {
      *R = 3;  // l2 and larger (the bench keeps l2..l4 unfused: 17.7 vs 3.6 + 11.4 us at l2)
      *T = 3;
    }
  }
  // the instantiated (R, T) shapes: the per-level choices above (warp_corr_band's list)
  const bool inst = (*R == 3 && *T == 1) || (*R == 2 && *T == (warp ? 3 : 1)) ||
                    (*R == 3 && *T == 3 && warp);
  if (!inst) return false;
  // a level whose all-channel staging exceeds the LDS runs as two launches (config-4 Sintel l1,
  // 128 channels x 32 columns: a lower band measured 2x slower than warp + row-band
  // correlation, profiles/r03e_band_fp16.txt)
  if (!make_geo(B, C, H, W, *R, *T, Greq, &P->g, lds)) return false;
  P->f1 = f1;
  P->x2 = x2;
  P->flow = flow;
  P->x2w = x2w;
  P->out = out;
  P->C = C;
  P->H = H;
  P->W = W;
  P->halfx = (float)((W - 1.0) / 2.0);
  P->halfy = (float)((H - 1.0) / 2.0);
  int ex;
  const float m = std::frexp(divisor, &ex);
  P->divisor = divisor;
  P->inv_divisor = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  return true;
}

}  // namespace band

// Whether the band kernel serves this problem (its geometry fits a workgroup).
bool warp_corr_band_accepts(int B, int C, int H, int W, int warp) {
  if (B == 0 || C == 0 || H == 0 || W == 0) return true;
  band::Prob P;
  size_t lds;
  int R = 0, T = 1;
  return band::make_prob(nullptr, nullptr, nullptr, nullptr, nullptr, B, C, H, W, (float)C, warp,
                         &R, &T, &P, &lds);
}

// Fused warp -> correlation for Correlation(pad == md in {8, 9}, k 1, s1 1, s2 2), fp32 or fp16
// storage (dtype 0 / 1), raster channel order.  hipErrorNotSupported when the level does not fit
// a band workgroup (the caller then runs the warp and correlation kernels separately).
// `warp` = 0 correlates x2 directly (flow and x2w unused).
hipError_t warp_corr_band(const void* f1, const void* x2, const void* flow, void* x2w, void* out,
                          int B, int C, int H, int W, float divisor, int warp, int dtype,
                          hipStream_t stream) {
  using namespace band;
  if (B == 0 || C == 0 || H == 0 || W == 0) return hipSuccess;
  if (dtype != 0 && dtype != 1) return hipErrorNotSupported;
  if (W < 2 || (size_t)B * C * H * W >= (1ull << 31) || (size_t)B * 81 * H * W >= (1ull << 31))
    return hipErrorNotSupported;
  int R = 0, T = 1;
  Prob P;
  size_t lds;
  if (!make_prob(f1, x2, flow, x2w, out, B, C, H, W, divisor, warp, &R, &T, &P, &lds))
    return hipErrorNotSupported;
#define PWC_BAND(RR, TT, WW)                                                                 \
  if (R == RR && T == TT && (warp != 0) == WW)                                               \
    return dtype == 1 ? launch<__half, RR, TT, WW>(P, lds, stream)                           \
                      : launch<float, RR, TT, WW>(P, lds, stream);
#define PWC_BAND32(RR, TT)                                                                   \
  if (R == RR && T == TT && !warp && dtype == 0) return launch<float, RR, TT, false>(P, lds, stream);
  // the per-level choices of make_prob: l0 (3, 1), l1 (2, 3) and l2 and larger (3, 3) fused in
  // both storage types; the plain correlation (corr_forward_path: fp32 l0 / l1) (3, 1), (2, 1)
  PWC_BAND(3, 1, true)
  PWC_BAND(2, 3, true)
  PWC_BAND(3, 3, true)
  PWC_BAND32(3, 1)
  PWC_BAND32(2, 1)
#undef PWC_BAND
#undef PWC_BAND32
  return hipErrorNotSupported;
}

hipError_t warp_corr_band_f32(const void* f1, const void* x2, const void* flow, void* x2w,
                              void* out, int B, int C, int H, int W, float divisor, int warp,
                              hipStream_t stream) {
  return warp_corr_band(f1, x2, flow, x2w, out, B, C, H, W, divisor, warp, 0, stream);
}

// Two fused warp -> correlation problems (warp = 1, fp32, raster) in ONE launch
// (warp_corr_band_pair); hipErrorNotSupported when either does not take a band workgroup, their
// (R, T) pair has no instantiation, or their LDS footprints do not fit one CU together -- the
// caller then launches them one after the other.
hipError_t warp_corr_band_pair(const BandProblem& a, const BandProblem& b, float divisor_a,
                               float divisor_b, int dtype, hipStream_t stream) {
  using namespace band;
  if (debug_knob("band_pair", 1) == 0 || !epi_is_default(current_epi()))
    return hipErrorNotSupported;
  if (dtype != 0 && dtype != 1) return hipErrorNotSupported;
  for (const BandProblem* q : {&a, &b})
    if (q->B == 0 || q->C == 0 || q->H == 0 || q->W == 0) return hipErrorNotSupported;
  int R0 = 0, T0 = 1, R1 = 0, T1 = 1;
  Prob P0, P1;
  size_t l0, l1;
  if (!make_prob(a.f1, a.x2, a.flow, a.x2w, a.out, a.B, a.C, a.H, a.W, divisor_a, 1, &R0, &T0,
                 &P0, &l0) ||
      !make_prob(b.f1, b.x2, b.flow, b.x2w, b.out, b.B, b.C, b.H, b.W, divisor_b, 1, &R1, &T1,
                 &P1, &l1))
    return hipErrorNotSupported;
  // the kernel allocates max(l0, l1) to every workgroup: two of them must fit one CU
  const size_t lds = l0 > l1 ? l0 : l1;
  if (2 * lds > 160 * 1024) return hipErrorNotSupported;
  const int n0 = P0.g.units * ((D + T0 - 1) / T0);
  const int n1 = P1.g.units * ((D + T1 - 1) / T1);
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
#define PWC_PAIR_E(E, A0, B0, A1, B1)                                                         \
  {                                                                                           \
    {  /* > 64 KiB dynamic LDS, once per device (capi.hip) */                                 \
      const hipError_t e = lds_limit(                                                         \
          reinterpret_cast<const void*>(&warp_corr_band_pair<E, A0, B0, A1, B1>), 160 * 1024);\
      if (e != hipSuccess) return e;                                                          \
    }                                                                                         \
    take_launch_events(&ev0, &ev1);                                                           \
    hipExtLaunchKernelGGL((warp_corr_band_pair<E, A0, B0, A1, B1>),                           \
                          dim3((unsigned)(n0 + n1)), dim3(NT), lds, stream, ev0, ev1, 0, P0,  \
                          P1, n0, current_epi());                                             \
    return hipGetLastError();                                                                 \
  }
#define PWC_PAIR(A0, B0, A1, B1)                                                              \
  if (R0 == A0 && T0 == B0 && R1 == A1 && T1 == B1) {                                         \
    if (dtype == 1) PWC_PAIR_E(__half, A0, B0, A1, B1)                                        \
    PWC_PAIR_E(float, A0, B0, A1, B1)                                                         \
  }
  PWC_PAIR(3, 1, 2, 3)  // PWC-Net l0 + l1 (384 x 448: 6 x 7 and 12 x 14)
  PWC_PAIR(2, 3, 3, 1)
#undef PWC_PAIR
#undef PWC_PAIR_E
  return hipErrorNotSupported;
}

hipError_t warp_corr_band_pair_f32(const BandProblem& a, const BandProblem& b, float divisor_a,
                                   float divisor_b, hipStream_t stream) {
  return warp_corr_band_pair(a, b, divisor_a, divisor_b, 0, stream);
}

}  // namespace pwc
