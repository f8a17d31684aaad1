// corr_rows.hip — correlation forward of model.py:24's configuration (pad == md in {8, 9},
// k 1, s1 1, s2 2: 81 displacement channels, /C) for the mid-sized pyramid levels; fp32
// storage (W % 4 == 0) or fp16 storage (W % 8 == 0: halves widened to fp32 on the way into
// LDS, fp32 arithmetic, fp16 stores -- BASELINE config 4's coarse Sintel levels).
//
//   out[n, tj*9+ti, y, x] = sum_c f1[n,c,y,x] * f2[n,c,y+2tj-8,x+2ti-8] / C, zeros outside
//   (correlation_cuda_kernel.cu:34-106 with kernel_size 1, stride1 1, stride2 2).
//
// Row-band decomposition.  Output row y only meets f2 rows of its own parity and output column
// x only f2 columns of its own parity, so one workgroup owns
//     one image  x  one row parity p  x  a band of R parity rows,   ALL 9 x 9 displacements,
// over FULL rows: it reads the band's R f1 rows and the R + 8 same-parity f2 rows they meet
// (1 + 8/R of the f2 bytes, no column halo: the zero columns of the reference's padding live in
// LDS), channels streamed through LDS in chunks of CK.  Rows are fetched as 16-byte buffer
// loads (one per lane, contiguous 448-B rows at l4) and split into even / odd columns on the
// way into LDS (parity-column space, where the displacement step 2ti is 1 and every lane's
// window is 3 aligned quads).  Rows outside the image come back as zeros from the buffer range
// check, so no LDS clear is needed per chunk.
//
// Optionally (TS = 2) the 9 displacement rows tj are split between two workgroups of a band
// (each stages the R + 4 or R + 3 f2 rows its tj meet).
// Compute: item = (tj, row, column parity, 4-pixel segment); per channel 1 f1 quad + 3 f2
// quads feed 36 FMAs (0.44 LDS floats per FMA).  G = NT / items channel groups meet in LDS in a
// fixed order (deterministic).  The result block is written row by row as 16-byte
// nontemporal stores (lane = 4 consecutive x).
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace rows {

constexpr int D = 9;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Geo {
  int Wq4;   // parity-column slots of an f1 row half (W/2 rounded up to 4)
  int Wf;    // f2 row half slots: Wq4 + 8
  int S;     // 4-pixel segments per row half
  int Q;     // 16-byte quads per image row (W / 4)
  int TS;    // displacement-row groups: a workgroup takes DT = ceil(9 / TS) rows tj
  int DT;
  int NR2;   // staged f2 rows: R + DT - 1
  int I;     // compute items: DT * R * 2 * S
  int G;     // channel groups
  int nb;    // bands per parity half
  int units; // B * 2 * nb * TS
  int ck;    // channels per chunk
  int f1f;   // floats of one chunk's f1 image: ck * R * 2 * Wq4
  int f2f;   // floats of one chunk's f2 image: ck * NR2 * 2 * Wf
  float inv_Q, inv_NR2, inv_I, inv_S, inv_W4;
  int census;  // measurement only (knob rows_census): phase stamps -> g_rows_census
};

// Phase timestamps (measurement only): s_memrealtime (100 MHz) of workgroup b's thread 0 as a
// branch-free buffer store (off unless g.census)
__device__ unsigned long long g_rows_census[4096 * 8];
typedef unsigned u32x2c __attribute__((ext_vector_type(2)));
// compiled only into the measurement build (`make CENSUS=1`)
#ifdef PWC_CENSUS
#define ROWS_MARK(k)                                                                        \
  do {                                                                                      \
    const bool on_ = g.census && threadIdx.x == 0 && blockIdx.x < 4096;                     \
    const unsigned long long ts_ = __builtin_amdgcn_s_memrealtime();                        \
    __builtin_amdgcn_raw_buffer_store_b64(                                                  \
        __builtin_bit_cast(u32x2c, ts_),                                                    \
        __builtin_amdgcn_make_buffer_rsrc((void*)g_rows_census, (short)0,                   \
                                          (int)sizeof(g_rows_census), 0x00020000),          \
        on_ ? (int)((blockIdx.x * 8 + (k)) * 8) : (int)0x80000000, 0, 0);                   \
  } while (0)
#else
#define ROWS_MARK(k) \
  do {               \
  } while (0)
#endif

__device__ __forceinline__ int qdiv(int x, float inv) {
  return (int)(((float)x + 0.5f) * inv);
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// One workgroup's band (`unit0` = its XCD-remapped index within its problem's grid).
template <typename T, int R, int NT, int ML1, int ML2>
__device__ __forceinline__ void rows_band(const T* __restrict__ f1, const T* __restrict__ f2,
                                          T* __restrict__ out, int C, int H, int W,
                                          float divisor, float inv_divisor, const Geo& g,
                                          const OutEpi& epi, const int unit0) {
  constexpr bool H16 = sizeof(T) == 2;
  constexpr int EPQ = 16 / (int)sizeof(T);  // pixels per 16-B quad
  constexpr int HPQ = EPQ / 2;              // parity slots per quad and column parity
  extern __shared__ __attribute__((aligned(16))) float lds[];
  ROWS_MARK(0);
  const int NR2 = g.NR2;
  const int t = threadIdx.x;
  const int tg = unit0 % g.TS, unit = unit0 / g.TS;    // displacement-row group
  const int tj0 = tg * g.DT;
  const int b = unit % g.nb, np = unit / g.nb;
  const int p = np & 1, n = np >> 1;
  const int hp = (H - p + 1) >> 1;
  const int r0 = b * R;
  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t img_bytes = (uint32_t)C * plane * (uint32_t)sizeof(T);
  const size_t img = (size_t)n * C * plane;
  const __amdgpu_buffer_rsrc_t rs1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(f1 + img), (short)0, (int)img_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(f2 + img), (short)0, (int)img_bytes, 0x00020000);
  float* f1s = lds;
  float* f2s = lds + g.f1f;
  constexpr uint32_t kOOB = 0x80000000u;

  // zero the f2 pad slots once: 4 on the left of each row half, and from column W/2 to the end
  // of the half on the right (Wq4 may exceed W/2); the row slots are rewritten every chunk
  {
    const int half_w = W >> 1;
    const int nright = (g.Wf - 4 - half_w) >> 1;  // f32x2 pieces (W/2 is even)
    const int per = 2 + nright;
    const int npieces = g.ck * NR2 * 2 * per;
    for (int i = t; i < npieces; i += NT) {
      const int rh = i / per, e = i - rh * per;
      const int col = e < 2 ? 2 * e : 4 + half_w + 2 * (e - 2);
      *reinterpret_cast<f32x2*>(f2s + rh * g.Wf + col) = f32x2{0.f, 0.f};
    }
  }

  // ---- per-thread staging plan (fixed over chunks).  f1 items = (channel, band row, quad),
  // f2 items = (channel, f2 row, quad): two lists so each load names one buffer resource ----
  const int tot1 = g.ck * R * g.Q, tot2 = g.ck * NR2 * g.Q;
  uint32_t vo1[ML1], vo2[ML2];
  int ld1[ML1], ld2[ML2], ch1[ML1], ch2[ML2];
#pragma unroll
  for (int j = 0; j < ML1; ++j) {
    const int itm = t + j * NT;
    const int rest = qdiv(itm, g.inv_Q), qd = itm - rest * g.Q;
    const int c = rest / R, rho = rest - c * R;
    const bool ok = itm < tot1 && r0 + rho < hp;
    vo1[j] = ok ? ((uint32_t)c * plane + (uint32_t)(2 * (r0 + rho) + p) * W + EPQ * qd) *
                      (uint32_t)sizeof(T)
                : kOOB;
    ld1[j] = itm < tot1 ? ((c * R + rho) * 2) * g.Wq4 + HPQ * qd : -1;
    ch1[j] = c;
  }
#pragma unroll
  for (int j = 0; j < ML2; ++j) {
    const int itm = t + j * NT;
    const int rest = qdiv(itm, g.inv_Q), qd = itm - rest * g.Q;
    const int c = qdiv(rest, g.inv_NR2), k = rest - c * NR2;
    const int rr = r0 - 4 + tj0 + k;
    const bool ok = itm < tot2 && rr >= 0 && rr < hp;
    vo2[j] = ok ? ((uint32_t)c * plane + (uint32_t)(2 * rr + p) * W + EPQ * qd) *
                      (uint32_t)sizeof(T)
                : kOOB;
    ld2[j] = itm < tot2 ? g.f1f + ((c * NR2 + k) * 2) * g.Wf + 4 + HPQ * qd : -1;
    ch2[j] = c;
  }

  // ---- compute item ----
  const int grp = qdiv(t, g.inv_I), it = t - grp * g.I;
  const bool active = grp < g.G;
  const int s = it - qdiv(it, g.inv_S) * g.S;
  int rest = qdiv(it, g.inv_S);
  const int q = rest & 1;
  rest >>= 1;
  const int r = rest % R, tt = rest / R;  // tj = tj0 + tt
  const int a_off = (r * 2 + q) * g.Wq4 + 4 * s;
  const int b_off = g.f1f + ((r + tt) * 2 + q) * g.Wf + 4 * s;
  const int s1c = R * 2 * g.Wq4, s2c = NR2 * 2 * g.Wf;  // floats per channel
  float acc[D][4];
#pragma unroll
  for (int ti = 0; ti < D; ++ti)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc[ti][kk] = 0.f;

  // the next chunk's loads are issued right after its staging slot frees up, so they are in
  // flight during the current chunk's compute
  f32x4 v1[ML1], v2[ML2];
  auto issue = [&](int cb) {
    const int cn = min(g.ck, C - cb);
    const int so = (int)((uint32_t)cb * plane * (uint32_t)sizeof(T));
#pragma unroll
    for (int j = 0; j < ML1; ++j)  // channels past C (last chunk) read zeros: range check
      v1[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs1, (int)(ch1[j] < cn ? vo1[j] : kOOB), so, 0));
#pragma unroll
    for (int j = 0; j < ML2; ++j)
      v2[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs2, (int)(ch2[j] < cn ? vo2[j] : kOOB), so, 0));
  };
  issue(0);
  for (int cb = 0; cb < C; cb += g.ck) {
    const int cn = min(g.ck, C - cb);
    if (cb > 0) lds_barrier();  // the previous chunk's compute is done with the staging
    // split into column parities (fp16: widened to fp32 here)
    auto put = [&](int dst, int half, const f32x4& v) {
      if constexpr (H16) {
        const f16x8 h = __builtin_bit_cast(f16x8, v);
        *reinterpret_cast<f32x4*>(lds + dst) =
            f32x4{(float)h[0], (float)h[2], (float)h[4], (float)h[6]};
        *reinterpret_cast<f32x4*>(lds + dst + half) =
            f32x4{(float)h[1], (float)h[3], (float)h[5], (float)h[7]};
      } else {
        *reinterpret_cast<f32x2*>(lds + dst) = f32x2{v.x, v.z};
        *reinterpret_cast<f32x2*>(lds + dst + half) = f32x2{v.y, v.w};
      }
    };
#pragma unroll
    for (int j = 0; j < ML1; ++j)
      if (ld1[j] >= 0) put(ld1[j], g.Wq4, v1[j]);
#pragma unroll
    for (int j = 0; j < ML2; ++j)
      if (ld2[j] >= 0) put(ld2[j], g.Wf, v2[j]);
    if (cb + g.ck < C) issue(cb + g.ck);
    lds_barrier();
    ROWS_MARK(cb == 0 ? 1 : 3);
    if (active) {
      const float* pa = f1s + a_off;
      const float* pb = lds + b_off;
      for (int c = grp; c < cn; c += g.G) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(pa + c * s1c);
        const f32x4 q0 = *reinterpret_cast<const f32x4*>(pb + c * s2c);
        const f32x4 q1 = *reinterpret_cast<const f32x4*>(pb + c * s2c + 4);
        const f32x4 q2 = *reinterpret_cast<const f32x4*>(pb + c * s2c + 8);
        const float w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                             q2.x, q2.y, q2.z, q2.w};
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int ti = 0; ti < D; ++ti)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) acc[ti][kk] = fmaf(av[kk], w[kk + ti], acc[ti][kk]);
      }
    }
  }
  lds_barrier();  // staging dead: partial sums reuse it
  ROWS_MARK(4);
  if (active) {
    f32x4* rp = reinterpret_cast<f32x4*>(lds) + (grp * g.I + it) * D;
#pragma unroll
    for (int ti = 0; ti < D; ++ti) rp[ti] = f32x4{acc[ti][0], acc[ti][1], acc[ti][2], acc[ti][3]};
  }
  lds_barrier();
  ROWS_MARK(5);

  // ---- epilogue: lane = 4 consecutive x of one (tj, ti, row); fixed-order group sum ----
  const int W4 = W >> 2;
  const int nout = g.DT * D * R * W4;
  const int gstride = g.I * D * 4;
  for (int o = t; o < nout; o += NT) {
    const int m = o - qdiv(o, g.inv_W4) * W4;  // x = 4m .. 4m+3
    int rr2 = qdiv(o, g.inv_W4);
    const int rowi = rr2 % R;
    rr2 /= R;
    const int ti = rr2 % D, tt = rr2 / D, tj = tj0 + tt;
    const int row = r0 + rowi;
    if (row >= hp || tj >= D) continue;
    // x = 4m + e: parity e & 1, parity slot i = 2m + (e >> 1) -> segment s = i >> 2, kk = i & 3
    const int i0 = 2 * m, sg = i0 >> 2, kk = i0 & 3;  // kk in {0, 2}
    const int it0 = ((tt * R + rowi) * 2 + 0) * g.S + sg;
    const int it1 = ((tt * R + rowi) * 2 + 1) * g.S + sg;
    const float* p0 = lds + (it0 * D + ti) * 4 + kk;
    const float* p1 = lds + (it1 * D + ti) * 4 + kk;
    f32x2 e0 = *reinterpret_cast<const f32x2*>(p0);
    f32x2 e1 = *reinterpret_cast<const f32x2*>(p1);
    for (int gg = 1; gg < g.G; ++gg) {
      e0 += *reinterpret_cast<const f32x2*>(p0 + gg * gstride);
      e1 += *reinterpret_cast<const f32x2*>(p1 + gg * gstride);
    }
    f32x4 v4 = f32x4{e0.x, e1.x, e0.y, e1.y};
    if (inv_divisor != 0.f)
      v4 *= inv_divisor;
    else
      v4 = f32x4{v4.x / divisor, v4.y / divisor, v4.z / divisor, v4.w / divisor};
    if (epi.slope != 1.f)  // model.py:84's leaky_relu, fused only when asked for
      v4 = f32x4{epi_act(v4.x, epi.slope), epi_act(v4.y, epi.slope), epi_act(v4.z, epi.slope),
                 epi_act(v4.w, epi.slope)};
    const size_t ib = epi.ostride ? (size_t)n * epi.ostride : (size_t)n * (D * D) * H * W;
    T* dst = out + ib + ((size_t)(tj * D + ti) * H + (2 * row + p)) * W + 4 * m;
    if constexpr (H16)
      *reinterpret_cast<f16x4*>(dst) =
          f16x4{(_Float16)v4.x, (_Float16)v4.y, (_Float16)v4.z, (_Float16)v4.w};
    else
      st_out4(dst, v4);
  }
  ROWS_MARK(6);
}

template <typename T, int R, int NT, int ML1, int ML2>
__global__ __launch_bounds__(NT, 1) void corr_fwd_rows(const T* __restrict__ f1,
                                                       const T* __restrict__ f2,
                                                       T* __restrict__ out, int C, int H,
                                                       int W, float divisor, float inv_divisor,
                                                       Geo g, OutEpi epi) {
  // neighbouring bands share an L2
  rows_band<T, R, NT, ML1, ML2>(f1, f2, out, C, H, W, divisor, inv_divisor, g, epi,
                                xcd_remap(blockIdx.x, gridDim.x));
}

// Two INDEPENDENT problems in one launch (pwc_corr_forward_group): blocks [0, nA) run problem
// A's bands, the rest problem B's, each remapped over its own grid.  One workgroup per CU
// either way (LDS = the larger plan's), so the pair shares one launch gap and B's bands fill
// the CUs A's smaller grid leaves idle.
struct RowsArgs {
  const void* f1;
  const void* f2;
  void* out;
  int C, H, W;
  float divisor, inv;
  Geo g;
};

template <typename T, int RA, int M1A, int M2A, int RB, int M1B, int M2B, int NT>
__global__ __launch_bounds__(NT, 1) void corr_fwd_rows_pair(RowsArgs a, RowsArgs b, int nA,
                                                            OutEpi epi) {
  const int bid = blockIdx.x;
  if (bid < nA)
    rows_band<T, RA, NT, M1A, M2A>((const T*)a.f1, (const T*)a.f2, (T*)a.out, a.C, a.H, a.W,
                                   a.divisor, a.inv, a.g, epi, xcd_remap(bid, nA));
  else
    rows_band<T, RB, NT, M1B, M2B>((const T*)b.f1, (const T*)b.f2, (T*)b.out, b.C, b.H, b.W,
                                   b.divisor, b.inv, b.g, epi,
                                   xcd_remap(bid - nA, (int)gridDim.x - nA));
}

}  // namespace rows

// Serves l2/l3-sized grids (7..24 parity rows per image) by default.  Measurement knobs: rows=0
// disables the kernel, rows=2 selects it at every size; rows_r / rows_ck / rows_ts force a
// configuration.
// dtype 0: fp32 storage, 1: fp16 (Sintel l0..l2 of config 4: every parity-row count, W % 8).
namespace rows {
struct Plan {
  Geo g;
  size_t lds;
  int R, per1, per2;
  float inv;
  bool h16;
};

static hipError_t plan(int B, int C, int H, int W, float divisor, int dtype, Plan* P) {
  const int mode = debug_knob("rows", 1);  // 0 off, 2 forced at every size (measurement)
  if (mode == 0 || (dtype != 0 && dtype != 1)) return hipErrorNotSupported;
  const bool h16 = dtype == 1;
  const int epq = h16 ? 8 : 4;
  if (W % epq != 0 || W < 8 || B == 0) return hipErrorNotSupported;
  if ((size_t)B * C * H * W >= (1ull << 30) || (size_t)B * 81 * H * W >= (1ull << 31))
    return hipErrorNotSupported;
  // measured (B=8 384x448, profiles/r02d_rows_sweep.txt): l2 (12 parity rows) R 1 / CK 48
  // 9.7 us against corr_pt.hip's 11.7, l3 (24) R 2 / CK 32 13.1 against 14.4 (CK 16); fp16
  // Sintel (B=16) l0 15.1 -> 12.9, l1 11.4 -> 10.1, l2 20.6 -> 19.9 against CK 16; the
  // l4-sized grids belong to corr_stream.hip
  const int hp0 = (H + 1) / 2;
  int R = hp0 <= 12 ? 1 : hp0 <= 24 ? 2 : 3, CK = hp0 <= 12 ? 48 : 32;
  if (debug_knob("rows_r", 0) > 0) {
    R = debug_knob("rows_r", R);
    CK = debug_knob("rows_ck", CK);
  } else if (h16) {
    R = hp0 <= 12 ? 1 : R;  // fp16 has no parity-tile / band kernel for the small levels
    if (hp0 > 24 && mode != 2) return hipErrorNotSupported;
  } else if (hp0 <= 6 || (hp0 > 24 && mode != 2)) {
    return hipErrorNotSupported;  // l0/l1-sized: the band kernel; l4-sized: the stream kernel
  }
  Geo g;
  g.Wq4 = ((W / 2) + 3) & ~3;
  g.Wf = g.Wq4 + 8;
  g.S = g.Wq4 / 4;
  g.Q = W / epq;
  // 13..24 parity rows: 3-row bands split into two displacement-row groups (tj 0-4 / 5-8:
  // 7 staged f2 rows instead of 11) when that fills the workgroup rounds better than 2-row
  // bands -- config-2 l3: 256 workgroups instead of 192, 14.2 -> 13.1 us
  // (profiles/r02e_rows_tj_groups.txt); Sintel fp16 l2 keeps 2-row bands (224 against 320)
  g.TS = 1;
  if (hp0 > 12 && hp0 <= 24 && debug_knob("rows_r", 0) == 0) {
    const long long u2 = (long long)B * 2 * ((hp0 + 1) / 2);
    const long long u3 = (long long)B * 2 * ((hp0 + 2) / 3) * 2;
    auto fill = [](long long u) { return (double)u / (256.0 * (double)((u + 255) / 256)); };
    if (fill(u3) > fill(u2)) R = 3, g.TS = 2;
  }
  g.TS = debug_knob("rows_ts", g.TS);
  if (g.TS < 1 || g.TS > D) return hipErrorNotSupported;
  g.DT = (D + g.TS - 1) / g.TS;
  g.TS = (D + g.DT - 1) / g.DT;  // no empty groups
  g.NR2 = R + g.DT - 1;
  g.I = g.DT * R * 2 * g.S;
  constexpr int NT = 768;
  if (g.I > NT || R < 1) return hipErrorNotSupported;
  g.G = NT / g.I;
  if (g.G > C) g.G = C;
  const int hp = (H + 1) / 2;
  g.nb = (hp + R - 1) / R;
  g.units = B * 2 * g.nb * g.TS;
  g.ck = CK < C ? CK : C;
  size_t lds = 0;
  for (;; g.ck = (g.ck + 1) / 2) {  // the largest chunk of channels that fits the LDS
    g.f1f = g.ck * R * 2 * g.Wq4;
    g.f2f = g.ck * g.NR2 * 2 * g.Wf;
    const size_t stage = (size_t)(g.f1f + g.f2f) * 4;
    const size_t red = (size_t)g.G * g.I * D * 16;
    lds = stage > red ? stage : red;
    if (lds <= 160 * 1024) break;
    if (g.ck <= 4) return hipErrorNotSupported;
  }
  const int per1 = (g.ck * R * g.Q + NT - 1) / NT;  // 16-B loads per thread per chunk
  const int per2 = (g.ck * g.NR2 * g.Q + NT - 1) / NT;
  g.inv_Q = 1.f / (float)g.Q;
  g.inv_NR2 = 1.f / (float)g.NR2;
  g.inv_I = 1.f / (float)g.I;
  g.inv_S = 1.f / (float)g.S;
  g.inv_W4 = 1.f / (float)(W / 4);
  g.census = debug_knob("rows_census", 0);
  int ex;
  const float mnt = std::frexp(divisor, &ex);
  const float inv = (mnt == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  P->g = g;
  P->lds = lds;
  P->R = R;
  P->per1 = per1;
  P->per2 = per2;
  P->inv = inv;
  P->h16 = h16;
  return hipSuccess;
}
}  // namespace rows

// The instantiated (storage type, band rows R, loads per thread M1 / M2) variants, first match
// wins: the launcher and the acceptance predicate below walk the same list.  Round 4 dropped the
// variants no default plan reaches: (3, 1, 4) and (2, 1, 3) sat behind (3, 2, 7) / (2, 2, 6) in
// the first-match order, and (4, 2, 8) needed the rows_r=4 knob (plan() picks R <= 3).
#define PWC_ROWS_VARIANTS(X)                                                  \
  X(float, 3, 2, 7) /* l4 at CK 16: 1.75 / 6.4 loads per thread per chunk */ \
  X(float, 2, 2, 6)                                                          \
  X(float, 1, 1, 5)                                                          \
  X(float, 2, 2, 8)                                                          \
  X(float, 1, 2, 8)                                                          \
  X(_Float16, 2, 1, 3)                                                       \
  X(_Float16, 2, 2, 6)                                                       \
  X(_Float16, 1, 1, 3)                                                       \
  X(_Float16, 1, 2, 5)

extern "C" __attribute__((visibility("default"))) int pwc_debug_rows_census(void* dst, int n) {
  if (dst == nullptr) {
    static unsigned long long zeros[4096 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(rows::g_rows_census), zeros, sizeof(zeros)) == hipSuccess;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(rows::g_rows_census),
                             sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}

// Whether corr_forward_rows serves this problem (a plan and an instantiated variant exist).
bool corr_rows_accepts(int B, int C, int H, int W, int dtype) {
  rows::Plan P;
  if (rows::plan(B, C, H, W, (float)C, dtype, &P) != hipSuccess) return false;
#define PWC_ROWS_OK(TT, RR, M1, M2) \
  if (sizeof(TT) == (P.h16 ? 2u : 4u) && P.R == RR && P.per1 <= M1 && P.per2 <= M2) return true;
  PWC_ROWS_VARIANTS(PWC_ROWS_OK)
#undef PWC_ROWS_OK
  return false;
}

hipError_t corr_forward_rows(const void* in1, const void* in2, void* out, int B, int C, int H,
                             int W, float divisor, int dtype, hipStream_t stream) {
  using namespace rows;
  Plan P;
  const hipError_t pe = plan(B, C, H, W, divisor, dtype, &P);
  if (pe != hipSuccess) return pe;
  const Geo& g = P.g;
  const size_t lds = P.lds;
  const int R = P.R, per1 = P.per1, per2 = P.per2;
  const float inv = P.inv;
  const bool h16 = P.h16;
  constexpr int NT = 768;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
#define PWC_ROWS(TT, RR, M1, M2)                                                              \
  if (sizeof(TT) == (h16 ? 2u : 4u) && R == RR && per1 <= M1 && per2 <= M2) {                 \
    {  /* > 64 KiB dynamic LDS, once per device (capi.hip) */                                 \
      const hipError_t e = lds_limit(                                                         \
          reinterpret_cast<const void*>(&corr_fwd_rows<TT, RR, NT, M1, M2>), 160 * 1024);     \
      if (e != hipSuccess) return e;                                                          \
    }                                                                                         \
    hipExtLaunchKernelGGL((corr_fwd_rows<TT, RR, NT, M1, M2>), dim3((unsigned)g.units),       \
                          dim3(NT), lds, stream, ev0, ev1, 0, (const TT*)in1, (const TT*)in2, \
                          (TT*)out, C, H, W, divisor, inv, g, current_epi());                 \
    return hipGetLastError();                                                                 \
  }
  PWC_ROWS_VARIANTS(PWC_ROWS)
#undef PWC_ROWS
  return hipErrorNotSupported;
}

// Two independent fp32 problems that each take the row-band kernel, as one launch; the
// variant pairs instantiated are the config-2 l2 (R 1) + l3 (R 3) ones.  hipErrorNotSupported
// = no such pair (the caller runs them one by one).  Values equal the single launches bit for
// bit (same workgroup body and plan).
hipError_t corr_forward_rows_pair(const void* a1, const void* a2, void* aout, int aB, int aC,
                                  int aH, int aW, const void* b1, const void* b2, void* bout,
                                  int bB, int bC, int bH, int bW, float adiv, float bdiv,
                                  hipStream_t stream) {
  using namespace rows;
  if (!epi_is_default(current_epi()) || debug_knob("rows_pair", 1) == 0)
    return hipErrorNotSupported;
  Plan pa, pb;
  if (plan(aB, aC, aH, aW, adiv, 0, &pa) != hipSuccess ||
      plan(bB, bC, bH, bW, bdiv, 0, &pb) != hipSuccess)
    return hipErrorNotSupported;
  const long long nA = pa.g.units, nB = pb.g.units;
  if (nA + nB >= (1ll << 31)) return hipErrorNotSupported;
  const size_t lds = pa.lds > pb.lds ? pa.lds : pb.lds;
  const RowsArgs A{a1, a2, aout, aC, aH, aW, adiv, pa.inv, pa.g};
  const RowsArgs Bq{b1, b2, bout, bC, bH, bW, bdiv, pb.inv, pb.g};
  constexpr int NT = 768;
#define PWC_ROWS_PAIR(RA, M1A, M2A, RB, M1B, M2B)                                             \
  if (pa.R == RA && pa.per1 <= M1A && pa.per2 <= M2A && pb.R == RB && pb.per1 <= M1B &&       \
      pb.per2 <= M2B) {                                                                       \
    {  /* > 64 KiB dynamic LDS, once per device (capi.hip) */                                 \
      const hipError_t e = lds_limit(                                                         \
          reinterpret_cast<const void*>(                                                      \
              &corr_fwd_rows_pair<float, RA, M1A, M2A, RB, M1B, M2B, NT>),                    \
          160 * 1024);                                                                      \
      if (e != hipSuccess) return e;                                                          \
    }                                                                                         \
    hipEvent_t ev0 = nullptr, ev1 = nullptr;                                                  \
    take_launch_events(&ev0, &ev1); /* the one-shot timing hook times this launch */          \
    hipExtLaunchKernelGGL((corr_fwd_rows_pair<float, RA, M1A, M2A, RB, M1B, M2B, NT>),        \
                          dim3((unsigned)(nA + nB)), dim3(NT), lds, stream, ev0, ev1, 0, A,   \
                          Bq, (int)nA, current_epi());                                        \
    return hipGetLastError();                                                                 \
  }
  // the variants the single launcher would pick (same first-match order: R 3 takes (2, 7)
  // before (1, 4); R 1 takes (1, 5))
  const bool a3 = pa.R == 3 && pa.per1 <= 2 && pa.per2 <= 7;
  const bool b3 = pb.R == 3 && pb.per1 <= 2 && pb.per2 <= 7;
  const bool a1v = pa.R == 1 && pa.per1 <= 1 && pa.per2 <= 5;
  const bool b1v = pb.R == 1 && pb.per1 <= 1 && pb.per2 <= 5;
  if (a1v && b3) {
    PWC_ROWS_PAIR(1, 1, 5, 3, 2, 7)
  }
  if (a3 && b1v) {
    PWC_ROWS_PAIR(3, 2, 7, 1, 1, 5)
  }
#undef PWC_ROWS_PAIR
  return hipErrorNotSupported;
}

}  // namespace pwc
