// corr_bwd_rows.hip — correlation backward of model.py:24's configuration (pad == md in {8, 9},
// k 1, s1 1, s2 2: 81 displacement channels, /C), fp32, as row-band gathers (no atomics).
//
//   g1[n,c,y,x]   = sum_t gO[n,t,y,x] * f2[n,c,y+2tj-8,x+2ti-8] / C            (cu:108-198)
//   g2[n,c,y',x'] = sum_t gO[n,t,y'-2tj+8,x'-2ti+8] * f1[n,c,y'-2tj+8,x'-2ti+8] / C
//                                                                                (cu:200-290)
// with t = tj*9 + ti and zero terms outside the image.  In parity space (y = 2Y+p, x = 2X+q)
// both are 9x9 stencils over ONE parity image, the structure of the forward (corr_rows.hip):
//   g1[c,Y,X]   = sum_{tj,ti} gO[t,Y,X]           * F2[c, Y+tj-4, X+ti-4]
//   g2[c,Y',X'] = sum_{tj,ti} gO[t,Y'-tj+4,X'-ti+4] * F1[c, Y'-tj+4, X'-ti+4]
// One workgroup owns one image x one row parity p x a band of R parity rows over full rows.
// It stages the R + 8 same-parity feature rows of a chunk of channels in LDS (split into
// column parities, 4 zero slots each side: the reference's zero padding), and each item
// (tj, band row, column parity, 4-pixel segment) holds the 36 gO values it needs in
// registers for the whole channel loop.  Per channel an item reads 3 aligned quads of one
// staged row and runs 36 FMAs (the forward's ratio); the 9 tj partials of every (channel,
// pixel) meet in LDS and are summed in tj order (deterministic), then stored row by row.
// gO is read once per gradient; the staged features (R+8)/R times, mostly from L2.
//
// VEC (W % 4 == 0, 16-B aligned rows): 16-byte buffer loads split into column parities on the
// way into LDS and 16-byte stores; otherwise dword loads/stores (any W, the l0/l1 levels).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "pwc_common.cuh"

namespace pwc {
namespace bwdrows {

constexpr int D = 9;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kOOB = 0x80000000u;

struct Geo {
  int R;     // parity rows per band
  int Wq4;   // slots of a staged row half: ceil(W/2) rounded up to 4
  int Wf;    // Wq4 + 8 (4 zero slots on each side)
  int S;     // 4-pixel segments per row half (Wq4 / 4)
  int I;     // items: 9 * R * 2 * S
  int G;     // channel groups
  int ck;    // channels per chunk (CT * G)
  int nb;    // bands per parity half
  int stf;   // staging floats: ck * (R + 8) * 2 * Wf
  int nld;   // staging load items per chunk: ck * (R + 8) * (W / 4 if VEC else W)
  int cps;   // channels per slice (grid.y), a multiple of ck
  int lw;    // load items per staged row: W / 4 (VEC) or W
  int census;  // measurement only (knob bwd_census): phase stamps -> g_bwd_census
  float inv_lw, inv_NR, inv_I, inv_S, inv_R;
};

__device__ __forceinline__ int qdiv(int x, float inv) { return (int)(((float)x + 0.5f) * inv); }

// Phase census (measurement only: a `make CENSUS=1` build + knob bwd_census): s_memrealtime
// (100 MHz) of thread 0 of workgroup b -> g_bwd_census[b * 8 + k], a branch-free buffer store.
// The product build compiles the marks out (each store would add to the waits on vmcnt).
typedef unsigned int u32x2b __attribute__((ext_vector_type(2)));
__device__ unsigned long long g_bwd_census[4096 * 8];
#ifdef PWC_CENSUS
#define BWD_MARK(k)                                                                          \
  do {                                                                                       \
    const unsigned lin_ = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;    \
    const bool on_ = g.census && threadIdx.x == 0 && lin_ < 4096;                            \
    const unsigned long long ts_ = __builtin_amdgcn_s_memrealtime();                         \
    __builtin_amdgcn_raw_buffer_store_b64(                                                   \
        __builtin_bit_cast(u32x2b, ts_),                                                     \
        __builtin_amdgcn_make_buffer_rsrc((void*)g_bwd_census, (short)0,                     \
                                          (int)sizeof(g_bwd_census), 0x00020000),            \
        on_ ? (int)((lin_ * 8 + (k)) * 8) : (int)0x80000000, 0, 0);                          \
  } while (0)
#else
#define BWD_MARK(k) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0));
}
__device__ __forceinline__ f32x4 ld4(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
}

// GRAD 1: feat = f2, result g1.  GRAD 2: feat = f1, result g2.  CT channels per item and
// chunk, ML staging loads per thread and chunk.
template <int GRAD, bool VEC, int CT, int ML, int NT>
__device__ __forceinline__ void corr_bwd_rows_body(const float* __restrict__ feat,
                                                   const float* __restrict__ gout,
                                                   float* __restrict__ gin, int C, int H,
                                                   int W, float divisor, float inv_divisor,
                                                   const Geo& g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* stg = lds;
  f32x4* part = reinterpret_cast<f32x4*>(lds + g.stf);
  const int t = threadIdx.x;
  BWD_MARK(0);
  const int R = g.R, NR = R + 8;
  const int unit = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring bands share an L2
  const int b = unit % g.nb, np = unit / g.nb;
  const int p = np & 1, n = np >> 1;
  const int hp = (H - p + 1) >> 1;
  const int r0 = b * R;
  if (r0 >= hp) return;  // odd H: the odd-row half has one row fewer (uniform per workgroup)
  const uint32_t plane = (uint32_t)(H * W);
  const __amdgpu_buffer_rsrc_t rsf = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(feat + (size_t)n * C * plane), (short)0, (int)((uint32_t)C * plane * 4u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t rsg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(gout + (size_t)n * (D * D) * plane), (short)0,
      (int)((uint32_t)(D * D) * plane * 4u), 0x00020000);

  // zero the whole staging once: pad slots and the columns past each half's width stay zero
  for (int i = t; i < g.stf / 4; i += NT) reinterpret_cast<f32x4*>(stg)[i] = f32x4{0, 0, 0, 0};

  // ---- staging plan (fixed over chunks): item = (channel, staged row, raster quad/col) ----
  uint32_t vo[ML];
  int ls[ML], lc[ML];
#pragma unroll
  for (int j = 0; j < ML; ++j) {
    const int itm = t + j * NT;
    const int rest = qdiv(itm, g.inv_lw), e = itm - rest * g.lw;
    const int c = qdiv(rest, g.inv_NR), k = rest - c * NR;
    const int rr = r0 - 4 + k;
    const bool ok = itm < g.nld && rr >= 0 && rr < hp;
    const int col = VEC ? 4 * e : e;
    vo[j] = ok ? ((uint32_t)c * plane + (uint32_t)(2 * rr + p) * W + col) * 4u : kOOB;
    // VEC: slot 4 + 2e of both halves; scalar: half e & 1, slot 4 + (e >> 1)
    ls[j] = itm < g.nld ? ((c * NR + k) * 2 + (VEC ? 0 : (e & 1))) * g.Wf + 4 +
                              (VEC ? 2 * e : (e >> 1))
                        : -1;
    lc[j] = c;
  }

  // ---- compute item (tj, band row r, column parity q, segment s) ----
  // Measured and not kept (r03h): items over three tj rows (the 3 tj summed in registers: a
  // third of the partial stores and epilogue reads, 108 gO registers, l4 as ONE round of
  // 6-row bands in 512-thread workgroups): l4 40.4 us against 36.7 -- its start-up 21 us
  // against 5.9 per round (both gradients' gO, 56 MB, loaded at once) -- and l3 27.8 against
  // 21.8 (profiles/r03h_corr_bwd_tg.txt)
  const int grp = qdiv(t, g.inv_I), it = t - grp * g.I;
  const bool active = grp < g.G;
  const int s = it - qdiv(it, g.inv_S) * g.S;
  int rest = qdiv(it, g.inv_S);
  const int q = rest & 1;
  rest >>= 1;
  const int r = rest - qdiv(rest, g.inv_R) * R, tj = qdiv(rest, g.inv_R);
  const int whq = (W - q + 1) >> 1;  // columns of this parity
  // the 36 gO values of this item, zero where the forward output does not exist.  Every load
  // is issued before the first use (straight-line code, one wait): loads and uses interleaved
  // per displacement made the compiler wait for each displacement's loads in turn (9
  // dependent memory round trips per workgroup start).
  float gv[D][4];
  constexpr int NQ = GRAD == 1 ? 2 : 3;  // quads per displacement (VEC)
  f32x4 raw[VEC ? D : 1][NQ];
  {
    const int Y = GRAD == 1 ? r0 + r : r0 + r - tj + 4;  // gO parity row
    const bool rok = active && Y >= 0 && Y < hp && r0 + r < hp;
#pragma unroll
    for (int ti = 0; ti < D; ++ti) {
      const int X0 = GRAD == 1 ? 4 * s : 4 * s - ti + 4;  // gO parity column of kk = 0
      const uint32_t rowoff = (uint32_t)(tj * D + ti) * plane + (uint32_t)(2 * Y + p) * W;
      if constexpr (VEC && GRAD == 1) {
        const uint32_t o = rok ? (rowoff + 8 * s) * 4u : kOOB;
        raw[ti][0] = ld4(rsg, o);
        raw[ti][1] = ld4(rsg, o + 16u);
      } else if constexpr (VEC) {
        // raster columns 2*X0 + q + 2kk (kk = 0..3) from three aligned quads [b, b + 12);
        // b = 2*X0 - 2*(ti & 1).  X0 < 0 only for ti >= 5, so rowoff + b stays >= 0 (the
        // quads then start in the previous plane's data, masked below)
        const uint32_t o = rok ? (rowoff + 2 * X0 - 2 * (ti & 1)) * 4u : kOOB;
#pragma unroll
        for (int k = 0; k < NQ; ++k) raw[ti][k] = ld4(rsg, o + 16u * k);
      } else {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int X = X0 + kk;
          const bool ok = rok && X >= 0 && X < whq;
          gv[ti][kk] = ld1(rsg, ok ? (rowoff + 2 * X + q) * 4u : kOOB);
        }
      }
    }
  }
  if constexpr (VEC) {
#pragma unroll
    for (int ti = 0; ti < D; ++ti) {
      if constexpr (GRAD == 1) {
        const f32x4 a = raw[ti][0], c4 = raw[ti][1];
        gv[ti][0] = q ? a.y : a.x;
        gv[ti][1] = q ? a.w : a.z;
        gv[ti][2] = q ? c4.y : c4.x;
        gv[ti][3] = q ? c4.w : c4.z;
      } else {
        const int X0 = 4 * s - ti + 4, sh = 2 * (ti & 1);
        const f32x4 a = raw[ti][0], bq = raw[ti][1], c4 = raw[ti][2];
        const float w12[12] = {a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w, c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int X = X0 + kk;
          const bool ok = X >= 0 && X < whq;
          const float v = q ? w12[sh + 2 * kk + 1] : w12[sh + 2 * kk];
          gv[ti][kk] = ok ? v : 0.f;
        }
      }
    }
  }
  // every gO value has landed before the chunk loop: left pending, the waits the compiler
  // places for them inside the loop also wait for the next chunk's staging loads
#pragma unroll
  for (int ti = 0; ti < D; ++ti)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) asm volatile("" : "+v"(gv[ti][kk]));
  const int krow = GRAD == 1 ? r + tj : r - tj + 8;  // staged feature row
  const int wbase = (krow * 2 + q) * g.Wf + 4 * s;
  const int cstride = NR * 2 * g.Wf;
  const int RS2 = R * 2 * g.S;
  const int pbase = (tj * R + r) * 2 * g.S + q * g.S + s;

  // channel slice of this workgroup (grid.y), chunks of ck; the next chunk's staging loads
  // are in flight during the current chunk's compute and epilogue
  const int cs = blockIdx.y * g.cps, ce = min(C, cs + g.cps);
  f32x4 vv[ML];
  float vs[ML];
  auto issue = [&](int cb) {
    const int cn = min(g.ck, ce - cb);
    const uint32_t so = (uint32_t)cb * plane * 4u;
#pragma unroll
    for (int j = 0; j < ML; ++j) {
      const uint32_t o = (lc[j] < cn ? vo[j] : kOOB) + so;
      if (VEC)
        vv[j] = ld4(rsf, o);
      else
        vs[j] = ld1(rsf, o);
    }
  };
  if (cs < ce) issue(cs);
  for (int cb = cs; cb < ce; cb += g.ck) {
    const int cn = min(g.ck, ce - cb);
    lds_barrier();  // the zeroing / the previous chunk's compute and epilogue are done
#pragma unroll
    for (int j = 0; j < ML; ++j) {
      if (ls[j] < 0) continue;
      if (VEC) {
        *reinterpret_cast<f32x2*>(stg + ls[j]) = f32x2{vv[j].x, vv[j].z};
        *reinterpret_cast<f32x2*>(stg + ls[j] + g.Wf) = f32x2{vv[j].y, vv[j].w};
      } else {
        stg[ls[j]] = vs[j];
      }
    }
    if (cb + g.ck < ce) issue(cb + g.ck);
    lds_barrier();
    BWD_MARK(cb == cs ? 1 : 3);  // chunk staged (1: the first -- gO registers landed too)
    if (active) {
      // channel j of the chunk: 3 window quads, 36 FMAs.  The next channel's quads are read
      // before this channel's FMAs (double-buffered; the partial store between channels would
      // otherwise pin each channel's reads behind the previous store).  No `c < cn` guard: a
      // short chunk's missing channels are staged as zeros and their partials never summed.
      auto rd = [&](int j, f32x4(&b)[3]) {
        const float* pw = stg + (grp + j * g.G) * cstride + wbase;
        b[0] = *reinterpret_cast<const f32x4*>(pw);
        b[1] = *reinterpret_cast<const f32x4*>(pw + 4);
        b[2] = *reinterpret_cast<const f32x4*>(pw + 8);
      };
      f32x4 bA[3], bB[3];
      rd(0, bA);
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        f32x4(&cur)[3] = (j & 1) ? bB : bA;
        f32x4(&nxt)[3] = (j & 1) ? bA : bB;
        if (j + 1 < CT) rd(j + 1, nxt);
        __builtin_amdgcn_sched_barrier(0);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float w[12] = {cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y,
                             cur[1].z, cur[1].w, cur[2].x, cur[2].y, cur[2].z, cur[2].w};
#pragma unroll
        for (int ti = 0; ti < D; ++ti)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            acc[kk] = fmaf(gv[ti][kk], w[GRAD == 1 ? kk + ti : kk + 8 - ti], acc[kk]);
        part[(grp + j * g.G) * (D * RS2) + pbase] = f32x4{acc[0], acc[1], acc[2], acc[3]};
      }
    }
    lds_barrier();
    BWD_MARK(cb == cs ? 2 : 4);  // chunk computed
    // ---- epilogue: the 9 tj partials of each (channel, pixel) summed in tj order ----
    // Exactly one output (quad) per thread (the launcher guarantees ck * R * lw <= NT):
    // threads past the last output redo the last one -- identical value, identical address --
    // so the number of stores is static (l4 37.8 -> 37.0 us, l3 20.8 -> 20.3 against a
    // runtime-counted store loop; holding the store back until the next chunk was staged
    // measured 40.4: profiles/r03h_corr_bwd_tg.txt)
    const int Rv = min(R, hp - r0);  // band rows inside the image (odd H: the last band)
    const float inv_Rv = 1.f / (float)Rv;
    if (VEC) {
      const int Q = W >> 2;
      const int o = min(t, cn * Rv * Q - 1);
      const int m = o - qdiv(o, g.inv_lw) * Q;  // raster quad: x = 4m .. 4m+3
      const int rc = qdiv(o, g.inv_lw);
      const int rr = rc - qdiv(rc, inv_Rv) * Rv, c = qdiv(rc, inv_Rv);
      const int i0 = 2 * m, sg = i0 >> 2, kk = i0 & 3;  // kk in {0, 2}
      const float* p0 =
          reinterpret_cast<const float*>(part + c * (D * RS2) + rr * 2 * g.S + sg) + kk;
      const float* p1 = p0 + 4 * g.S;  // column parity 1
      f32x2 e0 = *reinterpret_cast<const f32x2*>(p0);
      f32x2 e1 = *reinterpret_cast<const f32x2*>(p1);
#pragma unroll
      for (int j = 1; j < D; ++j) {
        e0 += *reinterpret_cast<const f32x2*>(p0 + 4 * j * RS2);
        e1 += *reinterpret_cast<const f32x2*>(p1 + 4 * j * RS2);
      }
      f32x4 v4 = f32x4{e0.x, e1.x, e0.y, e1.y};
      if (inv_divisor != 0.f)
        v4 *= inv_divisor;
      else
        v4 = f32x4{v4.x / divisor, v4.y / divisor, v4.z / divisor, v4.w / divisor};
      st_out4(gin + ((size_t)n * C + cb + c) * plane + (size_t)(2 * (r0 + rr) + p) * W + 4 * m,
              v4);
    } else {
      const int o = min(t, cn * Rv * W - 1);
      const int x = o - qdiv(o, g.inv_lw) * W;
      const int rc = qdiv(o, g.inv_lw);
      const int rr = rc - qdiv(rc, inv_Rv) * Rv, c = qdiv(rc, inv_Rv);
      const int qq = x & 1, X = x >> 1;
      const float* p0 = reinterpret_cast<const float*>(part + c * (D * RS2) + rr * 2 * g.S +
                                                       qq * g.S + (X >> 2)) +
                        (X & 3);
      float e = *p0;
#pragma unroll
      for (int j = 1; j < D; ++j) e += p0[4 * j * RS2];
      e = inv_divisor != 0.f ? e * inv_divisor : e / divisor;
      st_out1(gin + ((size_t)n * C + cb + c) * plane + (size_t)(2 * (r0 + rr) + p) * W + x, e);
    }
  }
  BWD_MARK(5);  // stores issued
}

// Both gradients in ONE launch: grid.z = 0 computes g1 from f2, grid.z = 1 g2 from f1 (the
// two are independent; at the coarse levels each alone fills a fraction of the chip, so one
// launch runs them side by side and saves a launch gap).  Measured and not kept (r03h): the two
// gradients and channel slices of a band adjacent on one XCD, so that both read the band's gO
// from one L2 in the same round (l4 36.7 -> 38.9 us).
template <bool VEC, int CT, int ML, int NT>
__global__ __launch_bounds__(NT, 1) void corr_bwd_rows(const float* __restrict__ f1,
                                                       const float* __restrict__ f2,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ g1,
                                                       float* __restrict__ g2, int C, int H,
                                                       int W, float divisor, float inv_divisor,
                                                       Geo g) {
  if (blockIdx.z == 0)
    corr_bwd_rows_body<1, VEC, CT, ML, NT>(f2, gout, g1, C, H, W, divisor, inv_divisor, g);
  else
    corr_bwd_rows_body<2, VEC, CT, ML, NT>(f1, gout, g2, C, H, W, divisor, inv_divisor, g);
}

}  // namespace bwdrows

// Measurement knobs (PWC_DEBUG / pwc_set_debug): bwd_rows=0 disables the kernel; bwd_r forces a
// band height, bwd_slices the channel slices.
hipError_t corr_backward_rows_f32(const void* in1, const void* in2, const void* gout, void* g1,
                                  void* g2, int B, int C, int H, int W, float divisor,
                                  hipStream_t stream) {
  using namespace bwdrows;
  const bool off = debug_knob("bwd_rows", 1) == 0;
  if (off || B == 0 || C == 0 || H == 0 || W < 2) return hipErrorNotSupported;
  if ((size_t)C * H * W >= (1ull << 29) || (size_t)81 * H * W >= (1ull << 29))
    return hipErrorNotSupported;
  const bool vec = W % 4 == 0 && (uintptr_t)in1 % 16 == 0 && (uintptr_t)in2 % 16 == 0 &&
                   (uintptr_t)gout % 16 == 0 && (uintptr_t)g1 % 16 == 0 &&
                   (uintptr_t)g2 % 16 == 0;
  const int hp = (H + 1) / 2;
  Geo g;
  g.Wq4 = (((W + 1) / 2) + 3) & ~3;
  g.Wf = g.Wq4 + 8;
  g.S = g.Wq4 / 4;
  // the tallest band (least restaging of the R + 8 feature rows); channel slices fill the chip.
  // CT (channels per item and chunk) 8 on the 16-B path; 2 on the dword path (l0 / l1: more,
  // shorter chunks give more slices -- 10.6 -> 9.4 us at l0, 12.0 -> 11.6 at l1;
  // profiles/r02e_corr_bwd_slices.txt)
  constexpr int NT = 768;
  int R = 1, CT = vec ? 8 : 2;
  for (int r : {3, 2, 1}) {
    if (9 * r * 2 * g.S > NT) continue;
    R = r;
    break;
  }
  R = debug_knob("bwd_r", R);
  g.R = R;
  g.I = 9 * R * 2 * g.S;
  if (R < 1 || g.I > NT) return hipErrorNotSupported;
  g.G = NT / g.I;
  if (g.G * CT > C) g.G = (C + CT - 1) / CT;
  g.nb = (hp + R - 1) / R;
  size_t lds = 0;
  for (;; --g.G) {  // fewest channel groups' worth of LDS that fits
    g.ck = CT * g.G;
    g.stf = g.ck * (R + 8) * 2 * g.Wf;
    lds = (size_t)g.stf * 4 + (size_t)g.ck * 9 * R * 2 * g.S * 16;
    if (lds <= 160 * 1024) break;
    if (g.G == 1) return hipErrorNotSupported;
  }
  g.lw = vec ? W / 4 : W;
  // the epilogue stores one output (quad) per thread and chunk
  if ((long long)g.ck * R * g.lw > NT) return hipErrorNotSupported;
  g.census = debug_knob("bwd_census", 0);
  g.nld = g.ck * (R + 8) * g.lw;
  // channel slices (grid.y) up to one workgroup per CU over both gradients (grid.z): the
  // slices of a band are independent (every gradient element is one channel's) but each
  // re-reads the band's gO.  Measured (B = 8, 384 x 448): l1 16.0 -> 12.3 us (CT 8, 3
  // slices), l2 17.0 -> 12.7 (2), l3 27.7 -> 23.2 (1), l0 / l4 unchanged (4 / 1)
  const long long bands = (long long)B * 2 * ((hp + R - 1) / R);
  const int nchunks = (C + g.ck - 1) / g.ck;
  int nsl = 1;
  while (nsl < nchunks && bands * 2 * (nsl + 1) <= 256) ++nsl;
  if (const int k = debug_knob("bwd_slices", 0)) nsl = std::max(1, std::min(nchunks, k));
  g.cps = ((nchunks + nsl - 1) / nsl) * g.ck;
  nsl = (C + g.cps - 1) / g.cps;
  g.inv_lw = 1.f / (float)g.lw;
  g.inv_NR = 1.f / (float)(R + 8);
  g.inv_I = 1.f / (float)g.I;
  g.inv_S = 1.f / (float)g.S;
  g.inv_R = 1.f / (float)R;
  const int ml = (g.nld + NT - 1) / NT;
  int ex;
  const float mnt = std::frexp(divisor, &ex);
  const float inv = (mnt == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  const unsigned units = (unsigned)(B * 2 * g.nb);
#define PWC_BWD(V, CTT, M)                                                                     \
  if (vec == V && CT == CTT && ml <= M) {                                                      \
    {  /* > 64 KiB dynamic LDS, once per device (capi.hip) */                                  \
      const hipError_t e = lds_limit(                                                          \
          reinterpret_cast<const void*>(&corr_bwd_rows<V, CTT, M, NT>), 160 * 1024);           \
      if (e != hipSuccess) return e;                                                           \
    }                                                                                          \
    hipLaunchKernelGGL((corr_bwd_rows<V, CTT, M, NT>), dim3(units, nsl, 2), dim3(NT), lds,     \
                       stream, (const float*)in1, (const float*)in2, (const float*)gout,       \
                       (float*)g1, (float*)g2, C, H, W, divisor, inv, g);                      \
    return hipGetLastError();                                                                  \
  }
  PWC_BWD(true, 8, 2)
  PWC_BWD(true, 8, 4)
  PWC_BWD(true, 8, 8)
  PWC_BWD(false, 2, 4)
  PWC_BWD(false, 2, 8)
#undef PWC_BWD
  return hipErrorNotSupported;
}

// measurement only: copy (dst) or clear (dst == null) the phase stamps of bwd_census launches
extern "C" __attribute__((visibility("default"))) int pwc_debug_bwd_census(void* dst, int n) {
  if (dst == nullptr) {
    static unsigned long long zeros[4096 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(bwdrows::g_bwd_census), zeros, sizeof(zeros)) ==
           hipSuccess;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(bwdrows::g_bwd_census),
                             sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}

}  // namespace pwc
