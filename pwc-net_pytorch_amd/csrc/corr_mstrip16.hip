// corr_mstrip16.hip — correlation forward of BASELINE config 4 (Sintel shape 448 x 1024, fp16
// storage, B = 16) on the matrix cores: the l4 level (32 x 112 x 256) of model.py:24's
// Correlation(9, 1, 9, 1, 2), fp16 in and out, fp32 sums.
//
// Semantics (correlation_cuda_kernel.cu:34-106 with k = 1, s1 = 1, pad = md = 9, s2 = 2; the
// reference has no fp16 path, so this is its arithmetic on fp16 storage: every product of two
// fp16 values is exact in fp32, sums are fp32, the result rounds to fp16 once):
//   out[n, (tj+4)*9 + (ti+4), y, x] = sum_c f1[n,c,y,x] * f2[n,c,y+2tj,x+2ti] / C
//
// The contraction.  Split the columns by parity, x = 2u + e: the displacement x + 2ti - 8 is
// then u + ti - 4 of the same parity, and for one output row y, one displacement row tj and one
// parity e the volume is a band of a GEMM over the channels:
//   D[u][u'] = sum_c f1[c, y, 2u+e] * f2[c, y+2tj-8, 2u'+e],   out(ti) = D[u][u + ti - 4].
// One v_mfma_f32_16x16x32_f16 (K = 32 = C) takes 16 u x 16 u'; the 9 diagonals of a 16-u block
// lie in two of them, u' from u0-4 (rows u0 .. u0+7) and from u0+4 (rows u0+8 .. u0+15):
// 28 % of the products are used, which still leaves the matrix cores far from the bound
// (288 MFMA per output row per CU, ~0.2 us; the VALU dot-product form took ~3 us).
//
// Operands come from LDS with ds_read_b64_tr_b16 (the transposed read: lane i of a 16-lane group
// receives pixel i of four channel rows), so the rows are staged planar per (parity, channel):
// [e][c][u] halves, 80 halves per row (40 dwords: any 8 consecutive channel rows of one read
// fall on distinct 8-dword bank groups).  The loader de-interleaves the parities (one 16-B load =
// 8 pixels of one channel -> 4 even + 4 odd halves, two v_perm each) and writes two 8-B runs.
//
// Diagonal extraction.  Rows 0-7 need the u' block at u0-4, rows 8-15 the one at u0+4: with the
// f1 operand split into its two row halves (the other half zeroed), both products accumulate
// into ONE tile, D = A_lo B_1 + A_hi B_2.  Lane l holds D[4(l>>4) + v][l & 15], v = 0..3; within
// its 16-lane row of lanes, output ti of row i sits in lane ti + (i mod 8), so two DPP row shifts
// per register (row_shl v on lane rows 0 and 2, row_shl 4+v on rows 1 and 3) bring all four u of
// a lane row to lane ti.  With both parities,
// lane (g, ti) then holds 8 consecutive pixels of plane ti: one 16-B store.
//
// Schedule.  A workgroup owns a 128-px column strip of 14 parity rows, one output row per STEP:
// step s reads f2 rows s .. s+8 of the chunk's window from an 11-slot LDS ring (row m in slot
// m % 11) and f1 row s from one of two buffers.  Four loader waves keep the next TWO steps' rows
// in flight in registers: between the barriers B_{s-1} and B_s they issue step s+2's loads and
// write step s's (loaded two steps earlier) into the slot step s-3 freed, so a load has two steps
// to land.  Eight compute waves (a 16-u block and a share of the 9 displacement rows each, both
// parities; two per SIMD, so one wave's MFMA and DPP latencies hide behind the other's) store
// each step's row while the next steps compute.
#include <hip/hip_ext.h>

#include <cmath>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace mstrip16 {

// volume store cache policy: 0 (write-back).  Nontemporal (2) stores wrote 86.1 MB per l4
// launch for 74.3 MB of volume (partial lines streamed out twice); write-back stores write
// 72.6 MB within the launch, the l4 kernel runs 3.79 -> 4.05 TB/s by its events, and config 4's
// step is unchanged (102.19 K pairs/s both, 4 alternating rounds;
// profiles/r06f_mstrip16_store_policy.txt).  Measurement builds may override.
#ifndef PWC_MS_STPOL
#define PWC_MS_STPOL 0
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4v __attribute__((__vector_size__(4 * sizeof(short))));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4;
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

// halves per staged (parity, channel) row: >= NU + 8 (the f2 halo), and RS/2 dwords = 8 (mod 16)
// so the eight channel rows one 32-lane half of a transposed read takes sit on distinct 8-dword
// bank groups
constexpr int row_halves(int nu) { return 2 * (16 * ((nu + 8 - 8 + 31) / 32) + 8); }

// C channels, TW-px strips, RCH parity rows (steps) per workgroup.  Config-4 l4: <32, 128, 14>
// (four 16-u blocks, the 9 displacement rows split 5 + 4 over two waves each); config-4 l3:
// <64, 64, 7> (two 16-u blocks, rows split 3 + 2 + 2 + 2; K = 64 as two MFMAs per block);
// config-4 l2: <96, 32, 4, 24> (one 16-u block, rows split 2 + 1 x 7 over eight waves; K = 96
// as three MFMAs; rows of 24 halves, NU + 8, so the ring fits the LDS -- at the cost of 2-way
// bank conflicts on some transposed reads: RS_ overrides the conflict-free stride).
// S1: stride-1 displacements (Correlation(4, 1, 4, 1, 1), CostVolumeLayer sr = 4): no column
// parity -- a staged row is ONE plane of the strip's pixels x0 - 8 .. x0 + TW + 8, the two tiles
// of a wave (the parities of stride 2) are two adjacent 16-px blocks, and the rows of the ring
// are consecutive image rows instead of one parity's.
template <int C_, int TW_, int RCH_, int RS_ = 0, bool S1_ = false>
struct Geo {
  static constexpr int C = C_, TW = TW_, RCH = RCH_;
  static constexpr bool S1 = S1_;
  static constexpr int HALO = S1 ? TW_ / 2 + 16 : 8;  // staged halves beyond NU of an f2 row
  static constexpr int KC = C / 32;                // MFMA K chunks
  static constexpr int NU = TW / 2;                // pixels per parity
  static constexpr int NUB = NU / 16;              // 16-u blocks
  static constexpr int TS = 8 / NUB;               // displacement-row splits per block
  static constexpr int RS = RS_ ? RS_ : row_halves(NU);
  // bytes from a row's parity-0 data to its parity-1 data (stride 1: to the next 16-px block)
  static constexpr int EB = S1 ? 32 : C * RS * 2;
  static constexpr int ROWB = S1 ? C * RS * 2 : 2 * EB;  // bytes per staged row
  static constexpr int NSL = 11;                   // f2 ring: a step's 9 rows + 2 staged ahead
  static constexpr int LDS_BYTES = (NSL + 2) * ROWB;
  static constexpr int NWC = NUB * TS;             // compute waves
  static constexpr int NWL = 4;                    // loader waves
  static constexpr int THREADS = 64 * (NWC + NWL);
  static constexpr int G2 = TW / 8 + 2;            // 8-px groups per f2 row (8-px halo each side)
  static constexpr int G1 = TW / 8;                // ... per f1 row
  static constexpr int IF2 = C * G2;               // 16-B load items per f2 row
  static constexpr int IF1 = C * G1;               // per f1 row
  static constexpr int LT = 64 * NWL;              // loader lanes
  static constexpr int NK2 = (IF2 + LT - 1) / LT;  // loader slots: f2 row, then f1 row
  static constexpr int NK1 = (IF1 + LT - 1) / LT;
  static constexpr int LB = NK2 + NK1;
  static_assert(NWC == 8 && NUB * 16 == NU && C % 32 == 0, "eight compute waves, 16-u blocks");
  static_assert((RS_ != 0 || (RS / 2) % 16 == 8) && RS >= NU + HALO && RS % (S1 ? 8 : 4) == 0,
                "8 channel rows on distinct bank groups (unless overridden)");
  static_assert(LDS_BYTES <= 160 * 1024 && THREADS <= 1024, "workgroup resources");
};
using GeoL4 = Geo<32, 128, 14>;
using GeoL3 = Geo<64, 64, 7>;
using GeoL2 = Geo<96, 32, 4, 24>;
// stride 1 (Corr4 / CostVolumeLayer) at config-4 l4 and l3: 14 / 7 image rows per workgroup;
// rows of TW + 16 halves, (RS / 2) = 8 (mod 16) dwords as above
using GeoS1L4 = Geo<32, 128, 14, 144, true>;
using GeoS1L3 = Geo<64, 64, 7, 80, true>;
using GeoS1L2 = Geo<96, 32, 4, 48, true>;

constexpr uint32_t kOOB = 0x80000000u;

struct Ctx {
  __amdgpu_buffer_rsrc_t rs1, rs2;  // this image's f1 / f2
  uint32_t plane_b;                 // channel plane bytes
  int H, W, Y0, py, x0;
  bool s1;                          // stride 1: rows are image rows, not one parity's
};

// A loader lane's items of one step: NK2 slots of the new f2 row (item i = lane + LT k, channel
// i / G2, 8-px group i % G2: consecutive lanes read contiguous bytes of one channel row), then
// NK1 slots of the f1 row.  Per lane the global offset without the row term and the LDS offset
// without the buffer base are fixed; each step adds uniform row terms, so a load instruction is
// all-f2 or all-f1 (a uniform buffer resource).
template <class G>
struct LaneItems {
  uint32_t g[G::LB];  // global byte offset of the item's 8 px in row 0, or kOOB
  int l[G::LB];       // LDS byte of its even run within a staged row, -1: no item
};

// Stride 1: LDS byte (within a staged row) of the 8 px at x = x0 + d of channel ch: f2 rows hold
// pixels x0 - 8 .., f1 rows x0 ..
template <class G>
__device__ __forceinline__ int s1_byte(int ch, int d, bool f2) {
  return (ch * G::RS + d + (f2 ? 8 : 0)) * 2;
}

template <class G>
__device__ __forceinline__ void lane_items(const Ctx& c, int lt, LaneItems<G>& it) {
#pragma unroll
  for (int k = 0; k < G::LB; ++k) {
    const bool f2 = k < G::NK2;
    const int i = lt + G::LT * (f2 ? k : k - G::NK2);
    const int per = f2 ? G::G2 : G::G1;
    const int ch = i / per, kk = i % per;
    const int x = f2 ? c.x0 - 8 + 8 * kk : c.x0 + 8 * kk;
    const bool have = f2 ? i < G::IF2 : i < G::IF1;
    it.g[k] = have && x >= 0 && x < c.W ? (uint32_t)ch * c.plane_b + (uint32_t)x * 2u : kOOB;
    if constexpr (G::S1)
      it.l[k] = have ? s1_byte<G>(ch, x - c.x0, f2) : -1;
    else
      it.l[k] = have ? (ch * G::RS + 4 * kk) * 2 : -1;
  }
}

// row term of parity row pr: byte offset of its first pixel, or kOOB outside the image
__device__ __forceinline__ uint32_t row_off(const Ctx& c, int pr) {
  const int y = c.s1 ? pr : 2 * pr + c.py;
  return pr >= 0 && y < c.H ? (uint32_t)y * (uint32_t)c.W * 2u : kOOB;
}

__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t rs, uint32_t g, uint32_t row) {
  const uint32_t off = (g | row) & kOOB ? kOOB : g + row;
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
}

// 8 pixels of one channel -> the 4 even and the 4 odd halves, one 8-B run in each parity plane
// (stride 1: the 8 pixels as they are)
template <class G>
__device__ __forceinline__ void item_store(char* lds, int lds_b, const u32x4& d) {
  if (lds_b < 0) return;
  if constexpr (G::S1) {
    *reinterpret_cast<u32x4*>(lds + lds_b) = d;
    return;
  }
  const u32x2 ev = {__builtin_amdgcn_perm(d.y, d.x, 0x05040100u),
                    __builtin_amdgcn_perm(d.w, d.z, 0x05040100u)};
  const u32x2 od = {__builtin_amdgcn_perm(d.y, d.x, 0x07060302u),
                    __builtin_amdgcn_perm(d.w, d.z, 0x07060302u)};
  *reinterpret_cast<u32x2*>(lds + lds_b) = ev;
  *reinterpret_cast<u32x2*>(lds + lds_b + G::EB) = od;
}

// Step st's loads: f2 window row st + 8 and f1 row st
template <class G>
__device__ __forceinline__ void step_issue(const Ctx& c, const LaneItems<G>& it, int st,
                                           u32x4 (&r)[G::LB]) {
  const uint32_t r2 = row_off(c, c.Y0 - 4 + st + 8), r1 = row_off(c, c.Y0 + st);
#pragma unroll
  for (int k = 0; k < G::LB; ++k)
    r[k] = k < G::NK2 ? load16(c.rs2, it.g[k], r2) : load16(c.rs1, it.g[k], r1);
}

template <class G>
__device__ __forceinline__ void step_write(char* lds, const LaneItems<G>& it, int st,
                                           const u32x4 (&r)[G::LB]) {
  const int b2 = ((st + 8) % G::NSL) * G::ROWB, b1 = (G::NSL + (st & 1)) * G::ROWB;
#pragma unroll
  for (int k = 0; k < G::LB; ++k)
    item_store<G>(lds, it.l[k] < 0 ? -1 : it.l[k] + (k < G::NK2 ? b2 : b1), r[k]);
}

// Both transposed reads of one 16 x 32 operand block: channels 4g + q, then 16 + 4g + q
template <class G>
__device__ __forceinline__ f16x8 tr_block(const char* lds, int byte) {
  typedef __attribute__((address_space(3))) char lchar;
  const lchar* p = (const lchar*)lds + byte;
  const s16x4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  const s16x4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 16 * G::RS * 2));
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(f16x8, v);
}

// Lane (g, ti) <- the diagonal ti of rows 4g .. 4g+3 (see the header).  Whole-vector bit casts:
// an element-wise bit_cast of a vector element miscompiles to element 0 with this toolchain.
template <int V>
__device__ __forceinline__ int diag_reg(int t) {
  int x = t;
  if constexpr (V > 0) x = __builtin_amdgcn_update_dpp(t, t, 0x100 + V, 0x5, 0xF, false);
  return __builtin_amdgcn_update_dpp(x, t, 0x104 + V, 0xA, 0xF, false);
}

__device__ __forceinline__ f32x4 diag(const f32x4& d) {
  const i32x4 a = __builtin_bit_cast(i32x4, d);
  i32x4 r;
  r[0] = diag_reg<0>(a[0]);
  r[1] = diag_reg<1>(a[1]);
  r[2] = diag_reg<2>(a[2]);
  r[3] = diag_reg<3>(a[3]);
  return __builtin_bit_cast(f32x4, r);
}

// The f1 operand with its rows 8-15 (lo = true) or 0-7 (lo = false) zeroed: rows 0-7 of the
// volume come from the u' block at u0 - 4 and rows 8-15 from the block at u0 + 4, so
// D = A_lo B_1 + A_hi B_2 accumulates both halves in one tile (row i = lane & 15 of A).
__device__ __forceinline__ f16x8 rows_half(const f16x8& a, bool keep) {
  const u32x4 v = __builtin_bit_cast(u32x4, a);
  const u32x4 z = {0u, 0u, 0u, 0u};
  return __builtin_bit_cast(f16x8, keep ? v : z);
}

#ifdef PWC_CENSUS
// measurement build only (make CENSUS=1): ablation mask from knob ms_abl -- 1: no operand reads,
// products or diagonals (zeros stored), 2: no stores, 4: the loader stages nothing after step 0
#define MS_ABL(bit) (abl & (bit))
#else
#define MS_ABL(bit) 0
#endif

// The operand blocks of one displacement row: [parity][u' block][K chunk]
template <class G>
struct BOps {
  f16x8 v[2][2][G::KC];
};

template <class G>
__device__ __forceinline__ void read_b(const char* lds, int f2b, BOps<G>& b) {
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < G::KC; ++k)
        b.v[e][h][k] =
            tr_block<G>(lds, f2b + e * G::EB + 16 * h + (G::S1 ? 8 : 0) + k * 32 * G::RS * 2);
}

// Displacement rows TJ0 .. TJ0 + NTJ - 1 of one output row: the next row's operand blocks are
// read while this row's products, diagonals and store run.
// PLAIN: no fused leaky_relu; POW2: the divisor is a power of two (an exact multiply by
// inv_divisor) -- both compile-time, so no uniform branch sits between the stores (a branch
// around the epilogue cost the compiler its vmcnt accounting across the stores)
template <class G, int TJ0, int NTJ, bool PLAIN, bool POW2>
__device__ __forceinline__ void tj_rows(const char* lds, int slot0, int lane_b,
                                        const f16x8 (&a)[2][2][G::KC],
                                        float inv_divisor, float divisor, float slope,
                                        __amdgpu_buffer_rsrc_t rso, uint32_t o0, uint32_t pstep,
                                        bool lane_ok, int jj, int abl, int layout) {
  if (MS_ABL(1)) {
    const u32x4 h = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int t = 0; t < NTJ; ++t)
      __builtin_amdgcn_raw_buffer_store_b128(
          h, rso, (int)(lane_ok ? o0 + (uint32_t)((TJ0 + t) * 9 + jj) * pstep : kOOB), 0,
          PWC_MS_STPOL);
    return;
  }
  int sl = slot0 + TJ0;
  sl = sl >= G::NSL ? sl - G::NSL : sl;
  BOps<G> bc, bn;
  read_b<G>(lds, sl * G::ROWB + lane_b, bc);
#pragma unroll
  for (int t = 0; t < NTJ; ++t) {
    const int tj = TJ0 + t;
    sl = sl + 1 == G::NSL ? 0 : sl + 1;
    if (t + 1 < NTJ) read_b<G>(lds, sl * G::ROWB + lane_b, bn);
    // both parities' tiles interleaved: consecutive MFMAs are independent
    f32x4 d[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int k = 0; k < G::KC; ++k)
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int pe = 0; pe < 2; ++pe)
          d[pe] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[pe][hb][k], bc.v[pe][hb][k], d[pe], 0,
                                                         0, 0);
    f32x4 e[2];
#pragma unroll
    for (int pe = 0; pe < 2; ++pe) {
      // exact 2^-k multiply; otherwise (C = 96, CostVolumeLayer's / 81) the quotient from the
      // reciprocal with one Newton correction (q + (r - q d) / d): within an fp32 ulp of the
      // division, which the fp16 rounding of the stored value absorbs -- a tenth of a division's
      // instructions
      const f32x4 r = diag(d[pe]);
      if constexpr (POW2) {
        e[pe] = r * inv_divisor;
      } else {
        const float rcp = 1.f / divisor;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float q = r[v] * rcp;
          e[pe][v] = __builtin_fmaf(__builtin_fmaf(-q, divisor, r[v]), rcp, q);
        }
      }
    }
    // output plane of (tj, ti = jj): raster (tj * 9 + ti) or CostVolumeLayer order (stride 1)
    const uint32_t pl = G::S1 && layout == kCvl ? (uint32_t)cvl_channel(tj - 4, min(jj, 8) - 4, 4)
                                                : (uint32_t)(tj * 9 + jj);
    if constexpr (G::S1) {
      // tile pe: pixels 32 ub + 16 pe + 4 g + v.  One permlane16 swap per dword gives lane row g
      // eight consecutive pixels: even rows block 0's x 8 (g / 2) .., odd rows block 1's -- one
      // 16-B store, 64 B per wave and plane (plain epilogue: the predicate declines a fused
      // leaky_relu for stride 1)
      uint32_t p0 = __builtin_bit_cast(uint32_t, h2_t{(_Float16)e[0][0], (_Float16)e[0][1]});
      uint32_t p1 = __builtin_bit_cast(uint32_t, h2_t{(_Float16)e[0][2], (_Float16)e[0][3]});
      uint32_t q0 = __builtin_bit_cast(uint32_t, h2_t{(_Float16)e[1][0], (_Float16)e[1][1]});
      uint32_t q1 = __builtin_bit_cast(uint32_t, h2_t{(_Float16)e[1][2], (_Float16)e[1][3]});
      asm volatile(
          "s_nop 1\n\t"
          "v_permlane16_swap_b32 %0, %2\n\t"
          "v_permlane16_swap_b32 %1, %3\n\t"
          "s_nop 1"
          : "+v"(p0), "+v"(p1), "+v"(q0), "+v"(q1));
      const u32x4 hs = {p0, p1, q0, q1};
      __builtin_amdgcn_raw_buffer_store_b128(hs, rso, (int)(lane_ok ? o0 + pl * pstep : kOOB), 0,
                                             PWC_MS_STPOL);
      if (t + 1 < NTJ) bc = bn;
      continue;
    }
    u32x4 h;
    if constexpr (PLAIN) {
#pragma unroll
      for (int v = 0; v < 4; ++v)
        h[v] = __builtin_bit_cast(uint32_t, h2_t{(_Float16)e[0][v], (_Float16)e[1][v]});
    } else {
#pragma unroll
      for (int v = 0; v < 4; ++v)
        h[v] = __builtin_bit_cast(uint32_t, h2_t{(_Float16)fmaxf(e[0][v], e[0][v] * slope),
                                                 (_Float16)fmaxf(e[1][v], e[1][v] * slope)});
    }
    const uint32_t off = o0 + pl * pstep;
    __builtin_amdgcn_raw_buffer_store_b128(h, rso, (int)(lane_ok ? off : kOOB), 0, PWC_MS_STPOL);
    if (t + 1 < NTJ) bc = bn;
  }
}

template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_fwd_mstrip16(
    const __half* __restrict__ in1, const __half* __restrict__ in2, __half* __restrict__ out,
    int H, int W, int nchunk, int ntx, float inv_divisor, float divisor, OutEpi epi, int abl,
    int layout) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // logical block = (n, row parity, chunk, strip), strip fastest (XCD neighbours share rows);
  // stride 1: (n, chunk, strip)
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % ntx;
  const int ch = (t / ntx) % nchunk;
  const int py = G::S1 ? 0 : (t / (ntx * nchunk)) & 1;
  const int n = t / (ntx * nchunk * (G::S1 ? 1 : 2));
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Ctx c;
  c.plane_b = (uint32_t)(H * W) * 2u;
  const uint32_t img_bytes = (uint32_t)G::C * c.plane_b;  // < 2^31 (launcher)
  const __half* img1 = in1 + (size_t)n * G::C * H * W;
  const __half* img2 = in2 + (size_t)n * G::C * H * W;
  c.rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)img1, (short)0, (int)img_bytes, 0x00020000);
  c.rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)img2, (short)0, (int)img_bytes, 0x00020000);
  c.H = H, c.W = W, c.Y0 = ch * G::RCH, c.py = py, c.x0 = tx * G::TW;
  c.s1 = G::S1;

  // step 0's window (f2 rows 0..8) and f1 row: every wave, one batch (item i of the 9 x IF2
  // window items: row i / IF2; then the f1 row)
  {
    constexpr int SK = (9 * G::IF2 + G::THREADS - 1) / G::THREADS;
    constexpr int S1 = (G::IF1 + G::THREADS - 1) / G::THREADS;
    u32x4 r[SK + S1];
    int b[SK + S1];
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      const int i = threadIdx.x + G::THREADS * k;
      const int m = i / G::IF2, j = i % G::IF2;
      const int chn = j / G::G2, kk = j % G::G2;
      const int x = c.x0 - 8 + 8 * kk;
      const bool have = m < 9;
      r[k] = load16(c.rs2,
                    have && x >= 0 && x < W ? (uint32_t)chn * c.plane_b + (uint32_t)x * 2u : kOOB,
                    row_off(c, c.Y0 - 4 + m));
      b[k] = !have ? -1
                   : m * G::ROWB + (G::S1 ? s1_byte<G>(chn, x - c.x0, true)
                                          : (chn * G::RS + 4 * kk) * 2);
    }
#pragma unroll
    for (int k = 0; k < S1; ++k) {
      const int i = threadIdx.x + G::THREADS * k;
      const int chn = i / G::G1, kk = i % G::G1;
      const int x = c.x0 + 8 * kk;
      const bool have = i < G::IF1;
      r[SK + k] = load16(c.rs1,
                         have && x < W ? (uint32_t)chn * c.plane_b + (uint32_t)x * 2u : kOOB,
                         row_off(c, c.Y0));
      b[SK + k] = !have ? -1
                        : G::NSL * G::ROWB + (G::S1 ? s1_byte<G>(chn, x - c.x0, false)
                                                    : (chn * G::RS + 4 * kk) * 2);
    }
#pragma unroll
    for (int k = 0; k < SK + S1; ++k) item_store<G>(lds, b[k], r[k]);
  }

  if (wave >= G::NWC) {
    // ---------------- loader waves ----------------
    LaneItems<G> it;
    lane_items<G>(c, threadIdx.x - 64 * G::NWC, it);
    u32x4 r[3][G::LB];
    if (G::RCH > 1) step_issue<G>(c, it, 1, r[1]);
    if (G::RCH > 2) step_issue<G>(c, it, 2, r[2]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B_0
#pragma unroll
    for (int s = 1; s < G::RCH; ++s) {
      // between B_{s-1} and B_s (step s-1 computing): step s+2's loads out, step s's rows in
      // (f2 row s+8 into the slot of row s-3, f1 into buffer s & 1, both last read by step s-2)
      if (s + 2 < G::RCH && !MS_ABL(4)) step_issue<G>(c, it, s + 2, r[(s + 2) % 3]);
      step_write<G>(lds, it, s, r[s % 3]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // B_s
    }
    return;
  }

  // ---------------- compute waves ----------------
  const int ub = wave % G::NUB;  // 16-u block: pixels x0 + 32 ub .. + 31
  const int th = wave / G::NUB;  // displacement-row split
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, jj = lane & 15;
  const int lane_b = ((4 * g + q) * G::RS + 4 * p) * 2 + (G::S1 ? 64 : 32) * ub;
  const bool lo_rows = (lane & 15) < 8;  // A rows 0-7 (lanes l & 15 < 8)
  // this lane's 8 output pixels (stride 1 after the swap: block g & 1 of the wave's two, 8 (g / 2)
  // into it)
  const int xs = G::S1 ? c.x0 + 32 * ub + 16 * (g & 1) + 8 * (g >> 1) : c.x0 + 32 * ub + 8 * g;
  const bool lane_ok = jj < 9 && xs < W && !MS_ABL(2);
  const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * 81 * H * W)), (short)0,
      (int)(81u * c.plane_b), 0x00020000);
  const float slope = epi.slope;
  const bool plain = slope == 1.f;  // no fused leaky_relu (stride 1: always, the predicate)
  // stride 2 divides by its compile-time C; stride 1 by C or, for CostVolumeLayer, 81
  const bool pow2 = G::S1 ? inv_divisor != 0.f : (G::C & (G::C - 1)) == 0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's share of step 0's staging
  int slot0 = 0;                                       // slot of window row s
  for (int s = 0; s < G::RCH; ++s) {
    __builtin_amdgcn_s_barrier();  // B_s: the step's rows are in LDS
    const int y = G::S1 ? c.Y0 + s : 2 * (c.Y0 + s) + py;
    if (y < H) {
      const int f1b = (G::NSL + (s & 1)) * G::ROWB + lane_b;
      f16x8 a[2][2][G::KC];  // [parity][rows 0-7 | rows 8-15][K chunk]
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int k = 0; k < G::KC; ++k) {
          const f16x8 v = tr_block<G>(lds, f1b + e * G::EB + k * 32 * G::RS * 2);
          a[e][0][k] = rows_half(v, lo_rows);
          a[e][1][k] = rows_half(v, !lo_rows);
        }
      const uint32_t o0 = ((uint32_t)y * W + xs) * 2u;
      const uint32_t pstep = c.plane_b;
      // the 9 displacement rows split over TS waves per block: 5 + 4, or 3 + 2 + 2 + 2
#define PWC_TJ1(A, N, PL, P2)                                                                 \
  tj_rows<G, A, N, PL, P2>(lds, slot0, lane_b, a, inv_divisor, divisor, slope, rso, o0, pstep, \
                           lane_ok, jj, abl, layout)
#define PWC_TJ(A, N)                                                                          \
  do {                                                                                        \
    if constexpr (G::S1) {                                                                    \
      if (pow2)                                                                               \
        PWC_TJ1(A, N, true, true);                                                            \
      else                                                                                    \
        PWC_TJ1(A, N, true, false);                                                           \
    } else {                                                                                  \
      constexpr bool P2 = (G::C & (G::C - 1)) == 0;                                           \
      if (plain)                                                                              \
        PWC_TJ1(A, N, true, P2);                                                              \
      else                                                                                    \
        PWC_TJ1(A, N, false, P2);                                                             \
    }                                                                                         \
  } while (0)
      if constexpr (G::TS == 2) {
        if (th == 0)
          PWC_TJ(0, 5);
        else
          PWC_TJ(5, 4);
      } else if constexpr (G::TS == 8) {
        switch (th) {
          case 0: PWC_TJ(0, 2); break;
          case 1: PWC_TJ(2, 1); break;
          case 2: PWC_TJ(3, 1); break;
          case 3: PWC_TJ(4, 1); break;
          case 4: PWC_TJ(5, 1); break;
          case 5: PWC_TJ(6, 1); break;
          case 6: PWC_TJ(7, 1); break;
          default: PWC_TJ(8, 1); break;
        }
      } else {
        static_assert(G::TS == 4, "tj splits");
        if (th == 0)
          PWC_TJ(0, 3);
        else if (th == 1)
          PWC_TJ(3, 2);
        else if (th == 2)
          PWC_TJ(5, 2);
        else
          PWC_TJ(7, 2);
      }
#undef PWC_TJ
#undef PWC_TJ1
    }
    slot0 = slot0 + 1 == G::NSL ? 0 : slot0 + 1;
  }
}

// workgroups of the grid: (n, row parity, chunk, strip), stride 1 without the parity
template <class G>
long long grid_blocks(int B, int H, int W) {
  const int rows = G::S1 ? H : (H + 1) / 2;
  return (long long)B * (G::S1 ? 1 : 2) * ((rows + G::RCH - 1) / G::RCH) *
         ((W + G::TW - 1) / G::TW);
}

template <class G>
bool accepts(const void* in1, const void* in2, const void* out, int B, int H, int W) {
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16) return false;
  if (W % 8 || W < 64 || H < 2 || (size_t)G::C * H * W * 2 >= 0x7ffffff0ull) return false;
  if ((size_t)81 * H * W * 2 >= 0x7ffffff0ull) return false;
  return grid_blocks<G>(B, H, W) >= 192;
}

template <class G>
hipError_t launch(const void* in1, const void* in2, void* out, int B, int H, int W, float inv,
                  float divisor, const OutEpi& epi, hipStream_t stream, int layout = kRaster) {
  const int nchunk = ((G::S1 ? H : (H + 1) / 2) + G::RCH - 1) / G::RCH;
  const int ntx = (W + G::TW - 1) / G::TW;
  const long long nblk = grid_blocks<G>(B, H, W);
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e =
        lds_limit(reinterpret_cast<const void*>(&corr_fwd_mstrip16<G>), G::LDS_BYTES);
    if (e != hipSuccess) return e;
  }
#ifdef PWC_CENSUS
  const int abl = debug_knob("ms_abl", 0);
#else
  const int abl = 0;
#endif
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);  // bench.py's live timing hook (one-shot)
  hipExtLaunchKernelGGL((corr_fwd_mstrip16<G>), dim3((unsigned)nblk), dim3(G::THREADS),
                        G::LDS_BYTES, stream, ev0, ev1, 0, (const __half*)in1,
                        (const __half*)in2, (__half*)out, H, W, nchunk, ntx, inv, divisor, epi, abl,
                        layout);
  return hipGetLastError();
}

}  // namespace mstrip16

// Whether the fp16 matrix-core strip kernel serves this problem: fp16 storage, model.py:24's
// stride-2 displacements in raster order (dr = 4, pad = md, k = 1, s1 = 1: the caller), C = 32
// (l4 geometry), 64 (l3) or 96 (l2), W a multiple of 8, 16-B aligned buffers, at least ~one
// workgroup per CU, and an output epilogue the kernel writes itself (leaky_relu slope <= 1:
// the max(v, slope v) form; a channel-slice stride that keeps 16-B stores aligned) -- so this
// predicate, corr_forward_path and the launcher agree (knob mstrip16=0: off).
// Stride 1 (Correlation(4, 1, 4, 1, 1) and CostVolumeLayer sr = 4; pad == md: the caller): C =
// 32 / 64 / 96, raster or CostVolumeLayer channel order, a plain output (no fused epilogue, no
// channel slice: those are the Corr9 model path's).
bool corr_mstrip16_accepts(const void* in1, const void* in2, const void* out, int B, int C,
                           int H, int W, int s2, int dtype, int layout) {
  if (dtype != 1 || debug_knob("mstrip16", 1) == 0) return false;
  const OutEpi epi = current_epi();
  if (s2 == 1) {
    if ((layout != kRaster && layout != kCvl) || epi.slope != 1.f || epi.ostride != 0 ||
        debug_knob("mstrip16_s1", 1) == 0)
      return false;
    if (C == 32) return mstrip16::accepts<mstrip16::GeoS1L4>(in1, in2, out, B, H, W);
    if (C == 64) return mstrip16::accepts<mstrip16::GeoS1L3>(in1, in2, out, B, H, W);
    if (C == 96) return mstrip16::accepts<mstrip16::GeoS1L2>(in1, in2, out, B, H, W);
    return false;
  }
  if (s2 != 2 || layout != kRaster) return false;
  if (!(epi.slope <= 1.f) || epi.ostride % 8) return false;
  if (C == 32) return mstrip16::accepts<mstrip16::GeoL4>(in1, in2, out, B, H, W);
  if (C == 64) return mstrip16::accepts<mstrip16::GeoL3>(in1, in2, out, B, H, W);
  if (C == 96) return mstrip16::accepts<mstrip16::GeoL2>(in1, in2, out, B, H, W);
  return false;
}

hipError_t corr_forward_mstrip16(const void* in1, const void* in2, void* out, int B, int C,
                                 int H, int W, int s2, int layout, float divisor,
                                 hipStream_t stream) {
  if (!corr_mstrip16_accepts(in1, in2, out, B, C, H, W, s2, 1, layout))
    return hipErrorNotSupported;
  int ex;
  const float mnt = std::frexp(divisor, &ex);
  // a power-of-two divisor is an exact multiply; otherwise the kernel divides (inv = 0: the
  // CostVolumeLayer's /81)
  const float inv = mnt == 0.5f ? std::ldexp(1.f, 1 - ex) : 0.f;
  const OutEpi epi = current_epi();  // slope and stride checked by the predicate
  // stride 2 takes its power-of-two decision from C at compile time: Correlation's k^2 C, k = 1
  if (s2 == 2 && divisor != (float)C) return hipErrorNotSupported;
  if (s2 == 1) {
    if (C == 32)
      return mstrip16::launch<mstrip16::GeoS1L4>(in1, in2, out, B, H, W, inv, divisor, epi,
                                                 stream, layout);
    if (C == 64)
      return mstrip16::launch<mstrip16::GeoS1L3>(in1, in2, out, B, H, W, inv, divisor, epi,
                                                 stream, layout);
    return mstrip16::launch<mstrip16::GeoS1L2>(in1, in2, out, B, H, W, inv, divisor, epi, stream,
                                               layout);
  }
  if (C == 32) return mstrip16::launch<mstrip16::GeoL4>(in1, in2, out, B, H, W, inv, divisor, epi,
                                                              stream);
  if (C == 64) return mstrip16::launch<mstrip16::GeoL3>(in1, in2, out, B, H, W, inv, divisor, epi,
                                                              stream);
  return mstrip16::launch<mstrip16::GeoL2>(in1, in2, out, B, H, W, inv, divisor, epi, stream);
}

}  // namespace pwc
