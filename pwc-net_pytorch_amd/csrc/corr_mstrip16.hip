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
// Diagonal extraction.  Lane l holds D[4(l>>4) + v][l & 15], v = 0..3.  Rows 0-7 come from the
// first product, 8-15 from the second; within its 16-lane row of lanes, output ti of row i sits in
// lane ti + (i mod 8), so two DPP row shifts per register (row_shl v on lane rows 0 and 2,
// row_shl 4+v on rows 1 and 3) bring all four u of a lane row to lane ti.  With both parities,
// lane (g, ti) then holds 8 consecutive pixels of plane ti: one 16-B store.
//
// Schedule.  A workgroup owns a 128-px column strip of 14 parity rows, one output row per STEP:
// step s reads f2 rows s .. s+8 of the chunk's window from an 11-slot LDS ring (row m in slot
// m % 11) and f1 row s from one of two buffers.  Four loader waves keep the next TWO steps' rows
// in flight in registers: between the barriers B_{s-1} and B_s they issue step s+2's loads and
// write step s's (loaded two steps earlier) into the slot step s-3 freed, so a load has two steps
// to land.  Four compute waves (one 16-u block each, both parities, all 9 tj) store each step's
// row while the next steps compute.
#include <hip/hip_ext.h>

#include <cmath>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace mstrip16 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4v __attribute__((__vector_size__(4 * sizeof(short))));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4;
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

struct Geo {
  static constexpr int C = 32;
  static constexpr int TW = 128;            // strip width (px)
  static constexpr int NU = TW / 2;         // pixels per parity
  static constexpr int RS = 80;             // halves per (parity, channel) row; f2 uses 72
  static constexpr int EB = C * RS * 2;     // bytes per parity plane of a staged row
  static constexpr int ROWB = 2 * EB;       // bytes per staged row
  static constexpr int RCH = 14;            // parity rows per workgroup = steps
  static constexpr int NSL = 11;            // f2 ring: a step's 9 rows + the 2 staged ahead
  static constexpr int LDS_BYTES = (NSL + 2) * ROWB;
  static constexpr int NWC = 4;             // compute waves: one 16-u block each
  static constexpr int NWL = 4;             // loader waves
  static constexpr int THREADS = 64 * (NWC + NWL);
  static constexpr int IF2 = C * (TW + 16) / 8;  // 16-B load items per f2 row (8-px halo each side)
  static constexpr int IF1 = C * TW / 8;         // per f1 row
  static constexpr int LT = 64 * NWL;            // loader lanes
  static constexpr int LB = (IF2 + IF1 + LT - 1) / LT;  // items per loader lane per step
  static_assert(NU == 16 * NWC, "one 16-u block per compute wave");
  static_assert((RS / 2) % 16 == 8 && RS >= NU + 8, "8 channel rows on distinct bank groups");
  static_assert(LDS_BYTES <= 160 * 1024 && THREADS <= 1024, "workgroup resources");
};

constexpr uint32_t kOOB = 0x80000000u;

struct Ctx {
  __amdgpu_buffer_rsrc_t rs1, rs2;  // this image's f1 / f2
  uint32_t plane_b;                 // channel plane bytes
  int H, W, Y0, py, x0;
};

// A loader lane's items of one step: NK2 slots of the new f2 row (item i = lane + LT k, channel
// i / 18, 8-px group i % 18: 18 consecutive lanes read 288 contiguous bytes of one channel row),
// then NK1 slots of the f1 row (channel i / 16).  Per lane the global offset without the row
// term and the LDS offset without the buffer base are fixed; each step adds uniform row terms, so
// a load instruction is all-f2 or all-f1 (a uniform buffer resource).
constexpr int NK2 = (Geo::IF2 + Geo::LT - 1) / Geo::LT;
constexpr int NK1 = Geo::IF1 / Geo::LT;
static_assert(NK1 * Geo::LT == Geo::IF1 && NK2 + NK1 == Geo::LB, "loader slots");

struct LaneItems {
  uint32_t g[Geo::LB];  // global byte offset of the item's 8 px in row 0, or kOOB
  int l[Geo::LB];       // LDS byte of its even run within a staged row, -1: no item
};

__device__ __forceinline__ void lane_items(const Ctx& c, int lt, LaneItems& it) {
#pragma unroll
  for (int k = 0; k < Geo::LB; ++k) {
    const bool f2 = k < NK2;
    const int i = lt + Geo::LT * (f2 ? k : k - NK2);
    const int per = f2 ? Geo::TW / 8 + 2 : Geo::TW / 8;
    const int ch = i / per, kk = i % per;
    const int x = f2 ? c.x0 - 8 + 8 * kk : c.x0 + 8 * kk;
    const bool have = f2 ? i < Geo::IF2 : true;
    it.g[k] = have && x >= 0 && x < c.W ? (uint32_t)ch * c.plane_b + (uint32_t)x * 2u : kOOB;
    it.l[k] = have ? (ch * Geo::RS + 4 * kk) * 2 : -1;
  }
}

// row term of parity row pr: byte offset of its first pixel, or kOOB outside the image
__device__ __forceinline__ uint32_t row_off(const Ctx& c, int pr) {
  const int y = 2 * pr + c.py;
  return pr >= 0 && y < c.H ? (uint32_t)y * (uint32_t)c.W * 2u : kOOB;
}

__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t rs, uint32_t g, uint32_t row) {
  const uint32_t off = (g | row) & kOOB ? kOOB : g + row;
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
}

// 8 pixels of one channel -> the 4 even and the 4 odd halves, one 8-B run in each parity plane
__device__ __forceinline__ void item_store(char* lds, int lds_b, const u32x4& d) {
  if (lds_b < 0) return;
  const u32x2 ev = {__builtin_amdgcn_perm(d.y, d.x, 0x05040100u),
                    __builtin_amdgcn_perm(d.w, d.z, 0x05040100u)};
  const u32x2 od = {__builtin_amdgcn_perm(d.y, d.x, 0x07060302u),
                    __builtin_amdgcn_perm(d.w, d.z, 0x07060302u)};
  *reinterpret_cast<u32x2*>(lds + lds_b) = ev;
  *reinterpret_cast<u32x2*>(lds + lds_b + Geo::EB) = od;
}

// Step st's loads: f2 window row st + 8 and f1 row st
__device__ __forceinline__ void step_issue(const Ctx& c, const LaneItems& it, int st,
                                           u32x4 (&r)[Geo::LB]) {
  const uint32_t r2 = row_off(c, c.Y0 - 4 + st + 8), r1 = row_off(c, c.Y0 + st);
#pragma unroll
  for (int k = 0; k < Geo::LB; ++k)
    r[k] = k < NK2 ? load16(c.rs2, it.g[k], r2) : load16(c.rs1, it.g[k], r1);
}

__device__ __forceinline__ void step_write(char* lds, const LaneItems& it, int st,
                                           const u32x4 (&r)[Geo::LB]) {
  const int b2 = ((st + 8) % Geo::NSL) * Geo::ROWB, b1 = (Geo::NSL + (st & 1)) * Geo::ROWB;
#pragma unroll
  for (int k = 0; k < Geo::LB; ++k)
    item_store(lds, it.l[k] < 0 ? -1 : it.l[k] + (k < NK2 ? b2 : b1), r[k]);
}

// Both transposed reads of one 16 x 32 operand block: channels 4g + q, then 16 + 4g + q
__device__ __forceinline__ f16x8 tr_block(const char* lds, int byte) {
  typedef __attribute__((address_space(3))) char lchar;
  const lchar* p = (const lchar*)lds + byte;
  const s16x4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  const s16x4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 16 * Geo::RS * 2));
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

__device__ __forceinline__ f32x4 diag(const f32x4& d1, const f32x4& d2, bool lo_half) {
  const i32x4 a = __builtin_bit_cast(i32x4, d1), b = __builtin_bit_cast(i32x4, d2);
  i32x4 r;
  r[0] = diag_reg<0>(lo_half ? a[0] : b[0]);
  r[1] = diag_reg<1>(lo_half ? a[1] : b[1]);
  r[2] = diag_reg<2>(lo_half ? a[2] : b[2]);
  r[3] = diag_reg<3>(lo_half ? a[3] : b[3]);
  return __builtin_bit_cast(f32x4, r);
}

template <int POL>
__global__ __launch_bounds__(Geo::THREADS, 1) void corr_fwd_mstrip16(
    const __half* __restrict__ in1, const __half* __restrict__ in2, __half* __restrict__ out,
    int H, int W, int nchunk, int ntx, float inv_divisor, OutEpi epi) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // logical block = (n, row parity, chunk, strip), strip fastest (XCD neighbours share rows)
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % ntx;
  const int ch = (t / ntx) % nchunk;
  const int py = (t / (ntx * nchunk)) & 1;
  const int n = t / (ntx * nchunk * 2);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Ctx c;
  c.plane_b = (uint32_t)(H * W) * 2u;
  const uint32_t img_bytes = (uint32_t)Geo::C * c.plane_b;  // < 2^31 (launcher)
  const __half* img1 = in1 + (size_t)n * Geo::C * H * W;
  const __half* img2 = in2 + (size_t)n * Geo::C * H * W;
  c.rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)img1, (short)0, (int)img_bytes, 0x00020000);
  c.rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)img2, (short)0, (int)img_bytes, 0x00020000);
  c.H = H, c.W = W, c.Y0 = ch * Geo::RCH, c.py = py, c.x0 = tx * Geo::TW;

  // step 0's window (f2 rows 0..8) and f1 row: every wave, one batch (item i of the 9 x IF2
  // window items: row i / IF2; then the f1 row over the first IF1 threads)
  {
    constexpr int SK = (9 * Geo::IF2 + Geo::THREADS - 1) / Geo::THREADS;
    static_assert(Geo::IF1 <= Geo::THREADS, "one f1 slot");
    u32x4 r[SK + 1];
    int b[SK + 1];
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      const int i = threadIdx.x + Geo::THREADS * k;
      const int m = i / Geo::IF2, j = i % Geo::IF2;
      const int ch = j / (Geo::TW / 8 + 2), kk = j % (Geo::TW / 8 + 2);
      const int x = c.x0 - 8 + 8 * kk;
      const bool have = m < 9;
      r[k] = load16(c.rs2, have && x >= 0 && x < W ? (uint32_t)ch * c.plane_b + (uint32_t)x * 2u
                                                   : kOOB,
                    row_off(c, c.Y0 - 4 + m));
      b[k] = have ? m * Geo::ROWB + (ch * Geo::RS + 4 * kk) * 2 : -1;
    }
    {
      const int i = threadIdx.x;
      const int ch = i / (Geo::TW / 8), kk = i % (Geo::TW / 8);
      const int x = c.x0 + 8 * kk;
      const bool have = i < Geo::IF1;
      r[SK] = load16(c.rs1, have && x < W ? (uint32_t)ch * c.plane_b + (uint32_t)x * 2u : kOOB,
                     row_off(c, c.Y0));
      b[SK] = have ? Geo::NSL * Geo::ROWB + (ch * Geo::RS + 4 * kk) * 2 : -1;
    }
#pragma unroll
    for (int k = 0; k <= SK; ++k) item_store(lds, b[k], r[k]);
  }

  if (wave >= Geo::NWC) {
    // ---------------- loader waves ----------------
    LaneItems it;
    lane_items(c, threadIdx.x - 64 * Geo::NWC, it);
    u32x4 r[3][Geo::LB];
    step_issue(c, it, 1, r[1]);
    step_issue(c, it, 2, r[2]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B_0
#pragma unroll
    for (int s = 1; s < Geo::RCH; ++s) {
      // between B_{s-1} and B_s (step s-1 computing): step s+2's loads out, step s's rows in
      // (f2 row s+8 into the slot of row s-3, f1 into buffer s & 1, both last read by step s-2)
      if (s + 2 < Geo::RCH) step_issue(c, it, s + 2, r[(s + 2) % 3]);
      step_write(lds, it, s, r[s % 3]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // B_s
    }
    return;
  }

  // ---------------- compute waves ----------------
  const int ub = wave;  // 16-u block: pixels x0 + 32 ub .. + 31
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, jj = lane & 15;
  const int lane_b = ((4 * g + q) * Geo::RS + 4 * p) * 2 + 32 * ub;
  const bool lo_half = lane < 32;
  const int xs = c.x0 + 32 * ub + 8 * g;  // this lane's 8 output pixels
  const bool lane_ok = jj < 9 && xs < W;
  const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * 81 * H * W)), (short)0,
      (int)(81u * c.plane_b), 0x00020000);
  const float slope = epi.slope;
  const bool plain = slope == 1.f;  // no fused leaky_relu
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's share of step 0's staging
  int slot0 = 0;                                       // slot of window row s
  for (int s = 0; s < Geo::RCH; ++s) {
    __builtin_amdgcn_s_barrier();  // B_s: the step's rows are in LDS
    const int y = 2 * (c.Y0 + s) + py;
    if (y < H) {
      const int f1b = (Geo::NSL + (s & 1)) * Geo::ROWB + lane_b;
      const f16x8 a0 = tr_block(lds, f1b);
      const f16x8 a1 = tr_block(lds, f1b + Geo::EB);
      const uint32_t o0 = ((uint32_t)y * W + xs) * 2u;
      // software pipeline over tj: the next displacement row's four operand blocks are read
      // while this row's products and diagonals run
      int sl = slot0;
      f16x8 bc[4], bn[4];
      {
        const int f2b = sl * Geo::ROWB + lane_b;
        bc[0] = tr_block(lds, f2b), bc[1] = tr_block(lds, f2b + 16);
        bc[2] = tr_block(lds, f2b + Geo::EB), bc[3] = tr_block(lds, f2b + Geo::EB + 16);
      }
#pragma unroll
      for (int tj = 0; tj < 9; ++tj) {
        sl = sl + 1 == Geo::NSL ? 0 : sl + 1;
        if (tj < 8) {
          const int f2b = sl * Geo::ROWB + lane_b;
          bn[0] = tr_block(lds, f2b), bn[1] = tr_block(lds, f2b + 16);
          bn[2] = tr_block(lds, f2b + Geo::EB), bn[3] = tr_block(lds, f2b + Geo::EB + 16);
        }
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 d10 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bc[0], z, 0, 0, 0);
        const f32x4 d20 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bc[1], z, 0, 0, 0);
        const f32x4 d11 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bc[2], z, 0, 0, 0);
        const f32x4 d21 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bc[3], z, 0, 0, 0);
        const f32x4 e0 = diag(d10, d20, lo_half) * inv_divisor;  // exact: 2^-k
        const f32x4 e1 = diag(d11, d21, lo_half) * inv_divisor;
        u32x4 h;
        if (plain) {
#pragma unroll
          for (int v = 0; v < 4; ++v)
            h[v] = __builtin_bit_cast(uint32_t, h2_t{(_Float16)e0[v], (_Float16)e1[v]});
        } else {
#pragma unroll
          for (int v = 0; v < 4; ++v)
            h[v] = __builtin_bit_cast(uint32_t, h2_t{(_Float16)fmaxf(e0[v], e0[v] * slope),
                                                     (_Float16)fmaxf(e1[v], e1[v] * slope)});
        }
        const uint32_t off = o0 + (uint32_t)((tj * 9 + jj) * H) * (uint32_t)W * 2u;
        __builtin_amdgcn_raw_buffer_store_b128(h, rso, (int)(lane_ok ? off : kOOB), 0, POL);
#pragma unroll
        for (int k = 0; k < 4; ++k) bc[k] = bn[k];
      }
    }
    slot0 = slot0 + 1 == Geo::NSL ? 0 : slot0 + 1;
  }
}

}  // namespace mstrip16

// Whether the fp16 MFMA strip kernel serves this problem: fp16 storage, model.py:24's stride-2
// displacements in raster order (dr = 4, pad = md, k = 1, s1 = 1: the caller), C = 32, W a
// multiple of 8, 16-B aligned buffers, at least ~one workgroup per CU (knob mstrip16=0: off).
bool corr_mstrip16_accepts(const void* in1, const void* in2, const void* out, int B, int C,
                           int H, int W, int s2, int dtype, int layout) {
  using G = mstrip16::Geo;
  if (dtype != 1 || s2 != 2 || layout != kRaster || C != G::C) return false;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16) return false;
  if (W % 8 || W < 64 || H < 2 || (size_t)C * H * W * 2 >= 0x7ffffff0ull) return false;
  if ((size_t)81 * H * W * 2 >= 0x7ffffff0ull) return false;
  if (debug_knob("mstrip16", 1) == 0) return false;
  const long long nblk = (long long)B * 2 * (((H + 1) / 2 + G::RCH - 1) / G::RCH) *
                         ((W + G::TW - 1) / G::TW);
  return nblk >= 192;
}

hipError_t corr_forward_mstrip16(const void* in1, const void* in2, void* out, int B, int C,
                                 int H, int W, float divisor, hipStream_t stream) {
  using G = mstrip16::Geo;
  if (!corr_mstrip16_accepts(in1, in2, out, B, C, H, W, 2, 1, kRaster))
    return hipErrorNotSupported;
  int ex;
  const float mnt = std::frexp(divisor, &ex);
  if (mnt != 0.5f) return hipErrorNotSupported;  // exact 1 / divisor multiply
  const float inv = std::ldexp(1.f, 1 - ex);
  const OutEpi epi = current_epi();
  if (!(epi.slope <= 1.f)) return hipErrorNotSupported;  // max(v, slope v) form
  if (epi.ostride % 8) return hipErrorNotSupported;      // 16-B stores
  const int nchunk = ((H + 1) / 2 + G::RCH - 1) / G::RCH;
  const int ntx = (W + G::TW - 1) / G::TW;
  const long long nblk = (long long)B * 2 * nchunk * ntx;
  if (nblk <= 0) return hipSuccess;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&mstrip16::corr_fwd_mstrip16<2>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);  // bench.py's live timing hook (one-shot)
  hipExtLaunchKernelGGL((mstrip16::corr_fwd_mstrip16<2>), dim3((unsigned)nblk),
                        dim3(G::THREADS), G::LDS_BYTES, stream, ev0, ev1, 0, (const __half*)in1,
                        (const __half*)in2, (__half*)out, H, W, nchunk, ntx, inv, epi);
  return hipGetLastError();
}

}  // namespace pwc
