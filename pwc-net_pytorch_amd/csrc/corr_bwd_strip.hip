// corr_bwd_strip.hip — correlation backward of model.py:24's configuration (pad == md in {8, 9},
// k 1, s1 1, s2 2: 81 displacement channels, /C) for the strip-sized fp32 levels (config 5's
// l2 / l3 / l4), both gradients in one launch, no atomics, no partial sums through LDS or HBM.
//
//   g1[n,c,y,x]   = sum_t gO[n,t,y,x] * f2[n,c,y+2tj-8,x+2ti-8] / C            (cu:108-198)
//   g2[n,c,y',x'] = sum_t gO[n,t,y'-2tj+8,x'-2ti+8] * f1[n,c,y'-2tj+8,x'-2ti+8] / C
//                                                                                (cu:200-290)
// with t = 9 tj + ti and zero terms outside the image.  A row only meets rows of its own parity.
//
// Why this shape.  corr_bwd_rows.hip gives every (tj, row, segment) item its
// 36 gO values in registers and reduces the nine tj partials of every (channel, pixel) through
// LDS: one partial store per 36 FMAs.  Here the displacement rows are the workgroup's STEPS: a
// workgroup owns R parity rows of one image parity, full width, ALL channels (so gO is staged
// once per gradient); lane = (row, 4-px segment, set of CS channels) with its 4 x CS gradient
// values in registers for the whole launch.  Step u (0..8) needs, for every row r of the band,
// the feature row r + u - 4 (f2 for g1: tj = u; f1 for g2: tj = 8 - u, the rows then coincide)
// and the nine gO planes of that tj at the rows of the band (g1) or at the feature rows (g2).
// The feature rows live in a ring of R + 2 LDS slots, the gO planes of a step in one of three
// LDS buffers; two loader waves (feature rows, gO) keep the next two steps' LDS-DMAs
// (buffer_load_dwordx4 ... lds; the range check gives the zero border) in flight while the
// compute waves run a step.  Per channel and step a lane reads 5 ds_read_b128 of its feature
// row and runs 18 v_pk_fma_f32 on the step's 36 gO values, which it reads once per step for all
// CS channels:
//   g1: acc[c][k] += gO[ti][x+k]          * f2w[c][x + 2ti - 8 + k]
//   g2: acc[c][k] += gO[ti][x+8-2ti+k]    * f1w[c][x + 8 - 2ti + k]
// (g2's gO quads are half-aligned for odd ti: two ds_read_b64).  The order of the sums is fixed
// (steps, channels, ti), so the result is repeatable bit for bit.
//
// Bound (profiles/r05n_corr_bwd_strip.txt): the steps run at the rate the LDS-DMAs land
// (~30 GB/s per CU, rows served mostly from the Infinity Cache: every 3-row band re-reads 8 halo
// rows), not at the LDS or VALU rate; the variants measured and not kept are listed there.
#include <hip/hip_runtime.h>

#include <cmath>

#include "pwc_common.cuh"

namespace pwc {
namespace bstrip {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kOOB = 0x80000000u;

// CW channels per workgroup, R parity rows per band, NSEG 4-px segments per row (W = 4 NSEG),
// CS channels per lane.
template <int CW_, int R_, int NSEG_, int CS_>
struct Geo {
  static constexpr int CW = CW_, R = R_, NSEG = NSEG_, CS = CS_;
  static constexpr int K = CW / CS;               // lanes per (row, segment)
  static constexpr int NTASK = R * NSEG * K;      // lanes with work
  static constexpr int NWC = (NTASK + 63) / 64;   // compute waves
  static constexpr int THREADS = 64 * (NWC + 2);  // + two loader waves (feature rows, gO)
  static constexpr int GQ = NSEG + 4;             // quads of a staged gO row: 2 zero quads each side
  // LDS bank slots (16 B) of one ds_read_b128 lane group of the feature-row reads: the slot of a
  // lane is (k CS CHS + s) mod 16 (ring slots are whole DMAs, = 0 mod 16).  Conflict degree
  // summed over every 16-lane group of the launch, for a channel-row stride CHS.
  static constexpr int conflicts(int chs) {
    int total = 0;
    for (int g0 = 0; g0 < NWC * 64; g0 += 16) {
      int cnt[16] = {}, worst = 1;
      for (int l = 0; l < 16; ++l) {
        const int t = g0 + l;
        if (t >= NTASK) break;  // idle lanes repeat the last task's address
        const int s = t % NSEG, k = (t / NSEG) % K;
        const int b = (k * CS * chs + s) % 16;
        ++cnt[b];
        worst = cnt[b] > worst ? cnt[b] : worst;
      }
      total += worst - 1;
    }
    return total;
  }
  static constexpr int pick_chs() {
    int best = NSEG + 4, bc = conflicts(NSEG + 4);
    for (int c = NSEG + 5; c < NSEG + 20; ++c)
      if (conflicts(c) < bc) best = c, bc = conflicts(c);
    return best;
  }
  static constexpr int CHS = pick_chs();  // quads per staged channel row (2 zero quads each side)
  static constexpr int SLOT = (CW * CHS + 63) / 64 * 64;  // quads per ring slot (whole DMAs)
  static constexpr int IPS = SLOT / 64;                   // DMAs per feature row
  static constexpr int NSLOT = R + 2;  // the rows of a step + the next two steps' new rows
  static constexpr int GBUF = (9 * R * GQ + 63) / 64 * 64;  // quads per gO buffer
  static constexpr int IPG = GBUF / 64;
  static constexpr int NGB = 3;  // gO buffers: the step's + the next two
  static constexpr int LDS_BYTES = (NSLOT * SLOT + NGB * GBUF) * 16;
  static_assert(CW % CS == 0 && NSEG >= 1, "geometry");
  static_assert(LDS_BYTES <= 160 * 1024 && THREADS <= 1024, "workgroup resources");
  static_assert(2 * IPS <= 63 && 2 * IPG <= 63, "two steps' DMAs of a loader within the 6-bit vmcnt");
  static_assert(((CS - 1) * CHS + 4) * 16 < 65536 && (8 * R * GQ + 4) * 16 < 65536,
                "ds offsets are instruction immediates");
};

#ifdef PWC_BSTRIP_CENSUS  // measurement build (tools/bstrip_census.py): phase stamps, 100 MHz
// slots: 0 entry, 1 .. 9 barriers B_0 .. B_8 passed, 10 last FMA, 11 stores issued (compute wave
// 0); 12 / 13 the feature / gO loader's prologue landed.  Kept in LDS behind the buffers (the
// step loop would index registers at run time) and copied out by compute wave 0 at the end.
__device__ unsigned long long g_bs_census[8192 * 16];
#define BSTAMP(slot)                                                                      \
  do {                                                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                       \
    if (lane == 0)                                                                        \
      asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds0 + G::LDS_BYTES + \
                                                               (uint32_t)(slot) * 8u),   \
                   "v"(t_)                                                                \
                   : "memory");                                                           \
  } while (0)
#define CENSUS_EXTRA 128
#else
#define BSTAMP(slot) \
  do {               \
  } while (0)
#define CENSUS_EXTRA 0
#endif

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ f32x4 lds_rd4(uint32_t a) {
  return *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>((uintptr_t)a);
}
__device__ __forceinline__ f32x2 lds_rd2(uint32_t a) {
  return *reinterpret_cast<const __attribute__((address_space(3))) f32x2*>((uintptr_t)a);
}

// workgroup barrier that is also a compiler barrier for memory operations (the builtin is not:
// LDS reads could move across it)
__device__ __forceinline__ void wg_barrier() { asm volatile("s_barrier" ::: "memory"); }

#ifndef PWC_BSTRIP_GO_AUX  // cache policy of the gO DMAs (measurement builds may override)
#define PWC_BSTRIP_GO_AUX 0
#endif
#ifndef PWC_BSTRIP_F_AUX  // cache policy of the feature-row DMAs
#define PWC_BSTRIP_F_AUX 0
#endif

template <int AUX = 0>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t lds, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)(uintptr_t)lds, 16, voff, 0, 0, AUX);
#endif
}

// 36 FMAs (18 v_pk_fma_f32) of one channel and step: acc[k] += sum_ti g[ti][k] * w[j(ti) + k],
// j = 2 ti (g1) or 16 - 2 ti (g2), w = the 20 feature values x-8 .. x+11 of the lane's segment.
template <int GRAD>
__device__ __forceinline__ void bwd_fma(float (&acc)[4], const f32x4 (&g)[9], const f32x4 (&w)[5]) {
#pragma unroll
  for (int ti = 0; ti < 9; ++ti) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = (GRAD == 1 ? 2 * ti : 16 - 2 * ti) + 2 * h;
      const f32x4 q = w[j >> 2];
      const f32x2 w2 = (j & 2) ? f32x2{q.z, q.w} : f32x2{q.x, q.y};
      const f32x2 a2 = h ? f32x2{g[ti].z, g[ti].w} : f32x2{g[ti].x, g[ti].y};
      f32x2 c2 = {acc[2 * h], acc[2 * h + 1]};
      c2 = __builtin_elementwise_fma(a2, w2, c2);
      acc[2 * h] = c2.x;
      acc[2 * h + 1] = c2.y;
    }
  }
}

struct Args {
  const float* f1;
  const float* f2;
  const float* gout;
  float* g1;
  float* g2;
  int C, H, W, nb, ns, B;
};

template <class G, int GRAD>
__device__ __forceinline__ void body(const Args& a, int n, int p, int band, int slice) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int H = a.H, W = a.W;
  const int hp = (H - p + 1) >> 1;  // parity rows of this parity
  const int r0 = band * G::R;
  if (r0 >= hp) return;  // odd H: the odd-row half may have a band fewer (uniform)
  const int c0 = slice * G::CW;
  const uint32_t plane_b = (uint32_t)(H * W) * 4u;
  const float* feat = (GRAD == 1 ? a.f2 : a.f1) + ((size_t)n * a.C + c0) * H * W;
  const uint32_t lds0 = lds_addr(lds);
  const uint32_t gbase = lds0 + (uint32_t)(G::NSLOT * G::SLOT) * 16u;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave == 0) BSTAMP(0);

  if (wave == G::NWC) {
    // ---------------- loader wave 1: feature rows ----------------
    const uint32_t feat_bytes = (uint32_t)G::CW * plane_b;
    uint32_t relw[G::IPS];
#pragma unroll
    for (int i = 0; i < G::IPS; ++i) {
      const int q4 = 64 * i + lane, cc = q4 / G::CHS, q = q4 % G::CHS;
      relw[i] = cc < G::CW && q >= 2 && q < G::NSEG + 2
                    ? (uint32_t)cc * plane_b + (uint32_t)(q - 2) * 16u
                    : kOOB;
    }
    // feature row m of the walk (parity row r0 - 4 + m) into ring slot m % NSLOT; DMAs from
    // index D0 on wait for a free vmcnt slot (the prologue's rows exceed 63)
    auto dma_row = [&](int m, int D0) {
      const int Y = r0 - 4 + m, yrow = 2 * Y + p;
      const bool ok = Y >= 0 && yrow < H;
      const uint32_t off = ok ? (uint32_t)yrow * (uint32_t)W * 4u : 0u;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)feat + off), (short)0, ok ? (int)(feat_bytes - off) : 0,
          0x00020000);
      const uint32_t dst = lds0 + (uint32_t)((m % G::NSLOT) * G::SLOT) * 16u;
#pragma unroll
      for (int i = 0; i < G::IPS; ++i) {
        if (D0 + i >= 63) asm volatile("s_waitcnt vmcnt(62)" ::: "memory");
        dma16<PWC_BSTRIP_F_AUX>(rs, dst + (uint32_t)i * 1024u, relw[i]);
      }
    };
    // prologue: steps 0 and 1 (rows 0 .. R), wait for step 0's
#pragma unroll
    for (int m = 0; m <= G::R; ++m) dma_row(m, m * G::IPS);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::IPS) : "memory");
    BSTAMP(12);
    wg_barrier();  // B_0
#pragma unroll 1
    for (int u = 0; u < 8; ++u) {
      if (u < 7) {  // step u + 2's new row, then wait for step u + 1's
        dma_row(u + G::R + 1, G::IPS);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::IPS) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      wg_barrier();  // B_{u+1}
    }
    return;
  }
  if (wave == G::NWC + 1) {
    // ---------------- loader wave 2: the gO planes of each step ----------------
    uint32_t relg[G::IPG];
    int rowg[G::IPG];
#pragma unroll
    for (int i = 0; i < G::IPG; ++i) {
      const int q4 = 64 * i + lane, ti = q4 / (G::R * G::GQ), rem = q4 % (G::R * G::GQ);
      const int q = rem % G::GQ;
      rowg[i] = rem / G::GQ;
      relg[i] = ti < 9 && q >= 2 && q < G::NSEG + 2
                    ? (uint32_t)ti * plane_b + (uint32_t)(q - 2) * 16u
                    : kOOB;
    }
    const __amdgpu_buffer_rsrc_t rsg = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.gout + (size_t)n * 81 * H * W), (short)0, (int)(81u * plane_b), 0x00020000);
    // the nine gO planes of step u into buffer u % 3
    auto dma_g = [&](int u) {
      const int plane0 = GRAD == 1 ? 9 * u : 9 * (8 - u);
      const uint32_t dst = gbase + (uint32_t)((u % G::NGB) * G::GBUF) * 16u;
#pragma unroll
      for (int i = 0; i < G::IPG; ++i) {
        const int Y = GRAD == 1 ? r0 + rowg[i] : r0 + rowg[i] + u - 4;
        const bool ok = relg[i] != kOOB && Y >= 0 && Y < hp;
        const uint32_t off =
            ok ? relg[i] + (uint32_t)plane0 * plane_b + (uint32_t)(2 * Y + p) * (uint32_t)W * 4u
               : kOOB;
        dma16<PWC_BSTRIP_GO_AUX>(rsg, dst + (uint32_t)i * 1024u, off);
      }
    };
    dma_g(0);
    dma_g(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::IPG) : "memory");
    BSTAMP(13);
    wg_barrier();  // B_0
#pragma unroll 1
    for (int u = 0; u < 8; ++u) {
      if (u < 7) {
        dma_g(u + 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::IPG) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      wg_barrier();  // B_{u+1}
    }
    return;
  }

  // ---------------- compute waves ----------------
  const int tl = wave * 64 + lane;
  const bool active = tl < G::NTASK;
  const int t = active ? tl : G::NTASK - 1;  // idle lanes duplicate a task, store nothing
  const int s = t % G::NSEG, k = (t / G::NSEG) % G::K, r = t / (G::NSEG * G::K);
  float acc[G::CS][4];
#pragma unroll
  for (int j = 0; j < G::CS; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[j][e] = 0.f;
  const uint32_t wlane = (uint32_t)(k * G::CS * G::CHS + s) * 16u;
  const uint32_t glane = gbase + (uint32_t)(r * G::GQ + s) * 16u;

  int gb = 0;  // gO buffer of the step (u % 3)
#pragma unroll 1
  for (int u = 0; u < 9; ++u) {
    const int slot = (r + u) % G::NSLOT;
    const uint32_t wa = lds0 + (uint32_t)(slot * G::SLOT) * 16u + wlane;
    const uint32_t ga = glane + (uint32_t)(gb * G::GBUF) * 16u;
    gb = gb == G::NGB - 1 ? 0 : gb + 1;
    wg_barrier();  // B_u: this step's rows landed, step u - 1 done everywhere
    if (wave == 0) BSTAMP(1 + u);
    f32x4 g[9];
#pragma unroll
    for (int ti = 0; ti < 9; ++ti) {
      const uint32_t pa = ga + (uint32_t)(ti * G::R * G::GQ) * 16u;
      if constexpr (GRAD == 1) {
        g[ti] = lds_rd4(pa + 2u * 16u);
      } else {
        const int m = ti >> 1;
        if (ti & 1) {
          const f32x2 lo = lds_rd2(pa + (uint32_t)(3 - m) * 16u + 8u);
          const f32x2 hi = lds_rd2(pa + (uint32_t)(4 - m) * 16u);
          g[ti] = f32x4{lo.x, lo.y, hi.x, hi.y};
        } else {
          g[ti] = lds_rd4(pa + (uint32_t)(4 - m) * 16u);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G::CS; ++j) {
      f32x4 w[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) w[i] = lds_rd4(wa + (uint32_t)(j * G::CHS + i) * 16u);
      bwd_fma<GRAD>(acc[j], g, w);
    }
  }
  if (wave == 0) BSTAMP(10);
  // ---- stores: one 16-B store per channel (whole rows across the segments' lanes) ----
  const int Y = r0 + r;
  if (active && Y < hp) {
    float* gimg = (GRAD == 1 ? a.g1 : a.g2) + ((size_t)n * a.C + c0 + k * G::CS) * H * W +
                  (size_t)(2 * Y + p) * W + 4 * s;
#pragma unroll
    for (int j = 0; j < G::CS; ++j) {
      f32x4 v;
      // / C, the geometry's compile-time channel count (the launcher checks divisor == C):
      // an exact 2^-k multiply, or the reference's fp32 division (cu:196, 288) for C = 96 --
      // as in the forward strips, no runtime select between the stores
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = (G::CW & (G::CW - 1)) == 0 ? acc[j][e] * (1.f / G::CW) : acc[j][e] / (float)G::CW;
      st_out4(gimg + (size_t)j * H * W, v);
    }
  }
#ifdef PWC_BSTRIP_CENSUS
  BSTAMP(11);
  if (wave == 0 && lane < 14) {
    const unsigned long long v = *reinterpret_cast<const __attribute__((address_space(3)))
                                                       unsigned long long*>(
        (uintptr_t)(lds0 + G::LDS_BYTES + (uint32_t)lane * 8u));
    g_bs_census[(size_t)blockIdx.x * 16 + lane] = v;
  }
#endif
}

// logical block = (gradient, n, row parity, band, channel slice), slice fastest: the slices of
// a band read the same gO rows and neighbouring bands share feature rows; xcd_remap keeps
// neighbours on one XCD (one L2)
template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_bwd_strip(Args a) {
  const int per_grad = a.B * 2 * a.nb * a.ns;
  int t = xcd_remap(blockIdx.x, gridDim.x);
  const int grad = t / per_grad;
  t -= grad * per_grad;
  const int slice = t % a.ns;
  const int band = (t / a.ns) % a.nb;
  const int p = (t / (a.ns * a.nb)) & 1;
  const int n = t / (a.ns * a.nb * 2);
  if (grad == 0)
    body<G, 1>(a, n, p, band, slice);
  else
    body<G, 2>(a, n, p, band, slice);
}

template <class G>
static hipError_t launch(const Args& a0, hipStream_t stream) {
  Args a = a0;
  a.nb = ((a.H + 1) / 2 + G::R - 1) / G::R;
  a.ns = a.C / G::CW;
  const long long nblk = 2LL * a.B * 2 * a.nb * a.ns;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e =
        lds_limit(reinterpret_cast<const void*>(&corr_bwd_strip<G>), G::LDS_BYTES + CENSUS_EXTRA);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((corr_bwd_strip<G>), dim3((unsigned)nblk), dim3(G::THREADS),
                     G::LDS_BYTES + CENSUS_EXTRA,
                     stream, a);
  return hipGetLastError();
}

// config 5 l4 (C = 32, W = 112): all channels (gO staged once per gradient), 3-row bands, 4
// channels per lane
#ifndef PWC_BWD_GEO4  // (measurement builds may override)
#define PWC_BWD_GEO4 32, 3, 28, 4
#endif
using GeoB4 = Geo<PWC_BWD_GEO4>;
// config 5 l3 (C = 64, W = 56)
#ifndef PWC_BWD_GEO3
#define PWC_BWD_GEO3 64, 3, 14, 8
#endif
using GeoB3 = Geo<PWC_BWD_GEO3>;
// config 5 l2 (C = 96, W = 28): 2-row bands (192 workgroups), 8 channels per lane -- in the
// training step 12.0 -> 11.2 us against corr_bwd_rows (3-row bands 13.0, 1-row 14.5, 4
// channels per lane 11.4; profiles/r05z_bwd_strip_l2.txt)
#ifndef PWC_BWD_GEO2
#define PWC_BWD_GEO2 96, 2, 7, 8
#endif
using GeoB2 = Geo<PWC_BWD_GEO2>;

}  // namespace bstrip

// Which geometry serves this problem (0: none): fp32 (the caller checks model.py:24's
// configuration: k 1, s1 1, s2 2, pad == md in {8, 9}, raster), 16-B aligned buffers, the
// widths and channel counts of the geometries, 32-bit buffer offsets, a grid of >= 192
// workgroups.  Knob bwd_strip=0 leaves every problem to corr_bwd_rows.hip, bwd_strip=2 drops
// the grid-size condition.
static int bwd_strip_plan(const void* in1, const void* in2, const void* gout, const void* g1,
                          const void* g2, int B, int C, int H, int W) {
  if (debug_knob("bwd_strip", 1) == 0 || B <= 0 || H < 2) return 0;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)gout % 16 ||
      (uintptr_t)g1 % 16 || (uintptr_t)g2 % 16)
    return 0;
  if ((size_t)81 * H * W * 4 >= 0x7ffffff0ull || (size_t)C * H * W * 4 >= 0x7ffffff0ull) return 0;
  // every geometry stages all C channels in one workgroup (CW = C: the kernel divides by CW);
  // and the grid must fill the chip: its latency-bound workgroups (9 dependent steps each) lose
  // to corr_bwd_rows.hip below ~192 of them (profiles/r06c_bwd_strip_small_batch.txt: B = 1 / 2
  // at l2-l4, B = 4 at l2 / l3 -- 8.4-13.2 against 10.4-15.9 us; B = 4 at l4, 256 workgroups,
  // 17.7 against 18.4)
  // (knob bwd_strip = 2: any grid -- the small-batch edge-case tests of the kernel)
  const bool any_grid = debug_knob("bwd_strip", 1) == 2;
  auto fills = [&](int R) {
    return any_grid || 2LL * B * 2 * (((H + 1) / 2 + R - 1) / R) >= 192;
  };
  if (C == 32 && W == 4 * bstrip::GeoB4::NSEG && C == bstrip::GeoB4::CW && fills(bstrip::GeoB4::R))
    return 4;
  if (C == 64 && W == 4 * bstrip::GeoB3::NSEG && C == bstrip::GeoB3::CW && fills(bstrip::GeoB3::R))
    return 3;
  if (C == 96 && W == 4 * bstrip::GeoB2::NSEG && C == bstrip::GeoB2::CW &&
      fills(bstrip::GeoB2::R) && debug_knob("bwd_strip_l2", 1) != 0)
    return 2;
  return 0;
}

bool corr_bwd_strip_accepts(const void* in1, const void* in2, const void* gout, const void* g1,
                            const void* g2, int B, int C, int H, int W) {
  return bwd_strip_plan(in1, in2, gout, g1, g2, B, C, H, W) != 0;
}

hipError_t corr_backward_strip_f32(const void* in1, const void* in2, const void* gout, void* g1,
                                   void* g2, int B, int C, int H, int W, float divisor,
                                   hipStream_t stream) {
  const int plan = bwd_strip_plan(in1, in2, gout, g1, g2, B, C, H, W);
  // the kernels divide by their compile-time C: Correlation's divisor k^2 C with k = 1 (any other
  // divisor goes on to corr_bwd_rows.hip)
  if (plan == 0 || divisor != (float)C) return hipErrorNotSupported;
  bstrip::Args a{(const float*)in1, (const float*)in2, (const float*)gout, (float*)g1, (float*)g2,
                 C, H, W, 0, 0, B};
  switch (plan) {
    case 4:
      return bstrip::launch<bstrip::GeoB4>(a, stream);
    case 3:
      return bstrip::launch<bstrip::GeoB3>(a, stream);
    case 2:
      return bstrip::launch<bstrip::GeoB2>(a, stream);
    default:
      return hipErrorNotSupported;
  }
}

#ifdef PWC_BSTRIP_CENSUS
extern "C" __attribute__((visibility("default"))) int pwc_debug_bstrip_census(void* dst, int n) {
  if (dst == nullptr) {
    static unsigned long long zeros[8192 * 16];
    return hipMemcpyToSymbol(HIP_SYMBOL(bstrip::g_bs_census), zeros, sizeof(zeros)) == hipSuccess;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(bstrip::g_bs_census),
                             sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}
#endif

}  // namespace pwc
