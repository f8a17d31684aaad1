// corr_cols.hip — correlation forward for the l4-sized grids (the paper's "level 2"):
// model.py:24's Correlation(9, 1, 9, 1, 2) in fp32, i.e. correlation_cuda_kernel.cu:34-106 with
// k = 1, s1 = 1, pad = md = 9, s2 = 2:
//   out[n, (tj+4)*9 + (ti+4), y, x] = sum_c f1[n,c,y,x] * f2[n,c,y+2tj,x+2ti] / C
// with zeros outside the image (the reference's zero-padded NHWC scratch, cu:10-32).
//
// Why this shape.  At B = 8 the l4 volume is 256 row bands of 3 parity rows, one
// per CU, and a band's 81 output planes (109 KB) can only be written once all C channels are
// summed.  One pass per band therefore serialises "stream the inputs + compute" and "drain the
// output".  Here a workgroup walks its band in column ITEMS (two 56-px halves at W = 112): item
// k's outputs leave the registers as soon as its last channel is summed -- plain vector stores,
// no LDS park -- and their drain to HBM overlaps item k+1's channel loop.
//
//   * loader waves (2): per stage of CC channels, buffer_load_dwordx4 ... lds (LDS-DMA) of the
//     item's f2 rows (R + 8 parity rows, 8 px of halo each side) and f1 rows into a ring of NS
//     stages; the buffer unit's range check yields the reference's zero border.  Each loader
//     keeps its share of up to AHEAD stages in flight (<= 63 DMAs: the 6-bit vmcnt).
//   * compute lanes: one (r, tj) unit per 16-lane ds_read_b128 group (MI355X_MICROARCH.md §LDS),
//     lane p of the group = 4-pixel segment p: per channel 5 window quads of f2 row r + tj and 1
//     f1 quad, 18 v_pk_fma_f32 into 4 px x 9 ti accumulators.  The 16 lanes of a group read 16
//     consecutive quads (conflict-free); idle positions repeat a neighbour's address (broadcast).
//     Reads run two channels ahead of the FMAs (three register buffers).
//   * one s_barrier per stage: it publishes the stage's landing (the loaders wait on vmcnt
//     first) and frees the slot read two stages earlier.
//   * output: per lane 9 stores of 16 B; a group writes 14 consecutive quads of one plane row.
#include <hip/hip_ext.h>

#include <cmath>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);

namespace cols {

#ifdef PWC_COLS_CENSUS  // tools/colbench.hip only: per-workgroup phase timestamps (100 MHz)
__device__ unsigned long long* g_census;
#define CENSUS(slot)                                                                   \
  do {                                                                                 \
    if ((threadIdx.x & 63) == 0)                                                       \
      g_census[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
// measurement ablations (colbench): 1 no stores, 2 no DMA, 4 no LDS reads, 8 no FMAs; read
// once per wave into `abl` (a global load inside the loader's loop would stall it)
__device__ int g_abl;
#define ABL_LOAD() const int abl = __builtin_amdgcn_readfirstlane(g_abl)
#define ABL(bit) ((abl & (bit)) != 0)
#else
#define CENSUS(slot) \
  do {               \
  } while (0)
#define ABL_LOAD() constexpr int abl = 0
#define ABL(bit) false
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int round64(int v) { return (v + 63) / 64 * 64; }

// R: parity rows per workgroup; TWQ: item width in quads (4 px); CC: channels per ring stage;
// NS: ring stages; NLD: loader waves.
template <int R_, int TWQ_, int CC_, int NS_, int NLD_, int AH_ = 8>
struct Geo {
  static constexpr int R = R_, TWQ = TWQ_, CC = CC_, NS = NS_, NLD = NLD_;
  static constexpr int F2R = R + 8;                    // f2 parity rows (tj = -4..4)
  static constexpr int Q2 = TWQ + 4;                   // f2 row quads: 8 px of halo each side
  static constexpr int Q1 = TWQ;                       // f1 row quads
  static constexpr int CH2 = F2R * Q2, CH1 = R * Q1;   // quads per channel
  static constexpr int F2PART = round64(CC * CH2), F1PART = round64(CC * CH1);
  static constexpr int STAGEQ = F2PART + F1PART;       // quads per ring stage
  static constexpr int I2 = F2PART / 64, I1 = F1PART / 64, IPS = I2 + I1;  // DMAs per stage
  static constexpr int IPL = (IPS + NLD - 1) / NLD;    // ... per loader wave
  static constexpr int NUNIT = 9 * R;                  // (r, tj) units, one per 16-lane group
  static constexpr int NCW = (NUNIT + 3) / 4;          // compute waves
  static constexpr int THREADS = 64 * (NCW + NLD);
  static constexpr int NK = NS * CC;                   // channels per unrolled round
  static constexpr int LDS_BYTES = NS * STAGEQ * 16;
  static constexpr int NBASE = (LDS_BYTES + 32767) / 32768;  // 32 KiB address windows
  // stages one loader keeps in flight: its DMAs <= 63 (vmcnt), and a slot is reissued only
  // after it was released (stage k-2's slot frees at barrier B_k)
  static constexpr int AHEAD0 = 63 / IPL < AH_ ? 63 / IPL : AH_;
  static constexpr int AHEAD = AHEAD0 < NS - 2 ? AHEAD0 : NS - 2;
  static_assert(TWQ <= 16, "a unit's segments fit one 16-lane group");
  static_assert(THREADS <= 1024 && LDS_BYTES <= 160 * 1024, "workgroup resources");
  static_assert(AHEAD >= 2 && NS >= 4 && NK % 2 == 0, "ring depth");
  static_assert(IPS % NLD == 0, "every loader wave owns IPL DMAs of each stage");
};

// 16-lane groups of ds_read_b128 (MI355X_MICROARCH.md, LDS table): hw lane -> (group, pos).
__device__ __forceinline__ void lane_group(int lane, int& g, int& p) {
  const int l = lane & 31, hi = lane >> 5;
  int gg, pp;
  if (l < 4) { gg = 0; pp = l; }
  else if (l < 12) { gg = 1; pp = l - 4; }
  else if (l < 16) { gg = 0; pp = l - 8; }
  else if (l < 20) { gg = 1; pp = l - 8; }
  else if (l < 28) { gg = 0; pp = l - 12; }
  else { gg = 1; pp = l - 16; }
  g = gg + 2 * hi;
  p = pp;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Buffer resource of one stage: the image plus the stage's first channel (`cbytes`), records to
// the image's end -- the range check then returns zeros for out-of-image offsets (0x80000000).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stage_rsrc(const void* img, uint32_t cbytes,
                                                             uint32_t img_bytes) {
  const int nrec = cbytes < img_bytes ? (int)(img_bytes - cbytes) : 0;
  const uint64_t b = (uint64_t)(uintptr_t)img + (uint64_t)cbytes;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo),
                                           (short)0, __builtin_amdgcn_readfirstlane(nrec),
                                           0x00020000);
}

// One LDS-DMA instruction: 16 B from `rs` + this lane's `rel` into 1 KiB of LDS at `lds_dst`.
__device__ __forceinline__ void dma1(__amdgpu_buffer_rsrc_t rs, uint32_t rel, uint32_t lds_dst) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)(uintptr_t)lds_dst, 16, rel, 0, 0, 0);
#endif
}

// s_waitcnt vmcnt(n * M), n in [0, 7] (immediates; larger n clamps to 63)
template <int M>
__device__ __forceinline__ void wait_vm_stages(int n) {
#define PWC_W(k)                                                                     \
  case k:                                                                            \
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k * M < 63 ? k * M : 63) : "memory"); \
    break;
  switch (n) {
    PWC_W(0) PWC_W(1) PWC_W(2) PWC_W(3) PWC_W(4) PWC_W(5) PWC_W(6)
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(7 * M < 63 ? 7 * M : 63) : "memory");
  }
#undef PWC_W
}

// Reads of one channel: 5 window quads at a + O .. a + O + 64 and the f1 quad at b + O1.
struct Ops {
  f32x4 w[5];
  f32x4 f;
};

template <int O, int O1>
__device__ __forceinline__ void read_a(uint32_t a, Ops& x) {
  static_assert(O >= 0 && O + 64 < 65536 && O1 >= 0 && O1 < 65536, "ds offset field");
  asm volatile(
      "ds_read_b128 %0, %2 offset:%3\n\t"
      "ds_read_b128 %1, %2 offset:%4"
      : "=&v"(x.w[0]), "=&v"(x.w[1])
      : "v"(a), "n"(O), "n"(O + 16)
      : "memory");
}
template <int O, int O1>
__device__ __forceinline__ void read_b(uint32_t a, Ops& x) {
  asm volatile(
      "ds_read_b128 %0, %2 offset:%3\n\t"
      "ds_read_b128 %1, %2 offset:%4"
      : "=&v"(x.w[2]), "=&v"(x.w[3])
      : "v"(a), "n"(O + 32), "n"(O + 48)
      : "memory");
}
template <int O, int O1>
__device__ __forceinline__ void read_c(uint32_t a, uint32_t b, Ops& x) {
  asm volatile(
      "ds_read_b128 %0, %2 offset:%4\n\t"
      "ds_read_b128 %1, %3 offset:%5"
      : "=&v"(x.w[4]), "=&v"(x.f)
      : "v"(a), "v"(b), "n"(O + 64), "n"(O1)
      : "memory");
}

// Wait until at most N LDS reads are outstanding; tie the channel's registers through the asm
// so the compiler neither reads them earlier nor reuses them meanwhile.
template <int N>
__device__ __forceinline__ void lgk_wait(Ops& x) {
  asm volatile("s_waitcnt lgkmcnt(%6)"
               : "+v"(x.w[0]), "+v"(x.w[1]), "+v"(x.w[2]), "+v"(x.w[3]), "+v"(x.w[4]),
                 "+v"(x.f)
               : "n"(N));
}

// acc[t][p] += f1[p] * f2[x + p + 2 (t - 4)], t = 0..8, p = 0..3: window element j = p + 2t
// (window quad 0 starts 8 px left of the segment); pixel pairs (p, p+1), p even, meet aligned
// element pairs, so each (t, pair) is one v_pk_fma_f32.  T0..T1: a chunk of displacements.
template <int T0, int T1>
__device__ __forceinline__ void fma_t(float (&acc)[9][4], const Ops& x) {
#pragma unroll
  for (int t = T0; t < T1; ++t) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * h + 2 * t;
      const f32x4 q = x.w[j >> 2];
      const f32x2 w2 = (j & 2) ? f32x2{q.z, q.w} : f32x2{q.x, q.y};
      const f32x2 a2 = h ? f32x2{x.f.z, x.f.w} : f32x2{x.f.x, x.f.y};
      f32x2 c2 = {acc[t][2 * h], acc[t][2 * h + 1]};
      c2 = __builtin_elementwise_fma(a2, w2, c2);
      acc[t][2 * h] = c2.x;
      acc[t][2 * h + 1] = c2.y;
    }
  }
}

// LDS byte offsets of channel K's f2 window / f1 quads inside an unrolled round of NS stages
// (the lane's own row / segment part lives in its base registers, one per 32 KiB window)
template <class G, int K>
struct Off {
  static constexpr int S = K / G::CC, J = K % G::CC;
  static constexpr int W2 = (S * G::STAGEQ + J * G::CH2) * 16;
  static constexpr int W1 = (S * G::STAGEQ + G::F2PART + J * G::CH1) * 16;
  static constexpr int WIN2 = W2 / 32768, IMM2 = W2 % 32768;
  static constexpr int WIN1 = W1 / 32768, IMM1 = W1 % 32768;
};

template <class G, int K>
__device__ __forceinline__ void read_ch(const uint32_t (&wa)[G::NBASE],
                                        const uint32_t (&fa)[G::NBASE], Ops& x, int part) {
  using O = Off<G, K>;
  if (part == 0) read_a<O::IMM2, O::IMM1>(wa[O::WIN2], x);
  if (part == 1) read_b<O::IMM2, O::IMM1>(wa[O::WIN2], x);
  if (part == 2) read_c<O::IMM2, O::IMM1>(wa[O::WIN2], fa[O::WIN1], x);
}

// Channel K of a round: (barrier when K+2 opens a stage), wait for K's reads, then K+2's reads
// interleaved with K's FMAs.  Buffers rotate K % 3, static because every round restarts its
// pipeline at K = 0 (a round is fully unrolled so every LDS offset is an immediate; the async
// read registers never cross a loop back-edge, where the compiler might copy or spill them
// before the data lands).
template <class G, int K, int M = 0>
__device__ __forceinline__ void round_step(const uint32_t (&wa)[G::NBASE],
                                           const uint32_t (&fa)[G::NBASE], float (&acc)[9][4],
                                           Ops (&ops)[3]) {
  if constexpr (K < G::NK) {
    constexpr int N2 = K + 2;
    constexpr bool PRE = N2 < G::NK && !(M & 1);  // M (measurement): 1 no reads, 2 no FMAs
    constexpr bool FM = !(M & 2);
    if constexpr (N2 < G::NK && N2 % G::CC == 0) __builtin_amdgcn_s_barrier();
    Ops& cur = ops[K % 3];
    Ops& nxt = ops[N2 % 3];
    if constexpr (K + 1 < G::NK)
      lgk_wait<6>(cur);  // channel K+1's six reads may still be in flight
    else
      lgk_wait<0>(cur);
    if constexpr (PRE) read_ch<G, N2>(wa, fa, nxt, 0);
    if constexpr (FM) fma_t<0, 3>(acc, cur);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRE) read_ch<G, N2>(wa, fa, nxt, 1);
    if constexpr (FM) fma_t<3, 6>(acc, cur);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRE) read_ch<G, N2>(wa, fa, nxt, 2);
    if constexpr (FM) fma_t<6, 9>(acc, cur);
    __builtin_amdgcn_sched_barrier(0);
    round_step<G, K + 1, M>(wa, fa, acc, ops);
  }
}

// Loader wave LD: DMA instructions [LD * IPL, (LD + 1) * IPL) of every stage (statically
// indexed, branch-free).  Per instruction and lane: the source row's element offset (or -1 when
// the row is outside the image) and the column relative to the item's first pixel; per item the
// column check picks the offset or the out-of-range value (the buffer unit's zero fill).
template <class G, int LD>
__device__ __forceinline__ void loader(const float* img1, const float* img2, uint32_t lds0, int lane,
                                       int Y0, int py, int H, int W, int nst, int total,
                                       uint32_t plane_b, uint32_t img_bytes, int abl) {
  constexpr uint32_t kOOB = 0x80000000u;
  if (LD == 0) CENSUS(1);  // loader entry
  int rowoff[G::IPL], xrel[G::IPL];
#pragma unroll
  for (int k = 0; k < G::IPL; ++k) {
    const int i = LD * G::IPL + k;
    const bool f2 = i < G::I2;
    const int g = (f2 ? 64 * i : 64 * (i - G::I2)) + lane;
    const int n_here = f2 ? G::CC * G::CH2 : G::CC * G::CH1;
    const int chq = f2 ? G::CH2 : G::CH1, rq = f2 ? G::Q2 : G::Q1;
    const int j = g / chq, q = g - j * chq;
    const int rho = q / rq, xq = q - rho * rq;
    const int prow = f2 ? Y0 - 4 + rho : Y0 + rho;
    const int srow = 2 * prow + py;
    const bool ok = i < G::IPS && g < n_here && prow >= 0 && srow < H;
    rowoff[k] = ok ? (j * H + srow) * W : -1;
    xrel[k] = f2 ? 4 * xq - 8 : 4 * xq;
  }
  if (LD == 0) CENSUS(2);  // loader offsets ready
  uint32_t rel[G::IPL];
  int rel_item = -1;
  auto issue = [&](int gs) {
    const int item = gs / nst, st = gs - item * nst;
    if (item != rel_item) {
      const int X0 = item * G::TWQ * 4;
#pragma unroll
      for (int k = 0; k < G::IPL; ++k) {
        const int x = X0 + xrel[k];
        rel[k] = (rowoff[k] >= 0 && x >= 0 && x < W) ? (uint32_t)(rowoff[k] + x) * 4u : kOOB;
      }
      rel_item = item;
    }
    if (ABL(2)) return;
    const uint32_t cb = (uint32_t)(st * G::CC) * plane_b;
    const uint32_t slot = lds0 + (uint32_t)((gs % G::NS) * G::STAGEQ * 16);
    const __amdgpu_buffer_rsrc_t rs2 = stage_rsrc(img2, cb, img_bytes);
    const __amdgpu_buffer_rsrc_t rs1 = stage_rsrc(img1, cb, img_bytes);
#pragma unroll
    for (int k = 0; k < G::IPL; ++k) {
      const int i = LD * G::IPL + k;
      if (i < G::IPS)
        dma1(i < G::I2 ? rs2 : rs1, rel[k],
             slot + (uint32_t)((i < G::I2 ? 64 * i : G::F2PART + 64 * (i - G::I2)) * 16));
    }
  };
  int issued = -1;
  while (issued + 1 < total && issued + 1 < G::AHEAD) issue(++issued);
  if (LD == 0) CENSUS(3);  // prologue DMAs issued
  for (int k = 0; k < total; ++k) {
    wait_vm_stages<G::IPL>(issued - k);  // stage k landed
    __builtin_amdgcn_s_barrier();        // B_k
    // B_k freed stage k-2's slot; keep up to AHEAD stages in flight beyond stage k
    while (issued + 1 < total && issued + 1 <= k + G::AHEAD) issue(++issued);
  }
  if (LD == 0) CENSUS(9);  // last stage landed
}

template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_fwd_cols(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    int C, int H, int W, int nband, int nitem, float divisor, float inv_divisor, OutEpi epi) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // logical block = (n, row parity, band), band fastest: the bands of one image parity share
  // halo rows, and xcd_remap keeps neighbours on one XCD (one L2)
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int band = t % nband;
  const int py = (t / nband) & 1;
  const int n = t / (2 * nband);
  const int Y0 = band * G::R;  // first parity row of the band
  const int nst = C / G::CC;   // stages per item
  const int total = nitem * nst;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t plane_b = plane * 4u;
  const uint32_t img_bytes = (uint32_t)C * plane_b;  // < 2^31 (launcher)
  const float* img1 = in1 + (size_t)n * C * plane;
  const float* img2 = in2 + (size_t)n * C * plane;
  const uint32_t lds0 = lds_addr(lds);
  ABL_LOAD();
  if (wave == 0) CENSUS(0);

  if (wave >= G::NCW) {
    // ---------------- loader waves ----------------
    if (wave == G::NCW)
      loader<G, 0>(img1, img2, lds0, lane, Y0, py, H, W, nst, total, plane_b, img_bytes, abl);
    else
      loader<G, 1>(img1, img2, lds0, lane, Y0, py, H, W, nst, total, plane_b, img_bytes, abl);
    return;
  }

  // ---------------- compute waves ----------------
  int g, p;
  lane_group(lane, g, p);
  const int u = wave * 4 + g;
  const int uu = u < G::NUNIT ? u : G::NUNIT - 1;
  const int r = uu / 9, tj = uu - 9 * r;
  const int seg = p < G::TWQ ? p : G::TWQ - 1;  // idle positions repeat segment TWQ-1
  const bool active = u < G::NUNIT && p < G::TWQ;
  uint32_t wa[G::NBASE], fa[G::NBASE];
#pragma unroll
  for (int k = 0; k < G::NBASE; ++k) {
    wa[k] = lds0 + (uint32_t)(k * 32768 + ((r + tj) * G::Q2 + seg) * 16);
    fa[k] = lds0 + (uint32_t)(k * 32768 + (r * G::Q1 + seg) * 16);
  }
  const int y = 2 * (Y0 + r) + py;
  const bool store = active && y < H;
  float* oimg = out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * 81 * plane);
  const int nround = C / G::NK;
  if (wave == 0) CENSUS(10);  // compute setup done

  for (int item = 0; item < nitem; ++item) {
    float acc[9][4];
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[a][k] = 0.f;
    for (int rd = 0; rd < nround; ++rd) {
      Ops ops[3];
      __builtin_amdgcn_s_barrier();  // stage 0 of the round landed
      if (wave == 0 && item == 0 && rd == 0) CENSUS(4);  // past B_0
#pragma unroll
      for (int part = 0; part < 3; ++part) read_ch<G, 0>(wa, fa, ops[0], part);
#pragma unroll
      for (int part = 0; part < 3; ++part) read_ch<G, 1>(wa, fa, ops[1], part);
#ifdef PWC_COLS_M  // measurement builds: 1 no LDS reads, 2 no FMAs, 3 neither
      round_step<G, 0, PWC_COLS_M>(wa, fa, acc, ops);
#else
      round_step<G, 0>(wa, fa, acc, ops);
#endif
    }
    if (wave == 0) CENSUS(item == 0 ? 5 : 7);  // item loop done
    // ---- this item's 81 planes, straight from registers (cu:100: / C) ----
    if (store && !ABL(1)) {
      if (inv_divisor != 0.f) {
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[a][k] *= inv_divisor;
      } else {
        // q = x * (1/d) plus one FMA residual correction (a non-power-of-2 C)
        const float rinv = 1.f / divisor;
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float q = acc[a][k] * rinv;
            acc[a][k] = fmaf(fmaf(-q, divisor, acc[a][k]), rinv, q);
          }
      }
      if (epi.slope != 1.f) {
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[a][k] = epi_act(acc[a][k], epi.slope);
      }
      // raster channel order (cu:98): plane (tj + 4) * 9 + ti + 4, ti = a - 4
      float* orow = oimg + ((size_t)(tj * 9) * H + y) * W + item * G::TWQ * 4 + 4 * seg;
#pragma unroll
      for (int a = 0; a < 9; ++a)
        st_out4(orow + (size_t)a * plane, st_f32x4{acc[a][0], acc[a][1], acc[a][2], acc[a][3]});
    }
    if (wave == 0 && item == 0) CENSUS(6);  // item 0's stores issued
  }
  if (wave == 0) CENSUS(8);
}

template <class G>
static hipError_t launch(const float* in1, const float* in2, float* out, int B, int C, int H,
                         int W, int nitem, float divisor, hipStream_t stream) {
  const int HP = (H + 1) / 2;  // parity rows; parity 0 has the extra row
  const int nband = (HP + G::R - 1) / G::R;
  const long long nblk = (long long)B * 2 * nband;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&corr_fwd_cols<G>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             G::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;  // exact when a power of 2
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);  // bench.py's live timing hook (one-shot)
  hipExtLaunchKernelGGL((corr_fwd_cols<G>), dim3((unsigned)nblk), dim3(G::THREADS),
                        G::LDS_BYTES, stream, ev0, ev1, 0, in1, in2, out, C, H, W, nband,
                        nitem, divisor, inv, current_epi());
  return hipGetLastError();
}

}  // namespace cols

// hipErrorNotSupported: a shape this kernel does not serve (the caller tries the next path).
// Serves fp32, k = 1, s1 = 1, pad = md with dr = 4 and s2 = 2 (model.py:24), rows split into
// items of 56 px (W = 112: two items), C a multiple of 32, 16-B aligned buffers, grids of at
// least ~one workgroup per CU.
hipError_t corr_forward_cols(const void* in1, const void* in2, void* out, int B, int C, int H,
                             int W, int layout, float divisor, hipStream_t stream) {
  using namespace cols;
  if (layout != kRaster) return hipErrorNotSupported;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16) return hipErrorNotSupported;
  if ((size_t)C * H * W * 4 >= 0x7ffffff0ull || C % 32) return hipErrorNotSupported;
  const long long nblk = (long long)B * 2 * ((((H + 1) / 2) + 2) / 3);
  if (nblk < 192) return hipErrorNotSupported;
  if (W % 56 == 0 && W / 56 <= 4) {
    using G = Geo<3, 14, 4, 8, 1>;
    return launch<G>((const float*)in1, (const float*)in2, (float*)out, B, C, H, W, W / 56,
                     divisor, stream);
  }
  return hipErrorNotSupported;
}

}  // namespace pwc
