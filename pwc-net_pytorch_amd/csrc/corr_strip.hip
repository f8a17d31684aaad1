// corr_strip.hip — correlation forward for the strip-sized fp32 grids of model.py:24's
// Correlation(9, 1, 9, 1, 2): BASELINE config 2's l4 (32 x 96 x 112), l3 (64 x 48 x 56) and l2
// (96 x 24 x 28) at B = 8.  Output rows are produced in STEPS so that their stores drain while
// the next rows compute.
//
// Semantics (correlation_cuda_kernel.cu:34-106 with k = 1, s1 = 1, pad = md = 9, s2 = 2):
//   out[n, (tj+4)*9 + (ti+4), y, x] = sum_c f1[n,c,y,x] * f2[n,c,y+2tj,x+2ti] / C
// with zeros outside the image (the reference's zero-padded scratch).
//
// Why this shape.  corr_stream.hip streams the channels of a 3-row band through
// an LDS ring; every output needs the last channel, so the l4 output only starts to drain after
// the loop.  Here a workgroup owns R parity rows of one image parity over a column strip (or the
// whole row), and ALL channels of the R + 8 f2 parity rows it meets stay resident in LDS.  The
// rows are produced NQD at a time: step s computes its rows, reduces, and issues the stores
// straight from the registers, and step s+1 starts at once (its rows were staged during step s).
// Step 0's f2 rows arrive channel pair by channel pair (the loader's first DMAs bring the first
// channels of every step-0 row), so step 0 computes behind the loads.
//
// Geometries (struct Geo): GeoL4 = 56-px strips of 6 rows (round 4); GeoF = whole 112-px rows
// (whole 448-B output rows: no 128-B line is shared by two workgroups), 6 rows in 3 steps, the
// 81 (tj, segment) tasks of a row split into two workgroups by displacement row; GeoF3 (C = 64,
// l3) = 3 rows in one step; GeoF2 (C = 96, l2) = 1 row, channels split in quarters.
//
//   * loader wave: each staged f2 row = whole 1-KiB LDS-DMAs (buffer_load_dwordx4 ... lds; the
//     buffer range check gives the zero border), <= 63 in flight, one s_barrier per landed group.
//   * compute waves: NQD groups of WPP waves (group q takes row NQD s + q); lane = (tj, 4-px
//     segment, channel part): per channel 5 ds_read_b128 of the f2 window and 18 v_pk_fma_f32
//     on f1 values the lane loaded itself (the next step's f1 prefetched into the register of
//     the channel just consumed).  Channel halves sit in lanes l and l + 32 and are summed by
//     v_permlane32_swap; quarters additionally by v_permlane16_swap.
//   * LDS row stride = NSEG (mod 16) quads: every ds_read_b128 lane group hits 16 distinct 16-B
//     bank slots (conflict-free; PMC SQ_LDS_BANK_CONFLICT = 0).
//   * stores: 16 B per lane (4 px of one displacement plane), consecutive segments in
//     consecutive lanes, nontemporal.
//   * blocks are remapped XCD-aware so the workgroups of one image parity share an L2.
#include <hip/hip_ext.h>

#include <cmath>
#include <type_traits>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace strip {

#ifdef PWC_STRIP_CENSUS  // tools/strip_bench.hip only: per-workgroup phase stamps (100 MHz)
// Stamps are kept in scalar registers and written once at the end of the wave: a global store
// inside the loop would enter the compute waves' vmcnt accounting and distort the timing.
// Layout per workgroup (64 slots): compute quad A (wave 0) 0..31, quad B (wave WPP) 32..63; in
// each, slot 0 = entry, 1 = first data, 2 + 3 s + {0,1,2} = step s loop done / reduced / stores
// issued; the loader's stamps are slots 61..63 of quad B's range (group 0, step-0 window, all).
__device__ unsigned long long* g_census;
#define STAMP(slot) (cen_t[(slot)] = __builtin_amdgcn_s_memrealtime())
// a runtime slot (the step loop): the stamp goes to LDS behind the window (a runtime index
// into the stamp registers would put them in scratch; a global store would join the vmcnt
// accounting).  Placed only where the wave has no LDS read in flight (after a step's loop).
#define CSTAMP(slot)                                                                        \
  do {                                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                         \
    const uint32_t a_ = lds0 + G::LDS_BYTES +                                               \
                        (uint32_t)(((wave == 0 ? 0 : wave == G::WPP ? 32 : 64) + (slot)) * 8); \
    asm volatile("ds_write_b64 %0, %1" ::"v"(a_), "v"(t_) : "memory");                     \
  } while (0)
#define CENSUS_DECL unsigned long long cen_t[32] = {}
#define CENSUS_FLUSH(lo, hi, base)                                                     \
  do {                                                                                 \
    if ((threadIdx.x & 63) == 0 && g_census != nullptr)                                \
      for (int k_ = (lo); k_ < (hi); ++k_)                                             \
        if (cen_t[k_]) g_census[blockIdx.x * 64 + (base) + k_] = cen_t[k_];            \
  } while (0)
#else
#define STAMP(slot) \
  do {              \
  } while (0)
#define CSTAMP(slot) \
  do {               \
  } while (0)
#define CENSUS_DECL \
  do {              \
  } while (0)
#define CENSUS_FLUSH(lo, hi, base) \
  do {                       \
  } while (0)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef PWC_STRIP_ABL
#define PWC_STRIP_ABL 0
#endif
#ifndef PWC_STRIP_STORE_AUX  // output store cache policy (measurement builds may override)
#define PWC_STRIP_STORE_AUX 2  // nontemporal
#endif
#ifndef PWC_STRIP_LAST_AUX  // the last step's stores
#define PWC_STRIP_LAST_AUX PWC_STRIP_STORE_AUX
#endif

// C channels, R output parity rows per workgroup, TW-px column strips; the 9 x NSEG (tj, 4-px
// segment) tasks of an output row split over TS workgroups (each stages only the f2 rows its tj
// meet); NQD output rows per step (two compute waves each); LA channels of LDS read-ahead.
// FULL: the strip is the whole image row (TW == W); a channel row then stages only its 2-quad
// left halo (zeros) before its data, and its right halo is the next channel row's left halo,
// so a row of all channels is 2 quads per channel shorter (+ 2 zero quads after the last); a
// channel row may carry extra zero quads on the right so that a staged row is whole DMAs.
// NCS: the channels of a task split over NCS lanes (2: halves in lanes l, l + 32; 4: quarters
// in the four 16-lane rows), summed by permlane swaps before the stores.
template <int C_, int R_, int TW_, int TS_ = 1, int NQD_ = 2, int LA_ = 1, bool FULL_ = false,
          int NCS_ = 2>
struct Geo {
  static constexpr int C = C_, R = R_, TW = TW_, TS = TS_, NQD = NQD_, LA = LA_, NCS = NCS_;
  static constexpr bool FULL = FULL_;
  static constexpr int CH = C / NCS;        // channels per lane
  static constexpr int S = 64 / NCS;        // task slots per wave
  static constexpr int NSEG = TW / 4;       // 4-px segments per strip row
  static constexpr int qr_full() {
    int q = TW / 4 + 2;
    while ((C * q) % 64) ++q;
    return q;
  }
  // quads per staged channel row: 8-px halo each side (shared between channel rows if FULL)
  static constexpr int QR = FULL ? qr_full() : (TW + 16) / 4;
  static constexpr int ROWQ = C * QR;       // quads per staged f2 row (all channels), DMA'd
  static constexpr int IPR = ROWQ / 64;     // LDS-DMAs per f2 row
  static constexpr int ZQ = FULL ? 2 : 0;   // zero quads after the DMA'd row (the last right halo)
  // row stride in quads, = NSEG (mod 16): a lane's quad index is then its task index
  // (tj NSEG + segment) + a constant, mod 16, so every ds_read_b128 lane group of 16
  // consecutive-task lanes hits 16 distinct 16-B bank slots (conflict-free)
  static constexpr int SIGMA = ROWQ + ZQ + ((NSEG % 16 - (ROWQ + ZQ) % 16) + 16) % 16;
  static constexpr int NTASK_ALL = 9 * NSEG;  // (tj, segment) tasks per output row
  static constexpr int NTASK = NTASK_ALL / TS;  // per workgroup of a task group
  static constexpr int tj_lo(int g) { return g * NTASK / NSEG; }
  static constexpr int tj_hi(int g) { return ((g + 1) * NTASK - 1) / NSEG; }
  static constexpr int tj_span() {
    int m = 0;
    for (int g = 0; g < TS; ++g) m = tj_hi(g) - tj_lo(g) + 1 > m ? tj_hi(g) - tj_lo(g) + 1 : m;
    return m;
  }
  static constexpr int TJS = tj_span();     // displacement rows a workgroup meets
  static constexpr int NROW = R + TJS - 1;  // f2 parity rows of the strip
  static constexpr int NSTEP = R / NQD;
  static constexpr int WIN = NQD + TJS - 1;  // f2 rows of step 0
  static constexpr int WPP = (NTASK + S - 1) / S;  // waves per output row (S task slots each)
  static constexpr int NWC = WPP * NQD;     // compute waves
  static constexpr int THREADS = 64 * (NWC + 1);
  static constexpr int LDS_BYTES = NROW * SIGMA * 16;
#ifdef PWC_STRIP_CENSUS
  static constexpr int LDS_ALLOC = LDS_BYTES + 96 * 8;  // + the step stamps (census build)
#else
  static constexpr int LDS_ALLOC = LDS_BYTES;
#endif
  static constexpr int NDMA = NROW * IPR;
  static constexpr int NBAR = IPR + NSTEP - 1;  // barriers every wave executes
  static_assert((NCS == 2 || NCS == 4) && C % NCS == 0 && TW % 4 == 0 && R % NQD == 0,
                "geometry");
  static_assert(NTASK_ALL % TS == 0, "task groups");
  static_assert(ROWQ % 64 == 0, "a staged row is whole DMAs");
  static_assert(LDS_ALLOC <= 160 * 1024 && THREADS <= 1024, "workgroup resources");
  static_assert(LA >= 1 && LA <= 2 && CH > LA, "read-ahead");
  // every read offset inside a step is an instruction immediate (16-bit); the step's row base
  // is in the address register
  static_assert(((C - 1) * QR + 4) * 16 < 65536, "ds offsets");
};

// Loader DMA d -> (f2 row m, DMA i of the row): step 0's rows group-major (group i of all
// rows before group i + 1), then the later rows whole.
template <class G>
constexpr int dma_row(int d) {
  return d < G::IPR * G::WIN ? d % G::WIN : G::WIN + (d - G::IPR * G::WIN) / G::IPR;
}
template <class G>
constexpr int dma_idx(int d) {
  return d < G::IPR * G::WIN ? d / G::WIN : (d - G::IPR * G::WIN) % G::IPR;
}
// DMAs that have landed before barrier j: group j of step 0's rows (j < IPR), then every row
// of step s = j - IPR + 1.
template <class G>
constexpr int dma_need(int j) {
  return j < G::IPR ? (j + 1) * G::WIN : G::IPR * (G::WIN + G::NQD * (j - G::IPR + 1));
}
// DMAs issued before barrier j's wait: never more than 63 in flight (the 6-bit vmcnt), counting
// every DMA not yet known to have landed (those before barrier j-1's wait are)
template <class G>
constexpr int dma_target(int j) {
  return (j > 0 ? dma_need<G>(j - 1) : 0) + 63 < G::NDMA ? (j > 0 ? dma_need<G>(j - 1) : 0) + 63
                                                         : G::NDMA;
}
// DMA group that completes channel pair k (LDS channel rows 2k, 2k+1) including what its
// reads touch: with FULL rows, channel row 2k+1's right halo is the next channel row's 2-quad
// left pad, which can open the next DMA group (the last pair's is the ZQ quads, written at
// kernel start)
template <class G>
constexpr int pair_group(int k) {
  const int g = (G::NCS * (k + 1) * G::QR + (G::FULL ? 2 : 0) - 1) / 64;
  return g < G::IPR - 1 ? g : G::IPR - 1;
}

// Step 0's barrier count must match the loader's: a compute wave takes one barrier at the step's
// start (group 0) and one more each time pair_group rises, the loader one per DMA group.  That
// holds iff pair_group starts at 0, rises by at most 1 per channel pair (NCS * QR + 2 <= 64:
// a pair never spans two whole DMA groups) and ends at the last group.
template <class G>
constexpr bool pair_groups_match_loader() {
  if (pair_group<G>(0) != 0 || pair_group<G>(G::CH - 1) != G::IPR - 1) return false;
  for (int k = 1; k < G::CH; ++k)
    if (pair_group<G>(k) - pair_group<G>(k - 1) > 1) return false;
  return true;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One row of the loader: the buffer resource starts at the row (zero records for a row
// outside the image: the whole DMA reads zeros).
struct RowRsrc {
  const float* img;
  uint32_t img_bytes, row_bytes;
  int P0, py, H;  // P0 = image parity row of staged row 0
#ifdef PWC_STRIP_CENSUS
  unsigned long long* cen;
#endif
};

template <class G, int D>
__device__ __forceinline__ void dma_one(const RowRsrc& rr, const uint32_t (&rel)[G::IPR],
                                        uint32_t lds0) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int m = dma_row<G>(D), i = dma_idx<G>(D);
  const int pr = rr.P0 + m;                // parity row of the image
  const int yrow = 2 * pr + rr.py;         // image row
  const bool ok = pr >= 0 && yrow < rr.H;
  const uint32_t off = ok ? (uint32_t)yrow * rr.row_bytes : 0u;
  const int nrec = ok ? (int)(rr.img_bytes - off) : 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)rr.img + off), (short)0, nrec, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)(uintptr_t)(lds0 + (uint32_t)((m * G::SIGMA + 64 * i) * 16)),
      16, rel[i], 0, 0, 0);
#endif
}

template <class G, int D, int E>
__device__ __forceinline__ void dma_range(const RowRsrc& rr, const uint32_t (&rel)[G::IPR],
                                          uint32_t lds0) {
  if constexpr (D < E) {
    dma_one<G, D>(rr, rel, lds0);
    dma_range<G, D + 1, E>(rr, rel, lds0);
  }
}

// Barrier j of the loader: issue up to dma_target(j), wait for dma_need(j), barrier.
template <class G, int J>
__device__ __forceinline__ void loader_from(const RowRsrc& rr, const uint32_t (&rel)[G::IPR],
                                            uint32_t lds0) {
  if constexpr (J < G::NBAR) {
    constexpr int from = J == 0 ? 0 : dma_target<G>(J - 1);
    constexpr int to = dma_target<G>(J);
    static_assert(to >= dma_need<G>(J) && to - dma_need<G>(J) <= 63, "DMA schedule");
    dma_range<G, from, to>(rr, rel, lds0);
    wait_vmcnt<to - dma_need<G>(J)>();
#ifdef PWC_STRIP_CENSUS
    if constexpr (J == 0) rr.cen[29] = __builtin_amdgcn_s_memrealtime();  // group 0
    if constexpr (J == G::IPR - 1) rr.cen[30] = __builtin_amdgcn_s_memrealtime();  // window
    if constexpr (J == G::NBAR - 1) rr.cen[31] = __builtin_amdgcn_s_memrealtime();  // all rows
#endif
    __builtin_amdgcn_s_barrier();
    loader_from<G, J + 1>(rr, rel, lds0);
  }
}

// Five ds_read_b128 of one channel's f2 window (immediate offset O).
template <int O>
__device__ __forceinline__ void read5(uint32_t a, f32x4 (&w)[5]) {
  static_assert(O >= 0 && O + 64 < 65536, "ds offset field");
  asm volatile(
      "ds_read_b128 %0, %5 offset:%6\n\t"
      "ds_read_b128 %1, %5 offset:%7\n\t"
      "ds_read_b128 %2, %5 offset:%8\n\t"
      "ds_read_b128 %3, %5 offset:%9\n\t"
      "ds_read_b128 %4, %5 offset:%10"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4])
      : "v"(a), "n"(O), "n"(O + 16), "n"(O + 32), "n"(O + 48), "n"(O + 64)
      : "memory");
}

// Wait until at most N LDS reads are outstanding; the window registers it completes are tied
// through the asm so the compiler neither reads them earlier nor reuses them meanwhile.
template <int N>
__device__ __forceinline__ void lgk_wait(f32x4 (&w)[5]) {
  asm volatile("s_waitcnt lgkmcnt(%5)"
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4])
               : "n"(N));
}

// Four v_permlane32_swap_b32 (a's lanes 32-63 <-> b's lanes 0-31) in one block: one s_nop
// pair covers the VALU -> permlane operand hazard on either side (no swap reads a register
// another writes).  Written as asm: with ROCm 7.2 the builtin's two results fold into one
// register when both feed one add (the sum read v + v), dropping the other half.
__device__ __forceinline__ void swap32x4(float& a0, float& b0, float& a1, float& b1, float& a2,
                                         float& b2, float& a3, float& b3) {
  asm volatile(
      "s_nop 1\n\t"
      "v_permlane32_swap_b32 %0, %1\n\t"
      "v_permlane32_swap_b32 %2, %3\n\t"
      "v_permlane32_swap_b32 %4, %5\n\t"
      "v_permlane32_swap_b32 %6, %7\n\t"
      "s_nop 1"
      : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3));
}

// Four v_permlane16_swap_b32 (a's odd 16-lane rows <-> b's even rows), hazards as above.
__device__ __forceinline__ void swap16x4(float& a0, float& b0, float& a1, float& b1, float& a2,
                                         float& b2, float& a3, float& b3) {
  asm volatile(
      "s_nop 1\n\t"
      "v_permlane16_swap_b32 %0, %1\n\t"
      "v_permlane16_swap_b32 %2, %3\n\t"
      "v_permlane16_swap_b32 %4, %5\n\t"
      "v_permlane16_swap_b32 %6, %7\n\t"
      "s_nop 1"
      : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3));
}

struct LaneCtx {
  uint32_t addr;                   // LDS byte address of (step-0 row qd + tj - tj_lo, channel half, segment)
  __amdgpu_buffer_rsrc_t rs1;      // f1 of this image
  uint32_t f1off;                  // f1 voffset of step 0 (or kOOB)
  uint32_t f1step;                 // f1 voffset increment per step
  uint32_t plane_b;                // channel plane bytes
  int nstep_ok;                    // steps whose output row exists
};

constexpr uint32_t kOOB = 0x80000000u;

// f1 voffset of step st (kOOB: nothing to load -- zeros), computed once per step: a select
// per channel load becomes a branch in the step loop, around which the compiler sinks the FMAs
template <class G>
__device__ __forceinline__ uint32_t f1_voff(const LaneCtx& lc, int st) {
  return st < lc.nstep_ok && lc.f1off != kOOB ? lc.f1off + (uint32_t)st * lc.f1step : kOOB;
}
template <class G>
__device__ __forceinline__ f32x4 load_f1(const LaneCtx& lc, uint32_t v, int k) {
  return __builtin_bit_cast(
      f32x4, __builtin_amdgcn_raw_buffer_load_b128(lc.rs1, (int)v, (int)(k * lc.plane_b), 0));
}

// Window buffer of channel k (LA + 1 rotating buffers)
template <class G, int K>
__device__ __forceinline__ f32x4 (&wbuf(f32x4 (&w)[G::LA + 1][5]))[5] {
  return w[K % (G::LA + 1)];
}

// Issue channel K's window reads (step 0: after the barrier that lands its DMA group).
template <class G, bool FIRST, int K>
__device__ __forceinline__ void issue_read(uint32_t a, f32x4 (&w)[G::LA + 1][5]) {
  if constexpr (FIRST && K > 0 && pair_group<G>(K) > pair_group<G>(K - 1))
    __builtin_amdgcn_s_barrier();
  read5<G::NCS * K * G::QR * 16>(a, wbuf<G, K>(w));
}

// Channel k of a step (FIRST: step 0, whose window lands group by group; PF: the next step's
// f1 is prefetched into f1[k]): the window reads of channel k + LA, wait for channel k's, its
// FMAs, the prefetch.
template <class G, bool FIRST, bool PF, int K>
__device__ __forceinline__ void channel(const LaneCtx& lc, uint32_t f1v, uint32_t a, float (&acc)[9][4],
                                        f32x4 (&f1)[G::CH], f32x4 (&w)[G::LA + 1][5]) {
  if constexpr (K < G::CH) {
    if constexpr (K + G::LA < G::CH) {
      // PWC_STRIP_ABL 2: no window reads after step 0 (measurement only)
      if constexpr (FIRST || !(PWC_STRIP_ABL & 2)) issue_read<G, FIRST, K + G::LA>(a, w);
      lgk_wait<5 * G::LA>(wbuf<G, K>(w));
    } else {
      lgk_wait<5 * (G::CH - 1 - K)>(wbuf<G, K>(w));
    }
    // PWC_STRIP_ABL 4: no FMAs, 8: no f1 prefetch (measurement only)
    if constexpr (!(PWC_STRIP_ABL & 4)) corr_fma_pairs_s2<9, 5>(acc, f1[K], wbuf<G, K>(w));
    if constexpr (PF && !(PWC_STRIP_ABL & 8)) f1[K] = load_f1<G>(lc, f1v, K);
    __builtin_amdgcn_sched_barrier(0);
    channel<G, FIRST, PF, K + 1>(lc, f1v, a, acc, f1, w);
  }
}

template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_fwd_strip(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    int H, int W, int ngrp, int ntx, OutEpi epi) {
  static_assert(pair_groups_match_loader<G>(), "step-0 barriers out of step with the loader");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // logical block = (n, row parity, row group, strip, task group), task group fastest: the
  // workgroups of one image parity are neighbours and xcd_remap keeps neighbours on one XCD
  // (shared f2 rows)
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tg = t % G::TS;
  const int tx = (t / G::TS) % ntx;
  const int grp = (t / (G::TS * ntx)) % ngrp;
  const int py = (t / (G::TS * ntx * ngrp)) & 1;
  const int n = t / (G::TS * ntx * ngrp * 2);
  const int Y0 = grp * G::R;  // first parity row of the group
  const int x0 = tx * G::TW;  // first pixel of the strip
  const int tjlo = tg * G::NTASK / G::NSEG;  // first displacement row of the task group
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t plane_b = (uint32_t)(H * W) * 4u;
  const uint32_t img_bytes = (uint32_t)G::C * plane_b;  // < 2^31 (launcher)
  const float* img1 = in1 + (size_t)n * G::C * H * W;
  const float* img2 = in2 + (size_t)n * G::C * H * W;
  const uint32_t lds0 = lds_addr(lds);
  CENSUS_DECL;
  STAMP(0);

  if (wave == G::NWC) {
    // ---------------- loader wave ----------------
    uint32_t rel[G::IPR];
#pragma unroll
    for (int i = 0; i < G::IPR; ++i) {
      const int qq = 64 * i + lane;            // quad of the staged row
      const int l = qq / G::QR, qx = qq % G::QR;  // LDS channel row, quad in it
      // channel k of every lane part adjacent: (k, k + CH, ...)
      const int c = l / G::NCS + G::CH * (l % G::NCS);
      const int px = x0 - 8 + 4 * qx;
      rel[i] = px >= 0 && px < W ? ((uint32_t)c * plane_b + (uint32_t)px * 4u) : kOOB;
    }
#ifdef PWC_STRIP_CENSUS
    const RowRsrc rr{img2, img_bytes, (uint32_t)W * 4u, Y0 - 4 + tjlo, py, H, cen_t};
#else
    const RowRsrc rr{img2, img_bytes, (uint32_t)W * 4u, Y0 - 4 + tjlo, py, H};
#endif
    loader_from<G, 0>(rr, rel, lds0);
    CENSUS_FLUSH(29, 32, 32);
    return;
  }

  // ---------------- compute waves ----------------
  const int qd = wave / G::WPP, wq = wave % G::WPP;
  const int slot = lane % G::S, chalf = lane / G::S;  // task slot, channel part
  const int gtask = G::S * wq + slot;             // task of this workgroup's group
  const bool active = gtask < G::NTASK;
  const int tt = tg * G::NTASK + (active ? gtask : G::NTASK - 1);  // idle slots duplicate a lane
  const int tj = tt / G::NSEG, seg = tt % G::NSEG;
  const int px = x0 + 4 * seg;
  LaneCtx lc;
  lc.addr = lds0 + (uint32_t)(((qd + tj - tjlo) * G::SIGMA + chalf * G::QR + seg) * 16);
  lc.rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)img1, (short)0, (int)img_bytes, 0x00020000);
  const int yrow0 = 2 * (Y0 + qd) + py;  // this quad's output row in step 0
  lc.f1off = px < W ? ((uint32_t)(chalf * G::CH) * plane_b + ((uint32_t)yrow0 * W + px) * 4u)
                    : kOOB;
  lc.f1step = (uint32_t)(2 * G::NQD * W) * 4u;
  lc.plane_b = plane_b;
  // steps whose output row (2 (Y0 + NQD st + qd) + py) lies inside the image
  lc.nstep_ok = yrow0 < H ? min(G::NSTEP, (H - 1 - yrow0) / (2 * G::NQD) + 1) : 0;

  if constexpr (G::ZQ > 0) {
    // the last channel row's right halo (never DMA'd): zero quads behind every staged row,
    // written before step 0's first barrier
    if (wave == 0 && lane < G::NROW * G::ZQ) {
      const uint32_t za = lds0 + (uint32_t)(((lane / G::ZQ) * G::SIGMA + G::ROWQ + lane % G::ZQ) * 16);
      asm volatile("ds_write_b128 %0, %1" ::"v"(za), "v"(f32x4{0.f, 0.f, 0.f, 0.f}) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  f32x4 f1[G::CH];
#pragma unroll
  for (int k = 0; k < G::CH; ++k) f1[k] = load_f1<G>(lc, f1_voff<G>(lc, 0), k);

  // output: one buffer resource over the image's 81 planes (< 2^31 bytes: the accepts
  // predicate); a store whose lane has nothing to write (idle task, row or strip outside the
  // image, the high half's fifth store) gets an out-of-range offset.  Every store instruction
  // is then unconditional, so the compiler's vmcnt count for the f1 prefetch stays exact across
  // steps (a branch around a store makes it assume the store-less path and wait for stores
  // still draining).
  float* oimg = out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * 81 * H * W);
  const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc(
      (void*)oimg, (short)0, (int)(81u * plane_b), 0x00020000);
  // leaky_relu (model.py:84) as max(v, slope v): equal to epi_act for slope <= 1 (the
  // predicate declines larger slopes), and the identity at slope 1, bit for bit
  const float slope = epi.slope;
  // one step: rows 2 (Y0 + NQD st + qd) + py; step 0 and the last step unrolled, the steps in
  // between one runtime loop body (an unrolled chain of steps lets the compiler stretch live
  // ranges across them and spill)
  auto step = [&](auto first_c, auto pf_c, int st) {
    constexpr bool FIRST = decltype(first_c)::value, PF = decltype(pf_c)::value;
    float acc[9][4];
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[a][e] = 0.f;
    f32x4 w[G::LA + 1][5];
    const uint32_t a = lc.addr + (uint32_t)(st * G::NQD * G::SIGMA * 16);
    __builtin_amdgcn_s_barrier();  // step 0: group 0 landed; later steps: their rows landed
    if (FIRST) STAMP(1);
    issue_read<G, FIRST, 0>(a, w);
    if constexpr (G::LA > 1) issue_read<G, FIRST, 1>(a, w);
    channel<G, FIRST, PF, 0>(lc, f1_voff<G>(lc, st + 1), a, acc, f1, w);
    CSTAMP(2 + 3 * st);  // loop done
    // channel parts: lanes l + S j (j < NCS) hold partial sums of the same task; permlane
    // swaps pair a register holding plane P in every lane with one holding plane Q: the lanes
    // of the lower half keep P's total, the upper half Q's.  Halves (NCS 2): pairs (ti, ti + 5),
    // the low half keeps ti 0-4, the high half 5-8.  Quarters (NCS 4): permlane32 pairs
    // (0,2) (1,3) (4,6) (5,7) (8,8), then permlane16 pairs: part j keeps planes j, 4 + j
    // (and part 0 plane 8).
    constexpr int NQ = G::NCS == 2 ? 5 : 3;  // stores per lane
    float res[NQ][4];
    int pl[NQ];  // displacement column ti of each store
    if constexpr (G::NCS == 2) {
#pragma unroll
      for (int ti = 0; ti < 5; ++ti) {
        float x[4], y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          x[e] = acc[ti][e], y[e] = ti < 4 ? acc[ti + 5][e] : acc[ti][e];
        swap32x4(x[0], y[0], x[1], y[1], x[2], y[2], x[3], y[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) res[ti][e] = x[e] + y[e];
        pl[ti] = ti + 5 * chalf;
      }
    } else {
      constexpr int PA[5] = {0, 1, 4, 5, 8}, PB[5] = {2, 3, 6, 7, 8};
      float r1[5][4];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        float x[4], y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = acc[PA[i]][e], y[e] = acc[PB[i]][e];
        swap32x4(x[0], y[0], x[1], y[1], x[2], y[2], x[3], y[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) r1[i][e] = x[e] + y[e];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        float x[4], y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = r1[2 * i][e], y[e] = i < 2 ? r1[2 * i + 1][e] : r1[4][e];
        swap16x4(x[0], y[0], x[1], y[1], x[2], y[2], x[3], y[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) res[i][e] = x[e] + y[e];
      }
      pl[0] = chalf, pl[1] = 4 + chalf, pl[2] = 8;
    }
    CSTAMP(3 + 3 * st);  // channel parts reduced
    const int yrow = yrow0 + 2 * G::NQD * st;
    const bool wr = active && px < W && st < lc.nstep_ok;
    const uint32_t o0 = (uint32_t)(((tj * 9) * H + yrow) * W + px) * 4u;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      u32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // exact 2^-k multiply, or the reference's fp32 division (cu:98-100) when C is not a
        // power of two (C = 96)
        // (the divisor is k^2 C = C here, a compile-time constant: the launcher checks)
        const float o = (G::C & (G::C - 1)) == 0 ? res[q][e] * (1.f / G::C)
                                                 : res[q][e] / (float)G::C;
        v[e] = __builtin_bit_cast(uint32_t, fmaxf(o, o * slope));
      }
      // measurement builds (tools/strip_bench, -DPWC_STRIP_ABL=mask): 1 = stores discarded
      const bool keep = G::NCS == 2 ? (q < 4 || chalf == 0) : (q < 2 || chalf == 0);
      const bool ok = !(PWC_STRIP_ABL & 1) && wr && keep;
      // nontemporal (aux 2): measured against sc1, nt sc1 and plain stores, 14.2 against
      // 17.0-19.9 us back to back (profiles/r04a_strip_store_policy.txt)
      // the last step's stores with PWC_STRIP_LAST_AUX (measurement builds)
      __builtin_amdgcn_raw_buffer_store_b128(v, rso, (int)(ok ? o0 + pl[q] * plane_b : kOOB), 0,
                                             PF ? PWC_STRIP_STORE_AUX : PWC_STRIP_LAST_AUX);
    }
    CSTAMP(4 + 3 * st);  // stores issued
  };
  step(std::true_type{}, std::integral_constant<bool, (G::NSTEP > 1)>{}, 0);
#pragma unroll 1
  for (int st = 1; st < G::NSTEP - 1; ++st) step(std::false_type{}, std::true_type{}, st);
  if constexpr (G::NSTEP > 1) step(std::false_type{}, std::false_type{}, G::NSTEP - 1);
#ifdef PWC_STRIP_CENSUS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  {
    const unsigned long long* st_ = reinterpret_cast<const unsigned long long*>(
        reinterpret_cast<const char*>(lds) + G::LDS_BYTES);
    const int b_ = wave == 0 ? 0 : 32;
    for (int k_ = 2; k_ < 2 + 3 * G::NSTEP; ++k_) cen_t[k_] = st_[b_ + k_];
  }
#endif
  if (wave == 0) CENSUS_FLUSH(0, 2 + 3 * G::NSTEP, 0);
  if (wave == G::WPP) CENSUS_FLUSH(0, 2 + 3 * G::NSTEP, 32);  // the second quad's first wave
}

template <class G>
static hipError_t launch(const void* in1, const void* in2, void* out, int B, int H, int W,
                         float divisor, hipStream_t stream) {
  const int hp0 = (H + 1) / 2;  // parity-0 rows (the larger parity)
  const int ngrp = (hp0 + G::R - 1) / G::R;
  const int ntx = (W + G::TW - 1) / G::TW;
  const long long nblk = (long long)B * 2 * ngrp * ntx * G::TS;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e = lds_limit(reinterpret_cast<const void*>(&corr_fwd_strip<G>), G::LDS_ALLOC);
    if (e != hipSuccess) return e;
  }
  // the kernel divides by its compile-time C: Correlation's divisor k^2 C with k = 1
  if (divisor != (float)G::C) return hipErrorNotSupported;
  const OutEpi epi = current_epi();
  if (!(epi.slope <= 1.f)) return hipErrorNotSupported;  // max(v, slope v) form
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);  // bench.py's live timing hook (one-shot)
  hipExtLaunchKernelGGL((corr_fwd_strip<G>), dim3((unsigned)nblk), dim3(G::THREADS),
                        G::LDS_ALLOC, stream, ev0, ev1, 0, (const float*)in1, (const float*)in2,
                        (float*)out, H, W, ngrp, ntx, epi);
  return hipGetLastError();
}

template <class G>
long long grid_blocks(int B, int H, int W) {
  return (long long)B * 2 * (((H + 1) / 2 + G::R - 1) / G::R) * ((W + G::TW - 1) / G::TW) * G::TS;
}

// 6 parity rows x 56-px strips per workgroup, all 9 displacement rows (14 staged f2 rows):
// widths that are other multiples of 56 (the 224-px stress shape)
using GeoL4 = Geo<32, 6, 56>;
// W = 112 (config 2 l4): whole 112-px rows, so every store of a displacement plane covers a
// whole 448-B image row (the 56-px strips left the 128-B lines at the strip seam and across
// the row-parity seam half-written by two workgroups: 7.2 against 5.9 us for the volume's
// stores alone, tools/store_probe.hip); 6 parity rows, the (tj, segment) tasks of a row split
// over two workgroups (10 staged f2 rows each)
using GeoF = Geo<32, 6, 112, 2, 2, 1, true>;
// C = 64, W = 56 (config 2 l3): the same whole-row form, 3 parity rows per workgroup (7 staged
// f2 rows, 112 KB), one step of six compute waves
using GeoF3 = Geo<64, 3, 56, 2, 3, 1, true>;
// C = 96, W = 28 (config 2 l2): one parity row per workgroup (9 staged f2 rows, 136 KB), the
// channels of a task in quarters (four compute waves, 24 channels per lane)
#ifndef PWC_STRIP_GEOF2  // (measurement builds may override)
#define PWC_STRIP_GEOF2 96, 1, 28, 1, 1, 1, true, 4
#endif
using GeoF2 = Geo<PWC_STRIP_GEOF2>;

}  // namespace strip

// Which strip geometry serves this problem (0: none): fp32, model.py:24's stride-2 displacements
// in raster order (dr = 4, pad = md, k = 1, s1 = 1: checked by the caller), 16-B aligned
// buffers, an output the kernel's 32-bit buffer addressing reaches, the max(v, slope v)
// epilogue, and at least about one workgroup per CU (smaller grids leave CUs idle: the stream
// and row-band kernels suit them better); C = 32 at W = 112 (whole rows) or a multiple of
// 56 (strips), C = 64 at W = 56 and C = 96 at W = 28 (whole rows).  Knobs: strip=0 disables the kernel
// (measurement of the stream / row-band kernels), strip_geo=4 selects the 56-px strips at
// W = 112, strip_l3=0 / strip_l2=0 leave C = 64 / 96 to the row-band kernel.
enum StripPlan : int { kStripNone = 0, kStripL4 = 1, kStripF = 2, kStripF3 = 3, kStripF2 = 4 };
static int strip_plan(const void* in1, const void* in2, const void* out, int B, int C, int H,
                      int W, int s2, int dtype, int layout) {
  if (dtype != 0 || s2 != 2 || layout != kRaster) return kStripNone;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16) return kStripNone;
  if (H < 2 || (size_t)C * H * W * 4 >= 0x7ffffff0ull) return kStripNone;
  // the 81-plane output is addressed through one 32-bit buffer resource whose out-of-range
  // sentinel is 2^31: it must stay below that (larger grids go to the size_t stream kernel)
  if ((size_t)81 * H * W * 4 >= 0x7ffffff0ull) return kStripNone;
  if (!(current_epi().slope <= 1.f)) return kStripNone;  // the max(v, slope v) epilogue
  if (debug_knob("strip", 1) == 0) return kStripNone;
  if (C == 32) {
    if (W == strip::GeoF::TW && debug_knob("strip_geo", 10) != 4 &&
        strip::grid_blocks<strip::GeoF>(B, H, W) >= 192)
      return kStripF;
    if (W % strip::GeoL4::TW == 0 && strip::grid_blocks<strip::GeoL4>(B, H, W) >= 192)
      return kStripL4;
  }
  if (C == 64 && W == strip::GeoF3::TW && debug_knob("strip_l3", 1) != 0 &&
      strip::grid_blocks<strip::GeoF3>(B, H, W) >= 192)
    return kStripF3;
  if (C == 96 && W == strip::GeoF2::TW && debug_knob("strip_l2", 1) != 0 &&
      strip::grid_blocks<strip::GeoF2>(B, H, W) >= 192)
    return kStripF2;
  return kStripNone;
}

bool corr_strip_accepts(const void* in1, const void* in2, const void* out, int B, int C, int H,
                        int W, int s2, int dtype, int layout) {
  return strip_plan(in1, in2, out, B, C, H, W, s2, dtype, layout) != kStripNone;
}

hipError_t corr_forward_strip(const void* in1, const void* in2, void* out, int B, int C, int H,
                              int W, float divisor, hipStream_t stream) {
  switch (strip_plan(in1, in2, out, B, C, H, W, 2, 0, kRaster)) {
    case kStripF:
      return strip::launch<strip::GeoF>(in1, in2, out, B, H, W, divisor, stream);
    case kStripF3:
      return strip::launch<strip::GeoF3>(in1, in2, out, B, H, W, divisor, stream);
    case kStripF2:
      return strip::launch<strip::GeoF2>(in1, in2, out, B, H, W, divisor, stream);
    case kStripL4:
      return strip::launch<strip::GeoL4>(in1, in2, out, B, H, W, divisor, stream);
    default:
      return hipErrorNotSupported;
  }
}

}  // namespace pwc
