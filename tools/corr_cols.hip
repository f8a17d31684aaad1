// corr_cols.hip — PROTOTYPE, not in the product library (measured slower than corr_stream.hip:
// profiles/r03a_cols4px_ablation.txt, r03a_cols2grp.txt).  Correlation forward for the l4-sized grids (the paper's "level 2"):
// model.py:24's Correlation(9, 1, 9, 1, 2) in fp32, i.e. correlation_cuda_kernel.cu:34-106 with
// k = 1, s1 = 1, pad = md = 9, s2 = 2:
//   out[n, (tj+4)*9 + (ti+4), y, x] = sum_c f1[n,c,y,x] * f2[n,c,y+2tj,x+2ti] / C
// with zeros outside the image (the reference's zero-padded NHWC scratch, cu:10-32).
//
// Why this shape.  At B = 8 the l4 volume is 256 row bands of 3 parity rows, one
// per CU, and a band's 81 output planes (109 KB) exist only once all C channels are summed: a
// one-pass band serialises "stream the inputs + compute" and "drain the output".  Here the band
// is cut into column ITEMS (two 56-px halves at W = 112) computed by two GROUPS of waves: group
// A sums item 0 at raised issue priority and then stores it straight from registers, while
// group B -- fed by the same loader stream -- sums item 1.  Item 0's drain to HBM overlaps item
// 1's channel loop, and a group blocked on store issue never stalls the other: the waves meet
// through LDS counters, not s_barrier.
//
//   * loader wave: per stage of CC channels, buffer_load_dwordx4 ... lds (LDS-DMA) of the
//     item's f2 rows (R + 8 parity rows, 8 px of halo each side) and f1 rows into a ring of NS
//     stages (the buffer unit's range check yields the zero border); keeps up to AHEAD stages
//     in flight (<= 63 DMAs: the 6-bit vmcnt), publishes each landed stage in an LDS counter and
//     reissues a slot once every wave of its consumer group has released it.
//   * compute lanes (per group, as corr_stream.hip): lane = (r, tj, 8-pixel segment); a 16-lane
//     ds_read_b128 group holds 7 segments of two units whose f2 rows differ by one (odd row
//     stride: conflict-free); per channel 6 window quads + 2 f1 quads, 36 v_pk_fma_f32 into
//     8 px x 9 ti accumulators; the next channel's reads are in flight during the FMAs.
//   * output: 18 stores of 16 B per lane, straight from the accumulators.
#include <hip/hip_ext.h>

#include <cmath>

#include "../pwc-net_pytorch_amd/csrc/pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);

namespace cols {

#ifdef PWC_COLS_CENSUS  // tools/colbench.hip only: per-workgroup phase timestamps (100 MHz)
__device__ unsigned long long* g_census;
#define CENSUS(slot)                                                                   \
  do {                                                                                 \
    if ((threadIdx.x & 63) == 0)                                                       \
      g_census[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime();           \
  } while (0)
// measurement ablations (colbench): 1 no stores, 2 no DMA; read once per wave
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

// R: parity rows per workgroup; TWQ: item width in quads (4 px, even); CC: channels per ring
// stage; NS: ring stages.
template <int R_, int TWQ_, int CC_, int NS_>
struct Geo {
  static constexpr int R = R_, TWQ = TWQ_, CC = CC_, NS = NS_;
  static constexpr int NSEG = TWQ / 2;                 // 8-pixel segments per unit
  static constexpr int S = (TWQ + 4) | 1;              // LDS row stride in quads (odd)
  static constexpr int F2R = R + 8;                    // f2 parity rows (tj = -4..4)
  static constexpr int CH2 = F2R * S, CH1 = R * S;     // quads per channel
  static constexpr int F2PART = round64(CC * CH2), F1PART = round64(CC * CH1);
  static constexpr int STAGEQ = F2PART + F1PART;       // quads per ring stage
  static constexpr int I2 = F2PART / 64, I1 = F1PART / 64, IPS = I2 + I1;  // DMAs per stage
  // a group's 27 units (r, tj) in 12 16-lane ds_read_b128 groups (3 waves): 12 unit pairs
  // (tj 2k, 2k+1) on positions 0-6 / 8-14, the 3 units tj = 8 spread over positions 7 / 15
  static constexpr int NPAIR = 4 * R;                  // unit pairs = 16-lane groups
  static constexpr int NWG = NPAIR / 4;                // waves per group
  static constexpr int NCW = 2 * NWG;                  // compute waves (two groups)
  static constexpr int THREADS = 64 * (NCW + 1);       // + the loader wave
  static constexpr int NK = NS * CC;                   // channels per unrolled round
  static constexpr int RING_B = NS * STAGEQ * 16;
  static constexpr int FLAG_B = 16 * (NS + 4);         // LDS counters (16-B spaced)
  static constexpr int LDS_BYTES = RING_B + FLAG_B;
  static constexpr int NBASE = (RING_B + 32767) / 32768;  // 32 KiB address windows
  static constexpr int AHEAD0 = 63 / IPS;
  static constexpr int AHEAD = AHEAD0 < NS - 1 ? AHEAD0 : NS - 1;
  static_assert(TWQ % 2 == 0 && NSEG == 7 && R == 3, "the lane map is built for 3 x 56 px");
  static_assert(THREADS <= 1024 && LDS_BYTES <= 160 * 1024, "workgroup resources");
  static_assert(AHEAD >= 1 && NK % 2 == 0, "ring depth");
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

// Lane -> (r, tj, 8-pixel segment) of a group's lane map.  16-lane group gi (0..11) = wave
// lw's ds_read_b128 group g: positions 0-6 hold segments 0-6 of unit (gi / 4, 2 (gi % 4)) and
// positions 8-14 those of (gi / 4, 2 (gi % 4) + 1): f2 rows one apart, so with an odd row stride
// their 16-B slots are disjoint mod 256 B (conflict-free).  Positions 7 and 15 take the 21
// segments of the three tj = 8 units, one each (at most one 2-way conflict per group); the 3
// spare positions repeat position 6 / 14's address (broadcast).
template <class G>
__device__ __forceinline__ void lane_job(int gi, int p, int& r, int& tj, int& seg, bool& active) {
  r = gi >> 2;
  tj = 2 * (gi & 3) + (p >= 8 ? 1 : 0);
  seg = p & 7;
  active = true;
  if ((p & 7) == 7) {
    const int q = 2 * gi + (p >> 3);  // spread slot 0..23
    if (q < 3 * G::NSEG) {
      r = q / G::NSEG;
      tj = 8;
      seg = q - r * G::NSEG;
    } else {
      seg = G::NSEG - 1;  // spare: position 6 / 14's address
      active = false;
    }
  }
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Buffer resource of one stage: the image plus the stage's first channel (`cbytes`), records to
// the image's end -- the range check returns zeros for out-of-image offsets (0x80000000).
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

// ---- LDS counters (the loader <-> group hand-offs; LDS ops of one wave complete in order) ----
__device__ __forceinline__ uint32_t lds_load_u32(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void lds_store_u32(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add_u32(uint32_t a, uint32_t v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// Wait until the loader has published stage `gs` as landed.  All of this wave's earlier LDS
// operations complete on the way (lgkmcnt(0)).  The poll loop lives inside one asm statement:
// as C++ loops inside the unrolled channel sequence they split it into blocks and the register
// allocator spilled hundreds of VGPRs (among them asynchronously written read targets).
__device__ __forceinline__ void wait_landed(uint32_t flag, int gs) {
  uint32_t v;
  int sv;
  asm volatile(
      "1:\n\t"
      "ds_read_b32 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %1, %0\n\t"
      "s_cmp_gt_i32 %1, %3\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n\t"
      "2:"
      : "=&v"(v), "=&s"(sv)
      : "v"(flag), "s"(__builtin_amdgcn_readfirstlane(gs))
      : "memory", "scc");
}

// ---- compute side ----
typedef float acc_t[9][8];

template <int O0, int O1>
__device__ __forceinline__ void read2(uint32_t a, uint32_t b, f32x4& x, f32x4& y) {
  static_assert(O0 >= 0 && O0 < 65536 && O1 >= 0 && O1 < 65536, "ds offset field");
  asm volatile(
      "ds_read_b128 %0, %2 offset:%4\n\t"
      "ds_read_b128 %1, %3 offset:%5"
      : "=&v"(x), "=&v"(y)
      : "v"(a), "v"(b), "n"(O0), "n"(O1)
      : "memory");
}

// Wait until at most N LDS reads are outstanding; tie the channel's registers through the asm
// so the compiler neither reads them earlier nor reuses them meanwhile.
template <int N>
__device__ __forceinline__ void lgk_wait(f32x4 (&w)[6], f32x4 (&f)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]),
                 "+v"(f[0]), "+v"(f[1])
               : "n"(N));
}

// displacements ti in [T0, T1) of one channel: acc[ti][p] += f1[p] * win[p + 2 ti], p = 0..7,
// win[0] = column x0 - 8: every pixel pair (p, p+1), p even, meets an aligned window pair ->
// one v_pk_fma_f32 (csrc/corr_stream.hip fma_ti<2>)
template <int T0, int T1>
__device__ __forceinline__ void fma_ti(acc_t& acc, const f32x4 (&w)[6], const f32x4 (&f)[2]) {
#pragma unroll
  for (int ti = T0; ti < T1; ++ti) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int p = 2 * h, j = p + 2 * ti;
      const f32x4 a = f[h >> 1];
      const f32x2 a2 = (h & 1) ? f32x2{a.z, a.w} : f32x2{a.x, a.y};
      const f32x4 q = w[j >> 2];
      const f32x2 w2 = (j & 2) ? f32x2{q.z, q.w} : f32x2{q.x, q.y};
      f32x2 c2 = {acc[ti][p], acc[ti][p + 1]};
      c2 = __builtin_elementwise_fma(a2, w2, c2);
      acc[ti][p] = c2.x;
      acc[ti][p + 1] = c2.y;
    }
  }
}

// channel K's reads inside an unrolled round (offsets relative to 32 KiB window bases)
template <class G, int K>
struct Off {
  static constexpr int S = K / G::CC, J = K % G::CC;
  static constexpr int W2 = (S * G::STAGEQ + J * G::CH2) * 16;
  static constexpr int W1 = (S * G::STAGEQ + G::F2PART + J * G::CH1) * 16;
  static constexpr int WIN2 = W2 / 32768, IMM2 = W2 % 32768;
  static constexpr int WIN1 = W1 / 32768, IMM1 = W1 % 32768;
};

template <class G>
struct Ctx {
  uint32_t wa[G::NBASE], fa[G::NBASE];  // window / f1 base address per 32 KiB window
  uint32_t landed, rel0;  // LDS counters: stages landed; released[0] (16-B spaced)
  int gs0;                // global stage index of the round's first stage
};

// One channel: its reads were issued during the previous channel's FMAs; the next channel's
// reads go out between this channel's FMA chunks.  At a stage's last channel the stage is
// released to the loader once its reads are done; before the next stage's first reads, the
// landing counter is polled.
template <class G, int K>
__device__ __forceinline__ void round_step(const Ctx<G>& cx, acc_t& acc, f32x4 (&wA)[6],
                                           f32x4 (&fA)[2], f32x4 (&wB)[6], f32x4 (&fB)[2]) {
  if constexpr (K < G::NK) {
    constexpr int NEXT = K + 1;
    f32x4(&wc)[6] = (K & 1) ? wB : wA;
    f32x4(&fc)[2] = (K & 1) ? fB : fA;
    f32x4(&wn)[6] = (K & 1) ? wA : wB;
    f32x4(&fn)[2] = (K & 1) ? fA : fB;
    lgk_wait<0>(wc, fc);  // this channel's reads
    if constexpr (K % G::CC == G::CC - 1)
      lds_add_u32(cx.rel0 + 16 * ((cx.gs0 + K / G::CC) % G::NS), 1);  // stage read: release
    if constexpr (NEXT < G::NK) {
      using O = Off<G, NEXT>;
#ifndef PWC_COLS_NOPOLL  // measurement build: no landing polls inside the round
      if constexpr (NEXT % G::CC == 0) wait_landed(cx.landed, cx.gs0 + NEXT / G::CC);
#endif
      read2<O::IMM2, O::IMM2 + 16>(cx.wa[O::WIN2], cx.wa[O::WIN2], wn[0], wn[1]);
      fma_ti<0, 2>(acc, wc, fc);
      __builtin_amdgcn_sched_barrier(0);
      read2<O::IMM2 + 32, O::IMM2 + 48>(cx.wa[O::WIN2], cx.wa[O::WIN2], wn[2], wn[3]);
      fma_ti<2, 4>(acc, wc, fc);
      __builtin_amdgcn_sched_barrier(0);
      read2<O::IMM2 + 64, O::IMM2 + 80>(cx.wa[O::WIN2], cx.wa[O::WIN2], wn[4], wn[5]);
      fma_ti<4, 6>(acc, wc, fc);
      __builtin_amdgcn_sched_barrier(0);
      read2<O::IMM1, O::IMM1 + 16>(cx.fa[O::WIN1], cx.fa[O::WIN1], fn[0], fn[1]);
      fma_ti<6, 9>(acc, wc, fc);
    } else {
      fma_ti<0, 9>(acc, wc, fc);
    }
    __builtin_amdgcn_sched_barrier(0);
    round_step<G, K + 1>(cx, acc, wA, fA, wB, fB);
  }
}

// Loader: DMA offsets per instruction and lane (branch-free), per item the column check picks
// the offset or the out-of-range value; issues stage after stage as ring slots are released,
// publishing each stage once landed.
template <class G>
__device__ __forceinline__ void loader(const float* img1, const float* img2, uint32_t lds0,
                                       uint32_t landed_a, uint32_t rel0, int lane, int Y0, int py,
                                       int H, int W, int nst, int total, uint32_t plane_b,
                                       uint32_t img_bytes, int abl) {
  constexpr uint32_t kOOB = 0x80000000u;
  int rowoff[G::IPS], xrel[G::IPS];
#pragma unroll
  for (int i = 0; i < G::IPS; ++i) {
    const bool f2 = i < G::I2;
    const int g = (f2 ? 64 * i : 64 * (i - G::I2)) + lane;
    const int n_here = f2 ? G::CC * G::CH2 : G::CC * G::CH1;
    const int chq = f2 ? G::CH2 : G::CH1;
    const int j = g / chq, q = g - j * chq;
    const int rho = q / G::S, xq = q - rho * G::S;  // slot quad xq holds column X0 - 8 + 4 xq
    const int prow = f2 ? Y0 - 4 + rho : Y0 + rho;
    const int srow = 2 * prow + py;
    const bool ok = g < n_here && xq < G::TWQ + 4 && prow >= 0 && srow < H;
    rowoff[i] = ok ? (j * H + srow) * W : -1;
    xrel[i] = 4 * xq - 8;
  }
  uint32_t rel[G::IPS];
  int rel_item = -1;
  auto issue = [&](int gs) {
    const int item = gs / nst, st = gs - item * nst;
    if (item != rel_item) {
      const int X0 = item * G::TWQ * 4;
#pragma unroll
      for (int i = 0; i < G::IPS; ++i) {
        const int x = X0 + xrel[i];
        rel[i] = (rowoff[i] >= 0 && x >= 0 && x < W) ? (uint32_t)(rowoff[i] + x) * 4u : kOOB;
      }
      rel_item = item;
    }
    if (ABL(2)) return;
    const uint32_t cb = (uint32_t)(st * G::CC) * plane_b;
    const uint32_t slot = lds0 + (uint32_t)((gs % G::NS) * G::STAGEQ * 16);
    const __amdgpu_buffer_rsrc_t rs2 = stage_rsrc(img2, cb, img_bytes);
    const __amdgpu_buffer_rsrc_t rs1 = stage_rsrc(img1, cb, img_bytes);
#pragma unroll
    for (int i = 0; i < G::IPS; ++i)
      dma1(i < G::I2 ? rs2 : rs1, rel[i],
           slot + (uint32_t)((i < G::I2 ? 64 * i : G::F2PART + 64 * (i - G::I2)) * 16));
  };
  // a slot is free for stage s once its previous use (stage s - NS) was released by all NWG
  // waves of that use's group: released[s % NS] counts NWG per use
  auto slot_free = [&](int s) {
    return s < G::NS || (int)lds_load_u32(rel0 + 16 * (s % G::NS)) >= (s / G::NS) * G::NWG;
  };
  int issued = -1, published = -1;
  CENSUS(1);
  while (published < total - 1) {
    while (issued + 1 < total && issued - published < G::AHEAD && slot_free(issued + 1)) {
      issue(++issued);
      if (issued == G::NS) CENSUS(13);  // group 1's first stage issued
    }
    if (published < issued) {
      if (ABL(4))
        wait_vm_stages<G::IPS>(0);
      else
        wait_vm_stages<G::IPS>(issued - published - 1);  // stage published + 1 landed
      ++published;
      lds_store_u32(landed_a, (uint32_t)(published + 1));
      if (published == 0) CENSUS(3);
      if (published == G::NS) CENSUS(12);  // group 1's first stage published
    } else {
      __builtin_amdgcn_s_sleep(2);  // every slot still held: wait for a release
    }
  }
  CENSUS(9);  // last stage published
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
  const uint32_t landed_a = lds0 + G::RING_B, rel0 = landed_a + 16;
  ABL_LOAD();
  if (wave == 0) CENSUS(0);
  if (threadIdx.x < G::NS + 1) lds_store_u32(landed_a + 16 * threadIdx.x, 0u);
  __syncthreads();  // counters zeroed (the only workgroup barrier)

  if (wave == G::NCW) {
    loader<G>(img1, img2, lds0, landed_a, rel0, lane, Y0, py, H, W, nst, total, plane_b,
              img_bytes, abl);
    return;
  }

  // ---------------- compute waves: group 0 = items 0, 2, ...; group 1 = items 1, 3, ... ----
  const int grp = wave / G::NWG, lw = wave - grp * G::NWG;
#ifndef PWC_COLS_NOPRIO
  if (grp == 0) __builtin_amdgcn_s_setprio(1);  // the item drained first computes first
#endif
  int g, p;
  lane_group(lane, g, p);
  int r, tj, seg;
  bool active;
  lane_job<G>(lw * 4 + g, p, r, tj, seg, active);
  Ctx<G> cx;
#pragma unroll
  for (int k = 0; k < G::NBASE; ++k) {
    // window: from pixel x0 - 8 (quad 2 seg of the slot row); f1: quad 2 seg + 2 of its row
    // (the f1 part's offset inside a stage is in Off::W1)
    cx.wa[k] = lds0 + (uint32_t)(k * 32768 + ((r + tj) * G::S + 2 * seg) * 16);
    cx.fa[k] = lds0 + (uint32_t)(k * 32768 + (r * G::S + 2 * seg + 2) * 16);
  }
  cx.landed = landed_a;
  cx.rel0 = rel0;
  const int y = 2 * (Y0 + r) + py;
  const bool store = active && y < H && !ABL(1);
  float* oimg = out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * 81 * plane);
  const int nround = C / G::NK;
  if (wave == 0) CENSUS(10);

  for (int item = grp; item < nitem; item += 2) {
    acc_t acc;
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[a][k] = 0.f;
    for (int rd = 0; rd < nround; ++rd) {
      cx.gs0 = item * nst + rd * G::NS;
      f32x4 wA[6], fA[2], wB[6], fB[2];
      wait_landed(cx.landed, cx.gs0);
      if (lw == 0 && item == 0 && rd == 0) CENSUS(4);  // stage 0 landed
      if (lw == 0 && item == 1 && rd == 0) CENSUS(2);  // group 1's first stage landed
      using O0 = Off<G, 0>;
      read2<O0::IMM2, O0::IMM2 + 16>(cx.wa[O0::WIN2], cx.wa[O0::WIN2], wA[0], wA[1]);
      read2<O0::IMM2 + 32, O0::IMM2 + 48>(cx.wa[O0::WIN2], cx.wa[O0::WIN2], wA[2], wA[3]);
      read2<O0::IMM2 + 64, O0::IMM2 + 80>(cx.wa[O0::WIN2], cx.wa[O0::WIN2], wA[4], wA[5]);
      read2<O0::IMM1, O0::IMM1 + 16>(cx.fa[O0::WIN1], cx.fa[O0::WIN1], fA[0], fA[1]);
      round_step<G, 0>(cx, acc, wA, fA, wB, fB);
    }
    if (lw == 0) CENSUS(item == 0 ? 5 : 7);  // item loop done (wave 0 of its group)
    // ---- this item's 81 planes, straight from registers (cu:100: / C) ----
    if (store) {
      if (inv_divisor != 0.f) {
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[a][k] *= inv_divisor;
      } else {
        // q = x * (1/d) plus one FMA residual correction (a non-power-of-2 C)
        const float rinv = 1.f / divisor;
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float q = acc[a][k] * rinv;
            acc[a][k] = fmaf(fmaf(-q, divisor, acc[a][k]), rinv, q);
          }
      }
      if (epi.slope != 1.f) {
#pragma unroll
        for (int a = 0; a < 9; ++a)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[a][k] = epi_act(acc[a][k], epi.slope);
      }
      // raster channel order (cu:98): plane (tj + 4) * 9 + ti + 4, ti = a - 4
      float* orow = oimg + ((size_t)(tj * 9) * H + y) * W + item * G::TWQ * 4 + 8 * seg;
#pragma unroll
      for (int a = 0; a < 9; ++a) {
        st_out4(orow + (size_t)a * plane, st_f32x4{acc[a][0], acc[a][1], acc[a][2], acc[a][3]});
        st_out4(orow + (size_t)a * plane + 4,
                st_f32x4{acc[a][4], acc[a][5], acc[a][6], acc[a][7]});
      }
    }
    if (lw == 0 && item == 0) CENSUS(6);  // item 0's stores issued
  }
  if (lw == 0) CENSUS(8 + grp * 3);       // 8: group 0 done, 11: group 1 done
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
// Serves fp32 model.py:24 correlation (k 1, s1 1, pad = md, dr 4, s2 2) in the raster channel
// order, rows cut into items of 56 px (W = 112 or 224: two or four items), C a multiple of 32,
// 16-B aligned buffers, grids of at least ~one workgroup per CU.
hipError_t corr_forward_cols(const void* in1, const void* in2, void* out, int B, int C, int H,
                             int W, int layout, float divisor, hipStream_t stream) {
  using namespace cols;
  if (layout != kRaster) return hipErrorNotSupported;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16) return hipErrorNotSupported;
  if ((size_t)C * H * W * 4 >= 0x7ffffff0ull || C % 32) return hipErrorNotSupported;
  const long long nblk = (long long)B * 2 * ((((H + 1) / 2) + 2) / 3);
  if (nblk < 192) return hipErrorNotSupported;
  if (W % 56 == 0 && (W / 56) % 2 == 0 && W / 56 <= 4) {
    using G = Geo<3, 14, 4, 8>;
    return launch<G>((const float*)in1, (const float*)in2, (float*)out, B, C, H, W, W / 56,
                     divisor, stream);
  }
  return hipErrorNotSupported;
}

}  // namespace pwc
