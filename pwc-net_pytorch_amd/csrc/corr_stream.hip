// corr_stream.hip — correlation forward for the large pyramid levels (l4 / the paper's "level
// 2" and up): row bands over column tiles, one loader wave streaming channels through an LDS
// ring, seven compute waves; fp32 or fp16 storage, stride-2 (model.py:24's Correlation(9, 1,
// 9, 1, 2)) or stride-1 (Correlation(4, 1, 4, 1, 1), CostVolumeLayer sr = 4) displacements.
//
// Semantics (correlation_cuda_kernel.cu:34-106 with k = 1, s1 = 1, pad = md, dr = 4, s2 = 2):
//   out[n, (tj+4)*9 + (ti+4), y, x] = sum_c f1[n,c,y,x] * f2[n,c,y+2tj,x+2ti] / C
// with zeros outside the image (the reference's zero-padded scratch).
//
// Why this shape: a row y of the output only meets f2 rows of y's parity, so a
// workgroup takes R output rows of ONE row parity (rows 2(Y0+r)+py, r < R) over the full width
// and needs R + 8 f2 rows (all nine tj) plus R f1 rows: at R = 3 the chip's 256 CUs get one
// workgroup each for B = 8 at 96 x 112 and every f2 row is staged ~3.7x instead of the 9x of
// 16 x 16 tiles, which is what bounded the per-CU LDS ingest of the tile kernels.  Full rows
// also make every output row segment a run of whole 128-B lines.
//
//   * loader wave: per channel, IPC buffer_load_dwordx4 ... lds (LDS-DMA, 1 KiB each) fill one
//     ring slot: f2 rows then f1 rows, each padded to S quads (2 zero quads either side = the
//     reference's zero border, produced by the buffer unit's range check; S odd).  It keeps
//     NS-2 channels in flight and releases a channel with s_barrier after a counted vmcnt.
//   * compute lane = (r, tj, 8-pixel segment): per channel 6 window quads of f2 row r+tj and
//     2 quads of f1 row r (ds_read_b128), 36 v_pk_fma_f32 into 8 px x 9 ti accumulators; the
//     next channel's reads are in flight during the current channel's FMAs.
//   * lane map: every ds_read_b128 lane group (16 lanes, MI355X_MICROARCH.md §LDS) holds <= 8
//     consecutive segments of one (r, tj) unit and <= 8 of a unit whose f2 row differs by one;
//     with S odd their 16 B slots mod 256 B are all distinct (conflict-free); idle positions
//     duplicate an active lane's address (broadcast).
//   * output: per lane 9 ti x 2 float4 nontemporal stores (whole rows per workgroup).
//   * blocks are remapped XCD-aware so the bands of one image parity share an L2 (their f2
//     halo rows overlap).
#include <hip/hip_ext.h>

#include <cmath>
#include <type_traits>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);

namespace stream {

#ifdef PWC_STREAM_CENSUS  // tools/sbench.hip only: per-workgroup phase timestamps (100 MHz)
__device__ unsigned long long* g_census;
#define CENSUS(slot)                                                                   \
  do {                                                                                 \
    if ((threadIdx.x & 63) == 0)                                                       \
      g_census[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
#else
#define CENSUS(slot) \
  do {               \
  } while (0)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int round64(int v) { return (v + 63) / 64 * 64; }

// T: storage type (float or __half; arithmetic fp32); S2: displacement stride (2: rows of ONE
// parity per workgroup; 1: consecutive rows); R: output rows per workgroup; TWP: column tile
// width in pixels (a lane owns an 8-pixel segment of it; wider images take several tiles);
// CC: channels per ring stage; NS: ring depth in stages.
// P2 (fp16 storage only): LDS holds channel PAIRS -- pixel x of channels (c, c+1) as one
// half2 dword, interleaved by the loader on the way in -- and every product pair is one
// v_dot2_f32_f16 (two fp16 products, fp32 accumulation): per channel pair the fp32 kernel's LDS
// traffic and instruction count.  fp16 storage always takes the pair layout.
template <typename T, int S2_, int R_, int TWP_, int CC_, int NS_, bool P2_ = false>
struct Geo {
  using Elem = T;
  static constexpr int S2 = S2_, R = R_, TWP = TWP_, CC = CC_, NS = NS_;
  static constexpr bool H16 = sizeof(T) == 2;            // fp16 storage (and output)
  static constexpr bool P2 = P2_;
  static_assert(P2 == H16, "fp16 storage is staged as channel pairs (and only fp16)");
  static constexpr int CPU = P2 ? 2 : 1;                 // channels per ring unit
  static constexpr int EPQ = 4;                          // LDS elements (dwords) per quad
  static constexpr int OEPQ = 16 / (int)sizeof(T);       // output pixels per 16-B quad
  static constexpr int NPY = S2 == 2 ? 2 : 1;            // row parities split over workgroups
  static constexpr int TWQ = TWP / EPQ;                  // tile quads per row (LDS)
  static constexpr int OTWQ = TWP / OEPQ;                // tile quads per output row
  static constexpr int HQ = 8 / EPQ;                     // halo quads each side (8 pixels)
  static constexpr int SQ = 8 / EPQ;                     // quads per 8-pixel segment
  static constexpr int NSEG = TWP / 8;
  static constexpr int NB = (NSEG + 7) / 8;              // segment blocks per unit
  // fp32: balanced blocks; fp16: whole 8-segment blocks (the park swizzle XORs 4 inside one)
  static constexpr int BS = H16 ? 8 : (NSEG + NB - 1) / NB;
  // LDS row stride in quads: a ds_read_b128 lane group holds 8 segments of unit A and 8 of a
  // unit whose row differs by one, so their 16-B slots (mod 256 B) are disjoint iff S is odd
  // (2 quads per segment)
  static constexpr int S = (TWQ + 2 * HQ) | 1;
  static constexpr int NWQ = S2 == 2 ? 6 : 4;            // window quads read per unit
  static constexpr int NFQ = 2;                          // f1 quads read per unit
  static constexpr int F2R = R + 8;                      // f2 rows (tj = -4..4)
  static constexpr int F2Q = round64(F2R * S);           // quads of the f2 part of a channel
  static constexpr int F1Q = round64(R * S);
  static constexpr int CHQ = F2Q + F1Q;                  // quads per channel
  static constexpr int CH_B = CHQ * 16;
  static constexpr int IPC = CHQ / 64;                   // DMA instructions per channel
  static constexpr int IF2 = F2Q / 64;                   // ... of which read f2
  static constexpr int NPAIR = 4 * R + (R + 1) / 2;      // unit pairs (see pair_units)
  static constexpr int NG = NPAIR * NB;                  // 16-lane groups
  static constexpr int NWC = (NG + 3) / 4;               // compute waves
  static constexpr int THREADS = 64 * (NWC + 1);         // + the loader wave
  static constexpr int SLOT_B = CC * CH_B;               // one ring stage
  static constexpr int RING_B = NS * SLOT_B;
  static constexpr int PRQ = H16 ? 8 * NB : TWQ;         // park row quads (output staging)
  // P2 loader: 8-pixel units (one 16-B global load per channel) of the staged rows
  static constexpr int UPR = (TWP + 16) / 8;             // units per staged row
  static constexpr int NU = (F2R + R) * UPR;             // units per channel pair
  static constexpr int NIT = (NU + 63) / 64;             // loader iterations per pair
  static constexpr int OUT_B = 81 * R * PRQ * 16;
  static constexpr int LDS_BYTES = RING_B > OUT_B ? RING_B : OUT_B;
  static constexpr int NBASE = (RING_B + 32767) / 32768;  // 32 KiB address windows
  // loader: wait until stage k landed = at most the later stages' DMAs outstanding, capped by
  // the 6-bit vmcnt (a smaller count only waits a little longer)
  static constexpr int WAITN = (NS - 3) * CC * IPC < 63 ? (NS - 3) * CC * IPC : 63;
  static_assert(S2 == 1 || S2 == 2, "displacement stride");
  static_assert(TWP % 8 == 0 && TWP % EPQ == 0 && BS <= 8, "8-pixel segments, <= 8 per block");
  static_assert(S % 2 == 1, "conflict-free row stride");
  static_assert(NS >= 4, "ring depth");
  static_assert(THREADS <= 1024 && LDS_BYTES <= 160 * 1024, "workgroup resources");
  static_assert(CH_B <= 32768, "a channel fits one 32 KiB window");
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

// Unit pair pi -> units (r, tj) A and B whose f2 rows (r + tj) differ by exactly one:
//   pi < 4R:  r = pi / 4, tj = 2 (pi % 4) and tj + 1 (tj index 0..8 = displacement + 4)
//   else:     tj = 8, r = 2m and 2m + 1 (m = pi - 4R); B is absent when 2m + 1 == R.
template <class G>
__device__ __forceinline__ void pair_units(int pi, int& ra, int& ta, int& rb, int& tb, bool& hasb) {
  if (pi < 4 * G::R) {
    ra = rb = pi >> 2;
    ta = 2 * (pi & 3);
    tb = ta + 1;
    hasb = true;
  } else {
    const int m = pi - 4 * G::R;
    ra = 2 * m;
    rb = 2 * m + 1;
    ta = tb = 8;
    hasb = rb < G::R;
  }
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Two ds_read_b128 at a + O0 and b + O1 (immediates).
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

// Wait until at most N LDS reads are outstanding; the registers it completes are tied through
// the asm so the compiler neither reads them earlier nor reuses them meanwhile.
template <int N>
__device__ __forceinline__ void lgk_wait(f32x4 (&w)[6], f32x4 (&f)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]),
                 "+v"(f[0]), "+v"(f[1])
               : "n"(N));
}

// fp32, displacements ti in [T0, T1) of one channel: acc[ti][p] += f1[p] * win[p + S2 ti],
// p = 0..7, win[0] = column x0 - 4 S2.  Stride 2: every pixel pair (p, p+1), p even, meets an
// aligned window pair -> v_pk_fma_f32.  Stride 1: odd ti meet misaligned pairs -> two
// v_fma_f32 (the same FMA throughput as one v_pk_fma_f32).
template <int S2, int T0, int T1>
__device__ __forceinline__ void fma_ti(float (&acc)[9][8], const f32x4 (&w)[6],
                                       const f32x4 (&f)[2]) {
#pragma unroll
  for (int ti = T0; ti < T1; ++ti) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int p = 2 * h, j = p + S2 * ti;
      const f32x4 a = f[h >> 1];
      const f32x2 a2 = (h & 1) ? f32x2{a.z, a.w} : f32x2{a.x, a.y};
      if ((j & 1) == 0) {
        const f32x4 q = w[j >> 2];
        const f32x2 w2 = (j & 2) ? f32x2{q.z, q.w} : f32x2{q.x, q.y};
        f32x2 c2 = {acc[ti][p], acc[ti][p + 1]};
        c2 = __builtin_elementwise_fma(a2, w2, c2);
        acc[ti][p] = c2.x;
        acc[ti][p + 1] = c2.y;
      } else {
        acc[ti][p] = fmaf(a2.x, w[j >> 2][j & 3], acc[ti][p]);
        acc[ti][p + 1] = fmaf(a2.y, w[(j + 1) >> 2][(j + 1) & 3], acc[ti][p + 1]);
      }
    }
  }
}

// Channel pairs: acc[ti][p] += f1[c][p] * w[c][p + S2 ti] + f1[c+1][p] * w[c+1][p + S2 ti]
// as one v_dot2_f32_f16 per (ti, p); every LDS dword is one pixel's (c, c+1) half2.
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
template <int S2, int T0, int T1>
__device__ __forceinline__ void fma_ti_p(float (&acc)[9][8], const f32x4 (&w)[6],
                                         const f32x4 (&f)[2]) {
#pragma unroll
  for (int ti = T0; ti < T1; ++ti) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int j = p + S2 * ti;  // window element (quad j / 4), as fma_ti
      // dword k of a quad as half2, built from the quad's 8 halves (bit-casting the k-th
      // float / u32 element straight to half2 compiles to the quad's FIRST dword for every k
      // with this toolchain -- checked in the ISA)
      const f16x8 fh = __builtin_bit_cast(f16x8, f[p >> 2]);
      const f16x8 wh = __builtin_bit_cast(f16x8, w[j >> 2]);
      const h2_t a = {fh[2 * (p & 3)], fh[2 * (p & 3) + 1]};
      const h2_t b = {wh[2 * (j & 3)], wh[2 * (j & 3) + 1]};
      acc[ti][p] = __builtin_amdgcn_fdot2(a, b, acc[ti][p], false);
    }
  }
}

// fp32 or channel-pair products of displacements [T0, T1)
template <class G, int T0, int T1>
__device__ __forceinline__ void fma_unit(float (&acc)[9][8], const f32x4 (&w)[6],
                                         const f32x4 (&f)[2]) {
  if constexpr (G::P2)
    fma_ti_p<G::S2, T0, T1>(acc, w, f);
  else
    fma_ti<G::S2, T0, T1>(acc, w, f);
}

// One DMA instruction of channel c's slot: `rel` = this lane's byte offset inside the channel
// plane (or kOOB: the buffer unit returns zeros), `img` = the image's f1 or f2 base.
__device__ __forceinline__ void dma1(const void* img, uint32_t cbytes, uint32_t img_bytes,
                                     uint32_t rel, uint32_t lds_dst) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int nrec = cbytes < img_bytes ? (int)(img_bytes - cbytes) : 0;
  const uint64_t b = (uint64_t)(uintptr_t)img + (uint64_t)cbytes;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
      __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, (__attribute__((address_space(3))) void*)(uintptr_t)lds_dst, 16, rel, 0, 0, 0);
#endif
}

template <class G>
__device__ __forceinline__ void load_stage(int st, uint32_t plane_b, uint32_t img_bytes,
                                           const void* img1, const void* img2,
                                           const uint32_t (&rel)[G::IPC], uint32_t lds0) {
  const uint32_t slot = lds0 + (uint32_t)((st % G::NS) * G::SLOT_B);
#pragma unroll
  for (int j = 0; j < G::CC; ++j) {
    const uint32_t cb = (uint32_t)(st * G::CC + j) * plane_b;
#pragma unroll
    for (int i = 0; i < G::IPC; ++i)
      dma1(i < G::IF2 ? img2 : img1, cb, img_bytes, rel[i],
           slot + (uint32_t)(j * G::CH_B + i * 1024));
  }
}

// One channel's reads (window quads then f1 quads, in pairs) interleaved with its FMA chunks:
// the next channel's reads go out between the current channel's FMA chunks, so the LDS queue
// never holds a wave's whole batch while its FMAs wait to issue.  M: measurement modes
// (launcher knob stream_abl >> 3): 1 no LDS reads, 2 no FMAs, 4 no barriers (only valid
// without DMA).
template <class G, int IMM, int M>
__device__ __forceinline__ void channel_body(uint32_t w_, uint32_t f_, float (&acc)[9][8],
                                             const f32x4 (&wc)[6], const f32x4 (&fc)[2],
                                             f32x4 (&wn)[6], f32x4 (&fn)[2]) {
  constexpr bool RD = !(M & 1), FM = !(M & 2);
  if constexpr (G::S2 == 2) {
    if constexpr (RD) read2<IMM, IMM + 16>(w_, w_, wn[0], wn[1]);
    if constexpr (FM) fma_unit<G, 0, 2>(acc, wc, fc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RD) read2<IMM + 32, IMM + 48>(w_, w_, wn[2], wn[3]);
    if constexpr (FM) fma_unit<G, 2, 4>(acc, wc, fc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RD) read2<IMM + 64, IMM + 80>(w_, w_, wn[4], wn[5]);
    if constexpr (FM) fma_unit<G, 4, 6>(acc, wc, fc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RD) read2<IMM, IMM + 16>(f_, f_, fn[0], fn[1]);
    if constexpr (FM) fma_unit<G, 6, 9>(acc, wc, fc);
  } else {
    if constexpr (RD) read2<IMM, IMM + 16>(w_, w_, wn[0], wn[1]);
    if constexpr (FM) fma_unit<G, 0, 3>(acc, wc, fc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RD) read2<IMM + 32, IMM + 48>(w_, w_, wn[2], wn[3]);
    if constexpr (FM) fma_unit<G, 3, 6>(acc, wc, fc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (RD) read2<IMM, IMM + 16>(f_, f_, fn[0], fn[1]);
    if constexpr (FM) fma_unit<G, 6, 9>(acc, wc, fc);
  }
  if constexpr (!FM) asm volatile("" ::"v"(wc[0]), "v"(wc[2]), "v"(fc[0]));
}

// Compute-wave loop over one unrolled round of NS stages x CC channels (so every LDS offset is
// an instruction immediate inside one of NBASE 32 KiB windows; the launcher requires
// C % (NS * CC) == 0).  Channel k: barrier when channel k+1 opens a stage, wait for k's reads,
// then k+1's reads interleaved with k's FMAs.  The last channel reads a stale slot
// (discarded) and meets the loader's closing barrier, so every round is the same code.
template <class G, int K, int M = 0>
__device__ __forceinline__ void compute_round(const uint32_t (&wa)[G::NBASE],
                                              const uint32_t (&fa)[G::NBASE], float (&acc)[9][8],
                                              f32x4 (&wA)[6], f32x4 (&fA)[2], f32x4 (&wB)[6],
                                              f32x4 (&fB)[2]) {
  constexpr int NK = G::NS * G::CC;
  if constexpr (K < NK) {
    constexpr int NEXT = ((K + 1) % NK);
    constexpr int OFF = (NEXT / G::CC) * G::SLOT_B + (NEXT % G::CC) * G::CH_B;
    constexpr int WIN = OFF / 32768, IMM = OFF % 32768;
    // buffers alternate by channel parity (NK even keeps it static per K)
    f32x4(&wc)[6] = (K & 1) ? wB : wA;
    f32x4(&fc)[2] = (K & 1) ? fB : fA;
    f32x4(&wn)[6] = (K & 1) ? wA : wB;
    f32x4(&fn)[2] = (K & 1) ? fA : fB;
    if constexpr (NEXT % G::CC == 0 && !(M & 4)) __builtin_amdgcn_s_barrier();
    lgk_wait<0>(wc, fc);  // this channel's reads (issued during the previous channel's FMAs)
    channel_body<G, IMM, M>(wa[WIN], fa[WIN], acc, wc, fc, wn, fn);
    // keep this channel's FMAs between its wait and the next channel's (left alone, the
    // scheduler sinks them past later reads and the live ranges overflow into scratch)
    __builtin_amdgcn_sched_barrier(0);
    compute_round<G, K + 1, M>(wa, fa, acc, wA, fA, wB, fB);
  }
}

template <class G, int M>
__device__ __forceinline__ void compute_loop(int C, int nst, const uint32_t (&wa)[G::NBASE],
                                             const uint32_t (&fa)[G::NBASE], float (&acc)[9][8],
                                             f32x4 (&wA)[6], f32x4 (&fA)[2], f32x4 (&wB)[6],
                                             f32x4 (&fB)[2]) {
  for (int c0 = 0; c0 < C; c0 += G::NS * G::CC)
    compute_round<G, 0, M>(wa, fa, acc, wA, fA, wB, fB);
  if constexpr ((M & 4) != 0)
    for (int k = 0; k < nst; ++k) __builtin_amdgcn_s_barrier();
}

template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_fwd_stream(
    const typename G::Elem* __restrict__ in1, const typename G::Elem* __restrict__ in2,
    typename G::Elem* __restrict__ out, int C, int H, int W, int Ho, int Wo, int nband,
    int ntx, int layout, float divisor, float inv_divisor, OutEpi epi, int abl) {
  using T = typename G::Elem;
  static_assert((G::NS * G::CC) % 2 == 0, "buffer parity repeats every round");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // logical block = (n, row parity, band, column tile), tile fastest: the tiles and bands of
  // one image (parity) are neighbours, and xcd_remap keeps neighbours on one XCD (shared halo)
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % ntx;
  const int band = (t / ntx) % nband;
  const int py = (t / (ntx * nband)) % G::NPY;
  const int n = t / (ntx * nband * G::NPY);
  const int Y0 = band * G::R;         // first (parity) row of the band
  const int X0Q = tx * G::TWQ;        // first quad of the column tile
  const int CU = C / G::CPU;          // ring units (channels, or channel pairs)
  const int nst = CU / G::CC;         // ring stages
  const int WQ = W / G::EPQ;          // image quads per row (LDS element units)

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t plane = (uint32_t)(H * W);
  const uint32_t plane_b = plane * (uint32_t)sizeof(T);
  const uint32_t img_bytes = (uint32_t)C * plane_b;  // < 2^31 (launcher)
  const T* img1 = in1 + (size_t)n * C * plane;
  const T* img2 = in2 + (size_t)n * C * plane;
  const uint32_t lds0 = lds_addr(lds);
  if (wave == 0) CENSUS(0);

  if (G::P2 && wave == G::NWC) {
    // ---------------- loader wave, channel pairs: register staging ----------------
    // 8-pixel units of channels c and c+1 (two 16-B loads; the buffer range check gives the
    // zero border) interleaved into half2 quads (v_perm) and written with ds_write_b128.
    // Stage s goes into its slot before B_{s+3-NS} ... i.e. up to stage k + NS - 3 is written
    // before barrier B_k: the slot it reuses was last read before B_{k-1}.
    constexpr uint32_t kOOB = 0x80000000u;
    constexpr int NU2 = G::F2R * G::UPR, NU1 = G::R * G::UPR;
    constexpr int NI2 = (NU2 + 63) / 64, NI1 = (NU1 + 63) / 64;
    const int X0 = tx * G::TWP;
    uint32_t rel2[NI2], rel1[NI1];
    int dq2[NI2], dq1[NI1];
#pragma unroll
    for (int it = 0; it < NI2 + NI1; ++it) {
      const bool f2 = it < NI2;
      const int u = (f2 ? it : it - NI2) * 64 + lane;
      const int rr = u / G::UPR, cu = u - rr * G::UPR;
      const int prow = f2 ? Y0 - 4 + rr : Y0 + rr;
      const int srow = G::S2 == 2 ? 2 * prow + py : prow;
      const int px = X0 - 8 + 8 * cu;
      const bool in = u < (f2 ? NU2 : NU1);
      const bool ok = in && prow >= 0 && srow < H && px >= 0 && px < W;
      const uint32_t rel = ok ? (uint32_t)(srow * W + px) * 2u : kOOB;
      const int dq = in ? (f2 ? 0 : G::F2Q) + rr * G::S + 2 * cu : -1;
      if (f2) rel2[it] = rel, dq2[it] = dq;
      else rel1[it - NI2] = rel, dq1[it - NI2] = dq;
    }
    const __amdgpu_buffer_rsrc_t rs1 =
        __builtin_amdgcn_make_buffer_rsrc((void*)img1, (short)0, (int)img_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs2 =
        __builtin_amdgcn_make_buffer_rsrc((void*)img2, (short)0, (int)img_bytes, 0x00020000);
    f32x4 a2[G::CC][NI2], b2[G::CC][NI2], a1[G::CC][NI1], b1[G::CC][NI1];
    auto issue = [&](int gs) {
#pragma unroll
      for (int j = 0; j < G::CC; ++j) {
        const int so = (int)((uint32_t)(2 * (gs * G::CC + j)) * plane_b);
#pragma unroll
        for (int it = 0; it < NI2; ++it) {
          a2[j][it] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs2, (int)rel2[it], so, 0));
          b2[j][it] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs2, (int)rel2[it],
                                                           so + (int)plane_b, 0));
        }
#pragma unroll
        for (int it = 0; it < NI1; ++it) {
          a1[j][it] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs1, (int)rel1[it], so, 0));
          b1[j][it] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs1, (int)rel1[it],
                                                           so + (int)plane_b, 0));
        }
      }
    };
    // (c, c+1) halves of pixel k -> one dword: low half from channel c
    auto put = [&](float* base, int dq, const f32x4& a, const f32x4& b) {
      if (dq < 0) return;
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 av = __builtin_bit_cast(u32x4, a), bv = __builtin_bit_cast(u32x4, b);
      const uint32_t ax = av.x, ay = av.y, az = av.z, aw = av.w;
      const uint32_t bx = bv.x, by = bv.y, bz = bv.z, bw = bv.w;
      const u32x4 q0 = {__builtin_amdgcn_perm(bx, ax, 0x05040100u),
                        __builtin_amdgcn_perm(bx, ax, 0x07060302u),
                        __builtin_amdgcn_perm(by, ay, 0x05040100u),
                        __builtin_amdgcn_perm(by, ay, 0x07060302u)};
      const u32x4 q1 = {__builtin_amdgcn_perm(bz, az, 0x05040100u),
                        __builtin_amdgcn_perm(bz, az, 0x07060302u),
                        __builtin_amdgcn_perm(bw, aw, 0x05040100u),
                        __builtin_amdgcn_perm(bw, aw, 0x07060302u)};
      *reinterpret_cast<u32x4*>(base + 4 * dq) = q0;
      *reinterpret_cast<u32x4*>(base + 4 * dq + 4) = q1;
    };
    auto write = [&](int gs) {
      float* slot = lds + (size_t)(gs % G::NS) * (G::SLOT_B / 4);
#pragma unroll
      for (int j = 0; j < G::CC; ++j) {
        float* base = slot + j * (G::CH_B / 4);
#pragma unroll
        for (int it = 0; it < NI2; ++it) put(base, dq2[it], a2[j][it], b2[j][it]);
#pragma unroll
        for (int it = 0; it < NI1; ++it) put(base, dq1[it], a1[j][it], b1[j][it]);
      }
    };
    if (abl & 2) {  // measurement: no staging (barriers only)
      for (int k = 0; k <= nst; ++k) __builtin_amdgcn_s_barrier();
    } else {
      if (nst > 0) issue(0);
      int nw = 0;  // next stage to write
      for (int k = 0; k <= nst; ++k) {
        const int upto = min(k + G::NS - 3, nst - 1);
        while (nw <= upto) {
          write(nw);
          ++nw;
          if (nw < nst) issue(nw);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B_k
      }
    }
  } else if (wave == G::NWC) {
    // ---------------- loader wave ----------------
    constexpr uint32_t kOOB = 0x80000000u;
    uint32_t rel[G::IPC];
#pragma unroll
    for (int i = 0; i < G::IPC; ++i) {
      const bool f2 = i < G::IF2;
      const int j = (f2 ? 64 * i : 64 * i - G::F2Q) + lane;
      // slot quad q of LDS row rho holds image quad X0Q - HQ + q (q < TWQ + 2 HQ; the rest of
      // the row is padding): halo quads come from the neighbouring tile or read zero
      const int rho = j / G::S, q = j % G::S, cq = X0Q - G::HQ + q;
      const int prow = f2 ? Y0 - 4 + rho : Y0 + rho;  // parity row (S2 = 2) or row
      const int srow = G::S2 == 2 ? 2 * prow + py : prow;
      const bool ok = rho < (f2 ? G::F2R : G::R) && q < G::TWQ + 2 * G::HQ && cq >= 0 &&
                      cq < WQ && prow >= 0 && srow < H;
      rel[i] = ok ? (uint32_t)(srow * W + G::EPQ * cq) * (uint32_t)sizeof(T) : kOOB;
    }
    if (abl & 2) {  // measurement: no DMA (barriers only)
      for (int k = 0; k <= nst; ++k) __builtin_amdgcn_s_barrier();
    } else {
      const int npro = nst < G::NS ? nst : G::NS;
      for (int st = 0; st < npro; ++st)
        load_stage<G>(st, plane_b, img_bytes, img1, img2, rel, lds0);
      // barrier B_k (k = 0..nst-1): stage k landed; after B_k (k >= 2) stage k-2's slot is
      // free.  B_nst closes the compute waves' last channel.
      for (int k = 0; k < nst; ++k) {
        const int issued = (k >= 2 ? k - 2 + G::NS : G::NS) - 1;  // last stage issued so far
        const int ahead = (issued < nst - 1 ? issued : nst - 1) - k;
        if (ahead >= G::NS - 3)
          wait_vmcnt<G::WAITN>();
        else
          wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (k >= 2 && k - 2 + G::NS < nst)
          load_stage<G>(k - 2 + G::NS, plane_b, img_bytes, img1, img2, rel, lds0);
      }
      CENSUS(1);                     // last stage landed
      __builtin_amdgcn_s_barrier();  // B_nst
    }
  } else {
    // ---------------- compute waves ----------------
    int g, p;
    lane_group(lane, g, p);
    const int gi = wave * 4 + g;  // 16-lane group index
    const int pi = gi / G::NB, blk = gi % G::NB;
    int ra, ta, rb, tb;
    bool hasb;
    pair_units<G>(pi < G::NPAIR ? pi : 0, ra, ta, rb, tb, hasb);
    const bool useb = p >= 8 && hasb;
    const int sp = p & 7;
    const int r = useb ? rb : ra, tj = useb ? tb : ta;
    const int seg = blk * G::BS + (sp < G::BS ? sp : 0);
    const bool active = gi < G::NG && sp < G::BS && seg < G::NSEG && (p < 8 || hasb);
    const int sg = seg < G::NSEG ? seg : 0;  // a duplicate address for idle lanes (broadcast)
    // window: from pixel x0 - 4 S2, i.e. padded pixel 8 seg + 8 - 4 S2 (fp32: quad 2 seg or
    // 2 seg + 1); f1: padded pixel 8 seg + 8
    const int wq = 2 * sg + (G::S2 == 2 ? 0 : 1);
    const int fq = 2 * sg + 2;
    uint32_t wa[G::NBASE], fa[G::NBASE];
#pragma unroll
    for (int k = 0; k < G::NBASE; ++k) {
      wa[k] = lds0 + (uint32_t)(k * 32768 + ((r + tj) * G::S + wq) * 16);
      fa[k] = lds0 + (uint32_t)(k * 32768 + (G::F2Q + r * G::S + fq) * 16);
    }

    float acc[9][8];
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[a][k] = 0.f;

    f32x4 wA[6], fA[2], wB[6], fB[2];
    if (abl & 1) {  // measurement: no LDS reads / FMAs (barriers only)
      for (int k = 0; k <= nst; ++k) __builtin_amdgcn_s_barrier();
      acc[0][0] = (float)C;
    } else {
      __builtin_amdgcn_s_barrier();  // B_0: stage 0 landed
      read2<0, 16>(wa[0], wa[0], wA[0], wA[1]);
      read2<32, 48>(wa[0], wa[0], wA[2], wA[3]);
      if constexpr (G::S2 == 2) read2<64, 80>(wa[0], wa[0], wA[4], wA[5]);
      read2<0, 16>(fa[0], fa[0], fA[0], fA[1]);
      switch (abl >> 3) {
        case 0: compute_loop<G, 0>(CU, nst, wa, fa, acc, wA, fA, wB, fB); break;
        case 1: compute_loop<G, 1>(CU, nst, wa, fa, acc, wA, fA, wB, fB); break;
        case 2: compute_loop<G, 2>(CU, nst, wa, fa, acc, wA, fA, wB, fB); break;
        case 5: compute_loop<G, 5>(CU, nst, wa, fa, acc, wA, fA, wB, fB); break;
        default: compute_loop<G, 6>(CU, nst, wa, fa, acc, wA, fA, wB, fB); break;
      }
      lgk_wait<0>(wA, fA);  // the last (discarded) reads
    }
    if (wave == 0) CENSUS(2);  // channel loop done
    // park the results in LDS as [oc][r][x] (the ring is dead once every wave is past B_nst
    // and its own last reads; the barrier below orders the writes after everyone's reads)
    __builtin_amdgcn_s_barrier();
    if (wave == 0) CENSUS(5);  // past the park barrier
    if (active) {
      // out = acc / C (cu:100): an exact multiply when C is a power of two (a uniform branch,
      // so the division sequence is not evaluated and discarded per value)
      if (inv_divisor != 0.f) {
#pragma unroll
        for (int ti = 0; ti < 9; ++ti)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[ti][k] *= inv_divisor;
      } else {
        // q = x * (1/d) plus one FMA residual correction: the correctly rounded quotient up to
        // rare last-ulp ties, at 3 VALU instead of the ~10 of an IEEE division (CostVolumeLayer
        // divides by 81, modules.py:74)
        const float rinv = 1.f / divisor;
#pragma unroll
        for (int ti = 0; ti < 9; ++ti)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float q = acc[ti][k] * rinv;
            acc[ti][k] = fmaf(fmaf(-q, divisor, acc[ti][k]), rinv, q);
          }
      }
      // the fused leaky_relu (model.py:84) only when asked for: a uniform branch, so the
      // plain volume parks its 72 values with no per-value compare / select
      auto park = [&](auto act_c) {
        constexpr bool ACT = decltype(act_c)::value;
#pragma unroll
        for (int ti = 0; ti < 9; ++ti) {
          const int oc = out_channel(layout, tj - 4, ti - 4, 4, 9, G::S2);
          f32x4* prow = reinterpret_cast<f32x4*>(lds) + (oc * G::R + r) * G::PRQ;
          if constexpr (G::H16) {
            // one quad per lane; odd segment blocks XOR 4 so the two blocks sharing a
            // ds_write_b128 lane group (8 consecutive lanes) hit disjoint 16-B slots
            f16x8 v;
#pragma unroll
            for (int e = 0; e < 8; ++e)
              v[e] = (_Float16)(ACT ? epi_act(acc[ti][e], epi.slope) : acc[ti][e]);
            prow[seg ^ (4 * (blk & 1))] = __builtin_bit_cast(f32x4, v);
          } else {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e)
                v[e] = ACT ? epi_act(acc[ti][4 * h + e], epi.slope) : acc[ti][4 * h + e];
              // odd segment blocks swap their two quads: the two blocks sharing a
              // ds_write_b128 lane group then hit disjoint 16-B slots
              prow[2 * seg + (h ^ (blk & 1))] = v;
            }
          }
        }
      };
      if (epi.slope == 1.f)
        park(std::false_type{});
      else
        park(std::true_type{});
    }
  }
  if (wave == G::NWC) __builtin_amdgcn_s_barrier();  // the loader's side of the park barrier
  __syncthreads();
  // ---------------- epilogue: whole output row segments, every wave, nontemporal ----------
  if (wave == 0) CENSUS(3);  // parked
  if (abl & 4) return;  // measurement: no stores
  T* oimg = out + (epi.ostride ? (size_t)n * epi.ostride : (size_t)n * 81 * Ho * Wo);
  constexpr int OT = G::OTWQ;  // output quads per tile row
  constexpr int NQ = 81 * G::R * OT;
  constexpr int PER = (NQ + G::THREADS - 1) / G::THREADS;
  const int OWQ = W / G::OEPQ, OX0Q = tx * OT;
  st_f32x4 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {  // all LDS reads first, then all stores
    const int q = threadIdx.x + i * G::THREADS;
    const int row = q / OT, xq = q - row * OT;
    int pq;
    if constexpr (G::H16) {
      pq = row * G::PRQ + (xq ^ (4 * ((xq / G::BS) & 1)));
    } else {
      const int seg = xq >> 1;
      pq = row * G::PRQ + 2 * seg + ((xq & 1) ^ ((seg / G::BS) & 1));
    }
    if (q < NQ) v[i] = *reinterpret_cast<const st_f32x4*>(lds + 4 * pq);
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int q = threadIdx.x + i * G::THREADS;
    const int oc = q / (G::R * OT);
    const int rem = q - oc * (G::R * OT);
    const int r = rem / OT, xq = OX0Q + rem - r * OT;
    const int y = G::S2 == 2 ? 2 * (Y0 + r) + py : Y0 + r;
    if (q < NQ && y < Ho && xq < OWQ)
      st_out4(reinterpret_cast<float*>(oimg + ((size_t)oc * Ho + y) * Wo + G::OEPQ * xq), v[i]);
  }
  if (wave == 0) CENSUS(4);  // stores issued
}

template <class G>
static hipError_t launch(const void* in1, const void* in2, void* out, int B, int C, int H, int W,
                         int layout, float divisor, hipStream_t stream) {
  using T = typename G::Elem;
  const int HP = G::S2 == 2 ? (H + 1) / 2 : H;  // (parity) rows; parity 0 has the extra row
  const int nband = (HP + G::R - 1) / G::R;
  const int ntx = (W + G::TWP - 1) / G::TWP;
  const long long nblk = (long long)B * G::NPY * nband * ntx;
  if (nblk <= 0) return hipSuccess;
  if (C <= 0 || C % (G::NS * G::CC * G::CPU)) return hipErrorNotSupported;  // whole rounds
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e =
        lds_limit(reinterpret_cast<const void*>(&corr_fwd_stream<G>), G::LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;  // exact when a power of 2
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);  // bench.py's live timing hook (one-shot)
  hipExtLaunchKernelGGL((corr_fwd_stream<G>), dim3((unsigned)nblk), dim3(G::THREADS),
                        G::LDS_BYTES, stream, ev0, ev1, 0, (const T*)in1, (const T*)in2,
                        (T*)out, C, H, W, H, W, nband, ntx, layout, divisor, inv, current_epi(),
                        debug_knob("stream_abl", 0));
  return hipGetLastError();
}

template <typename T, int S2, int TWP>
static hipError_t pick(const void* in1, const void* in2, void* out, int B, int C, int H, int W,
                       int layout, float divisor, hipStream_t stream) {
  // ring: CC channels per stage x NS stages.  4 x 4 (half the barriers per channel) measured
  // best or equal at every shape served in back-to-back launches (config-2 l4 fp32 19.6 ->
  // 17.2 us against 2 x 8; Corr4, Sintel fp32/fp16 l3/l4; profiles/r02d_stream_ring_sweep.txt),
  // where one launch's store tail overlaps the next one's loop; inside the bench step, where
  // it cannot, all three rings measure the same 19.1-19.4 us (profiles/r02d_bench_ring_ab.txt)
  // fp16: channel pairs through v_dot2_f32_f16 (corr_stream_accepts guarantees C % 16 == 0)
  if constexpr (sizeof(T) == 2) {
    // 4-row bands when 3-row bands give few workgroups (about one round): config-4 Sintel
    // l3 (B=16, 64 x 56 x 128) 41.6 -> 28.0 us; l4 (1216 workgroups) stays at 3 (63.3 against
    // 66.4 us; 2 rows 75.4); profiles/r02e_stream_fp16_rows.txt
    const int hp = S2 == 2 ? (H + 1) / 2 : H;
    const long long nblk3 = (long long)B * (S2 == 2 ? 2 : 1) * ((hp + 2) / 3) *
                            ((W + TWP - 1) / TWP);
    if (debug_knob("stream_r", nblk3 <= 384 ? 4 : 3) == 4)
      return launch<Geo<T, S2, 4, TWP, 2, 4, true>>(in1, in2, out, B, C, H, W, layout, divisor,
                                                    stream);
    return launch<Geo<T, S2, 3, TWP, 2, 4, true>>(in1, in2, out, B, C, H, W, layout, divisor,
                                                  stream);
  } else if constexpr (S2 == 1) {
    // stride-1 displacements (Corr4, CostVolumeLayer): the 4 x 4 ring needs more than the 256
    // VGPRs (~640 spilled to scratch), 2 x 4 none, at the same time (l4 16.9-17.0 us against
    // 16.9-17.3 over 300 launches each; profiles/r02e_corr4_ring.txt)
    return launch<Geo<T, S2, 3, TWP, 2, 4>>(in1, in2, out, B, C, H, W, layout, divisor, stream);
  } else {
    return launch<Geo<T, S2, 3, TWP, 4, 4>>(in1, in2, out, B, C, H, W, layout, divisor, stream);
  }
}

}  // namespace stream

// hipErrorNotSupported: a shape this kernel does not serve (the caller tries the next path).
// Serves k = 1, s1 = 1, pad = md (output = input size) with dr = 4: s2 = 2 (model.py:24's
// Correlation(9,1,9,1,2)) or s2 = 1 (Correlation(4,1,4,1,1), CostVolumeLayer(sr=4) with the
// CVL channel order); fp32 or fp16 storage (dtype 0 / 1); W a multiple of 4 (fp32) or 8
// (fp16) and 16-B aligned pointers; C a multiple of 16; grids of at least ~one workgroup per
// CU (smaller grids have faster homes: corr_pt / corr_rows).
// Whether corr_forward_stream serves this problem (also the pairing predicate of the group
// entry, capi.hip, through corr_forward_path).
bool corr_stream_accepts(const void* in1, const void* in2, const void* out, int B, int C, int H,
                         int W, int s2, int dtype) {
  const int epq = dtype == 1 ? 8 : 4;
  if (dtype != 0 && dtype != 1) return false;
  if ((uintptr_t)in1 % 16 || (uintptr_t)in2 % 16 || (uintptr_t)out % 16 || W % epq) return false;
  if ((size_t)C * H * W * (16 / epq) >= 0x7ffffff0ull || C % 16) return false;
  const int twp = (W % 112 == 0 || W < 112) ? 112 : 128;  // column tile width in pixels
  const long long nblk = (long long)B * (s2 == 2 ? 2 : 1) *
                         (((s2 == 2 ? (H + 1) / 2 : H) + 2) / 3) * ((W + twp - 1) / twp);
  return nblk >= 192 && W >= 64 && (s2 == 1 || s2 == 2);
}

bool corr_strip_accepts(const void*, const void*, const void*, int, int, int, int, int, int, int);
hipError_t corr_forward_strip(const void*, const void*, void*, int, int, int, int, float,
                              hipStream_t);
bool corr_mstrip16_accepts(const void*, const void*, const void*, int, int, int, int, int, int,
                           int);
hipError_t corr_forward_mstrip16(const void*, const void*, void*, int, int, int, int, int, int,
                                 float, hipStream_t);

hipError_t corr_forward_stream(const void* in1, const void* in2, void* out, int B, int C, int H,
                               int W, int s2, int dtype, int layout, float divisor,
                               hipStream_t stream) {
  // fp16 storage, C = 32 / 64 / 96 (config-4 l4 / l3 / l2; stride 1: C = 32 / 64): the
  // matrix-core strip kernel (corr_mstrip16.hip), which also takes grids the stream kernel
  // declines
  if (corr_mstrip16_accepts(in1, in2, out, B, C, H, W, s2, dtype, layout)) {
    const hipError_t e =
        corr_forward_mstrip16(in1, in2, out, B, C, H, W, s2, layout, divisor, stream);
    if (e != hipErrorNotSupported) return e;
  }
  // fp32 model-config grids of C = 32 (config 2 l4) and C = 64 at W = 56 (config 2 l3): the
  // strip kernel (corr_strip.hip), also where the stream kernel would decline the grid
  if (corr_strip_accepts(in1, in2, out, B, C, H, W, s2, dtype, layout)) {
    const hipError_t e = corr_forward_strip(in1, in2, out, B, C, H, W, divisor, stream);
    if (e != hipErrorNotSupported) return e;
  }
  if (!corr_stream_accepts(in1, in2, out, B, C, H, W, s2, dtype)) return hipErrorNotSupported;
  const int twp = (W % 112 == 0 || W < 112) ? 112 : 128;  // column tile width in pixels
  using namespace stream;
#define PWC_PICK(T)                                                                            \
  if (s2 == 2)                                                                                 \
    return twp == 112 ? pick<T, 2, 112>(in1, in2, out, B, C, H, W, layout, divisor, stream)    \
                      : pick<T, 2, 128>(in1, in2, out, B, C, H, W, layout, divisor, stream);   \
  if (s2 == 1)                                                                                 \
    return twp == 112 ? pick<T, 1, 112>(in1, in2, out, B, C, H, W, layout, divisor, stream)    \
                      : pick<T, 1, 128>(in1, in2, out, B, C, H, W, layout, divisor, stream);
  if (dtype == 0) {
    PWC_PICK(float)
  } else {
    PWC_PICK(__half)
  }
#undef PWC_PICK
  return hipErrorNotSupported;
}

}  // namespace pwc
