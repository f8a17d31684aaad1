// warp_bwd.hip — WarpingLayer backward (modules.py:31-42; ATen grid_sampler_2d_backward with the
// reference's grid chain, bilinear, zeros, align_corners=True) for wide images: grad_x and
// grad_flow from one tile kernel plus a small finishing kernel, with a caller workspace
// (pwc_warp_backward_ws).
//
// One workgroup (512 threads: two per tile pixel, each half of a chunk's channels) owns
// (image n, 16 x 16 tile T of pixels, a group of channels).  It reads the flow of T's 32 x 32
// window (T plus an 8-pixel margin) once and builds, in LDS, the list of window pixels p whose
// bilinear corners land on each tile pixel q (counting sort with per-wave counters: the list
// order, and so every sum, is fixed -- deterministic).  The channels stream through LDS in
// chunks of CC (x and grad_out over the window, buffer loads two chunks ahead):
//   grad_x[q]   = sum over q's list of w * grad_out[p]                (plain stores, once each)
//   grad_flow_p += grad_out[p] * d(bilinear)/d(ix, iy) from x at p's four corners
// Every global load and store of the chunk loop is a branch-free buffer operation (range check
// instead of a branch): a skipped one would make the compiler wait for vmcnt(0) and drain the
// prefetch at every chunk.  With several channel groups each leaves its grad_flow partial in
// the workspace and warp_bwd_finish adds them in group order.  Corners beyond the margin
// (|flow| > ~8 px): their x values are re-read from global memory after the chunk loop, and
// the grad_x contributions of pixels outside their corner's tile window go to per-wave lists
// that warp_bwd_finish adds with fp32 atomics -- after every tile's plain stores (the kernel
// boundary orders them; per-workgroup agent-scope fences would write back the XCD's L2).
#include <hip/hip_runtime.h>

#include "warp_sample.cuh"

namespace pwc {
namespace wbwd {

constexpr int NT = 512;   // two threads per tile pixel (each half of a chunk's channels)
constexpr int TS = 16;            // tile side
constexpr int MG = 8;             // margin
constexpr int WS = TS + 2 * MG;   // window side (32)
constexpr int WN = WS * WS;       // window pixels (1024)
constexpr int MAXE = 4 * WN;      // list entries (each window pixel has 4 corners)
constexpr size_t kHead = 256;     // workspace: header, then partials / far lists / far counts
#ifndef PWC_WBWD_CC  // channels per chunk (measurement builds may override)
#define PWC_WBWD_CC 4
#endif
constexpr int CC = PWC_WBWD_CC;
constexpr int MINWG = CC <= 4 ? 2 : 1;  // workgroups per CU the LDS allows

struct Args {
  const float* x;
  const float* flow;
  const float* gout;
  float* gx;
  float* gflow;
  int B, C, H, W;
  float halfx, halfy;
  int ntx, ntiles, ng, cpg;
  float* part;        // ng * B * 2 * H * W grad_flow partials (ng > 1)
  unsigned* far;      // per workgroup and wave: 256 far-corner entries
  unsigned* farcnt;   // per workgroup and wave: the number of entries
  int nwg;
  int census;         // measurement only (knob warp_bwd_census): phase stamps -> g_wbwd_census
};

// Phase timestamps (measurement only): s_memrealtime (100 MHz) of workgroup b's thread 0
__device__ unsigned long long g_wbwd_census[4096 * 16];
// (a branch-free buffer store: a conditional store would cost the chunk loop its precise
// vmcnt waits -- see warp_bwd_tile)
// Product builds compile the marks and the ablation bits out (`make CENSUS=1` keeps them).
#ifdef PWC_CENSUS
#define WB_MARKC(k, cond)                                                                   \
  do {                                                                                      \
    const bool on_ = a.census && (cond) && threadIdx.x == 0 && blockIdx.x < 4096;           \
    const unsigned long long ts_ = __builtin_amdgcn_s_memrealtime();                        \
    __builtin_amdgcn_raw_buffer_store_b64(                                                  \
        __builtin_bit_cast(u32x2_t, ts_), census_rsrc(),                                    \
        on_ ? (int)((blockIdx.x * 16 + (k)) * 8) : (int)0x80000000, 0, 0);                  \
  } while (0)
#define WB_MARK(k) WB_MARKC(k, true)
#define WB_ABL(bit) (a.census & (bit))
#else
#define WB_MARKC(k, cond) \
  do {                    \
  } while (0)
#define WB_MARK(k) \
  do {             \
  } while (0)
#define WB_ABL(bit) 0
#endif
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t census_rsrc() {
  return __builtin_amdgcn_make_buffer_rsrc((void*)g_wbwd_census, (short)0,
                                           (int)sizeof(g_wbwd_census), 0x00020000);
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() also waits for every outstanding
// global load and store of the wave (gfx9 counts both in vmcnt), which would drain the next
// chunks' prefetches at every chunk; the compiler's own vmcnt waits cover register uses.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void tile_window(int tile, int ntx, int& ty0, int& tx0) {
  ty0 = (tile / ntx) * TS;
  tx0 = (tile - (tile / ntx) * ntx) * TS;
}

// corner k (0: (y0, x0), 1: (y0, x0+1), 2: (y0+1, x0), 3: (y0+1, x0+1)) weight, ATen's order
__device__ __forceinline__ float corner_w(const Bilinear& b, int k) {
  return k == 0 ? b.wx0 * b.wy0 : k == 1 ? b.wx1 * b.wy0 : k == 2 ? b.wx0 * b.wy1 : b.wx1 * b.wy1;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CC, bool V4>
__global__ __launch_bounds__(NT, MINWG) void warp_bwd_tile(Args a) {
  constexpr int NW = NT / 64;     // waves
  constexpr int HC = CC / 2;      // channels of a chunk per half (threads t, t + 256)
  __shared__ int cnt[NW][256];
  __shared__ int wsum[4];
  __shared__ int sst[256], sln[256];
  __shared__ float red[2][256];
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  float* xs = dyn;                                     // [channel][window pixel]
  float* gs = dyn + WN * CC;
  int2* lent = reinterpret_cast<int2*>(dyn + 2 * WN * CC);  // (window pixel, weight bits)
  const int t = threadIdx.x, wave = t >> 6, q = t & 255, hf = t >> 8;
  WB_MARK(0);
  const int H = a.H, W = a.W, C = a.C;
  const unsigned plane = (unsigned)(H * W);
  // neighbouring tiles (shared halo rows) on one XCD
  const int u = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = u % a.ntiles, rest = u / a.ntiles;
  const int cg = rest % a.ng, n = rest / a.ng;
  int ty0, tx0;
  tile_window(tile, a.ntx, ty0, tx0);
  const int wy0 = ty0 - MG, wx0 = tx0 - MG;
  const float* fl = a.flow + (size_t)(2 * n) * plane;
  for (int i = t; i < NW * 256; i += NT) (&cnt[0][0])[i] = 0;

  // ---- every flow load first: 2 window pixels per thread and the own (tile) pixel q ----
  constexpr int WPT = WN / NT;
  const int oy = ty0 + (q >> 4), ox = tx0 + (q & 15);
  const bool own = oy < H && ox < W;
  const unsigned opix = own ? (unsigned)(oy * W + ox) : 0u;
  float fu[WPT], fv[WPT];
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int wl = t + i * NT;
    const int py = min(max(wy0 + (wl >> 5), 0), H - 1), px = min(max(wx0 + (wl & 31), 0), W - 1);
    fu[i] = fl[(unsigned)(py * W + px)];
    fv[i] = fl[plane + (unsigned)(py * W + px)];
  }
  const float ou = fl[opix], ov = fl[plane + opix];
  // ---- channel chunks ----
  const int cs = cg * a.cpg, ce = min(C, cs + a.cpg);
  float gix = 0.f, giy = 0.f;
  // staging: thread t loads (row, quad) q of the window of array hf (0: x, 1: grad_out) for
  // every chunk channel
  const int sr = q >> 3, sq = q & 7;
  const int sy = wy0 + sr, sx = wx0 + 4 * sq;
  const bool rowok = sy >= 0 && sy < H;
  // buffer loads over image n of this half's array: out-of-window quads, rows outside the
  // image and channels past the group come back as zeros from the range check -- no branches,
  // so the number of loads in flight is static and the compiler waits for exactly the chunk
  // it needs (a skipped load would force vmcnt(0), draining the next chunk's prefetch)
  const int hfu = __builtin_amdgcn_readfirstlane(hf);  // wave-uniform: a scalar resource
  const float* src = (hfu ? a.gout : a.x) + (size_t)n * C * plane;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)src, (short)0, (int)((unsigned)C * plane * 4u), 0x00020000);
  constexpr unsigned kOOB = 0x80000000u;
  float* dst = hfu ? gs : xs;
  const __amdgpu_buffer_rsrc_t rsgx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.gx + (size_t)n * C * plane), (short)0, (int)((unsigned)C * plane * 4u),
      0x00020000);
  auto issue = [&](f32x4 (&v)[CC], int cb) {
#pragma unroll
    for (int c = 0; c < CC; ++c) {
      const int ch = cb + c;
      const bool ok = ch < ce && rowok && !WB_ABL(2);
      if (V4) {  // W % 4 == 0 and wx0 % 4 == 0: a quad is wholly inside or outside the row
        const unsigned off = ok && sx >= 0 && sx < W
                                 ? ((unsigned)ch * plane + (unsigned)(sy * W + sx)) * 4u
                                 : kOOB;
        v[c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned off = ok && sx + e >= 0 && sx + e < W
                                   ? ((unsigned)ch * plane + (unsigned)(sy * W + sx + e)) * 4u
                                   : kOOB;
          v[c][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0));
        }
      }
    }
  };
  // the first two chunks' loads fly during the list build
  f32x4 va[CC], vb[CC];
  issue(va, cs);
  issue(vb, cs + CC);
  lds_barrier();  // counters cleared

  // ---- list build: the 4 corners of each window pixel that land in the tile ----
  int slot[WPT][4], rank[WPT][4];
  float wt[WPT][4];
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int wl = t + i * NT;
    const int py = wy0 + (wl >> 5), px = wx0 + (wl & 31);
#pragma unroll
    for (int k = 0; k < 4; ++k) slot[i][k] = -1, wt[i][k] = 0.f, rank[i][k] = 0;
    if (py < 0 || py >= H || px < 0 || px >= W) continue;
    const Bilinear b = bilinear(src_coord(fu[i], px, W, a.halfx),
                                src_coord(fv[i], py, H, a.halfy), H, W);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cy = b.y0 + (k >> 1), cx = b.x0 + (k & 1);
      if (cy >= 0 && cy < H && cx >= 0 && cx < W && cy >= ty0 && cy < ty0 + TS && cx >= tx0 &&
          cx < tx0 + TS) {
        slot[i][k] = (cy - ty0) * TS + (cx - tx0);
        wt[i][k] = corner_w(b, k);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < WPT; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (slot[i][k] >= 0) rank[i][k] = atomicAdd(&cnt[wave][slot[i][k]], 1);
  lds_barrier();
  // exclusive scan over the 256 tile pixels (waves 0-3: thread t = tile pixel t), waves in order
  if (t < 256) {
    int len = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) len += cnt[w][t];
    int incl = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(incl, d, 64);
      if ((t & 63) >= d) incl += o;
    }
    if ((t & 63) == 63) wsum[wave] = incl;
    sln[t] = len;
    sst[t] = incl - len;  // within the wave; the waves' offsets are added below
  }
  lds_barrier();
  if (t < 256) {
    int start = sst[t];
    for (int w = 0; w < wave; ++w) start += wsum[w];
    sst[t] = start;
    int run = start;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int c = cnt[w][t];
      cnt[w][t] = run;
      run += c;
    }
  }
  lds_barrier();
#pragma unroll
  for (int i = 0; i < WPT; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (slot[i][k] >= 0)
        lent[cnt[wave][slot[i][k]] + rank[i][k]] = int2{t + i * NT, __float_as_int(wt[i][k])};
  const int start = sst[q], len = sln[q];
  WB_MARK(1);

  // ---- the own pixel p = tile pixel q (grad_flow) ----
  const int owl = ((q >> 4) + MG) * WS + (q & 15) + MG;
  Bilinear ob{};
  int cw[4];            // corner's window pixel, -1: outside the window (global), -2: masked
  unsigned cpix[4];
  const unsigned wgid = blockIdx.x;
  const __amdgpu_buffer_rsrc_t rsfar = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.far + ((size_t)wgid * NW + wave) * 256), (short)0, 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsfcnt = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.farcnt + (size_t)wgid * NW), (short)0, NW * 4, 0x00020000);
  int nfar = 0;
  if (own) ob = bilinear(src_coord(ou, ox, W, a.halfx), src_coord(ov, oy, H, a.halfy), H, W);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int cy = ob.y0 + (k >> 1), cx = ob.x0 + (k & 1);
    const bool in = own && cy >= 0 && cy < H && cx >= 0 && cx < W;
    const int ly = cy - wy0, lx = cx - wx0;
    cw[k] = !in ? -2 : (ly >= 0 && ly < WS && lx >= 0 && lx < WS) ? ly * WS + lx : -1;
    cpix[k] = in ? (unsigned)(cy * W + cx) : 0u;
    // far corner for grad_x: p lies outside the window of the tile that owns the corner
    bool far = false;
    if (in && cg == 0 && hf == 0) {
      int qy0, qx0;
      tile_window((cy / TS) * a.ntx + cx / TS, a.ntx, qy0, qx0);
      far = oy < qy0 - MG || oy >= qy0 + TS + MG || ox < qx0 - MG || ox >= qx0 + TS + MG;
    }
    // this wave's far entries go to its own region (64 lanes x 4 corners) in lane order;
    // branch-free buffer stores (a skipped store would cost the chunk loop its vmcnt waits)
    const unsigned long long fm = __builtin_amdgcn_ballot_w64(far);
    const int below = __builtin_amdgcn_mbcnt_hi((unsigned)(fm >> 32),
                                                __builtin_amdgcn_mbcnt_lo((unsigned)fm, 0u));
    const unsigned code = (((unsigned)n * plane + opix) << 2) | (unsigned)k;
    __builtin_amdgcn_raw_buffer_store_b32(code, rsfar,
                                          far ? (nfar + below) * 4 : (int)0x80000000, 0, 0);
    nfar += __builtin_popcountll(fm);
  }
  // the wave's far-entry count (lane 0; waves of the second half have none)
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)nfar, rsfcnt,
                                        (t & 63) == 0 ? wave * 4 : (int)0x80000000, 0, 0);
  lds_barrier();  // the list is complete
  // the first 12 list entries in registers for every chunk (random N(0, 2^2)-px flows give
  // ~4 per tile pixel; 12 keeps the waves with a longer list rare at 4 waves per SIMD)
  constexpr int KE = 12;
  int2 ent[KE];
#pragma unroll
  for (int j = 0; j < KE; ++j) ent[j] = j < len ? lent[start + j] : int2{0, 0};
  WB_MARK(2);

  // one chunk: its registers -> LDS, the chunk two ahead into the same registers, arithmetic
  // census bit 16: sub-phase marks of chunks 2 and 3 (slots 3-8, 9-14) instead of chunk ends
  auto process = [&](f32x4 (&v)[CC], int cb) {
    [[maybe_unused]] const int ci = (cb - cs) / CC;
#define WB_SUB(j) WB_MARKC((ci == 2 ? 3 : 9) + (j), WB_ABL(16) && (ci == 2 || ci == 3))
    WB_SUB(0);
    lds_barrier();  // the previous chunk's readers are done
    WB_SUB(1);
#pragma unroll
    for (int c = 0; c < CC; ++c)  // planar [channel][window pixel]: conflict-free 16-B writes
      *reinterpret_cast<f32x4*>(dst + c * WN + sr * WS + 4 * sq) = v[c];
    lds_barrier();
    WB_MARKC(3 + min(ci, 11), !WB_ABL(16));
    WB_SUB(2);
    // unconditional: past the group's last channel the loads come back as zeros from the range
    // check -- a skipped issue would leave the compiler's vmcnt count unsure at the next chunk,
    // and it would then wait for the chunk after the one it needs as well
    issue(v, cb + 2 * CC);
    WB_SUB(3);
    // grad_x of tile pixel q, this half's channels of the chunk
    const int c0 = hf * HC;
    float acc[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) acc[c] = 0.f;
    const int lenx = WB_ABL(4) ? 0 : len;
    // the register entries without a branch: every LDS read of them is in flight at once
    // (an `if (j < len)` per entry serialised one LDS round trip per entry); entries past the
    // list are {0, 0} and leave the sum as it is (a select, not a multiply by a zero weight)
    float gv[KE][HC];
#pragma unroll
    for (int j = 0; j < KE; ++j)
#pragma unroll
      for (int c = 0; c < HC; ++c) gv[j][c] = gs[(c0 + c) * WN + ent[j].x];
#pragma unroll
    for (int j = 0; j < KE; ++j) {
      const float w = __int_as_float(ent[j].y);
#pragma unroll
      for (int c = 0; c < HC; ++c) {
        const float s = acc[c] + gv[j][c] * w;
        acc[c] = j < lenx ? s : acc[c];
      }
    }
    for (int e = start + KE; e < start + lenx; ++e) {
      const int2 en = lent[e];
      const float w = __int_as_float(en.y);
#pragma unroll
      for (int c = 0; c < HC; ++c) acc[c] += gs[(c0 + c) * WN + en.x] * w;
    }
#pragma unroll
    for (int c = 0; c < HC; ++c) {  // branch-free: off-image pixels / past-group channels drop
      const int ch = cb + c0 + c;
      const unsigned off = own && ch < ce && !WB_ABL(8)
                               ? ((unsigned)ch * plane + opix) * 4u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[c]), rsgx, (int)off, 0, 0);
    }
    WB_SUB(4);
    if (own) {
      // grad_flow of p over this half's channels (x at the corners, masked outside the image)
      // (corners outside the window: zero here, added after the chunk loop)
      float r[4][HC];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < HC; ++c) r[k][c] = cw[k] >= 0 ? xs[(c0 + c) * WN + max(cw[k], 0)] : 0.f;
#pragma unroll
      for (int c = 0; c < HC; ++c) {
        const float go = gs[(c0 + c) * WN + owl];
        gix += go * ((r[1][c] - r[0][c]) * ob.wy0 + (r[3][c] - r[2][c]) * ob.wy1);
        giy += go * ((r[2][c] - r[0][c]) * ob.wx0 + (r[3][c] - r[1][c]) * ob.wx1);
      }
    }
    WB_SUB(5);
#undef WB_SUB
  };
  for (int cb = cs; cb < ce; cb += 2 * CC) {  // an odd chunk count's last chunk is all zeros
    process(va, cb);
    process(vb, cb + CC);
  }
  // pixels with a corner outside the window (|flow| beyond the margin): their grad_flow over
  // this group's channels again from global memory, exactly (the loop above left such corners
  // at zero, so the difference is added).  A wave-uniform branch, after the loop.
  const bool outw = cw[0] == -1 || cw[1] == -1 || cw[2] == -1 || cw[3] == -1;
  if (__builtin_amdgcn_ballot_w64(outw) != 0 && outw && hf == 0) {
    float dx = 0.f, dy = 0.f;
    for (int c = cs; c < ce; ++c) {
      const float* xp = a.x + ((size_t)n * C + c) * plane;
      float rf[4], rz[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        rf[k] = cw[k] == -2 ? 0.f : xp[cpix[k]];
        rz[k] = cw[k] == -1 ? 0.f : rf[k];
      }
      const float go = a.gout[((size_t)n * C + c) * plane + opix];
      dx += go * (((rf[1] - rf[0]) * ob.wy0 + (rf[3] - rf[2]) * ob.wy1) -
                  ((rz[1] - rz[0]) * ob.wy0 + (rz[3] - rz[2]) * ob.wy1));
      dy += go * (((rf[2] - rf[0]) * ob.wx0 + (rf[3] - rf[1]) * ob.wx1) -
                  ((rz[2] - rz[0]) * ob.wx0 + (rz[3] - rz[1]) * ob.wx1));
    }
    gix += dx;
    giy += dy;
  }
  WB_MARK(15);
  // the two halves' grad_flow partials, in half order
  if (hf == 1) red[0][q] = gix, red[1][q] = giy;
  lds_barrier();
  if (hf == 1) return;
  gix += red[0][q];
  giy += red[1][q];

  // ---- grad_flow: direct, or this group's partial for warp_bwd_finish ----
  if (!own) return;
  if (a.ng == 1) {
    const float mx = (float)(W - 1) / 2.f, my = (float)(H - 1) / 2.f;
    a.gflow[(size_t)(2 * n) * plane + opix] = (gix * mx) / a.halfx;
    a.gflow[(size_t)(2 * n + 1) * plane + opix] = (giy * my) / a.halfy;
  } else {
    float* pp = a.part + ((size_t)(cg * a.B + n) * 2) * plane;
    pp[opix] = gix;
    pp[plane + opix] = giy;
  }
}

// grad_flow from the channel groups' partials (fixed group order), then the far corners' grad_x
// contributions (fp32 atomics onto warp_bwd_tile's plain stores).
__global__ __launch_bounds__(256) void warp_bwd_finish(Args a) {
  const int H = a.H, W = a.W, C = a.C;
  const unsigned plane = (unsigned)(H * W);
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (a.ng > 1 && gid < (unsigned)a.B * plane) {
    const unsigned n = gid / plane, pix = gid - n * plane;
    float sx = 0.f, sy = 0.f;
    int g = 0;
    for (; g + 8 <= a.ng; g += 8) {  // 16 loads in flight, then the fixed-order sum
      float vx[8], vy[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* q = a.part + ((size_t)((g + j) * a.B + n) * 2) * plane;
        vx[j] = q[pix];
        vy[j] = q[plane + pix];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sx += vx[j], sy += vy[j];
    }
    for (; g < a.ng; ++g) {
      const float* q = a.part + ((size_t)(g * a.B + n) * 2) * plane;
      sx += q[pix];
      sy += q[plane + pix];
    }
    const float mx = (float)(W - 1) / 2.f, my = (float)(H - 1) / 2.f;
    a.gflow[(size_t)(2 * n) * plane + pix] = (sx * mx) / a.halfx;
    a.gflow[(size_t)(2 * n + 1) * plane + pix] = (sy * my) / a.halfy;
  }
  // far corners: block b takes the 8 wave lists of tile workgroups b, b + gridDim.x, ...; 32
  // threads per list, every count loaded at once (a per-list load -> loop chain made this
  // kernel's tail)
  const int nl = NT / 64, v = threadIdx.x >> 5, tl = threadIdx.x & 31;
  for (int wg = blockIdx.x; wg < a.nwg && v < nl; wg += gridDim.x) {
    const unsigned nf = a.farcnt[(size_t)wg * nl + v];
    const unsigned* lst = a.far + ((size_t)wg * nl + v) * 256;
    for (unsigned e = tl; e < nf; e += 32) {
      const unsigned code = lst[e];
      const int k = (int)(code & 3u);
      const unsigned gp = code >> 2, nn = gp / plane, pix = gp - nn * plane;
      const int py = (int)(pix / (unsigned)W), px = (int)pix - py * W;
      const float* fn = a.flow + (size_t)(2 * nn) * plane;
      const Bilinear b = bilinear(src_coord(fn[pix], px, W, a.halfx),
                                  src_coord(fn[plane + pix], py, H, a.halfy), H, W);
      const int cy = b.y0 + (k >> 1), cx = b.x0 + (k & 1);
      const float w = corner_w(b, k);
      const unsigned q = (unsigned)(cy * W + cx);
      for (int c0 = 0; c0 < C; c0 += 8) {  // 8 loads in flight, then their atomics
        float g[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          g[i] = c0 + i < C ? a.gout[((size_t)nn * C + c0 + i) * plane + pix] : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (c0 + i < C) atomicAdd(a.gx + ((size_t)nn * C + c0 + i) * plane + q, g[i] * w);
      }
    }
  }
}

struct Plan {
  int ntx, ntiles, ng, cpg, nwg;
  size_t part_off, far_off, cnt_off, bytes;
};

static bool plan(int B, int C, int H, int W, Plan* p) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return false;
  if ((size_t)B * H * W * 4 >= (1ull << 31) || (size_t)B * C * H * W >= (1ull << 31)) return false;
  // the tile kernel's buffer resources cover one image in 32-bit byte counts
  if ((size_t)C * H * W * 4 >= (1ull << 31)) return false;
  p->ntx = (W + TS - 1) / TS;
  p->ntiles = p->ntx * ((H + TS - 1) / TS);
  const long long tiles = (long long)B * p->ntiles;
  // channel groups: at most 512 workgroups (two per CU: one round), at least 4 channels each
  const int cc = CC;
  long long ng = 512 / tiles;
  const long long maxg = (C + cc - 1) / cc;
  if (ng > maxg) ng = maxg;
  if (ng < 1) ng = 1;
  if (const int k = debug_knob("warp_bwd_groups", 0)) ng = k;
  int cpg = (int)((C + ng - 1) / ng);
  cpg = (cpg + cc - 1) / cc * cc;
  p->cpg = cpg;
  p->ng = (C + cpg - 1) / cpg;
  if (tiles * p->ng >= (1ll << 31)) return false;
  size_t off = kHead;
  p->part_off = off;
  if (p->ng > 1) off += (size_t)p->ng * B * 2 * H * W * 4;
  p->nwg = (int)(tiles * p->ng);
  p->far_off = off;
  off += (size_t)p->nwg * (NT / 64) * 256 * 4;
  p->cnt_off = off;
  off += (size_t)p->nwg * (NT / 64) * 4;
  p->bytes = off;
  return true;
}

}  // namespace wbwd

extern "C" __attribute__((visibility("default"))) int pwc_debug_wbwd_census(void* dst, int n) {
  if (dst == nullptr) {
    static unsigned long long zeros[4096 * 16];
    return hipMemcpyToSymbol(HIP_SYMBOL(wbwd::g_wbwd_census), zeros, sizeof(zeros)) == hipSuccess;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(wbwd::g_wbwd_census),
                             sizeof(unsigned long long) * (size_t)n) == hipSuccess;
}

// The tile path's choice (warp_backward_tiles_f32): W >= 56 by default (config 5's l3 and l4;
// at l3 23.4 vs 24.6 us for the list-gather path since round 5's branch-free chunk loop,
// profiles/r05u_warp_bwd_tile_chunks.txt); knob warp_bwd_tiles = 0 never, 2 always.
static bool tiles_wanted(int W) {
  const int mode = debug_knob("warp_bwd_tiles", 1);
  return !(mode == 0 || (mode == 1 && W < 56));
}

// 0 whenever the tile path would decline, so the narrow levels pass no workspace
size_t warp_backward_workspace_size(int B, int C, int H, int W) {
  wbwd::Plan p;
  return tiles_wanted(W) && wbwd::plan(B, C, H, W, &p) ? p.bytes : 0;
}

// hipErrorNotSupported: no plan (or no workspace) -- the caller runs warp_backward_f32.
hipError_t warp_backward_tiles_f32(const void* x, const void* flow, const void* gout, void* gx,
                                   void* gflow, int B, int C, int H, int W, void* ws,
                                   size_t ws_bytes, hipStream_t stream) {
  using namespace wbwd;
  // measured (B=8 384x448, profiles/r03c_warp_bwd_tiles.txt, r05u_*): l4 (96 x 112) 34.9 ->
  // 26.4 us, l3 24.6 -> 23.4; l2..l0 slower (the tile workgroup's list build + per-chunk
  // barriers are a fixed latency that the multi-kernel path does not pay) -- W >= 56 by
  // default; knob warp_bwd_tiles = 0 never, 2 always (tests)
  if (!tiles_wanted(W)) return hipErrorNotSupported;
  Plan p;
  if (!plan(B, C, H, W, &p) || ws == nullptr || ws_bytes < p.bytes) return hipErrorNotSupported;
  char* w = (char*)ws;
  hipError_t e = hipSuccess;
  Args a;
  a.x = (const float*)x;
  a.flow = (const float*)flow;
  a.gout = (const float*)gout;
  a.gx = (float*)gx;
  a.gflow = (float*)gflow;
  a.B = B, a.C = C, a.H = H, a.W = W;
  a.halfx = (float)((W - 1.0) / 2.0);
  a.halfy = (float)((H - 1.0) / 2.0);
  a.ntx = p.ntx, a.ntiles = p.ntiles, a.ng = p.ng, a.cpg = p.cpg;
  a.part = (float*)(w + p.part_off);
  a.far = (unsigned*)(w + p.far_off);
  a.farcnt = (unsigned*)(w + p.cnt_off);
  a.nwg = p.nwg;
  a.census = debug_knob("warp_bwd_census", 0);
  const unsigned grid = (unsigned)(B * p.ntiles * p.ng);
  constexpr size_t lds = (size_t)2 * WN * CC * sizeof(float) + (size_t)MAXE * sizeof(int2);
  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
  for (const void* f : {reinterpret_cast<const void*>(&warp_bwd_tile<CC, true>),
                        reinterpret_cast<const void*>(&warp_bwd_tile<CC, false>)}) {
    e = lds_limit(f, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (W % 4 == 0)
    hipLaunchKernelGGL((warp_bwd_tile<CC, true>), dim3(grid), dim3(NT), lds, stream, a);
  else
    hipLaunchKernelGGL((warp_bwd_tile<CC, false>), dim3(grid), dim3(NT), lds, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  unsigned fin = (unsigned)(((size_t)B * H * W + 255) / 256);
  if (fin < (unsigned)p.nwg) fin = (unsigned)p.nwg < 1024u ? (unsigned)p.nwg : 1024u;
  hipLaunchKernelGGL(warp_bwd_finish, dim3(fin), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace pwc
