// warp.hip — bilinear flow warp (WarpingLayer) forward / backward for gfx950.
//
// Semantics: WarpingLayer.forward, modules.py:31-42 of daigo0927/PWC-Net_pytorch:
//   flow_n = flow / ((size-1)/2);  grid = get_grid(x) + flow_n  (utils.py:3-8: linspace(-1,1))
//   out = F.grid_sample(x, grid)   with torch==0.4.0 semantics (requirements.txt:62):
//   bilinear, zeros padding, align_corners=True: ix = ((gx + 1) / 2) * (W - 1).
// The reference builds the base grid on the host and copies it to the device on every call
// (modules.py:40) and runs ~5 elementwise kernels + a permute before grid_sampler_2d; here the
// whole normalisation chain is recomputed in registers, in the same fp32 operation order
// (no FMA contraction), so sample coordinates match the reference chain.
// Backward follows ATen grid_sampler_2d_backward: grad_x by fp32 atomics (scatter), grad of
// the sample point by the bilinear derivative; d(ix)/d(u) = ((W-1)/2) / ((W-1)/2) = 1.
#include <cstdlib>

#include "warp_sample.cuh"

namespace pwc {

// One thread per output pixel and CB channels (grid.y splits the channels).  32-bit indexing
// (the launcher checks B*C*H*W < 2^31).
template <typename T, int CB>
struct WarpGroup {  // one channel group's raw corner values
  float r[CB][4];
};

template <typename T, int CB>
__device__ __forceinline__ void warp_load(WarpGroup<T, CB>& g, const T* __restrict__ x,
                                          unsigned n, int C, unsigned plane, int c0, int W,
                                          const Pairs& kp, const Corners& kc) {
  if (W >= 2) {
    float lo[CB][2], hi[CB][2];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = min(c0 + i, C - 1);
      const T* p = x + ((unsigned)(n * C + c)) * plane;
      load_pair(p + kp.i0, lo[i][0], hi[i][0]);
      load_pair(p + kp.i1, lo[i][1], hi[i][1]);
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      g.r[i][0] = kp.l_lo ? lo[i][0] : hi[i][0];
      g.r[i][1] = kp.r_lo ? lo[i][0] : hi[i][0];
      g.r[i][2] = kp.l_lo ? lo[i][1] : hi[i][1];
      g.r[i][3] = kp.r_lo ? lo[i][1] : hi[i][1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int c = min(c0 + i, C - 1);
      const T* p = x + ((unsigned)(n * C + c)) * plane;
      g.r[i][0] = to_f32(p[kc.i00]);
      g.r[i][1] = to_f32(p[kc.i01]);
      g.r[i][2] = to_f32(p[kc.i10]);
      g.r[i][3] = to_f32(p[kc.i11]);
    }
  }
}

// model.py:78: F.upsample(flow, scale_factor=2, mode='bilinear') * 2 under torch 0.4
// (align_corners=False: ATen upsample_bilinear2d, area_pixel_compute_source_index with scale
// 1/2, source index clamped at 0, right/bottom tap clamped to the last row/column), the same
// fp32 operation order as ATen's kernel, then the exact *2.  `f` is one [h][w] plane.
struct UpTap {
  int i00, i01, i10, i11;
  float l0y, l1y, l0x, l1x;
};

__device__ __forceinline__ UpTap up2_taps(int oy, int ox, int h, int w) {
#pragma clang fp contract(off)
  const float sy = fmaxf(0.5f * ((float)oy + 0.5f) - 0.5f, 0.f);
  const float sx = fmaxf(0.5f * ((float)ox + 0.5f) - 0.5f, 0.f);
  const int y0 = (int)sy, x0 = (int)sx;
  const int yp = y0 < h - 1 ? 1 : 0, xp = x0 < w - 1 ? 1 : 0;
  UpTap t;
  t.l1y = sy - (float)y0;
  t.l0y = 1.f - t.l1y;
  t.l1x = sx - (float)x0;
  t.l0x = 1.f - t.l1x;
  t.i00 = y0 * w + x0;
  t.i01 = y0 * w + x0 + xp;
  t.i10 = (y0 + yp) * w + x0;
  t.i11 = (y0 + yp) * w + x0 + xp;
  return t;
}

template <typename T>
__device__ __forceinline__ float up2_value(const T* __restrict__ f, const UpTap& t) {
#pragma clang fp contract(off)
  const float v = t.l0y * (t.l0x * to_f32(f[t.i00]) + t.l1x * to_f32(f[t.i01])) +
                  t.l1y * (t.l0x * to_f32(f[t.i10]) + t.l1x * to_f32(f[t.i11]));
  return v * 2.f;
}

// One thread per output pixel; grid.y splits the channels into slices of NG groups of CB
// channels, and a thread walks its slice's groups with the next group's gathers in flight
// while the current one is blended and stored.  32-bit indexing (the launcher checks
// B*C*H*W < 2^31).
// UP: `flow` is the coarse [B][2][H/2][W/2] flow of the previous level, upsampled in registers
// (model.py:78); the channel-slice-0 threads also write the upsampled flow to `flow_up` when
// it is not null (model.py:89/91 concatenates it).
// The body of one (pixel block bx, channel slice cy) of warp_fwd_kernel; the grouped launch
// (warp_fwd_group) runs it on each problem's own block range.
template <typename T, int CB, int NG, bool UP>
__device__ __forceinline__ void warp_fwd_block(const T* __restrict__ x,
                                               const T* __restrict__ flow, T* __restrict__ out,
                                               int B, int C, int H, int W, float halfx,
                                               float halfy, T* __restrict__ flow_up,
                                               unsigned bx, unsigned cy) {
  const unsigned plane = (unsigned)(H * W);
  const unsigned idx = bx * 256u + threadIdx.x;
  if (idx >= (unsigned)B * plane) return;
  const unsigned n = idx / plane;
  const unsigned pix = idx - n * plane;
  const int py = (int)(pix / (unsigned)W);
  const int px = (int)pix - py * W;
  float u, v;
  if constexpr (UP) {
    const int h = H >> 1, w = W >> 1;
    const UpTap tp = up2_taps(py, px, h, w);
    const unsigned cplane = (unsigned)(h * w);
    u = up2_value(flow + (2 * n + 0) * cplane, tp);
    v = up2_value(flow + (2 * n + 1) * cplane, tp);
    if constexpr (sizeof(T) == 4) {  // round like a stored fp32 flow, then use it
      if (flow_up != nullptr && cy == 0) {
        flow_up[(2 * n + 0) * plane + pix] = u;
        flow_up[(2 * n + 1) * plane + pix] = v;
      }
    } else {  // storage rounding first: the reference warps with the stored upsampled flow
      const T ut = from_f32<T>(u), vt = from_f32<T>(v);
      if (flow_up != nullptr && cy == 0) {
        flow_up[(2 * n + 0) * plane + pix] = ut;
        flow_up[(2 * n + 1) * plane + pix] = vt;
      }
      u = to_f32(ut);
      v = to_f32(vt);
    }
  } else {
    u = to_f32(flow[(2 * n + 0) * plane + pix]);
    v = to_f32(flow[(2 * n + 1) * plane + pix]);
  }
  const float ix = src_coord(u, px, W, halfx);
  const float iy = src_coord(v, py, H, halfy);
  const Bilinear b = bilinear(ix, iy, H, W);
  const float w00 = b.wx0 * b.wy0, w01 = b.wx1 * b.wy0;  // feed fma operands: not fusable
  const float w10 = b.wx0 * b.wy1, w11 = b.wx1 * b.wy1;
  const Pairs kp = pairs(b, H, W);
  const Corners kc = corners(b, H, W);
  const float m00 = kc.m00, m01 = kc.m01, m10 = kc.m10, m11 = kc.m11;
  const int cs = (int)cy * CB * NG;
  WarpGroup<T, CB> g[2];
  warp_load(g[0], x, n, C, plane, cs, W, kp, kc);
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    const int c0 = cs + gi * CB;
    if (gi + 1 < NG) warp_load(g[(gi + 1) & 1], x, n, C, plane, c0 + CB, W, kp, kc);
    const WarpGroup<T, CB>& cur = g[gi & 1];
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      float acc = 0.f;
      acc = fmaf(masked(cur.r[i][0], m00), w00, acc);
      acc = fmaf(masked(cur.r[i][1], m01), w01, acc);
      acc = fmaf(masked(cur.r[i][2], m10), w10, acc);
      acc = fmaf(masked(cur.r[i][3], m11), w11, acc);
      if (c0 + i < C) {
        T* o = out + ((unsigned)(n * C + c0 + i)) * plane + pix;
        if constexpr (sizeof(T) == 4)
          st_out1(reinterpret_cast<float*>(o), acc);
        else
          *o = from_f32<T>(acc);
      }
    }
  }
}

template <typename T, int CB, int NG, bool XCD, bool UP = false>
__global__ __launch_bounds__(256) void warp_fwd_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ flow,
                                                       T* __restrict__ out, int B, int C, int H,
                                                       int W, float halfx, float halfy,
                                                       T* __restrict__ flow_up = nullptr) {
  // XCD: consecutive pixel blocks (which gather overlapping source rows) share an L2
  const unsigned bx = XCD ? (unsigned)xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  warp_fwd_block<T, CB, NG, UP>(x, flow, out, B, C, H, W, halfx, halfy, flow_up, bx,
                                blockIdx.y);
}

// Up to kWarpGroupMax independent warps in ONE launch (pwc_warp_forward_group): problem i owns
// the flat blocks [start[i], start[i+1]), laid out as its (channel slice, pixel block) grid, so
// a launch gap and each small grid's tail are shared.  The XCD remap runs over the flat grid:
// consecutive pixel blocks of one problem still share an L2.
constexpr int kWarpGroupMax = 4;
template <typename T>
struct WarpGroupArgs {
  const T* x[kWarpGroupMax];
  const T* flow[kWarpGroupMax];
  T* out[kWarpGroupMax];
  int B[kWarpGroupMax], C[kWarpGroupMax], H[kWarpGroupMax], W[kWarpGroupMax];
  float halfx[kWarpGroupMax], halfy[kWarpGroupMax];
  unsigned gx[kWarpGroupMax];
  unsigned start[kWarpGroupMax + 1];
  int n;
};

template <typename T, int CB, int NG>
__global__ __launch_bounds__(256) void warp_fwd_group(WarpGroupArgs<T> a) {
  const unsigned g = (unsigned)xcd_remap(blockIdx.x, gridDim.x);
  // scalar selects (uniform per workgroup), no dynamic indexing of the argument struct
  const T *x = a.x[0], *flow = a.flow[0];
  T* out = a.out[0];
  int B = a.B[0], C = a.C[0], H = a.H[0], W = a.W[0];
  float hx = a.halfx[0], hy = a.halfy[0];
  unsigned gx = a.gx[0], s0 = 0;
#pragma unroll
  for (int i = 1; i < kWarpGroupMax; ++i) {
    if (i < a.n && g >= a.start[i]) {
      x = a.x[i], flow = a.flow[i], out = a.out[i];
      B = a.B[i], C = a.C[i], H = a.H[i], W = a.W[i];
      hx = a.halfx[i], hy = a.halfy[i], gx = a.gx[i], s0 = a.start[i];
    }
  }
  const unsigned local = g - s0;
  const unsigned cy = local / gx;
  warp_fwd_block<T, CB, NG, false>(x, flow, out, B, C, H, W, hx, hy, nullptr, local - cy * gx,
                                   cy);
}

// ---- backward without a scatter over HBM (fp32) ----
// grad_x as a gather: a workgroup owns a TH x TW tile of grad_x (one pixel per thread) for
// CC channels.  Every output pixel within M of the tile (its candidate window) recomputes its
// sample (the forward's chain) and keeps the corners that fall in the tile; a counting sort in
// LDS turns these into one list of (source pixel, bilinear weight) per tile pixel.  MODE 4:
// each wave counts into its own row of slot counters, so a list holds wave 0's entries, then
// wave 1's, ... each wave's in (candidate round, corner, lane) order -- a fixed order with no
// sort (an LDS atomic orders one instruction's lanes by lane).  MODE 0: one shared counter row
// (arrival order) and an insertion sort by source pixel.  Per channel a thread then sums
// gO * weight over its list in registers (MODE 2: buffer loads at scalar channel offsets, two
// entries in flight) and writes its grad_x element with a plain coalesced store: every
// element is written once (no memset, no atomics, fixed summation order).  A corner whose pixel lies
// outside the corner tile's candidate window (flow beyond ~M pixels) is left to
// warp_bwd_flow, which adds it with a global atomic after this kernel (ATen's
// grid_sampler_2d_backward adds every corner that way).
constexpr int kBwdM = 8;

__device__ __forceinline__ bool bwd_in_window(int py, int px, int cy, int cx, int th, int tw) {
  const int ty0 = (cy / th) * th, tx0 = (cx / tw) * tw;
  return py >= ty0 - kBwdM && py < ty0 + th + kBwdM && px >= tx0 - kBwdM &&
         px < tx0 + tw + kBwdM;
}

// WHOLE > 0: the candidates are every pixel of the image (H * W <= WHOLE): no sample can miss its
// tile, so no corner is left to a far pass (l2-sized images; the 8-px margin window of an 8 x 32
// tile holds 1152 candidates there, more than the 672 pixels of the image).
template <int TW, int CC, int MODE, int WHOLE = 0>
__device__ __forceinline__ void warp_bwd_gx_body(const float* __restrict__ flow,
                                                 const float* __restrict__ gout,
                                                 float* __restrict__ gx, int C, int H, int W,
                                                 float halfx, float halfy, int ntx, int bx,
                                                 int by, int bz) {
  constexpr int TH = 256 / TW, M = kBwdM;
  constexpr int WW = TW + 2 * M, NCAND = WHOLE ? WHOLE : (TH + 2 * M) * WW;
  constexpr int K = (NCAND + 255) / 256;
  constexpr int MAXL = 4 * NCAND;
  constexpr bool WAVEC = (MODE & 4) != 0;  // per-wave slot counters: list order fixed, no sort
  __shared__ int cnt[WAVEC ? 4 * 256 : 256];
  __shared__ int wsum[4];
  __shared__ unsigned lpix[MAXL];
  __shared__ float lw[MAXL];
  const int t = threadIdx.x;
  const int tx = bx % ntx, ty = bx / ntx;
  const int n = by, c0 = bz * CC;
  const int y0 = ty * TH, x0 = tx * TW;
  const unsigned plane = (unsigned)(H * W);
  const int cw = WAVEC ? (t >> 6) * 256 : 0;  // this wave's counter row
  cnt[t] = 0;
  if (WAVEC) cnt[256 + t] = cnt[512 + t] = cnt[768 + t] = 0;
  int slot[K][4];
  float wt[K][4];
  unsigned pix[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int cand = t + j * 256;
    const int py = WHOLE ? cand / W : y0 - M + cand / WW;
    const int px = WHOLE ? cand - (cand / W) * W : x0 - M + cand % WW;
    pix[j] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) slot[j][k] = -1, wt[j][k] = 0.f;
    if ((WHOLE ? cand >= H * W : cand >= NCAND) || py < 0 || py >= H || px < 0 || px >= W)
      continue;
    pix[j] = (unsigned)(py * W + px);
    const float u = flow[(2 * n + 0) * plane + pix[j]];
    const float v = flow[(2 * n + 1) * plane + pix[j]];
    const Bilinear b = bilinear(src_coord(u, px, W, halfx), src_coord(v, py, H, halfy), H, W);
    const float w[4] = {b.wx0 * b.wy0, b.wx1 * b.wy0, b.wx0 * b.wy1, b.wx1 * b.wy1};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cy = b.y0 + (k >> 1), cx = b.x0 + (k & 1);
      if (cy >= 0 && cy < H && cx >= 0 && cx < W && cy >= y0 && cy < y0 + TH && cx >= x0 &&
          cx < x0 + TW) {
        slot[j][k] = (cy - y0) * TW + (cx - x0);
        wt[j][k] = w[k];
      }
    }
  }
  __syncthreads();
  // counting sort by tile pixel
  int pos[K][4];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      pos[j][k] = slot[j][k] >= 0 ? atomicAdd(&cnt[cw + slot[j][k]], 1) : 0;
  __syncthreads();
  int wc[4] = {cnt[t], 0, 0, 0};
  if (WAVEC) wc[1] = cnt[256 + t], wc[2] = cnt[512 + t], wc[3] = cnt[768 + t];
  const int len = wc[0] + wc[1] + wc[2] + wc[3];
  int incl = len;  // inclusive scan: within the wave, then over the 4 waves
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d, 64);
    if ((t & 63) >= d) incl += o;
  }
  if ((t & 63) == 63) wsum[t >> 6] = incl;
  __syncthreads();
  for (int w = 0; w < (t >> 6); ++w) incl += wsum[w];
  const int start = incl - len;
  cnt[t] = start;
  if (WAVEC) {
    cnt[256 + t] = start + wc[0];
    cnt[512 + t] = start + wc[0] + wc[1];
    cnt[768 + t] = start + wc[0] + wc[1] + wc[2];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (slot[j][k] >= 0) {
        const int e = cnt[cw + slot[j][k]] + pos[j][k];
        lpix[e] = pix[j];
        lw[e] = wt[j][k];
      }
  __syncthreads();
  // my list, sorted by source pixel (insertion sort: a few entries)
  for (int i = start + 1; i < (WAVEC ? 0 : start + len); ++i) {
    const unsigned pk = lpix[i];
    const float wk = lw[i];
    int j = i - 1;
    while (j >= start && lpix[j] > pk) {
      lpix[j + 1] = lpix[j];
      lw[j + 1] = lw[j];
      --j;
    }
    lpix[j + 1] = pk;
    lw[j + 1] = wk;
  }
  const int yy = y0 + t / TW, xx = x0 + t % TW;
  if (yy >= H || xx >= W) return;
  const int cn = min(CC, C - c0);
  const float* go = gout + ((unsigned)(n * C + c0)) * plane;
  float acc[CC];
#pragma unroll
  for (int i = 0; i < CC; ++i) acc[i] = 0.f;
  int e0 = start;
  if (MODE & 2) {
    // channel planes at scalar offsets of one buffer resource, two list entries in flight
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)go, (short)0, (int)((unsigned)cn * plane * 4u), 0x00020000);
    for (; e0 + 1 < start + len; e0 += 2) {
      const unsigned p0 = lpix[e0], p1 = lpix[e0 + 1];
      const float w0 = lw[e0], w1 = lw[e0 + 1];
      float g0[CC], g1[CC];
#pragma unroll
      for (int i = 0; i < CC; ++i) {
        g0[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rs, (int)(p0 * 4u), (int)(i * plane * 4u), 0));
        g1[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rs, (int)(p1 * 4u), (int)(i * plane * 4u), 0));
      }
#pragma unroll
      for (int i = 0; i < CC; ++i) acc[i] += g0[i] * w0;
#pragma unroll
      for (int i = 0; i < CC; ++i) acc[i] += g1[i] * w1;
    }
  }
  for (int e = e0; e < start + len; ++e) {
    const unsigned p = lpix[e];
    const float w = lw[e];
    float g[CC];
#pragma unroll
    for (int i = 0; i < CC; ++i) g[i] = go[(unsigned)min(i, cn - 1) * plane + p];
#pragma unroll
    for (int i = 0; i < CC; ++i) acc[i] += g[i] * w;
  }
  float* o = gx + ((unsigned)(n * C + c0)) * plane + (unsigned)(yy * W + xx);
#pragma unroll
  for (int i = 0; i < CC; ++i)
    if (i < cn) o[(unsigned)i * plane] = acc[i];
}

template <int TW, int CC, int MODE = 0>
__global__ __launch_bounds__(256) void warp_bwd_gx_lists(const float* __restrict__ flow,
                                                         const float* __restrict__ gout,
                                                         float* __restrict__ gx, int C, int H,
                                                         int W, float halfx, float halfy,
                                                         int ntx) {
  warp_bwd_gx_body<TW, CC, MODE>(flow, gout, gx, C, H, W, halfx, halfy, ntx, blockIdx.x,
                                 blockIdx.y, blockIdx.z);
}

// grad_flow per pixel + the corners warp_bwd_gx_lists left out.  A block holds 256 / NG
// pixels x NG channel groups (lanes of a wave = consecutive pixels of one group); group g
// takes channels [g*cpg, (g+1)*cpg) and the NG partial sums meet in LDS in group order
// (deterministic; NG = 1 is ATen's channel loop order).
// NOFAR: the far corners are left to warp_bwd_far (a merged launch cannot order its atomics
// after the grad_x tiles' plain stores)
template <int CB, int NG, bool PAIRS, bool NOFAR = false>
__device__ __forceinline__ void warp_bwd_flow_body(const float* __restrict__ x,
                                                   const float* __restrict__ flow,
                                                   const float* __restrict__ gout,
                                                   float* __restrict__ gx,
                                                   float* __restrict__ gflow, int B, int C,
                                                   int H, int W, float halfx, float halfy,
                                                   int cpg, int th, int tw, unsigned blk) {
  constexpr int PX = 256 / NG;
  __shared__ float red[NG > 1 ? 2 * 256 : 1];
  const unsigned plane = (unsigned)(H * W);
  const int grp = threadIdx.x / PX, pl = threadIdx.x - grp * PX;
  const unsigned idx = blk * (unsigned)PX + pl;
  const bool live = idx < (unsigned)B * plane;
  if (NG == 1 && !live) return;
  const unsigned idc = live ? idx : 0u;  // idle lanes of the last block sample pixel 0
  const unsigned n = idc / plane;
  const unsigned pix = idc - n * plane;
  const int py = (int)(pix / (unsigned)W);
  const int px = (int)pix - py * W;
  const float u = flow[(2 * n + 0) * plane + pix];
  const float v = flow[(2 * n + 1) * plane + pix];
  const float ix = src_coord(u, px, W, halfx);
  const float iy = src_coord(v, py, H, halfy);
  const Bilinear b = bilinear(ix, iy, H, W);
  const Corners k = corners(b, H, W);
  const Pairs kp = pairs(b, H, W);
  const float w00 = b.wx0 * b.wy0, w01 = b.wx1 * b.wy0;
  const float w10 = b.wx0 * b.wy1, w11 = b.wx1 * b.wy1;
  // corners outside their tile's candidate window (rare: |flow| beyond ~kBwdM)
  const bool o00 = k.m00 != 0.f && !bwd_in_window(py, px, b.y0, b.x0, th, tw);
  const bool o01 = k.m01 != 0.f && !bwd_in_window(py, px, b.y0, b.x0 + 1, th, tw);
  const bool o10 = k.m10 != 0.f && !bwd_in_window(py, px, b.y0 + 1, b.x0, th, tw);
  const bool o11 = k.m11 != 0.f && !bwd_in_window(py, px, b.y0 + 1, b.x0 + 1, th, tw);
  const bool outl = !NOFAR && (o00 || o01 || o10 || o11);
  float gix = 0.f, giy = 0.f;
  const int cs = grp * cpg, ce = live ? min(C, cs + cpg) : cs;
  for (int c0 = cs; c0 < ce; c0 += CB) {
    float r[CB][4], go[CB];
    if (PAIRS && W >= 2) {  // both corners of a sample row from one 8-byte load
      WarpGroup<float, CB> wg;
      warp_load(wg, x, n, C, plane, c0, W, kp, k);
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        r[i][0] = masked(wg.r[i][0], k.m00);
        r[i][1] = masked(wg.r[i][1], k.m01);
        r[i][2] = masked(wg.r[i][2], k.m10);
        r[i][3] = masked(wg.r[i][3], k.m11);
        const int c = min(c0 + i, ce - 1);
        go[i] = (c0 + i < ce) ? gout[((unsigned)(n * C + c)) * plane + pix] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = min(c0 + i, ce - 1);
        const float* p = x + ((unsigned)(n * C + c)) * plane;
        r[i][0] = masked(p[k.i00], k.m00);
        r[i][1] = masked(p[k.i01], k.m01);
        r[i][2] = masked(p[k.i10], k.m10);
        r[i][3] = masked(p[k.i11], k.m11);
        go[i] = (c0 + i < ce) ? gout[((unsigned)(n * C + c)) * plane + pix] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      if (c0 + i >= ce) break;
      if (outl) {
        float* q = gx + ((unsigned)(n * C + c0 + i)) * plane;
        if (o00) atomicAdd(q + k.i00, go[i] * w00);
        if (o01) atomicAdd(q + k.i01, go[i] * w01);
        if (o10) atomicAdd(q + k.i10, go[i] * w10);
        if (o11) atomicAdd(q + k.i11, go[i] * w11);
      }
      gix += go[i] * ((r[i][1] - r[i][0]) * b.wy0 + (r[i][3] - r[i][2]) * b.wy1);
      giy += go[i] * ((r[i][2] - r[i][0]) * b.wx0 + (r[i][3] - r[i][1]) * b.wx1);
    }
  }
  if (NG > 1) {
    red[threadIdx.x] = gix;
    red[256 + threadIdx.x] = giy;
    __syncthreads();
    if (grp != 0 || !live) return;
    for (int j = 1; j < NG; ++j) {
      gix += red[j * PX + pl];
      giy += red[256 + j * PX + pl];
    }
  }
  const float mx = (float)(W - 1) / 2.f, my = (float)(H - 1) / 2.f;
  gflow[(2 * n + 0) * plane + pix] = (gix * mx) / halfx;
  gflow[(2 * n + 1) * plane + pix] = (giy * my) / halfy;
}

template <int CB, int NG, bool PAIRS = false>
__global__ __launch_bounds__(256) void warp_bwd_flow(const float* __restrict__ x,
                                                     const float* __restrict__ flow,
                                                     const float* __restrict__ gout,
                                                     float* __restrict__ gx,
                                                     float* __restrict__ gflow, int B, int C,
                                                     int H, int W, float halfx, float halfy,
                                                     int cpg, int th, int tw) {
  warp_bwd_flow_body<CB, NG, PAIRS>(x, flow, gout, gx, gflow, B, C, H, W, halfx, halfy, cpg, th,
                                    tw, (unsigned)xcd_remap(blockIdx.x, gridDim.x));
}

// Images that fit one grad_x tile (l0 / l1): the two kernels in ONE launch, side by side --
// the first ngx workgroups build the lists and gather grad_x, the rest compute grad_flow.
// With the tile covering the whole image every in-image corner lies in its tile's window, so
// there are no far corners and no atomics, and the two halves are independent.
template <int TW, int CC, int MODE, int CB, int NG, bool PAIRS>
__global__ __launch_bounds__(256) void warp_bwd_small(const float* __restrict__ x,
                                                      const float* __restrict__ flow,
                                                      const float* __restrict__ gout,
                                                      float* __restrict__ gx,
                                                      float* __restrict__ gflow, int B, int C,
                                                      int H, int W, float halfx, float halfy,
                                                      int cpg, int ngx, int ncg) {
  const int b = blockIdx.x;
  if (b < ngx) {
    warp_bwd_gx_body<TW, CC, MODE>(flow, gout, gx, C, H, W, halfx, halfy, 1, 0, b / ncg,
                                   b % ncg);
  } else {
    const int nf = (int)gridDim.x - ngx;
    warp_bwd_flow_body<CB, NG, PAIRS>(x, flow, gout, gx, gflow, B, C, H, W, halfx, halfy, cpg,
                                      256 / TW, TW, (unsigned)xcd_remap(b - ngx, nf));
  }
}

// Multi-tile images: grad_x tiles and grad_flow side by side in one launch (both are gather
// kernels far below the chip's memory rate, so together they fill it better), the far corners
// in a small pass after it (warp_bwd_far).
template <int TW, int CC, int MODE, int CB, int NG, bool PAIRS, int WHOLE = 0>
__global__ __launch_bounds__(256) void warp_bwd_merged(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ gx,
                                                       float* __restrict__ gflow, int B, int C,
                                                       int H, int W, float halfx, float halfy,
                                                       int cpg, int ntx, int ntiles, int ngx) {
  const int b = blockIdx.x;
  if (b < ngx) {
    const int rest = b / ntiles;
    warp_bwd_gx_body<TW, CC, MODE, WHOLE>(flow, gout, gx, C, H, W, halfx, halfy, ntx,
                                          b % ntiles, rest % B, rest / B);
  } else {
    const int nf = (int)gridDim.x - ngx;
    warp_bwd_flow_body<CB, NG, PAIRS, true>(x, flow, gout, gx, gflow, B, C, H, W, halfx, halfy,
                                            cpg, 256 / TW, TW, (unsigned)xcd_remap(b - ngx, nf));
  }
}

// The corners warp_bwd_merged's tiles left out (sample point beyond ~kBwdM pixels of its
// corner's tile): one thread per pixel, global atomics as ATen's scatter, after the tiles.
__global__ __launch_bounds__(256) void warp_bwd_far(const float* __restrict__ flow,
                                                    const float* __restrict__ gout,
                                                    float* __restrict__ gx, int B, int C, int H,
                                                    int W, float halfx, float halfy, int th,
                                                    int tw) {
  // grid.y = groups of 8 channels: a far pixel's channels are spread over workgroups, and each
  // thread issues its 8 grad_out loads before its atomics (a load -> atomic chain per channel
  // made this pass's tail: up to 50 us at C = 96, one thread doing every channel)
  const unsigned plane = (unsigned)(H * W);
  const unsigned idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= (unsigned)B * plane) return;
  const unsigned n = idx / plane, pix = idx - n * plane;
  const int py = (int)(pix / (unsigned)W), px = (int)pix - py * W;
  const float u = flow[(2 * n + 0) * plane + pix];
  const float v = flow[(2 * n + 1) * plane + pix];
  const Bilinear b = bilinear(src_coord(u, px, W, halfx), src_coord(v, py, H, halfy), H, W);
  const Corners k = corners(b, H, W);
  const bool o00 = k.m00 != 0.f && !bwd_in_window(py, px, b.y0, b.x0, th, tw);
  const bool o01 = k.m01 != 0.f && !bwd_in_window(py, px, b.y0, b.x0 + 1, th, tw);
  const bool o10 = k.m10 != 0.f && !bwd_in_window(py, px, b.y0 + 1, b.x0, th, tw);
  const bool o11 = k.m11 != 0.f && !bwd_in_window(py, px, b.y0 + 1, b.x0 + 1, th, tw);
  if (!(o00 || o01 || o10 || o11)) return;
  const float w00 = b.wx0 * b.wy0, w01 = b.wx1 * b.wy0;
  const float w10 = b.wx0 * b.wy1, w11 = b.wx1 * b.wy1;
  const int c0 = (int)blockIdx.y * 8;
  float g[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    g[i] = c0 + i < C ? gout[((unsigned)(n * C + c0 + i)) * plane + pix] : 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (c0 + i >= C) break;
    float* q = gx + ((unsigned)(n * C + c0 + i)) * plane;
    if (o00) atomicAdd(q + k.i00, g[i] * w00);
    if (o01) atomicAdd(q + k.i01, g[i] * w01);
    if (o10) atomicAdd(q + k.i10, g[i] * w10);
    if (o11) atomicAdd(q + k.i11, g[i] * w11);
  }
}


template <typename T>
hipError_t warp_forward_win_t(const void*, const void*, void*, int, int, int, int, hipStream_t);

template <typename T>
hipError_t warp_forward_t(const void* x, const void* flow, void* out, int B, int C, int H,
                          int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0 || C == 0) return hipSuccess;
  if (npix * (size_t)(C > 2 ? C : 2) >= (1ull << 31)) return hipErrorInvalidValue;
  // large grids: the LDS-window kernel (warp_fwd_win.hip) where it takes the shape (knob
  // warp_win = 2: any grid, for tests and measurement)
  if (npix >= 16384 || debug_knob("warp_win", 1) == 2) {
    const hipError_t e = warp_forward_win_t<T>(x, flow, out, B, C, H, W, stream);
    if (e != hipErrorNotSupported) return e;
  }
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  const unsigned gx = (unsigned)((npix + 255) / 256);
#define PWC_WARP_LAUNCH(CB, NG, XCD)                                                          \
  hipLaunchKernelGGL((warp_fwd_kernel<T, CB, NG, XCD>),                                       \
                     dim3(gx, (unsigned)((C + CB * NG - 1) / (CB * NG))), dim3(256), 0, stream, \
                     (const T*)x, (const T*)flow, (T*)out, B, C, H, W, halfx, halfy)
  // fp16 storage on large grids: a thread walks 4 groups of 2 channels (its gathers of the next
  // group in flight while one is blended) -- config-4 Sintel l4 34.0 -> 28.0 us, l3 18.9 ->
  // 16.2, l2 9.2 -> 8.4 (profiles/r02e_warp_fp16_cfg.txt); fp32 on large grids: 8 channels per
  // thread (config-2 l3 5.57 -> 5.32 us, l4 equal; l2 stays at 4: 3.52 against 3.68 --
  // profiles/r02e_warp_fp32_cfg.txt).  Other shapes measured in round 2 were removed.
  // (if constexpr: a variant the storage type never takes is not instantiated)
  if (npix < 16384)
    PWC_WARP_LAUNCH(4, 1, true);
  else if constexpr (sizeof(T) == 2)
    PWC_WARP_LAUNCH(2, 4, true);
  else
    PWC_WARP_LAUNCH(8, 1, true);
#undef PWC_WARP_LAUNCH
  return hipGetLastError();
}

// Independent warps in one launch, kWarpGroupMax problems per launch (pwc_warp_forward_group).
// The channels-per-thread choice follows the largest problem (warp_forward_t's large-grid
// choice); each output element is the same fmaf chain as a separate call, bit for bit.
template <typename T>
hipError_t warp_forward_group_t(const WarpProblem* probs, int count, hipStream_t stream) {
  for (int i0 = 0; i0 < count; i0 += kWarpGroupMax) {
    WarpGroupArgs<T> a{};
    size_t big = 0;
    int n = 0;
    unsigned total = 0;
    bool cb8 = false;
    for (int i = i0; i < count && i < i0 + kWarpGroupMax; ++i) {
      const size_t npix = (size_t)probs[i].B * probs[i].H * probs[i].W;
      if (npix > big) big = npix;
    }
    // fp32 large grids: 8 channels per thread; fp16 large grids: 4 groups of 2; else 4 x 1
    cb8 = big >= 16384;
    const int cpt = cb8 ? 8 : 4;
    for (int i = i0; i < count && i < i0 + kWarpGroupMax; ++i) {
      const WarpProblem& q = probs[i];
      const size_t npix = (size_t)q.B * q.H * q.W;
      if (npix == 0 || q.C == 0) continue;
      if (npix * (size_t)(q.C > 2 ? q.C : 2) >= (1ull << 31)) return hipErrorInvalidValue;
      const unsigned gx = (unsigned)((npix + 255) / 256);
      const unsigned gy = (unsigned)((q.C + cpt - 1) / cpt);
      if ((unsigned long long)total + (unsigned long long)gx * gy >= (1ull << 31))
        return hipErrorInvalidValue;
      a.x[n] = (const T*)q.x;
      a.flow[n] = (const T*)q.flow;
      a.out[n] = (T*)q.out;
      a.B[n] = q.B, a.C[n] = q.C, a.H[n] = q.H, a.W[n] = q.W;
      a.halfx[n] = (float)((q.W - 1.0) / 2.0);
      a.halfy[n] = (float)((q.H - 1.0) / 2.0);
      a.gx[n] = gx;
      a.start[n] = total;
      total += gx * gy;
      ++n;
    }
    if (n == 0) continue;
    a.start[n] = total;
    a.n = n;
    if (!cb8)
      hipLaunchKernelGGL((warp_fwd_group<T, 4, 1>), dim3(total), dim3(256), 0, stream, a);
    else if constexpr (sizeof(T) == 4)
      hipLaunchKernelGGL((warp_fwd_group<T, 8, 1>), dim3(total), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((warp_fwd_group<T, 2, 4>), dim3(total), dim3(256), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
template hipError_t warp_forward_group_t<float>(const WarpProblem*, int, hipStream_t);
template hipError_t warp_forward_group_t<__half>(const WarpProblem*, int, hipStream_t);
template hipError_t warp_forward_group_t<__hip_bfloat16>(const WarpProblem*, int, hipStream_t);

hipError_t warp_backward_f32(const void* x, const void* flow, const void* gout, void* gx,
                             void* gflow, int B, int C, int H, int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0) return hipSuccess;
  if (npix * (size_t)(C > 2 ? C : 2) >= (1ull << 31)) return hipErrorInvalidValue;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  // Round 2's measured choices (profiles/r02d_bwd_knobs.txt, r02e_warp_bwd_modes.txt,
  // r02e_warp_bwd_small.txt); the other tile shapes, list-build modes, dword-corner flow loads
  // and the ATen-shaped atomic scatter were removed from the library in round 3.
  // wide rows (l4: 96 x 112 at 384 x 448) take 16 x 16 tiles of 16 channels and two channel
  // groups in warp_bwd_flow; narrower images 8 x 32 tiles of 8 channels
  const bool wide = W >= 96;
  // channel groups for grids with few pixels (the coarse levels): ~64K threads or 16 groups
  int ng = 1;
  while (ng < 16 && npix * ng < 65536 && C >= 8 * ng * 2) ng *= 2;
  if (C > 0) {
    // images inside one grad_x tile (l0 6 x 7 in 8 x 32, l1 12 x 14 in 16 x 16): grad_x and
    // grad_flow in one merged launch (warp_bwd_small; knob warp_bwd_small=0: the general path)
    const int tws = (H <= 8 && W <= 32) ? 32 : (H <= 16 && W <= 16) ? 16 : 0;
    if (tws && ng == 16 && debug_knob("warp_bwd_small", 1)) {
      const int cc = tws == 32 ? 8 : 16, ncg = (C + cc - 1) / cc, ngx = B * ncg;
      const int cpg = (C + ng - 1) / ng;
      const unsigned nflow = (unsigned)((npix * ng + 255) / 256);
      const dim3 grid((unsigned)ngx + nflow);
      if (tws == 32)
        hipLaunchKernelGGL((warp_bwd_small<32, 8, 6, 8, 16, true>), grid, dim3(256), 0, stream,
                           (const float*)x, (const float*)flow, (const float*)gout, (float*)gx,
                           (float*)gflow, B, C, H, W, halfx, halfy, cpg, ngx, ncg);
      else
        hipLaunchKernelGGL((warp_bwd_small<16, 16, 6, 8, 16, true>), grid, dim3(256), 0, stream,
                           (const float*)x, (const float*)flow, (const float*)gout, (float*)gx,
                           (float*)gflow, B, C, H, W, halfx, halfy, cpg, ngx, ncg);
      return hipGetLastError();
    }
  }
  if (wide && ng == 1 && C >= 32) ng = 2;
  const int cpg = (C + ng - 1) / ng;
  const unsigned nflow = (unsigned)((npix * ng + 255) / 256);
  if (C > 0 && debug_knob("warp_bwd_merge", 1)) {
    // grad_x tiles and grad_flow in one launch + the far-corner pass, where both halves fit
    // about one round of the chip together: l2 (456 workgroups) 17.5 -> 13.1 us, l3 (720, 16 x
    // 16 tiles from 48-px rows) 23.3 -> 21.7; l4 (1344) measured slower
    const bool t16 = W >= 48;
    const int TWm = t16 ? 16 : 32, CCm = t16 ? 16 : 8, THm = 256 / TWm;
    const int ntx = (W + TWm - 1) / TWm, nty = (H + THm - 1) / THm, ntiles = ntx * nty;
    const int ngx = ntiles * B * ((C + CCm - 1) / CCm);
    if ((long long)ngx + nflow <= 800) {
      bool done = false;
      // images of <= 768 pixels: every pixel is a candidate of every tile -- no far corners,
      // no far pass (config-5 l2: 12.4 -> 9.4 us, training step 228.4 -> 225.6 us on one box;
      // knob warp_bwd_whole=0: the margin windows + warp_bwd_far)
      const bool whole = (long long)H * W <= 768 && debug_knob("warp_bwd_whole", 1) != 0;
#define PWC_MERGED(T16, TW_, CC_, NG_, WH_)                                                     \
  if (!done && t16 == T16 && ng == NG_ && whole == (WH_ != 0)) {                                \
    hipLaunchKernelGGL((warp_bwd_merged<TW_, CC_, 6, 8, NG_, true, WH_>),                       \
                       dim3((unsigned)ngx + nflow), dim3(256), 0, stream, (const float*)x,      \
                       (const float*)flow, (const float*)gout, (float*)gx, (float*)gflow, B, C, \
                       H, W, halfx, halfy, cpg, ntx, ntiles, ngx);                              \
    done = true;                                                                                \
  }
      PWC_MERGED(false, 32, 8, 8, 0)
      PWC_MERGED(false, 32, 8, 4, 0)
      PWC_MERGED(false, 32, 8, 2, 0)
      PWC_MERGED(true, 16, 16, 4, 0)
      PWC_MERGED(true, 16, 16, 2, 0)
      PWC_MERGED(true, 16, 16, 1, 0)
      PWC_MERGED(false, 32, 8, 8, 768)
      PWC_MERGED(false, 32, 8, 4, 768)
      PWC_MERGED(false, 32, 8, 2, 768)
      PWC_MERGED(true, 16, 16, 4, 768)
      PWC_MERGED(true, 16, 16, 2, 768)
      PWC_MERGED(true, 16, 16, 1, 768)
#undef PWC_MERGED
      if (done && whole) return hipGetLastError();
      if (done) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(warp_bwd_far,
                           dim3((unsigned)((npix + 255) / 256), (unsigned)((C + 7) / 8)),
                           dim3(256), 0, stream, (const float*)flow, (const float*)gout,
                           (float*)gx, B, C, H, W, halfx, halfy, THm, TWm);
        return hipGetLastError();
      }
    }
  }
  // two launches: grad_x tiles (list build with per-wave slot counters, buffer-load gathers two
  // entries deep), then grad_flow with the far corners
  const int TW = wide ? 16 : 32, th = 256 / TW;
  if (C > 0) {
    const int ntx = (W + TW - 1) / TW, nty = (H + th - 1) / th;
    if (wide)
      hipLaunchKernelGGL((warp_bwd_gx_lists<16, 16, 6>),
                         dim3((unsigned)(ntx * nty), (unsigned)B, (unsigned)((C + 15) / 16)),
                         dim3(256), 0, stream, (const float*)flow, (const float*)gout, (float*)gx,
                         C, H, W, halfx, halfy, ntx);
    else
      hipLaunchKernelGGL((warp_bwd_gx_lists<32, 8, 6>),
                         dim3((unsigned)(ntx * nty), (unsigned)B, (unsigned)((C + 7) / 8)),
                         dim3(256), 0, stream, (const float*)flow, (const float*)gout, (float*)gx,
                         C, H, W, halfx, halfy, ntx);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const unsigned blocks = nflow;
#define PWC_FLOW(NGV)                                                                          \
  if (ng == NGV) {                                                                             \
    hipLaunchKernelGGL((warp_bwd_flow<8, NGV, true>), dim3(blocks), dim3(256), 0, stream,      \
                       (const float*)x, (const float*)flow, (const float*)gout, (float*)gx,    \
                       (float*)gflow, B, C, H, W, halfx, halfy, cpg, th, TW);                  \
    return hipGetLastError();                                                                  \
  }
  PWC_FLOW(1)
  PWC_FLOW(2)
  PWC_FLOW(4)
  PWC_FLOW(8)
  PWC_FLOW(16)
#undef PWC_FLOW
  return hipErrorNotSupported;
}

// model.py:78 + :80 in one launch: x2_warp = warp(x2, up2(flow_coarse) * 2), flow_up written
// when not null.  H and W are the fine (x2) sizes, both even.
template <typename T>
hipError_t upsample_warp_forward_t(const void* x, const void* flow_coarse, void* flow_up,
                                   void* out, int B, int C, int H, int W, hipStream_t stream) {
  const size_t npix = (size_t)B * H * W;
  if (npix == 0) return hipSuccess;
  if ((H | W) & 1) return hipErrorInvalidValue;
  if (npix * (size_t)(C > 2 ? C : 2) >= (1ull << 31)) return hipErrorInvalidValue;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
  const unsigned gx = (unsigned)((npix + 255) / 256);
  constexpr int CB = 4;
  const unsigned gy = C > 0 ? (unsigned)((C + CB - 1) / CB) : 1u;
  hipLaunchKernelGGL((warp_fwd_kernel<T, CB, 1, true, true>), dim3(gx, gy), dim3(256), 0, stream,
                     (const T*)x, (const T*)flow_coarse, (T*)out, B, C, H, W, halfx, halfy,
                     (T*)flow_up);
  return hipGetLastError();
}

// Backward of model.py:78 (adjoint of up2 * 2, fp32): grad_coarse[n,ch,Y,X] = 2 * sum of
// grad_up[n,ch,oy,ox] * tap weight over the fine pixels whose taps reach (Y,X) -- as a gather
// over the fine rows/columns within 2 of (2Y, 2X) (each coarse pixel is tapped by at most 4
// fine rows x 4 fine columns), fixed order: no atomics, deterministic.
__global__ __launch_bounds__(256) void flow_up2_bwd_kernel(const float* __restrict__ gup,
                                                           float* __restrict__ gc, int B,
                                                           int H, int W) {
  const int h = H >> 1, w = W >> 1;
  const unsigned idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= (unsigned)(B * 2 * h * w)) return;
  const int X = (int)(idx % (unsigned)w);
  const int Y = (int)((idx / (unsigned)w) % (unsigned)h);
  const unsigned nc = idx / (unsigned)(h * w);
  const float* g = gup + nc * (unsigned)(H * W);
  const int tgt = Y * w + X;
  float acc = 0.f;
  for (int oy = max(0, 2 * Y - 2); oy <= min(H - 1, 2 * Y + 2); ++oy)
    for (int ox = max(0, 2 * X - 2); ox <= min(W - 1, 2 * X + 2); ++ox) {
      const UpTap t = up2_taps(oy, ox, h, w);
      float wt = 0.f;  // ATen adds the four tap weights separately (taps may coincide)
      if (t.i00 == tgt) wt += t.l0y * t.l0x;
      if (t.i01 == tgt) wt += t.l0y * t.l1x;
      if (t.i10 == tgt) wt += t.l1y * t.l0x;
      if (t.i11 == tgt) wt += t.l1y * t.l1x;
      if (wt != 0.f) acc += (2.f * g[oy * W + ox]) * wt;
    }
  gc[idx] = acc;
}

hipError_t flow_up2_backward_f32(const void* grad_up, void* grad_coarse, int B, int H, int W,
                                 hipStream_t stream) {
  const size_t n = (size_t)B * 2 * (H / 2) * (W / 2);
  if (n == 0) return hipSuccess;
  if ((H | W) & 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(flow_up2_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const float*)grad_up, (float*)grad_coarse, B, H, W);
  return hipGetLastError();
}

template hipError_t upsample_warp_forward_t<float>(const void*, const void*, void*, void*, int,
                                                   int, int, int, hipStream_t);
template hipError_t upsample_warp_forward_t<__half>(const void*, const void*, void*, void*, int,
                                                    int, int, int, hipStream_t);
template hipError_t upsample_warp_forward_t<__hip_bfloat16>(const void*, const void*, void*,
                                                            void*, int, int, int, int,
                                                            hipStream_t);

template hipError_t warp_forward_t<float>(const void*, const void*, void*, int, int, int, int,
                                          hipStream_t);
template hipError_t warp_forward_t<__half>(const void*, const void*, void*, int, int, int, int,
                                           hipStream_t);
template hipError_t warp_forward_t<__hip_bfloat16>(const void*, const void*, void*, int, int,
                                                   int, int, hipStream_t);

}  // namespace pwc
