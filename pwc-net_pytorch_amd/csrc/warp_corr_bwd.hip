// warp_corr_bwd.hip — the backward of one coarse pyramid level (model.py:80-83 with model.py:24's
// Correlation(pad 9 (or 8), k 1, md = pad, s1 1, s2 2)) in ONE launch, for images a workgroup
// holds whole (the l0 / l1 levels: <= 256 pixels):
//   g1  = d corr / d x1         correlation_cuda_kernel.cu:108-198 (Correlation_backward_input1)
//   gw  = d corr / d x2_warp    cu:200-290 (Correlation_backward_input2), plus the gradient that
//                               arrives on x2_warp itself (WarpCorrelationFunction.backward)
//   gx2, gflow = WarpingLayer backward of gw (modules.py:31-42 -> ATen grid_sampler_2d_backward,
//                bilinear, zeros, align_corners=True, through utils.py:3-8's grid chain)
// gw stays in LDS: the two-launch path (pwc_corr_backward + pwc_warp_backward_ws) writes it to
// HBM and reads it back, and its two dependent launches are each a latency chain at these sizes
// (l0 9.6 + 5.4 us, l1 11.5 + 7.2 us in the config-5 step, profiles/r05_final_train_step.json).
//
// One workgroup = (image n, a group of 4 NQ channels, NQ = 4 / 2 / 1 as many as fit one thread
// per (channel quad, pixel) in 256); thread t = (quad t / HW, pixel t % HW).  All of the image's
// 81 cost-volume gradient planes (<= 81 KB) and the group's x1 / x2_warp / x2 channels
// (pixel-major float4 quads) are staged in LDS at once, then per pixel and quad:
//   g1[c][p]  = sum_d gO[d][p] * x2w[c][p + d] / C                      (d ascending, 81 terms)
//   gw[c][p]  = sum_d gO[d][p - d] * x1[c][p - d] / C  (+ g_x2w[c][p])  (zero outside the image)
// then the grid_sample backward inside the image: grad_x2[c][q] = sum over q's (source pixel,
// weight) list of w * gw[c][p] -- the lists come from a counting sort with per-wave counters
// (fixed order, as warp_bwd_tile) -- and the group's share of grad_flow[p] (x2 at p's four
// corners from LDS).  Every corner of an in-image sample lies in the image, so there are no far
// corners.  grad_flow sums over all channel groups: each workgroup stores its partial (agent-
// scope stores, written through to the coherent level) and bumps image n's counter; the
// workgroup that arrives last adds the partials in group order (deterministic: the result does
// not depend on arrival order) and resets the counter, so the counters are zero after every
// call (the caller zeroes them once).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "warp_sample.cuh"

namespace pwc {
namespace cbwd {

constexpr int NT = 512;    // threads: up to three displacement-row groups of (quad, pixel)
constexpr int MAXP = 256;  // quads x pixels per group (one thread each)
constexpr int D = 9;       // displacements per axis
constexpr int ND = D * D;  // cost-volume planes
constexpr int NW = NT / 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const float* f1;
  const float* x2;
  const float* flow;
  const float* x2w;
  const float* gc;    // [B][81][H][W]
  const float* gxw;   // gradient arriving on x2_warp, or null
  float* g1;
  float* gx2;
  float* gflow;
  float* part;        // [ng][B][2][HW] grad_flow partials
  unsigned* cnt;      // [B] arrival counters (zero before and after)
  int B, C, H, W, ng;
  float halfx, halfy, divisor;
  float inv_hw, inv_w, inv_wp, inv_pp, inv_qhw;  // 1/d for qdiv
  int ntg;  // displacement-row groups (thread groups splitting the 9 rows)
  int abl;  // measurement only (knob wcb_abl): 1 no correlation sums, 2 no lists / grad_x2,
            // 4 no grad_flow reduction, 8 gO loads out of range (zeros), 16 no border clear,
            // 32 no partial stores / arrival
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// x / d for 0 <= x < 2^20 from a host-computed float 1/d (exact: (x + 0.5) / d lies at least
// 0.5/d from an integer, beyond the float error; a runtime integer division is ~30 VALU)
__device__ __forceinline__ int qdiv(int x, float inv) { return (int)(((float)x + 0.5f) * inv); }

// LDS floats: gO pixel-major (81 per pixel) with 8 zero guard pixels each side, x1 / x2_warp
// as NQ zero-bordered planes of float4 quads ((H + 16) x (W + 16): every displacement of an
// in-image pixel lands inside), x2 / gw as NQ plain quad planes, the other displacement-row
// groups' partial sums ([2 groups][2][NQ HW] quads), per-wave slot counters, list starts /
// lengths, list pixels and weights (4 per source pixel), a [2][NT] reduction buffer, the
// arrival broadcast
__host__ __device__ constexpr int lds_floats(int h, int w, int nq) {
  return ((ND * (h * w + 16) + 3) & ~3) + 2 * 4 * nq * (h + 16) * (w + 16) + 2 * 4 * nq * h * w +
         16 * nq * h * w + NW * h * w + 2 * h * w + 2 * 4 * h * w + 2 * NT + 4;
}

// V4: gO copied in 16-B loads (HW % 4 == 0); NGO: gO loads per thread (all in flight at once;
// those past the end read zeros from the range check); NQ: channel quads per workgroup.  Thread
// t = (displacement-row group t / (NQ HW), quad, pixel): the ntg <= 3 groups each sum a third
// (or half) of the 9 displacement rows -- the sums' dependent chain is the kernel's longest
// phase, and one (quad, pixel) per thread leaves most SIMDs with one wave -- and group 0 adds the
// others' partial sums in group order, then carries on alone.
// (one or two waves per SIMD: registers for a whole displacement row's reads in flight -- at
// the default occupancy target the scheduler waited for each term's reads in turn)
template <bool V4, int NGO, int NQ>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 2)))
void warp_corr_bwd_small(Args a) {
  constexpr int CGW = 4 * NQ;  // channels per workgroup
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int H = a.H, W = a.W, C = a.C, HW = H * W;
  const int t = threadIdx.x, wave = t >> 6;
  const int u = xcd_remap(blockIdx.x, gridDim.x);  // an image's groups on one XCD (shared gO)
  const int n = u / a.ng, g = u - n * a.ng, c0 = g * CGW;
  const int Wp = W + 16, PP = (H + 16) * Wp;      // bordered quad plane
  float* go = lds;                                 // [(HW + 16) pixels][81], guard 8 + 8
  f32x4* f1p = reinterpret_cast<f32x4*>(lds + ((ND * (HW + 16) + 3) & ~3));  // [NQ][PP]
  f32x4* f2p = f1p + NQ * PP;
  f32x4* xq = f2p + NQ * PP;                       // [NQ][HW]
  f32x4* gwq = xq + NQ * HW;
  f32x4* comb = gwq + NQ * HW;                     // [2 groups][2][NQ * HW]
  int* cnt = reinterpret_cast<int*>(comb + 4 * NQ * HW);  // [NW][HW]
  int* sst = cnt + NW * HW;                          // list start / length per pixel
  int* sln = sst + HW;
  int* lp = sln + HW;                                // [4 * HW] source pixel of a list entry
  float* lw = reinterpret_cast<float*>(lp + 4 * HW);
  float* red = lw + 4 * HW;                          // [2][NT]
  int* arrival = reinterpret_cast<int*>(red + 2 * NT);
  const unsigned plane = (unsigned)HW;
  const int qhw = NQ * HW;
  const int tg = qdiv(t, a.inv_qhw), rq = t - tg * qhw;  // displacement-row group, (quad, pixel)
  const int k = qdiv(rq, a.inv_hw);                     // this thread's channel quad
  const bool act = tg < a.ntg;  // sums a share of the displacements
  const bool own = t < qhw;     // group 0: the (quad, pixel) owner
  const bool pix0 = t < HW;     // group 0, quad 0: one thread per pixel (lists, scan)
  const int p = act ? rq - k * HW : 0;
  const int kq = act ? k * HW : 0;  // quad plane offsets in LDS
  const int kp = act ? k * PP : 0;
  const int py = qdiv(p, a.inv_w), px = p - py * W;

  // ---- every load first: flow, the quad's channels, the gradient on x2_warp, gO ----
  const float* fl = a.flow + (size_t)(2 * n) * plane;
  const float fu = fl[p], fv = fl[plane + p];
  const size_t cb = ((size_t)n * C + c0 + 4 * (own ? k : 0)) * plane;
  float v1[4], v2[4], vx[4], ve[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v1[c] = a.f1[cb + (size_t)c * plane + p];
    v2[c] = a.x2w[cb + (size_t)c * plane + p];
    vx[c] = a.x2[cb + (size_t)c * plane + p];
    ve[c] = a.gxw ? a.gxw[cb + (size_t)c * plane + p] : 0.f;
  }
  // gO of image n: 81 * HW contiguous floats, copied flat ([d][pixel])
  const unsigned gbytes = (unsigned)(ND * HW) * 4u;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.gc + (size_t)n * ND * plane), (short)0, (int)gbytes, 0x00020000);
  constexpr int GV = V4 ? 4 : 1;
  typedef typename std::conditional<V4, f32x4, float>::type GT;
  GT gq[NGO];
#pragma unroll
  for (int j = 0; j < NGO; ++j) {
    const unsigned off = (a.abl & 8) ? 0x80000000u : (unsigned)((j * NT + t) * GV) * 4u;
    if constexpr (V4)
      gq[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)off, 0, 0));
    else
      gq[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, (int)off, 0, 0));
  }
  for (int i = t; i < NW * HW; i += NT) cnt[i] = 0;
  // the bordered planes' zero border (the interior is written below: no overlap) and gO's
  // guard pixels
  for (int i = t; i < ((a.abl & 16) ? 0 : NQ * PP); i += NT) {
    const int r = i - qdiv(i, a.inv_pp) * PP, ry = qdiv(r, a.inv_wp);
    const int yy = ry - 8, xx = r - ry * Wp - 8;
    if (yy < 0 || yy >= H || xx < 0 || xx >= W)
      f1p[i] = f2p[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int i = t; i < 16 * ND; i += NT) go[i < 8 * ND ? i : HW * ND + i] = 0.f;
  if (own) {
    f1p[kp + (py + 8) * Wp + px + 8] = f32x4{v1[0], v1[1], v1[2], v1[3]};
    f2p[kp + (py + 8) * Wp + px + 8] = f32x4{v2[0], v2[1], v2[2], v2[3]};
    xq[kq + p] = f32x4{vx[0], vx[1], vx[2], vx[3]};
  }
  // gO transposed to pixel-major (81 floats per pixel: an odd dword stride, so a wave's
  // pixels fall on distinct banks)
#pragma unroll
  for (int j = 0; j < NGO; ++j) {
    const int i = (j * NT + t) * GV;
    if constexpr (V4) {
      int d = qdiv(i, a.inv_hw), q = i - d * HW;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (i + e < ND * HW) go[(q + 8) * ND + d] = gq[j][e];
        if (++q == HW) q = 0, ++d;
      }
    } else {
      const int d = qdiv(i, a.inv_hw), q = i - d * HW;
      if (i < ND * HW) go[(q + 8) * ND + d] = gq[j];
    }
  }
  // the sample of this pixel (warp.hip's chain) and its in-image corners
  const Bilinear b = bilinear(src_coord(fu, px, W, a.halfx), src_coord(fv, py, H, a.halfy), H, W);
  const float wk[4] = {b.wx0 * b.wy0, b.wx1 * b.wy0, b.wx0 * b.wy1, b.wx1 * b.wy1};
  int slot[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cy = b.y0 + (j >> 1), cx = b.x0 + (j & 1);
    slot[j] = own && cy >= 0 && cy < H && cx >= 0 && cx < W ? cy * W + cx : -1;
  }
  lds_barrier();

  // ---- the correlation gradients, 81 displacements each ----
  // branch-free: every read is issued (at p when the displacement leaves the image, with a
  // zero gradient weight), so a displacement row's 36 LDS reads are in flight together (a
  // branch per displacement serialised one LDS round trip per term)
  //   g1: x2_warp from the bordered plane (zero outside the image) times p's own gO[d]
  //   gw: x1 from the bordered plane times gO[d] at p - d; when the row p - d leaves the image
  //       the gO reads stay on p's row (finite values against the border's zeros), and a
  //       column overflow reads the neighbouring row or a guard pixel (likewise finite)
  // so every term is added (outside ones are exact zeros) and all offsets inside a
  // displacement row are compile-time: a row's 36 LDS reads go out back to back
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  const int tjlo = act ? (tg * D + a.ntg / 2) / a.ntg : 0;
  const int tjhi = act ? ((tg + 1) * D + a.ntg / 2) / a.ntg : 0;
#pragma unroll 1
  for (int tj = tjlo; tj < ((a.abl & 1) ? tjlo : tjhi); ++tj) {
    const int dy = 2 * tj - 8;
    const bool r2 = py - dy >= 0 && py - dy < H;
    const int dyr = r2 ? dy : 0;
    const float* A1 = go + (p + 8) * ND + tj * D;                    // + ti
    const f32x4* B1 = f2p + kp + (py + 8 + dy) * Wp + px;             // + 2 ti
    const float* A2 = go + (p - dyr * W) * ND + tj * D + 8;           // + (8 - ti) * 161
    const f32x4* B2 = f1p + kp + (py + 8 - dy) * Wp + px;             // + 16 - 2 ti
    float a1[D], a2[D];
    f32x4 b1[D], b2[D];
#pragma unroll
    for (int ti = 0; ti < D; ++ti) {
      a1[ti] = A1[ti];
      b1[ti] = B1[2 * ti];
      a2[ti] = A2[(8 - ti) * (2 * ND - 1)];
      b2[ti] = B2[16 - 2 * ti];
    }
#pragma unroll
    for (int ti = 0; ti < D; ++ti) {
      s1 += a1[ti] * b1[ti];
      s2 += a2[ti] * b2[ti];
    }
  }
  // the other groups' shares, added in group order
  if (act && tg > 0) {
    comb[(2 * (tg - 1)) * qhw + rq] = s1;
    comb[(2 * (tg - 1) + 1) * qhw + rq] = s2;
  }
  lds_barrier();
  if (own) {
    for (int g2 = 1; g2 < a.ntg; ++g2) {
      s1 += comb[(2 * (g2 - 1)) * qhw + t];
      s2 += comb[(2 * (g2 - 1) + 1) * qhw + t];
    }
  }
  f32x4 gw;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    gw[c] = s2[c] / a.divisor + ve[c];
    s1[c] = s1[c] / a.divisor;
  }
  // this quad's share of grad_flow[p] (x2 at p's corners)
  float gix = 0.f, giy = 0.f;
  if (own) {
    f32x4 r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      r[j] = slot[j] >= 0 ? xq[kq + slot[j]] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      gix += gw[c] * ((r[1][c] - r[0][c]) * b.wy0 + (r[3][c] - r[2][c]) * b.wy1);
      giy += gw[c] * ((r[2][c] - r[0][c]) * b.wx0 + (r[3][c] - r[1][c]) * b.wx1);
    }
    gwq[kq + p] = gw;
    if (NQ > 1) red[t] = gix, red[NT + t] = giy;
  }
  // counting sort of the (source pixel, corner) entries by target pixel, per-wave counters
  // (the quad-0 threads: one per pixel)
  int rank[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    rank[j] = pix0 && slot[j] >= 0 ? atomicAdd(&cnt[wave * HW + slot[j]], 1) : 0;
  if (NQ > 1) lds_barrier();
  // the workgroup's partial of grad_flow[p] (quads in order), out first: the arrival counter
  // moves once every partial has landed, and its round trip then runs under the list build
  // and the grad_x2 gathers
  if (pix0) {
    if (NQ > 1) {
#pragma unroll
      for (int j = 1; j < NQ; ++j) gix += red[j * HW + p], giy += red[NT + j * HW + p];
    }
    float* pp = a.part + ((size_t)(g * a.B + n) * 2) * plane;
    if (!(a.abl & 32)) {
      __hip_atomic_store(pp + p, gix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pp + plane + p, giy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // every partial store has completed (written through to the coherent level) before the
  // counter moves
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  unsigned old = 0;
  if (t == 0 && !(a.abl & 32))
    old = __hip_atomic_fetch_add(a.cnt + n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // g1: plain stores (the launcher requires C % (4 NQ) == 0)
  if (own) {
#pragma unroll
    for (int c = 0; c < 4; ++c) a.g1[cb + (size_t)c * plane + p] = s1[c];
  }
  // list starts: exclusive scan of the list lengths over the target pixels (thread t = pixel
  // t for t < HW), then per-wave offsets inside each list
  __shared__ int wsum[NW];
  int wc[NW], len = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wc[w] = pix0 ? cnt[w * HW + p] : 0;
    len += wc[w];
  }
  int incl = len;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if ((t & 63) >= o) incl += v;
  }
  if ((t & 63) == 63) wsum[wave] = incl;
  lds_barrier();
  for (int w = 0; w < wave; ++w) incl += wsum[w];
  if (pix0) {
    int run = incl - len;
    sst[p] = run;
    sln[p] = len;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      cnt[w * HW + p] = run;
      run += wc[w];
    }
  }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (pix0 && slot[j] >= 0) {
      const int e = cnt[wave * HW + slot[j]] + rank[j];
      lp[e] = p;
      lw[e] = wk[j];
    }
  lds_barrier();

  // ---- grad_x2 of pixel p, this quad, over p's list ----
  if (own) {
    const int start = sst[p], end = start + ((a.abl & 2) ? 0 : sln[p]);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e = start; e < end; ++e) acc += gwq[kq + lp[e]] * lw[e];
#pragma unroll
    for (int c = 0; c < 4; ++c) a.gx2[cb + (size_t)c * plane + p] = acc[c];
  }
  if (t == 0) *arrival = (int)old;
  lds_barrier();
  if (*arrival != a.ng - 1 || (a.abl & 4)) return;
  // ---- the last group of image n: grad_flow = the partials in group order; thread t takes
  // pixel t % HW and the slice t / HW of the groups, slices added in order ----
  if (t == 0) __hip_atomic_store(a.cnt + n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nsl = NT / HW, per = (a.ng + nsl - 1) / nsl;
  const int sl = qdiv(t, a.inv_hw), sp = t - sl * HW;
  float sx = 0.f, sy = 0.f;
  if (sl < nsl) {
    const int g0 = sl * per, g1e = min(a.ng, g0 + per);
    for (int j = g0; j < g1e; j += 16) {  // 32 loads in flight, then the fixed-order sum
      float vxs[16], vys[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int gg = min(j + i, g1e - 1);
        const float* q = a.part + ((size_t)(gg * a.B + n) * 2) * plane;
        vxs[i] = __hip_atomic_load(q + sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vys[i] = __hip_atomic_load(q + plane + sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (j + i < g1e) sx += vxs[i], sy += vys[i];
    }
    red[t] = sx;
    red[NT + t] = sy;
  }
  lds_barrier();
  if (sl != 0) return;
  for (int j = 1; j < nsl; ++j) sx += red[j * HW + sp], sy += red[NT + j * HW + sp];
  const float mx = (float)(W - 1) / 2.f, my = (float)(H - 1) / 2.f;
  a.gflow[(size_t)(2 * n) * plane + sp] = (sx * mx) / a.halfx;
  a.gflow[(size_t)(2 * n + 1) * plane + sp] = (sy * my) / a.halfy;
}

// y += x (the two-launch path's gradient on x2_warp)
__global__ __launch_bounds__(256) void add_f32(float* __restrict__ y, const float* __restrict__ x,
                                               size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    y[i] += x[i];
}

}  // namespace cbwd

hipError_t add_inplace_f32(void* y, const void* x, size_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  size_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cbwd::add_f32, dim3((unsigned)blocks), dim3(256), 0, stream, (float*)y,
                     (const float*)x, n);
  return hipGetLastError();
}

// Workspace of the one-launch path: the grad_flow partials (0 when it does not apply).
// gO loads per thread of the instantiation serving H * W pixels (0: none)
static int gload_class(long long hw) {
  if (hw % 4 == 0) {
    const long long n = (cbwd::ND * hw + 4 * cbwd::NT - 1) / (4 * cbwd::NT);
    return n <= 4 ? 4 : n <= 7 ? 7 : n <= 11 ? 11 : 0;
  }
  const long long n = (cbwd::ND * hw + cbwd::NT - 1) / cbwd::NT;
  return n <= 7 ? 7 : n <= 12 ? 12 : 0;
}

// channel quads per workgroup: the most that fit one thread per (quad, pixel) and divide C
static int quads(int C, long long hw) {
  for (int nq : {4, 2, 1})
    if (nq * hw <= cbwd::MAXP && C % (4 * nq) == 0) return nq;
  return 0;
}

bool warp_corr_bwd_small_accepts(int B, int C, int H, int W) {
  using namespace cbwd;
  const long long hw = (long long)H * W;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || hw > MAXP || quads(C, hw) == 0) return false;
  if ((long long)B * C * hw >= (1ll << 31) || gload_class(hw) == 0) return false;
  if ((long long)lds_floats(H, W, quads(C, hw)) * 4 > 160 * 1024) return false;  // LDS
  return debug_knob("warp_corr_bwd", 1) != 0;
}

size_t warp_corr_bwd_small_workspace(int B, int C, int H, int W) {
  if (!warp_corr_bwd_small_accepts(B, C, H, W)) return 0;
  const int ng = C / (4 * quads(C, (long long)H * W));
  return (size_t)ng * B * 2 * H * W * sizeof(float);
}

// the reachable (gO load class, quads) instantiations: quads 4 need <= 64 pixels, 2 <= 128
static const void* pick_kernel(int hw, int nq) {
  using namespace cbwd;
#define WCB_K(V, G, Q) reinterpret_cast<const void*>(&warp_corr_bwd_small<V, G, Q>)
  const int gc = gload_class(hw);
  if (hw % 4 == 0) {  // 16-B copy: <= 100 / 176 / 256 pixels
    if (gc == 4) return nq == 4 ? WCB_K(true, 4, 4) : nq == 2 ? WCB_K(true, 4, 2) : WCB_K(true, 4, 1);
    if (gc == 7) return nq == 2 ? WCB_K(true, 7, 2) : WCB_K(true, 7, 1);
    return WCB_K(true, 11, 1);
  }
  // scalar copy: <= 44 / 75 pixels
  if (gc == 7) return nq == 4 ? WCB_K(false, 7, 4) : nq == 2 ? WCB_K(false, 7, 2) : WCB_K(false, 7, 1);
  return nq == 4 ? WCB_K(false, 12, 4) : nq == 2 ? WCB_K(false, 12, 2) : WCB_K(false, 12, 1);
#undef WCB_K
}

// hipErrorNotSupported: not this path (the caller runs the two launches)
hipError_t warp_corr_bwd_small(const void* in1, const void* x2, const void* flow,
                               const void* x2w, const void* grad_corr, const void* grad_x2w,
                               void* grad_in1, void* grad_x2, void* grad_flow, int B, int C,
                               int H, int W, float divisor, void* ws, size_t ws_bytes,
                               void* counters, hipStream_t stream) {
  using namespace cbwd;
  if (!warp_corr_bwd_small_accepts(B, C, H, W) || counters == nullptr || ws == nullptr ||
      ws_bytes < warp_corr_bwd_small_workspace(B, C, H, W))
    return hipErrorNotSupported;
  const int hw = H * W, nq = quads(C, hw);
  Args a;
  a.f1 = (const float*)in1;
  a.x2 = (const float*)x2;
  a.flow = (const float*)flow;
  a.x2w = (const float*)x2w;
  a.gc = (const float*)grad_corr;
  a.gxw = (const float*)grad_x2w;
  a.g1 = (float*)grad_in1;
  a.gx2 = (float*)grad_x2;
  a.gflow = (float*)grad_flow;
  a.part = (float*)ws;
  a.cnt = (unsigned*)counters;
  a.B = B, a.C = C, a.H = H, a.W = W;
  a.ng = C / (4 * nq);
  a.halfx = (float)((W - 1.0) / 2.0);
  a.halfy = (float)((H - 1.0) / 2.0);
  a.divisor = divisor;
  a.abl = debug_knob("wcb_abl", 0);
  a.inv_hw = 1.f / (float)(H * W);
  a.inv_w = 1.f / (float)W;
  a.inv_wp = 1.f / (float)(W + 16);
  a.inv_pp = 1.f / (float)((H + 16) * (W + 16));
  a.inv_qhw = 1.f / (float)(nq * hw);
  a.ntg = NT / (nq * hw) < 3 ? NT / (nq * hw) : 3;
  const size_t lds = (size_t)lds_floats(H, W, nq) * sizeof(float);
  const void* f = pick_kernel(hw, nq);
  hipError_t e = lds_limit(f, (int)lds);
  if (e != hipSuccess) return e;
  void* args[] = {&a};
  return hipLaunchKernel(f, dim3((unsigned)(B * a.ng)), dim3(NT), args, lds, stream);
}

}  // namespace pwc
