// corr_small.hip — correlation forward for the smallest pyramid levels (stride-2 displacements,
// dr = 4, any row alignment) on gfx950.
//
// Semantics: correlation_cuda_kernel.cu:34-106 of daigo0927/PWC-Net_pytorch with kernel_size 1,
// stride1 1, stride2 2, max_displacement / stride2 = 4 (model.py:24):
//   out[n, tc, oy, ox] = sum_c f1[n,c,oy+off,ox+off] * f2[n,c,oy+off+2tj,ox+off+2ti] / divisor
// zeros outside the image, off = max_displacement - pad_size.
//
// PWC-Net's l0 / l1 (6x7 and 12x14 pixels, 192 / 128 channels at 384x448) have rows that are
// not 16-B aligned and a few hundred output pixels per image, so the work is all channels and
// the cost is getting them onto enough CUs.  One workgroup = one row parity of one image (the
// parity halves never meet: an output row only sees f2 rows of its own parity) x one slice of
// the channels; the WHOLE parity half of the slice is staged in LDS at once (rows and columns
// outside the image are written as zeros, so there is no halo traffic at all), one batch of
// loads per thread.  Inside the workgroup the 8 waves form K channel groups that each
// accumulate 8 pixels x 9 ti per lane over their channels (the corr_pt.hip inner loop: 2 f1 +
// 6 f2 quads, 72 FMAs per channel), and meet in LDS (fixed order).  With nsplit > 1 channel
// slices, each slice writes raw partial sums and corr_reduce_splits (corr_fwd.hip) adds them in
// slice order: deterministic.
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>

#include "pwc_common.cuh"

namespace pwc {

hipError_t corr_reduce_splits_f32(const void* partial, void* out, size_t n, int nsplit,
                                  float divisor, float inv_divisor, hipStream_t stream);
void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip

namespace sm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int K_>
struct SmCfg {
  static constexpr int K = K_, NW = 8, WPG = NW / K, THREADS = 64 * NW, D = 9, DR = 4;
  static constexpr int ITEMS = 64 * WPG;  // output items (tj, row, segment) per group
  static constexpr int RED_BYTES = 18 * THREADS * 16;
};

struct SmGeo {
  int hp;    // parity rows staged (ceil(Ho / 2))
  int nseg;  // 8-pixel segments per row
  int x2;    // f2 LDS row floats: columns -8 .. 8*nseg+7
  int f1x;   // f1 LDS row floats: 8*nseg
  int f2f;   // f2 floats per channel: (hp + 8) * x2
  int chf;   // floats per channel
};

#ifdef PWC_SMALL_ABLATION  // bits: 1 = no global loads, 2 = no FMA work, 4 = no reduce/stores
__constant__ int g_sm_abl;
#define SM_ABL(b) (g_sm_abl & (b))
#else
#define SM_ABL(b) 0
#endif

template <class G>
__global__ __launch_bounds__(G::THREADS, 1) void corr_fwd_small(
    const float* __restrict__ in1, const float* __restrict__ in2, float* __restrict__ out,
    float* __restrict__ partial, int B, int C, int H, int W, int Ho, int Wo, int off, int layout,
    float divisor, float inv_divisor, int cps, int chk, SmGeo g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if (SM_ABL(8)) return;
  const int unit = blockIdx.x;  // (n, p); grid.y = channel slice
  const int p = unit & 1, n = unit >> 1;
  const int slice = blockIdx.y;
  const int c0 = slice * cps;
  const int cu = min(C, c0 + cps) - c0;  // channels of this slice
  const size_t plane = (size_t)H * W;
  const float* f1n = in1 + ((size_t)n * C + c0) * plane;
  const float* f2n = in2 + ((size_t)n * C + c0) * plane;

  // ---- channels stream through two LDS buffers of `chk` channels (LDS-DMA, buffer_load_dword
  // ... lds): job = one LDS row (f2 rows, then f1 rows, of a channel), wave wv takes rows
  // rr = wv, wv + 8, ..., lane = column; the DMA writes lane i's dword at the row base + 4i,
  // elements outside the image read 0 through the buffer range check, lanes past the row
  // width are masked off.  All of a chunk's rows are in flight at once, and chunk c+1 loads
  // while chunk c is consumed.  (Per-row setup, then one vector add + one scalar add per
  // channel: the scalar unit is shared by the CU's waves, and per-job integer division there
  // cost ~10 us.) ----
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rpc = g.hp + 8 + g.hp;  // LDS rows per channel
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds;
  const int nchunk = (cu + chk - 1) / chk;
  (void)rpc; (void)lds0;
  // Register staging of the in-image elements only (off == 0, checked by the launcher): thread
  // t owns within-channel element w = t % E of channels t / E, t / E + 512 / E, ... (E = the
  // 2 * rows * W elements of one channel's parity half), so the element -> LDS mapping is
  // computed once; the halo rows / columns stay zero from the initial clear and are never
  // written again.  One batch of loads per chunk (all in flight), then the LDS writes.
  const int hpp = (Ho - p + 1) / 2;           // parity rows that exist
  const int E = 2 * hpp * W;                  // in-image elements per channel
  const int cpt = E > 0 ? G::THREADS / E : 0;  // channels per pass of the block
  const int w = E > 0 ? (int)threadIdx.x % E : 0, cofs = E > 0 ? (int)threadIdx.x / E : cpt;
  int gsrc = 0, ldst = 0;
  bool is1 = false;
  if (E > 0) {
    const int half = hpp * W;
    is1 = w >= half;
    const int e = is1 ? w - half : w;
    const int r = e / W, x = e - r * W;
    gsrc = (2 * r + p) * W + x;
    ldst = is1 ? g.f2f + r * g.f1x + x : (r + G::DR) * g.x2 + x + 2 * G::DR;
  }
  const bool act = cofs < cpt;
  {  // clear both chunk buffers (halo zeros)
    f32x4* z = reinterpret_cast<f32x4*>(lds);
    const int nq = (2 * chk * g.chf) >> 2;
    for (int i = threadIdx.x; i < nq; i += G::THREADS) z[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  auto stage = [&](int chunk) {
    const int cb = chunk * chk, ce = min(cu, cb + chk);
    float* buf = lds + (chunk & 1) * chk * g.chf;
    constexpr int MAXP = 32;
    float v[MAXP];
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int c = cb + cofs + i * cpt;
      if (act && c < ce && !SM_ABL(1))
        v[i] = (is1 ? f1n : f2n)[(size_t)c * plane + gsrc];
    }
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int c = cb + cofs + i * cpt;
      if (act && c < ce) buf[(c - cb) * g.chf + ldst] = SM_ABL(1) ? 0.f : v[i];
    }
  };

  // ---- compute: group grp takes chunk channels grp, grp + K, ... ----
  const int grp = wave / G::WPG;
  const int item = (wave % G::WPG) * 64 + lane;
  const int per_tj = g.hp * g.nseg;
  const bool valid = item < G::D * per_tj;
  const int it = valid ? item : 0;
  const int tj = it / per_tj, rem = it - tj * per_tj;
  const int r = rem / g.nseg, s = rem - r * g.nseg;
  const int rho = r + tj;

  float lo[G::D][4], hi[G::D][4];
#pragma unroll
  for (int a = 0; a < G::D; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q) lo[a][q] = hi[a][q] = 0.f;

  const f32x4* l4 = reinterpret_cast<const f32x4*>(lds);
  const int f1q = (g.f2f + r * g.f1x + 8 * s) >> 2;  // quad index of the lane's f1 quads
  const int f2q = (rho * g.x2 + 8 * s) >> 2;         // first window quad
  const int chq = g.chf >> 2;
  stage(0);
  for (int chunk = 0; chunk < nchunk; ++chunk) {
    __syncthreads();  // chunk is in LDS; the other buffer is free (chunk-1 consumed)
    if (chunk + 1 < nchunk) stage(chunk + 1);
    const int ce = min(cu - chunk * chk, chk);
    const f32x4* bb = l4 + (chunk & 1) * chk * chq;
    for (int c = grp; c < ce && !SM_ABL(2); c += G::K) {
      const f32x4* b = bb + c * chq;
      const f32x4 a0 = b[f1q], a1 = b[f1q + 1];
      const f32x4 w[6] = {b[f2q], b[f2q + 1], b[f2q + 2], b[f2q + 3], b[f2q + 4], b[f2q + 5]};
      const f32x4 wl[5] = {w[0], w[1], w[2], w[3], w[4]};
      const f32x4 wh[5] = {w[1], w[2], w[3], w[4], w[5]};
      corr_fma_pairs_s2<G::D, 5>(lo, a0, wl);
      corr_fma_pairs_s2<G::D, 5>(hi, a1, wh);
    }
  }

  // ---- K partial sums meet in LDS ([v][group][item]); group grp finalises v == grp mod K ----
  if (SM_ABL(4)) {
    float z = 0.f;
    for (int a = 0; a < G::D; ++a)
      for (int q = 0; q < 4; ++q) z += lo[a][q] + hi[a][q];
    if (z == 1234.5f) out[0] = z;
    return;
  }
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(lds);
#pragma unroll
  for (int v = 0; v < 18; ++v) {
    const int ti = v >> 1;
    const f32x4 q = (v & 1) ? f32x4{hi[ti][0], hi[ti][1], hi[ti][2], hi[ti][3]}
                            : f32x4{lo[ti][0], lo[ti][1], lo[ti][2], lo[ti][3]};
    red[(v * G::K + grp) * G::ITEMS + item] = q;
  }
  __syncthreads();
  // Finalise: group grp sums the K partials of slots v == grp mod K (group order: fixed) and
  // parks the results in LDS in output order [oc][parity row][x]; then the whole workgroup
  // writes that block row by row (coalesced: lane = x).  Storing straight from the lanes
  // scattered 4-B writes over 81 planes (~6 us at l1).
  const int OC = G::D * G::D;
  const bool split = gridDim.y > 1;
  const bool pow2 = inv_divisor != 0.f;
  constexpr int NV = (18 + G::K - 1) / G::K;
  f32x4 res[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = grp + i * G::K;
    if (v < 18) {
      f32x4 q = red[(v * G::K) * G::ITEMS + item];
#pragma unroll
      for (int gg = 1; gg < G::K; ++gg) q += red[(v * G::K + gg) * G::ITEMS + item];
      if (!split) {
        if (pow2)
          q *= inv_divisor;
        else
          q /= divisor;
      }
      res[i] = q;
    }
  }
  __syncthreads();  // every wave has read its partials: the LDS becomes the output block
  // (hpp: parity rows that exist, above)
  float* blk = lds;                  // [oc][r][x], Wo floats per row
  if (valid && r < hpp) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = grp + i * G::K;
      if (v < 18) {
        const int ti = v >> 1, h = v & 1;
        const int oc = out_channel(layout, tj - G::DR, ti - G::DR, G::DR, G::D, 2);
        const int x = 8 * s + 4 * h;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (x + e < Wo) blk[(oc * g.hp + r) * Wo + x + e] = res[i][e];
      }
    }
  }
  __syncthreads();
  // nsplit == 1: the output itself (parity rows Wo floats apart).  Split: this workgroup's
  // partial block [oc][r][x] stored densely at partial[slice][n][p] (one contiguous run;
  // scattered partial rows wrote ~5 us slower), gathered back by sm_reduce.
  const size_t pblk = (size_t)OC * g.hp * Wo;
  float* base = split ? partial + (((size_t)slice * B + n) * 2 + p) * pblk
                      : out + (size_t)n * OC * Ho * Wo;
  const int ystr = split ? 1 : 2, yoff = split ? 0 : p, pstr = split ? g.hp : Ho;
  const int nrows = OC * hpp;
  // lane -> (row of the wave-instruction, x): rows of Wo floats packed 64 / WX per instruction
  // (WX = Wo rounded up to a power of two <= 64); no per-element integer division
  const int lw = 32 - __builtin_clz((unsigned)(Wo - 1) | 1u);  // log2(WX)
  const int wx = 1 << lw, rpi = 64 >> lw;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int x = ln & (wx - 1), sub = ln >> lw;
  int rr = 0, oc = 0;  // (oc, rr) of row wv * rpi + sub, advanced by 8 * rpi rows per step
  {
    const int row0 = wv * rpi + sub;
    oc = row0 / hpp;
    rr = row0 - oc * hpp;
  }
  const int step_oc = (8 * rpi) / hpp, step_rr = (8 * rpi) - step_oc * hpp;
  for (int row = wv * rpi + sub; row < nrows + 8 * rpi; row += 8 * rpi) {
    if (row < nrows && x < Wo)
      st_out1(base + ((size_t)oc * pstr + ystr * rr + yoff) * Wo + x, blk[(oc * g.hp + rr) * Wo + x]);
    oc += step_oc;
    rr += step_rr;
    if (rr >= hpp) {
      rr -= hpp;
      ++oc;
    }
  }
}

// out[n][oc][y][x] = (sum over slices k, in order, of partial[k][n][y & 1][oc][y >> 1][x]) /
// divisor; one thread per output element (coalesced writes, contiguous reads along x).
__global__ __launch_bounds__(256) void sm_reduce(const float* __restrict__ partial,
                                                 float* __restrict__ out, int B, int Ho, int Wo,
                                                 int hp, int nsplit, float divisor,
                                                 float inv_divisor) {
  const size_t total = (size_t)B * 81 * Ho * Wo;
  const size_t pblk = (size_t)81 * hp * Wo, pslice = (size_t)B * 2 * pblk;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (size_t)gridDim.x * 256) {
    const int x = (int)(i % Wo);
    const size_t t = i / Wo;
    const int y = (int)(t % Ho);
    const size_t t2 = t / Ho;
    const int oc = (int)(t2 % 81);
    const int n = (int)(t2 / 81);
    const size_t src = ((size_t)n * 2 + (y & 1)) * pblk + ((size_t)oc * hp + (y >> 1)) * Wo + x;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < nsplit) v[k] = partial[k * pslice + src];
    float sum = v[0];
#pragma unroll
    for (int k = 1; k < 16; ++k)
      if (k < nsplit) sum += v[k];
    st_out1(out + i, inv_divisor != 0.f ? sum * inv_divisor : sum / divisor);
  }
}

template <class G>
static hipError_t launch_small(const void* in1, const void* in2, void* out, int B, int C, int H,
                               int W, int Ho, int Wo, int off, int layout, float divisor,
                               int nsplit, void* partial, hipStream_t stream) {
  SmGeo g;
  g.hp = (Ho + 1) / 2;
  g.nseg = (Wo + 7) / 8;
  g.x2 = 8 * g.nseg + 16;
  g.f1x = 8 * g.nseg;
  g.f2f = (g.hp + 8) * g.x2;
  g.chf = g.f2f + g.hp * g.f1x;
  if (G::D * g.hp * g.nseg > G::ITEMS) return hipErrorNotSupported;
  if (nsplit < 1) nsplit = 1;
  const int cps = (C + nsplit - 1) / nsplit;
  nsplit = (C + cps - 1) / cps;
  // two chunk buffers within the LDS (the K-group reduction reuses it afterwards)
  int chk = (int)(163840 / (2 * 4 * (size_t)g.chf));
  if (chk > cps) chk = cps;
  {  // register staging: at most 32 passes of 512 / E channels per chunk
    const int E = 2 * ((Ho + 1) / 2) * W;
    const int cpt = E > 0 ? G::THREADS / E : 0;
    if (cpt < 1) return hipErrorNotSupported;
    if (chk > 32 * cpt) chk = 32 * cpt;
  }
  if (off != 0) return hipErrorNotSupported;
  if (chk < 1) return hipErrorNotSupported;
  const size_t data = (size_t)2 * chk * g.chf * 4;
  const size_t lds = data > (size_t)G::RED_BYTES ? data : (size_t)G::RED_BYTES;
  if (lds > 163840) return hipErrorNotSupported;
  if (nsplit > 1 && !partial) return hipErrorNotSupported;
  if (nsplit > 16) return hipErrorNotSupported;
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e = lds_limit(reinterpret_cast<const void*>(&corr_fwd_small<G>), 163840);
    if (e != hipSuccess) return e;
  }
  int ex;
  const float m = std::frexp(divisor, &ex);
  const float inv = (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL((corr_fwd_small<G>), dim3((unsigned)(2 * B), (unsigned)nsplit),
                        dim3(G::THREADS), lds, stream, ev0, ev1, 0, (const float*)in1,
                        (const float*)in2, (float*)out, (float*)partial, B, C, H, W, Ho, Wo,
                        off, layout, divisor, inv, cps, chk, g);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nsplit == 1) return e;
  const size_t total = (size_t)B * 81 * Ho * Wo;
  hipLaunchKernelGGL(sm_reduce, dim3((unsigned)std::min<size_t>((total + 255) / 256, 4096)),
                     dim3(256), 0, stream, (const float*)partial, (float*)out, B, Ho, Wo, g.hp,
                     nsplit, divisor, inv);
  return hipGetLastError();
}

}  // namespace sm

// Small-image correlation (stride-2, dr = 4).  `max_splits` bounds the channel slices (the
// caller's workspace holds max_splits partial volumes); hipErrorNotSupported when the image
// is too large for one parity half per workgroup.
hipError_t corr_forward_small_f32(const void* in1, const void* in2, void* out, int B, int C,
                                  int H, int W, int Ho, int Wo, int off, int dr, int s2,
                                  int layout, float divisor, int max_splits, void* partial,
                                  hipStream_t stream) {
  if (!(dr == 4 && s2 == 2)) return hipErrorNotSupported;
  if ((size_t)B * C * H * W >= (1ull << 31)) return hipErrorNotSupported;
  const int hp = (Ho + 1) / 2, nseg = (Wo + 7) / 8;
  const int items = 9 * hp * nseg;
  // channel slices: enough workgroups to spread the staging loads (~128), at least 8
  // channels per slice, within the workspace
  // channel slices: enough workgroups to spread the staging (~128), at least 8 channels per
  // slice, within the workspace (measured at l0 / l1, B = 8: 8 slices + reduce beat one
  // workgroup per parity half with every channel streamed through LDS, 10 vs 15 us at l0)
  int nsplit = 1;
  if (partial && max_splits > 1) {
    nsplit = (128 + 2 * B - 1) / (2 * B);
    if (nsplit > C / 8) nsplit = C / 8;
    if (nsplit > max_splits) nsplit = max_splits;
    if (nsplit < 1) nsplit = 1;
  }
  if (const int k = debug_knob("small_splits", 0)) nsplit = k;
  // a slice's partial block holds 2 * ceil(Ho / 2) rows: stay inside the caller's workspace,
  // sized for max_splits volumes of Ho rows
  if (nsplit > 1) {
    const long long fit = partial ? (long long)max_splits * Ho / (2 * hp) : 1;
    if (nsplit > fit) nsplit = (int)(fit < 1 ? 1 : fit);
  }
  if (items <= 64)
    return sm::launch_small<sm::SmCfg<8>>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout,
                                          divisor, nsplit, partial, stream);
  if (items <= 128)
    return sm::launch_small<sm::SmCfg<4>>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout,
                                          divisor, nsplit, partial, stream);
  if (items <= 256)
    return sm::launch_small<sm::SmCfg<2>>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout,
                                          divisor, nsplit, partial, stream);
  return hipErrorNotSupported;
}

}  // namespace pwc
