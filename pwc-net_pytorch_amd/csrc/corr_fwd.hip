// corr_fwd.hip — cost-volume correlation forward for gfx950 (MI355X).
//
// Semantics: correlation_cuda_kernel.cu:34-106 of daigo0927/PWC-Net_pytorch (values),
// correlation_cuda.c:20-34 (shapes).  For kernel_size == 1, stride1 == 1 the output pixel
// (oy, ox) pairs f1 at (oy+off, ox+off) with f2 at (oy+off+tj*s2, ox+off+ti*s2),
// off = max_displacement - pad_size, zero outside the image (the reference's zero-padded
// NHWC scratch, cu:10-32, is never materialised here).
//
// Tiled kernel (k == 1, s1 == 1; template displacement radius DR and stride S):
//   * one workgroup = one TY x TX output tile of one image, D*TY*NG threads
//     (thread = output row ty, pixel group g, displacement row tj);
//   * channels stream through a double-buffered LDS tile in chunks of CC: the f1 tile and
//     the f2 tile with a DR*S halo are read from HBM once per workgroup, coalesced along W
//     (float4 where aligned), and de-interleaved by x mod S so every lane's f2 window for
//     its PX same-phase pixels is PX+2*DR contiguous floats (ds_read_b128, row stride 48
//     dwords => conflict-free for the b128 lane groups);
//   * each thread accumulates PX x D outputs in registers (fp32 FMA chain over C);
//   * blocks are remapped XCD-aware so neighbouring tiles (shared halo rows) share an L2.
// Generic kernel: any (pad, k, md, s1, s2), one thread per output element; used for the
// rarely-used configurations the tiled kernel does not instantiate.
#include <hip/hip_ext.h>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "pwc_common.cuh"

namespace pwc {

void take_launch_events(hipEvent_t* start, hipEvent_t* stop);  // capi.hip


constexpr int kMaxSplits = 16;  // channel splits per tile (workspace budget)

template <int DR_, int S_, int GS_, int PX_, int NQ_, int TY_, int CC_>
struct CorrTile {
  static constexpr int DR = DR_, S = S_, GS = GS_, PX = PX_, NQ = NQ_, TY = TY_, CC = CC_;
  static constexpr int D = 2 * DR + 1;
  static constexpr int HALO = DR * S;
  static constexpr int NG = GS * NQ;         // pixel groups per tile row
  static constexpr int TX = NG * PX;         // tile width (pixels)
  static constexpr int R2 = TY + 2 * HALO;   // f2 tile rows
  static constexpr int X2 = TX + 2 * HALO;   // f2 tile columns
  static constexpr int NW = (GS == S) ? PX + 2 * DR : PX + 2 * DR * S;  // f2 window / lane
  static constexpr int THREADS = TY * NG * D;
  // row strides (floats): f2 rows padded to 16 (mod 32) dwords so that the four rows a
  // ds_read_b128 lane group touches land on disjoint 16-bank slices; f1 rows are 16 wide.
  static constexpr int RS2 = ((X2 + 15) / 32) * 32 + 16;
  static constexpr int RS1 = TX;
  static constexpr int F2_FLOATS = CC * R2 * RS2;
  static constexpr int F1_FLOATS = CC * TY * RS1;
  static constexpr int BUF_FLOATS = F2_FLOATS + F1_FLOATS;
  static constexpr int LDS_BYTES = 2 * BUF_FLOATS * 4;
  static_assert(PX == 4, "lane windows are handled as float4 quads");
  static_assert(GS == 1 || GS == S, "pixel grouping: consecutive or same-phase");
  static_assert(X2 % (4 * GS) == 0, "f2 tile row must split into whole quads per phase");
  static_assert(THREADS % 64 == 0, "whole wavefronts");
  static_assert(THREADS <= 1024, "workgroup size");
  static_assert(RS2 >= X2, "row stride");
};

// LDS float index of tile element (xh) within a row, layout [quad][phase][4].
template <class G>
__device__ __forceinline__ int lds_col(int xh) {
  const int p = xh % G::GS;
  const int m = xh / G::GS;
  return ((m >> 2) * G::GS + p) * 4 + (m & 3);
}

template <class G, typename T>
struct Stager {
  // float4 "slots" of the f2 and f1 tiles for one channel chunk, spread over the block.
  static constexpr int SLOTS2 = G::CC * G::R2 * (G::X2 / 4);
  static constexpr int SLOTS1 = G::CC * G::TY * (G::TX / 4);
  static constexpr int IT2 = (SLOTS2 + G::THREADS - 1) / G::THREADS;
  static constexpr int IT1 = (SLOTS1 + G::THREADS - 1) / G::THREADS;
  float4 r2[IT2];
  float4 r1[IT1];

  __device__ __forceinline__ static float4 load4(const T* __restrict__ base, int y, int x,
                                                 int H, int W, bool vec_ok) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y < 0 || y >= H) return v;
    const T* row = base + (size_t)y * W;
    if (vec_ok && x >= 0 && x + 3 < W) {
      if constexpr (sizeof(T) == 4) {
        v = *reinterpret_cast<const float4*>(row + x);
      } else {
        const uint2 raw = *reinterpret_cast<const uint2*>(row + x);
        const T* h = reinterpret_cast<const T*>(&raw);
        v = make_float4(to_f32(h[0]), to_f32(h[1]), to_f32(h[2]), to_f32(h[3]));
      }
      return v;
    }
    float e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int xx = x + i;
      e[i] = (xx >= 0 && xx < W) ? to_f32(row[xx]) : 0.f;
    }
    return make_float4(e[0], e[1], e[2], e[3]);
  }

  // Issue the global loads of chunk c0 (channels c0 .. c0+CC-1, those >= C read as zero) into
  // registers.
  __device__ __forceinline__ void load(const T* __restrict__ f1n, const T* __restrict__ f2n,
                                       int c0, int C, int H, int W, int y1, int x1,
                                       bool vec_ok) {
    const size_t plane = (size_t)H * W;
#pragma unroll
    for (int it = 0; it < IT2; ++it) {
      const int s = threadIdx.x + it * G::THREADS;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s < SLOTS2) {
        const int q4 = s % (G::X2 / 4);
        const int rr = (s / (G::X2 / 4)) % G::R2;
        const int cc = s / ((G::X2 / 4) * G::R2);
        const int c = c0 + cc;
        if (c < C)
          v = load4(f2n + (size_t)c * plane, y1 - G::HALO + rr, x1 - G::HALO + 4 * q4, H, W,
                    vec_ok);
      }
      r2[it] = v;
    }
#pragma unroll
    for (int it = 0; it < IT1; ++it) {
      const int s = threadIdx.x + it * G::THREADS;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s < SLOTS1) {
        const int q4 = s % (G::TX / 4);
        const int rr = (s / (G::TX / 4)) % G::TY;
        const int cc = s / ((G::TX / 4) * G::TY);
        const int c = c0 + cc;
        if (c < C) v = load4(f1n + (size_t)c * plane, y1 + rr, x1 + 4 * q4, H, W, vec_ok);
      }
      r1[it] = v;
    }
  }

  // Scatter the registers into one LDS buffer in the de-interleaved [quad][phase][4] layout.
  __device__ __forceinline__ void store(float* __restrict__ buf) const {
    float* F2 = buf;
    float* F1 = buf + G::F2_FLOATS;
#pragma unroll
    for (int it = 0; it < IT2; ++it) {
      const int s = threadIdx.x + it * G::THREADS;
      if (s < SLOTS2) {
        const int q4 = s % (G::X2 / 4);
        const int rr = (s / (G::X2 / 4)) % G::R2;
        const int cc = s / ((G::X2 / 4) * G::R2);
        float* row = F2 + (cc * G::R2 + rr) * G::RS2;
        const float e[4] = {r2[it].x, r2[it].y, r2[it].z, r2[it].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) row[lds_col<G>(4 * q4 + i)] = e[i];
      }
    }
#pragma unroll
    for (int it = 0; it < IT1; ++it) {
      const int s = threadIdx.x + it * G::THREADS;
      if (s < SLOTS1) {
        const int q4 = s % (G::TX / 4);
        const int rr = (s / (G::TX / 4)) % G::TY;
        const int cc = s / ((G::TX / 4) * G::TY);
        float* row = F1 + (cc * G::TY + rr) * G::RS1;
        const float e[4] = {r1[it].x, r1[it].y, r1[it].z, r1[it].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) row[lds_col<G>(4 * q4 + i)] = e[i];
      }
    }
  }
};

// blockIdx.y = channel split k: channels [k*cps, min(C,(k+1)*cps)); with gridDim.y > 1 the raw
// sums go to partial[k][n][oc][oy][ox] (fp32) for corr_reduce_splits.
template <class G, typename T>
__global__ __launch_bounds__(G::THREADS) void corr_fwd_tiled(
    const T* __restrict__ in1, const T* __restrict__ in2, T* __restrict__ out, int B, int C,
    int H, int W, int Ho, int Wo, int off, int layout, float divisor, int n_ty, int n_tx,
    int vec_ok_i, int cps, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const bool vec_ok = vec_ok_i != 0;

  const int nblk = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nblk);
  const int tx_tile = t % n_tx;
  const int ty_tile = (t / n_tx) % n_ty;
  const int n = t / (n_tx * n_ty);
  const int oy0 = ty_tile * G::TY, ox0 = tx_tile * G::TX;
  const int y1 = oy0 + off, x1 = ox0 + off;  // f1 tile origin (unpadded image coordinates)

  // thread role
  const int g = threadIdx.x % G::NG;
  const int ty = (threadIdx.x / G::NG) % G::TY;
  const int tjx = threadIdx.x / (G::NG * G::TY);  // 0 .. D-1, wave-uniform when NG*TY % 64 == 0
  const int p = g % G::GS;
  const int q = g / G::GS;

  const size_t plane = (size_t)H * W;
  const T* f1n = in1 + (size_t)n * C * plane;
  const T* f2n = in2 + (size_t)n * C * plane;

  float acc[G::D][G::PX];
#pragma unroll
  for (int a = 0; a < G::D; ++a)
#pragma unroll
    for (int k = 0; k < G::PX; ++k) acc[a][k] = 0.f;

  Stager<G, T> st;
  const int c_begin = blockIdx.y * cps;
  const int c_end = min(C, c_begin + cps);
  const int nchunks = (c_end - c_begin + G::CC - 1) / G::CC;
  st.load(f1n, f2n, c_begin, c_end, H, W, y1, x1, vec_ok);
  st.store(lds);
  __syncthreads();

  // lane-constant LDS offsets
  const int f2_row = ty + tjx * G::S;  // f2 tile row of this thread's displacement row
  const int f2_off = f2_row * G::RS2 + (q * G::GS + p) * 4;  // first quad of the window
  const int f1_off = ty * G::RS1 + (q * G::GS + p) * 4;

  for (int ch = 0; ch < nchunks; ++ch) {
    const float* buf = lds + (ch & 1) * G::BUF_FLOATS;
    if (ch + 1 < nchunks)
      st.load(f1n, f2n, c_begin + (ch + 1) * G::CC, c_end, H, W, y1, x1, vec_ok);
#pragma unroll
    for (int cc = 0; cc < G::CC; ++cc) {
      const float* F2 = buf + cc * G::R2 * G::RS2 + f2_off;
      const float* F1 = buf + G::F2_FLOATS + cc * G::TY * G::RS1 + f1_off;
      const float4 a4 = *reinterpret_cast<const float4*>(F1);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
      float w[G::NW];
#pragma unroll
      for (int u = 0; u < G::NW / 4; ++u) {
        const float4 b4 = *reinterpret_cast<const float4*>(F2 + u * 4 * G::GS);
        w[4 * u + 0] = b4.x;
        w[4 * u + 1] = b4.y;
        w[4 * u + 2] = b4.z;
        w[4 * u + 3] = b4.w;
      }
#pragma unroll
      for (int ti = 0; ti < G::D; ++ti)
#pragma unroll
        for (int k = 0; k < G::PX; ++k) {
          const int j = (G::GS == G::S) ? (k + ti) : (k + G::S * ti);
          acc[ti][k] = fmaf(av[k], w[j], acc[ti][k]);
        }
    }
    if (ch + 1 < nchunks) st.store(lds + ((ch + 1) & 1) * G::BUF_FLOATS);
    __syncthreads();
  }

  // epilogue: out[n][ch][oy][ox] = acc / divisor  (cu:100 divides by k*k*C)
  const int oy = oy0 + ty;
  if (oy >= Ho) return;
  const int OC = G::D * G::D;
  const int tj = tjx - G::DR;
  if (gridDim.y > 1) {
    float* pk = partial + (size_t)blockIdx.y * B * OC * Ho * Wo;
#pragma unroll
    for (int ti = 0; ti < G::D; ++ti) {
      const int oc = out_channel(layout, tj, ti - G::DR, G::DR, G::D, G::S);
      float* prow = pk + (((size_t)n * OC + oc) * Ho + oy) * Wo;
#pragma unroll
      for (int k = 0; k < G::PX; ++k) {
        const int ox = ox0 + q * G::GS * G::PX + p + G::GS * k;
        if (ox < Wo) prow[ox] = acc[ti][k];
      }
    }
    return;
  }
#pragma unroll
  for (int ti = 0; ti < G::D; ++ti) {
    const int oc = out_channel(layout, tj, ti - G::DR, G::DR, G::D, G::S);
    T* orow = out + (((size_t)n * OC + oc) * Ho + oy) * Wo;
    if constexpr (G::GS == 1) {
      const int ox = ox0 + q * G::PX;
      if (sizeof(T) == 4 && vec_ok && ox + 3 < Wo) {
        float4 v = make_float4(acc[ti][0] / divisor, acc[ti][1] / divisor,
                               acc[ti][2] / divisor, acc[ti][3] / divisor);
        *reinterpret_cast<float4*>(orow + ox) = v;
        continue;
      }
    }
#pragma unroll
    for (int k = 0; k < G::PX; ++k) {
      const int ox = ox0 + q * G::GS * G::PX + p + G::GS * k;
      if (ox < Wo) orow[ox] = from_f32<T>(acc[ti][k] / divisor);
    }
  }
}

// Generic kernel: one thread per output element, literal cu:34-106 arithmetic.
template <typename T>
__global__ void corr_fwd_generic(const T* __restrict__ in1, const T* __restrict__ in2,
                                 T* __restrict__ out, int B, int C, int H, int W, int Ho,
                                 int Wo, int pad, int kr, int md, int s1, int s2, int dr,
                                 int layout, float divisor) {
  const int D = 2 * dr + 1, OC = D * D;
  const size_t total = (size_t)B * OC * Ho * Wo;
  const size_t plane = (size_t)H * W;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const int ox = idx % Wo;
    const int oy = (idx / Wo) % Ho;
    const int tc = (idx / ((size_t)Wo * Ho)) % OC;
    const int n = idx / ((size_t)Wo * Ho * OC);
    const int tj = tc / D - dr, ti = tc % D - dr;
    const int y1 = oy * s1 + md + kr - pad, x1 = ox * s1 + md + kr - pad;  // unpadded
    const int y2 = y1 + tj * s2, x2 = x1 + ti * s2;
    float sum = 0.f;
    for (int j = -kr; j <= kr; ++j)
      for (int i = -kr; i <= kr; ++i) {
        const int ya = y1 + j, xa = x1 + i, yb = y2 + j, xb = x2 + i;
        if (ya < 0 || ya >= H || xa < 0 || xa >= W || yb < 0 || yb >= H || xb < 0 || xb >= W)
          continue;
        const T* pa = in1 + (size_t)n * C * plane + (size_t)ya * W + xa;
        const T* pb = in2 + (size_t)n * C * plane + (size_t)yb * W + xb;
        for (int c = 0; c < C; ++c) sum = fmaf(to_f32(pa[c * plane]), to_f32(pb[c * plane]), sum);
      }
    const int oc = layout == kCvl ? cvl_channel(tj * s2, ti * s2, dr) : tc;
    out[(((size_t)n * OC + oc) * Ho + oy) * Wo + ox] = from_f32<T>(sum / divisor);
  }
}

// Split-channel reduction: out[i] = (sum_k partial[k][i]) / divisor, k ascending (fixed order,
// deterministic).  inv_divisor != 0 when the divisor is a power of two (exact scale).
// out[i] = (sum_k partial[k][i]) / divisor, k = 0..nsplit-1 in order (deterministic).  All of
// a thread's nsplit loads are issued before the in-order sum (nsplit <= kMaxSplits), four
// consecutive elements per thread when n % 4 == 0.
template <typename T>
__global__ __launch_bounds__(256) void corr_reduce_splits(const float* __restrict__ partial,
                                                          T* __restrict__ out, size_t n,
                                                          int nsplit, float divisor,
                                                          float inv_divisor) {
  const bool vec = (n % 4) == 0;
  const size_t nv = vec ? n / 4 : n;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv;
       i += (size_t)gridDim.x * blockDim.x) {
    if (vec) {
      float4 v[kMaxSplits];
#pragma unroll
      for (int k = 0; k < kMaxSplits; ++k)
        if (k < nsplit) v[k] = reinterpret_cast<const float4*>(partial + (size_t)k * n)[i];
      float4 s = v[0];
#pragma unroll
      for (int k = 1; k < kMaxSplits; ++k)
        if (k < nsplit) {
          s.x += v[k].x;
          s.y += v[k].y;
          s.z += v[k].z;
          s.w += v[k].w;
        }
      const float r[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        out[4 * i + e] = from_f32<T>(inv_divisor != 0.f ? r[e] * inv_divisor : r[e] / divisor);
    } else {
      float v[kMaxSplits];
#pragma unroll
      for (int k = 0; k < kMaxSplits; ++k)
        if (k < nsplit) v[k] = partial[(size_t)k * n + i];
      float s = v[0];
#pragma unroll
      for (int k = 1; k < kMaxSplits; ++k)
        if (k < nsplit) s += v[k];
      out[i] = from_f32<T>(inv_divisor != 0.f ? s * inv_divisor : s / divisor);
    }
  }
}

static float exact_inverse(float divisor) {
  int ex;
  const float m = std::frexp(divisor, &ex);
  return (m == 0.5f) ? std::ldexp(1.f, 1 - ex) : 0.f;
}

template <typename T>
static hipError_t corr_reduce_splits_t(const void* partial, void* out, size_t n, int nsplit,
                                       float divisor, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (nsplit < 1 || nsplit > kMaxSplits) return hipErrorInvalidValue;
  const size_t nv = (n % 4 == 0) ? n / 4 : n;
  size_t blocks = (nv + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(corr_reduce_splits<T>, dim3((unsigned)blocks), dim3(256), 0, stream,
                     (const float*)partial, (T*)out, n, nsplit, divisor,
                     exact_inverse(divisor));
  return hipGetLastError();
}

hipError_t corr_reduce_splits_f32(const void* partial, void* out, size_t n, int nsplit,
                                  float divisor, float inv_divisor, hipStream_t stream) {
  (void)inv_divisor;
  return corr_reduce_splits_t<float>(partial, out, n, nsplit, divisor, stream);
}

// Channel splits for a grid of `base_blocks` workgroups: none once the grid alone gives every
// CU a workgroup; otherwise aim at two workgroups per CU (512), at most one split per channel
// chunk and at most `max_splits` (the caller sizes max_splits so that the partial volumes stay
// within the workspace budget, corr_workspace_bytes).
static int corr_pick_splits(long long base_blocks, int nchunks, int max_splits) {
  if (base_blocks <= 0 || base_blocks >= 256) return 1;
  long long k = (512 + base_blocks - 1) / base_blocks;
  if (k > nchunks) k = nchunks;
  if (k > max_splits) k = max_splits;
  return k < 1 ? 1 : (int)k;
}

// ------------------------------------------------------------------------------------
// host-side launchers
// ------------------------------------------------------------------------------------
using Corr9 = CorrTile</*DR*/ 4, /*S*/ 2, /*GS*/ 2, /*PX*/ 4, /*NQ*/ 2, /*TY*/ 16, /*CC*/ 4>;
using Corr4 = CorrTile</*DR*/ 4, /*S*/ 1, /*GS*/ 1, /*PX*/ 4, /*NQ*/ 4, /*TY*/ 16, /*CC*/ 4>;

template <class G, typename T>
static hipError_t launch_tiled(const void* in1, const void* in2, void* out, int B, int C,
                               int H, int W, int Ho, int Wo, int off, int layout,
                               float divisor, int max_splits, void* partial,
                               hipStream_t stream) {
  const int n_ty = (Ho + G::TY - 1) / G::TY;
  const int n_tx = (Wo + G::TX - 1) / G::TX;
  const long long nblk = (long long)B * n_ty * n_tx;
  if (nblk <= 0) return hipSuccess;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  // float4 loads/stores need 16-B aligned rows and halo-aligned tile origins.
  const size_t align = 4 * sizeof(T);
  const bool vec_ok = (W % 4 == 0) && (Wo % 4 == 0) && (off % 4 == 0) && (G::HALO % 4 == 0) &&
                      ((uintptr_t)in1 % align == 0) && ((uintptr_t)in2 % align == 0) &&
                      ((uintptr_t)out % 16 == 0);
  {  // > 64 KiB dynamic LDS: opted in once per device (lds_limit, capi.hip)
    const hipError_t e =
        lds_limit(reinterpret_cast<const void*>(&corr_fwd_tiled<G, T>), G::LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  const int nchunks = (C + G::CC - 1) / G::CC;
  int nsplit = partial ? corr_pick_splits(nblk, nchunks, max_splits) : 1;
  const int cps = ((nchunks + nsplit - 1) / nsplit) * G::CC;
  nsplit = C > 0 ? (C + cps - 1) / cps : 1;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);  // bench.py's live timing hook (one-shot)
  hipExtLaunchKernelGGL((corr_fwd_tiled<G, T>), dim3((unsigned)nblk, (unsigned)nsplit),
                        dim3(G::THREADS), G::LDS_BYTES, stream, ev0, ev1, 0, (const T*)in1,
                        (const T*)in2, (T*)out, B, C, H, W, Ho, Wo, off, layout, divisor, n_ty,
                        n_tx, vec_ok ? 1 : 0, cps, (float*)partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nsplit == 1) return e;
  return corr_reduce_splits_t<T>(partial, out, (size_t)B * G::D * G::D * Ho * Wo, nsplit,
                                 divisor, stream);
}

template <typename T>
static hipError_t launch_generic(const void* in1, const void* in2, void* out, int B, int C,
                                 int H, int W, int Ho, int Wo, int pad, int kr, int md, int s1,
                                 int s2, int dr, int layout, float divisor,
                                 hipStream_t stream) {
  const int D = 2 * dr + 1;
  const size_t total = (size_t)B * D * D * Ho * Wo;
  if (total == 0) return hipSuccess;
  const int threads = 256;
  size_t blocks = (total + threads - 1) / threads;
  if (blocks > 65536) blocks = 65536;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  take_launch_events(&ev0, &ev1);
  hipExtLaunchKernelGGL(corr_fwd_generic<T>, dim3((unsigned)blocks), dim3(threads), 0, stream,
                        ev0, ev1, 0, (const T*)in1, (const T*)in2, (T*)out, B, C, H, W, Ho, Wo,
                        pad, kr, md, s1, s2, dr, layout, divisor);
  return hipGetLastError();
}

// corr_pt.hip
hipError_t corr_forward_pt_f32(const void* in1, const void* in2, void* out, int B, int C, int H,
                               int W, int Ho, int Wo, int off, int dr, int s2, int layout,
                               float divisor, int groups, hipStream_t stream);

// corr_small.hip
hipError_t corr_forward_small_f32(const void* in1, const void* in2, void* out, int B, int C,
                                  int H, int W, int Ho, int Wo, int off, int dr, int s2,
                                  int layout, float divisor, int max_splits, void* partial,
                                  hipStream_t stream);

// Channel-split budget: nsplit partial volumes of B*OC*Ho*Wo floats, nsplit <= kMaxSplits and
// nsplit * volume <= kSplitBudget; no workspace once the 16x16 tiles alone fill the chip.
constexpr size_t kSplitBudget = 16u << 20;

int corr_max_splits(int B, int OC, int Ho, int Wo) {
  const long long tiles = (long long)B * ((Ho + 15) / 16) * ((Wo + 15) / 16);
  const size_t vol = (size_t)B * OC * Ho * Wo * sizeof(float);
  if (tiles >= 256 || vol == 0) return 1;
  size_t k = kSplitBudget / vol;
  if (k > (size_t)kMaxSplits) k = kMaxSplits;
  return k < 2 ? 1 : (int)k;
}

size_t corr_workspace_bytes(int B, int OC, int Ho, int Wo) {
  const int k = corr_max_splits(B, OC, Ho, Wo);
  return k > 1 ? (size_t)k * B * OC * Ho * Wo * sizeof(float) : 0;
}

// knob corr_pt=0 disables the parity-tile kernel (measurement of the older paths).
static bool pt_disabled() { return debug_knob("corr_pt", 1) == 0; }

// The band kernel of warp_corr.hip (without the warp) serves model.py:24's correlation at the
// smallest levels (parity half of <= 6 rows: l0, l1 at 384x448; measured 6.8 / 7.8 us against
// 11.0 / 13.4 us for corr_small + its reduce).  Knob corr_band=0 disables it (measurement).
static bool band_enabled() { return debug_knob("corr_band", 1) != 0; }

hipError_t warp_corr_band_f32(const void*, const void*, const void*, void*, void*, int, int, int,
                              int, float, int, hipStream_t);

hipError_t corr_forward_rows(const void*, const void*, void*, int, int, int, int, float, int,
                             hipStream_t);

// corr_stream.hip: full-width row bands + loader wave (the l4-sized grids; it decides).
hipError_t corr_forward_stream(const void*, const void*, void*, int, int, int, int, int, int,
                               int, float, hipStream_t);
bool corr_stream_accepts(const void*, const void*, const void*, int, int, int, int, int, int);
bool corr_mstrip16_accepts(const void*, const void*, const void*, int, int, int, int, int, int,
                           int);
bool corr_strip_accepts(const void*, const void*, const void*, int, int, int, int, int, int, int);
bool corr_rows_accepts(int, int, int, int, int);
bool warp_corr_band_accepts(int, int, int, int, int);

// The first stages of corr_forward_t's dispatch as one predicate: which of the stream, band and
// row-band kernels serves a problem (kPathOther: a later stage).  corr_forward_t launches in this
// order, and the group entry (capi.hip) pairs two problems in one row-band launch only when both
// would take the row-band kernel alone -- so a grouped result equals the single call's.
int corr_forward_path(const void* in1, const void* in2, const void* out, int B, int C, int H,
                      int W, int pad, int k, int md, int s1, int s2, int layout, int dtype) {
  const bool half = dtype == 1;
  if (k != 1 || s1 != 1) return kPathOther;
  // the stream entry (corr_stream.hip) also runs the strip kernels: fp16 Corr9 grids the
  // matrix-core strip takes go there even where the stream kernel itself would decline
  if ((dtype == 0 || half) && pad == md && md / s2 == 4 && (s2 == 1 || s2 == 2) &&
      (corr_stream_accepts(in1, in2, out, B, C, H, W, s2, half ? 1 : 0) ||
       corr_mstrip16_accepts(in1, in2, out, B, C, H, W, s2, dtype, layout) ||
       corr_strip_accepts(in1, in2, out, B, C, H, W, s2, dtype, layout)))
    return kPathStream;
  const bool c9 = layout == kRaster && s2 == 2 && pad == md && (md == 8 || md == 9);
  if (c9 && dtype == 0 && band_enabled() && (H + 1) / 2 <= 6 &&
      warp_corr_band_accepts(B, C, H, W, 0))
    return kPathBand;
  if (c9 && (dtype == 0 || half) && (uintptr_t)in1 % 16 == 0 && (uintptr_t)in2 % 16 == 0 &&
      (uintptr_t)out % 16 == 0 && corr_rows_accepts(B, C, H, W, half ? 1 : 0))
    return kPathRows;
  return kPathOther;
}

// corr_rows.hip (row bands over full rows) serves l2/l3-sized grids (it decides; PWC_DEBUG knob `rows`).

// `workspace` (>= corr_workspace_bytes) enables channel splitting for grids too small to fill
// the chip; null keeps one workgroup per tile over all channels.
template <typename T>
hipError_t corr_forward_t(const void* in1, const void* in2, void* out, int B, int C, int H,
                          int W, int Ho, int Wo, int pad, int k, int md, int s1, int s2,
                          int layout, float divisor, void* workspace, hipStream_t stream,
                          int force_generic) {
  const int kr = (k - 1) / 2;
  const int dr = md / s2;
  const int D = 2 * dr + 1;
  const int max_splits = workspace ? corr_max_splits(B, D * D, Ho, Wo) : 1;
  if (max_splits <= 1) workspace = nullptr;
  // a strided / activated output (pwc_corr_forward_into) is written by the band, row-band,
  // parity-tile and stream kernels only; every other path declines before launching
  const bool epi_def = epi_is_default(current_epi());
  constexpr bool kHalf = std::is_same<T, __half>::value;
  const int path = force_generic == 0 && (sizeof(T) == 4 || kHalf)
                       ? corr_forward_path(in1, in2, out, B, C, H, W, pad, k, md, s1, s2, layout,
                                           kHalf ? 1 : 0)
                       : kPathOther;
  if (path == kPathStream) {
    const hipError_t e = corr_forward_stream(in1, in2, out, B, C, H, W, s2, kHalf ? 1 : 0,
                                             layout, divisor, stream);
    // a strip launcher declines a divisor other than its compile-time C (no C ABI entry passes
    // one: Correlation divides by k^2 C); where no stream geometry takes such a grid either,
    // the later stages below serve it
    if (e != hipErrorNotSupported) return e;
  }
  if (path == kPathBand)
    return warp_corr_band_f32(in1, in2, nullptr, nullptr, out, B, C, H, W, divisor, 0, stream);
  if (path == kPathRows)
    return corr_forward_rows(in1, in2, out, B, C, H, W, divisor, kHalf ? 1 : 0, stream);
  if (force_generic == 0 && k == 1 && s1 == 1 && sizeof(T) == 4) {
    // stride-2 displacements with 16-B aligned rows (l2..l4 of PWC-Net): parity tiles
    // (corr_pt.hip), channel groups chosen by grid size
    if (dr == 4 && s2 == 2 && W % 4 == 0 && (md - pad) % 4 == 0 && !pt_disabled()) {
      const hipError_t e = corr_forward_pt_f32(in1, in2, out, B, C, H, W, Ho, Wo, md - pad, dr,
                                               s2, layout, divisor, 0, stream);
      if (e != hipErrorNotSupported) return e;
    }
    // the smallest levels (l0, l1: a few hundred pixels, unaligned rows): whole parity halves
    // per workgroup, channel slices over the workspace (corr_small.hip)
    if (dr == 4 && s2 == 2 && 9 * ((Ho + 1) / 2) * ((Wo + 7) / 8) <= 256 && !pt_disabled() &&
        epi_def) {
      const hipError_t e = corr_forward_small_f32(in1, in2, out, B, C, H, W, Ho, Wo, md - pad,
                                                  dr, s2, layout, divisor, max_splits,
                                                  workspace, stream);
      if (e != hipErrorNotSupported) return e;
    }
  }
  if (!epi_def) return hipErrorNotSupported;
  if (force_generic != 1 && k == 1 && s1 == 1 && dr == 4) {
    const int off = md - pad;
    if (s2 == 2)
      return launch_tiled<Corr9, T>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor,
                                    max_splits, workspace, stream);
    if (s2 == 1)
      return launch_tiled<Corr4, T>(in1, in2, out, B, C, H, W, Ho, Wo, off, layout, divisor,
                                    max_splits, workspace, stream);
  }
  return launch_generic<T>(in1, in2, out, B, C, H, W, Ho, Wo, pad, kr, md, s1, s2, dr, layout,
                           divisor, stream);
}

#define PWC_INST(T)                                                                          \
  template hipError_t corr_forward_t<T>(const void*, const void*, void*, int, int, int, int,   \
                                        int, int, int, int, int, int, int, int, float, void*,  \
                                        hipStream_t, int);
PWC_INST(float)
PWC_INST(__half)
PWC_INST(__hip_bfloat16)
#undef PWC_INST

}  // namespace pwc
