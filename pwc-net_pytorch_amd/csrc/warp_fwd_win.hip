// warp_fwd_win.hip — forward flow warp (WarpingLayer, modules.py:31-42; grid_sample bilinear,
// zeros, align_corners=True) of large grids through an LDS window.
//
// warp_fwd_kernel gathers every corner of every channel from global memory: under the bench's
// N(0, 2^2)-px flows a 64-lane pair gather touches ~56 cache lines, and the vector L1's tag
// lookups, not HBM, bound it (profiles/r02i_warp_fwd_flowscale_pmc.txt).  Here a workgroup owns
// one image n x a TH x TW tile of output pixels x a slice of the channels.  Each pixel's sample
// (the reference's coordinate chain) is computed once; the slice's channels then stream through
// LDS in chunks of CC: the chunk's window (the tile plus an M = 8 px margin on every side) comes
// in with 16-byte coalesced buffer loads -- the next chunk's loads in flight while this one is
// blended and stored -- and every pixel takes its four corners from LDS.  A corner outside the
// image points at a zero slot of the chunk plane (the reference's zeros padding); a pixel whose
// corners leave the window (|flow| beyond the margin) reads them from global memory instead,
// behind a wave-uniform branch -- exact for any flow, fast for the small ones.
//
// Bit-identical to warp_fwd_kernel: the same sample chain (warp_sample.cuh), the same corner
// values (a valid corner reads x at its own pixel either way; warp.hip's pair loads only change
// how it is fetched; a masked corner is +0 either way), the same fmaf order and store rounding.
#include "warp_sample.cuh"

namespace pwc {
namespace wwin {

constexpr int NT = 256;  // threads per workgroup
constexpr int M = 8;     // window margin (pixels) on every side of the tile

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Workgroup barrier for LDS hand-offs only (__syncthreads() would also wait for the next
// chunk's loads in flight).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS operations
  __builtin_amdgcn_s_barrier();
}

template <typename T, int TH, int TW, int CC>
struct Geo {
  static constexpr int ES = (int)sizeof(T);
  static constexpr int Q = 16 / ES;                 // elements per 16-byte quad
  static constexpr int WH = TH + 2 * M, WW = TW + 2 * M;
  static constexpr int PS = WH * WW;                // LDS slots per chunk channel
  static constexpr int QR = WW / Q, NQ = WH * QR;   // quads per window row / per channel
  static constexpr int QPT = (NQ + NT - 1) / NT;    // quads per thread per channel
  static constexpr int NPIX = TH * TW, PPT = (NPIX + NT - 1) / NT;
  static_assert(TW % Q == 0 && M % Q == 0, "quads never straddle the tile or the image edge");
};

template <typename T, int TH, int TW, int CC>
__global__ __launch_bounds__(NT) void warp_fwd_win(const T* __restrict__ x,
                                                  const T* __restrict__ flow,
                                                  T* __restrict__ out, int C, int H, int W,
                                                  float halfx, float halfy, int ntx, int ntiles,
                                                  int nslices, int cps) {
  using G = Geo<T, TH, TW, CC>;
  constexpr int ES = G::ES, Q = G::Q, WH = G::WH, WW = G::WW, PS = G::PS;
  constexpr int QR = G::QR, NQ = G::NQ, QPT = G::QPT, NPIX = G::NPIX, PPT = G::PPT;
  __shared__ __attribute__((aligned(16))) T win[CC * PS];

  const int t = threadIdx.x;
  // tiles of one (image, channel slice) consecutive on one XCD: their halos meet in one L2
  const int u = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = u % ntiles, rest = u / ntiles;
  const int s = rest % nslices, n = rest / nslices;
  const int ty0 = (tile / ntx) * TH, tx0 = (tile % ntx) * TW;
  const int wy0 = ty0 - M, wx0 = tx0 - M;
  const unsigned plane = (unsigned)(H * W);
  const int cs = s * cps, ce = min(C, cs + cps);

  // ---- the flow of this thread's pixels first (the coordinate chain then waits for these
  // alone), then the first chunk's window ----
  const T* fl = flow + (size_t)(2 * n) * plane;
  float fu[PPT], fv[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int i = t + k * NT;
    const int r = i / TW, col = i - r * TW;
    const int oy = ty0 + r, ox = tx0 + col;
    const unsigned pix = i < NPIX && oy < H && ox < W ? (unsigned)(oy * W + ox) : 0u;
    fu[k] = to_f32(fl[pix]);
    fv[k] = to_f32(fl[plane + pix]);
  }

  // ---- the window loads of a chunk: out-of-image quads, channels past the slice and idle
  // slots read zeros from the range check (a fixed number of loads in flight) -- so window
  // cells outside the image hold the reference's zero padding ----
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + (size_t)n * C * plane), (short)0, (int)((unsigned)C * plane * (unsigned)ES),
      0x00020000);
  constexpr unsigned kOOB = 0x80000000u;
  unsigned qoff[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int qi = t + j * NT;
    const int wr = qi / QR, wq = qi - wr * QR;
    const int gy = wy0 + wr, gx = wx0 + wq * Q;
    const bool ok = qi < NQ && gy >= 0 && gy < H && gx >= 0 && gx < W;
    qoff[j] = ok ? (unsigned)(gy * W + gx) * ES : kOOB;
  }
  u32x4 v[CC][QPT];
  auto issue = [&](int cb) {
#pragma unroll
    for (int c = 0; c < CC; ++c)
#pragma unroll
      for (int j = 0; j < QPT; ++j) {
        const unsigned off = cb + c < ce && qoff[j] != kOOB
                                 ? qoff[j] + (unsigned)(cb + c) * plane * ES : kOOB;
        v[c][j] = __builtin_bit_cast(u32x4,
                                     __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
      }
  };
  issue(cs);

  // ---- each pixel's sample, once: coordinates, window slot and weights.  The corners are
  // taken at their unclamped positions: one outside the image is a zero cell of the window,
  // which is exactly the reference's masked corner (+0). ----
  int a[PPT];
  float w[PPT][4];
  bool live[PPT];
  unsigned long long farm[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int i = t + k * NT;
    const int r = i / TW, col = i - r * TW;
    const int oy = ty0 + r, ox = tx0 + col;
    live[k] = i < NPIX && oy < H && ox < W;
    const float ix = src_coord(fu[k], ox, W, halfx);
    const float iy = src_coord(fv[k], oy, H, halfy);
    const Bilinear b = bilinear(ix, iy, H, W);
    w[k][0] = b.wx0 * b.wy0;  // feed fma operands: not fusable
    w[k][1] = b.wx1 * b.wy0;
    w[k][2] = b.wx0 * b.wy1;
    w[k][3] = b.wx1 * b.wy1;
    // (no "+ 1" on the corner: a saturated conversion of a huge coordinate must not wrap)
    const bool inw = b.y0 >= wy0 && b.y0 < wy0 + WH - 1 && b.x0 >= wx0 && b.x0 < wx0 + WW - 1;
    a[k] = inw ? (b.y0 - wy0) * WW + (b.x0 - wx0) : 0;
    farm[k] = __builtin_amdgcn_ballot_w64(live[k] && !inw);  // wave-uniform
    if (!inw) a[k] = -1;  // the global branch below
  }

  const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + (size_t)n * C * plane), (short)0, (int)((unsigned)C * plane * (unsigned)ES),
      0x00020000);

  // ---- the chunks ----
  for (int cb = cs; cb < ce; cb += CC) {
    lds_barrier();  // the previous chunk's readers are done
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
      const int qi = t + j * NT;
      if (qi < NQ) {
        const int wr = qi / QR, wq = qi - wr * QR;
#pragma unroll
        for (int c = 0; c < CC; ++c)
          *reinterpret_cast<u32x4*>(&win[c * PS + wr * WW + wq * Q]) = v[c][j];
      }
    }
    lds_barrier();
    // the next chunk's loads fly under this chunk's blends and stores (past the slice: zeros)
    issue(cb + CC);
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int i = t + k * NT;
      const int r = i / TW, col = i - r * TW;
      const int oy = ty0 + r, ox = tx0 + col;
      const unsigned opix = (unsigned)(oy * W + ox);
      const int ak = max(a[k], 0);
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        const T* wc = win + c * PS + ak;
        float v00 = to_f32(wc[0]), v01 = to_f32(wc[1]);
        float v10 = to_f32(wc[WW]), v11 = to_f32(wc[WW + 1]);
        if (farm[k] != 0) {
          if (live[k] && a[k] < 0) {
            // outside the window: warp_fwd_kernel's own gathers (clamped, masked)
            const Bilinear b = bilinear(src_coord(fu[k], ox, W, halfx),
                                        src_coord(fv[k], oy, H, halfy), H, W);
            const Corners kc = corners(b, H, W);
            const T* p = x + ((size_t)n * C + min(cb + c, C - 1)) * plane;
            v00 = masked(to_f32(p[kc.i00]), kc.m00);
            v01 = masked(to_f32(p[kc.i01]), kc.m01);
            v10 = masked(to_f32(p[kc.i10]), kc.m10);
            v11 = masked(to_f32(p[kc.i11]), kc.m11);
          }
        }
        float acc = 0.f;
        acc = fmaf(v00, w[k][0], acc);
        acc = fmaf(v01, w[k][1], acc);
        acc = fmaf(v10, w[k][2], acc);
        acc = fmaf(v11, w[k][3], acc);
        // branch-free buffer stores (a skipped store would leave the compiler unsure how many
        // operations are in flight, and it would wait for the next chunk's loads as well)
        const unsigned off = live[k] && cb + c < ce
                                 ? ((unsigned)(cb + c) * plane + opix) * ES : kOOB;
        if constexpr (ES == 4)  // nontemporal, as warp_fwd_kernel's st_out1
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc), rso, (int)off, 0, 2);
        else
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, from_f32<T>(acc)),
                                                rso, (int)off, 0, 0);
      }
    }
  }
}

}  // namespace wwin

// The window path of warp_forward_t (large grids).  Measured (tools/kbench.py --ops warp,
// graph-replayed, profiles/r06k_warp_fwd_window.txt): config 4 (fp16, B = 16, 448 x 1024)
// l2 / l3 / l4 8.5 / 16.9 / 29.9 -> 7.6 / 12.7 / 20.8 us with 8-row tiles and 4-channel chunks;
// fp32 (config 2 l3 / l4, 2-channel chunks) 5.7 / 9.0 -> 6.1 / 8.9 -- fp32 keeps the gathers and
// this kernel is instantiated for 16-bit storage only.  hipErrorNotSupported when it declines
// (fp32; rows not a whole number of 16-byte quads; a plane too large for one buffer resource;
// fewer than 64 tiles unless knob warp_win = 2; knob warp_win = 0) -- the caller then runs
// warp_fwd_kernel.
template <typename T>
hipError_t warp_forward_win_t(const void* x, const void* flow, void* out, int B, int C, int H,
                              int W, hipStream_t stream) {
  if constexpr (sizeof(T) == 4) {
    return hipErrorNotSupported;
  } else {
  using namespace wwin;
  constexpr int Q = 16 / (int)sizeof(T);
  const int mode = debug_knob("warp_win", 1);
  if (mode == 0) return hipErrorNotSupported;
  if (W % Q != 0 || B <= 0 || C <= 0 || H <= 0) return hipErrorNotSupported;
  if ((size_t)C * H * W * sizeof(T) >= (1ull << 31)) return hipErrorNotSupported;
  // tile width: 56 where it divides the row and 64 does not (W = 112, 56), else 64
  const bool t56 = W % 56 == 0 && W % 64 != 0;
  constexpr int TH = 8, CC = 4;
  const int TW = t56 ? 56 : 64;
  const int ntx = (W + TW - 1) / TW, nty = (H + TH - 1) / TH;
  const int ntiles = ntx * nty;
  const long long units = (long long)B * ntiles;
  if (mode == 1 && units < 64) return hipErrorNotSupported;
  // channel slices: about 2048 workgroups (eight per CU), at least two chunks each where the
  // channels allow (config 4: l2 768 workgroups x 2 chunks, l3 1792 x 2, l4 2688 x 3)
  const int nchunks = (C + CC - 1) / CC;
  const long long target = debug_knob("warp_win_wgs", 2048);
  long long ns = (target + units - 1) / units;
  if (ns > nchunks / 2) ns = nchunks / 2;
  if (ns < 1) ns = 1;
  const int cpc = (int)((nchunks + ns - 1) / ns);  // chunks per slice
  const int cps = cpc * CC;
  const int nslices = (C + cps - 1) / cps;
  const unsigned long long grid = (unsigned long long)units * nslices;
  if (grid >= (1ull << 31)) return hipErrorNotSupported;
  const float halfx = (float)((W - 1.0) / 2.0), halfy = (float)((H - 1.0) / 2.0);
#define PWC_WIN(TW_)                                                                          \
  hipLaunchKernelGGL((warp_fwd_win<T, TH, TW_, CC>), dim3((unsigned)grid), dim3(NT), 0, stream, \
                     (const T*)x, (const T*)flow, (T*)out, C, H, W, halfx, halfy, ntx, ntiles,  \
                     nslices, cps)
  if (t56)
    PWC_WIN(56);
  else
    PWC_WIN(64);
#undef PWC_WIN
  return hipGetLastError();
  }
}

template hipError_t warp_forward_win_t<float>(const void*, const void*, void*, int, int, int, int,
                                              hipStream_t);
template hipError_t warp_forward_win_t<__half>(const void*, const void*, void*, int, int, int,
                                               int, hipStream_t);
template hipError_t warp_forward_win_t<__hip_bfloat16>(const void*, const void*, void*, int, int,
                                                       int, int, hipStream_t);

}  // namespace pwc
