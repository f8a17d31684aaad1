// colbench.hip -- standalone check + timing + phase census of the l4 column-item correlation
// (tools/corr_cols.hip, a rejected prototype kept for the record), no torch.  B=8, C=32, 96x112 fp32 (config 2's l4): full compare with an
// fp64 CPU restatement of correlation_cuda_kernel.cu:34-106, then per-launch hipExtLaunchKernel
// event times over 6 rotating buffer sets (> the 256 MiB Infinity Cache) and per-workgroup
// s_memrealtime phase stamps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPWC_COLS_CENSUS -o tools/colbench tools/colbench.hip
//   tools/colbench [iters]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "corr_cols.hip"

namespace pwc {
hipEvent_t g_e0 = nullptr, g_e1 = nullptr;
void take_launch_events(hipEvent_t* a, hipEvent_t* b) {
  *a = g_e0;
  *b = g_e1;
  g_e0 = g_e1 = nullptr;
}
OutEpi current_epi() { return OutEpi{0, 1.f}; }
hipError_t lds_limit(const void* k, int bytes) {  // one device here
  return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
int debug_knob(const char*, int def) { return def; }
}  // namespace pwc

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)

// variants: cols::launch over other geometries (measurement)
static hipError_t run_variant(int v, const float* a, const float* b, float* o, int B, int C,
                              int H, int W) {
  using namespace pwc::cols;
  switch (v) {
    case 1: return launch<Geo<3, 14, 4, 4>>(a, b, o, B, C, H, W, W / 56, (float)C, 0);
    default: return pwc::corr_forward_cols(a, b, o, B, C, H, W, 0, (float)C, 0);
  }
}

int main(int argc, char** argv) {
  const int B = 8, C = 32, H = 96, W = 112, iters = argc > 1 ? std::atoi(argv[1]) : 200;
  const int abl = argc > 2 ? std::atoi(argv[2]) : 0, variant = argc > 3 ? std::atoi(argv[3]) : 0;
  const int chk_abl = abl & 4;  // the check runs with the sync-only ablation bits
  const size_t nin = (size_t)B * C * H * W, nout = (size_t)B * 81 * H * W;
  const int NSET = 6;
  std::vector<float*> f1(NSET), f2(NSET), out(NSET);
  std::vector<float> h1(nin), h2(nin);
  unsigned s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xffff) / 32768.f - 1.f; };
  for (size_t i = 0; i < nin; ++i) h1[i] = rnd();
  for (size_t i = 0; i < nin; ++i) h2[i] = rnd();
  for (int k = 0; k < NSET; ++k) {
    CK(hipMalloc(&f1[k], nin * 4));
    CK(hipMalloc(&f2[k], nin * 4));
    CK(hipMalloc(&out[k], nout * 4));
    CK(hipMemcpy(f1[k], h1.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(f2[k], h2.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemset(out[k], 0xff, nout * 4));  // NaN poison
  }
  const int nblk = B * 2 * 16;
  constexpr int NSL = 16;
  unsigned long long* cen;
  CK(hipMalloc(&cen, (size_t)(iters + 1) * nblk * NSL * 8));
  CK(hipMemset(cen, 0, (size_t)(iters + 1) * nblk * NSL * 8));
  auto set_census = [&](int i) {
    unsigned long long* p = cen + (size_t)i * nblk * NSL;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::cols::g_census), &p, sizeof(p)));
  };
  // ---- correctness ----
  set_census(iters);
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::cols::g_abl), &chk_abl, sizeof(int)));
  CK(run_variant(variant, f1[0], f2[0], out[0], B, C, H, W));
  CK(hipDeviceSynchronize());
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::cols::g_abl), &abl, sizeof(int)));
  std::vector<float> ho(nout);
  CK(hipMemcpy(ho.data(), out[0], nout * 4, hipMemcpyDeviceToHost));
  double maxerr = 0, maxref = 0;
  long bad = 0, bad_tj[9] = {0}, bad_x[2] = {0}, bad_y[2] = {0};
  for (int n = 0; n < B; ++n)
    for (int tj = -4; tj <= 4; ++tj)
      for (int ti = -4; ti <= 4; ++ti)
        for (int y = 0; y < H; ++y)
          for (int x = 0; x < W; ++x) {
            const int y2 = y + 2 * tj, x2 = x + 2 * ti;
            double acc = 0;
            if (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W)
              for (int c = 0; c < C; ++c)
                acc += (double)h1[((size_t)(n * C + c) * H + y) * W + x] *
                       (double)h2[((size_t)(n * C + c) * H + y2) * W + x2];
            acc /= C;
            const float g = ho[(((size_t)n * 81 + (tj + 4) * 9 + ti + 4) * H + y) * W + x];
            const double e = std::fabs((double)g - acc);
            if (!(e <= 1e-5)) {
              if (bad < 6)
                std::printf("bad n=%d tj=%d ti=%d y=%d x=%d got=%g ref=%g\n", n, tj, ti, y, x,
                            (double)g, acc);
              ++bad_tj[tj + 4];
              ++bad_x[x / 56];
              ++bad_y[y % 2];
              ++bad;
            }
            if (e > maxerr || e != e) maxerr = e != e ? 1e30 : std::max(maxerr, e);
            maxref = std::max(maxref, std::fabs(acc));
          }
  std::printf("bad by tj: %ld %ld %ld %ld %ld %ld %ld %ld %ld; by item: %ld %ld; by parity %ld %ld\n",
              bad_tj[0], bad_tj[1], bad_tj[2], bad_tj[3], bad_tj[4], bad_tj[5], bad_tj[6],
              bad_tj[7], bad_tj[8], bad_x[0], bad_x[1], bad_y[0], bad_y[1]);
  std::printf("{\"check\": \"corr9 l4 B=8 vs fp64\", \"max_abs_err\": %.3e, \"max_abs_ref\": %.3f, \"bad\": %ld}\n",
              maxerr, maxref, bad);
#ifndef PWC_COLS_M
  if (bad) return 1;  // (measurement builds compute wrong values on purpose)
#endif
  // ---- timing ----
  std::vector<hipEvent_t> e0(iters), e1(iters);
  for (int i = 0; i < iters; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  for (int i = 0; i < 50; ++i)
    CK(run_variant(variant, f1[i % NSET], f2[i % NSET], out[i % NSET], B, C, H, W));
  CK(hipDeviceSynchronize());
  for (int i = 0; i < iters; ++i) {
    set_census(i);
    pwc::g_e0 = e0[i];
    pwc::g_e1 = e1[i];
    CK(run_variant(variant, f1[i % NSET], f2[i % NSET], out[i % NSET], B, C, H, W));
  }
  CK(hipDeviceSynchronize());
  std::vector<double> ev(iters);
  for (int i = 0; i < iters; ++i) {
    float ms;
    CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
    ev[i] = ms * 1e3;
  }
  std::vector<double> sorted = ev;
  std::sort(sorted.begin(), sorted.end());
  double mean_ev = 0;
  for (double v : ev) mean_ev += v;
  mean_ev /= iters;
  std::vector<unsigned long long> c((size_t)iters * nblk * NSL);
  CK(hipMemcpy(c.data(), cen, c.size() * 8, hipMemcpyDeviceToHost));
  // per slot: mean over workgroups of (stamp - the workgroup's wave-0 start), and the max over
  // workgroups of (stamp - the launch's earliest start)
  constexpr int NN = 14;
  const char* names[NN] = {"start", "loader_loop", "grp1_start", "stage0_published", "stage0_seen",
                           "item0_loop", "item0_stored", "item1_loop", "grp0_done",
                           "last_published", "compute_ready", "grp1_done",
                           "stage8_published", "stage8_issued"};
  double mean[NN] = {0}, mx[NN] = {0};
  for (int i = 0; i < iters; ++i) {
    const unsigned long long* L = c.data() + (size_t)i * nblk * NSL;
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < nblk; ++b) t0 = std::min(t0, L[b * NSL]);
    for (int k = 0; k < NN; ++k) {
      unsigned long long m = 0;
      for (int b = 0; b < nblk; ++b) {
        mean[k] += (double)(long long)(L[b * NSL + k] - L[b * NSL]) * 0.01 / nblk / iters;
        m = std::max(m, L[b * NSL + k] - t0);
      }
      mx[k] += m * 0.01 / iters;
    }
  }
  const double bytes = (2.0 * nin + nout) * 4;
  std::printf("{\"kernel\": \"corr_fwd_cols l4 B=8\", \"variant\": %d, \"abl\": %d, \"event_us_mean\": %.2f, "
              "\"event_us_min\": %.2f, \"frac_8TBs\": %.3f", variant, abl, mean_ev, sorted[0],
              bytes / (mean_ev * 1e-6) / 8e12);
  for (int k = 1; k < NN; ++k) std::printf(", \"%s\": [%.2f, %.2f]", names[k], mean[k], mx[k]);
  std::printf("}\n");
  return 0;
}
