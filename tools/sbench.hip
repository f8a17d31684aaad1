// sbench.hip -- standalone timing + phase census of the l4 stream correlation kernel
// (csrc/corr_stream.hip), no torch.  Per launch: hipExtLaunchKernel event time; per
// workgroup: s_memrealtime at start, loader's last landing, loop end, parked, stores issued.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPWC_STREAM_CENSUS -o tools/sbench tools/sbench.hip
//   PWC_DEBUG=stream_abl=.. tools/sbench [iters]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../pwc-net_pytorch_amd/csrc/corr_stream.hip"

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
int debug_knob(const char* name, int def) {
  const char* e = std::getenv("PWC_DEBUG");
  if (!e) return def;
  std::string s(e), n(name);
  size_t p = s.find(n + "=");
  return p == std::string::npos ? def : std::atoi(s.c_str() + p + n.size() + 1);
}
}  // namespace pwc

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)

int main(int argc, char** argv) {
  const int B = 8, C = 32, H = 96, W = 112, iters = argc > 1 ? std::atoi(argv[1]) : 100;
  const size_t nin = (size_t)B * C * H * W, nout = (size_t)B * 81 * H * W;
  const int NS = 6;
  std::vector<float*> f1(NS), f2(NS), out(NS);
  std::vector<float> h(nin);
  for (size_t i = 0; i < nin; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
  for (int s = 0; s < NS; ++s) {
    CK(hipMalloc(&f1[s], nin * 4));
    CK(hipMalloc(&f2[s], nin * 4));
    CK(hipMalloc(&out[s], nout * 4));
    CK(hipMemcpy(f1[s], h.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(f2[s], h.data(), nin * 4, hipMemcpyHostToDevice));
  }
  const int nblk = B * 2 * 16;
  unsigned long long* cen;
  CK(hipMalloc(&cen, (size_t)iters * nblk * 8 * 8));
  CK(hipMemset(cen, 0, (size_t)iters * nblk * 8 * 8));
  std::vector<hipEvent_t> e0(iters), e1(iters);
  for (int i = 0; i < iters; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  for (int i = 0; i < 10; ++i) {
    unsigned long long* p = cen;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::stream::g_census), &p, sizeof(p)));
    CK(pwc::corr_forward_stream(f1[i % NS], f2[i % NS], out[i % NS], B, C, H, W, 2, 0, 0, 32.f, 0));
  }
  CK(hipDeviceSynchronize());
  for (int i = 0; i < iters; ++i) {
    unsigned long long* p = cen + (size_t)i * nblk * 8;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::stream::g_census), &p, sizeof(p)));
    pwc::g_e0 = e0[i];
    pwc::g_e1 = e1[i];
    CK(pwc::corr_forward_stream(f1[i % NS], f2[i % NS], out[i % NS], B, C, H, W, 2, 0, 0, 32.f, 0));
  }
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> c((size_t)iters * nblk * 8);
  CK(hipMemcpy(c.data(), cen, c.size() * 8, hipMemcpyDeviceToHost));
  double ev = 0;
  for (int i = 0; i < iters; ++i) {
    float ms;
    CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
    ev += ms * 1e3;
  }
  // per launch: phase spans relative to the earliest workgroup start (10 ns ticks -> us)
  double span_start = 0, land = 0, loop = 0, park = 0, issued = 0, loopdur = 0, pbar = 0;
  for (int i = 0; i < iters; ++i) {
    const unsigned long long* L = c.data() + (size_t)i * nblk * 8;
    unsigned long long t0 = ~0ull, t0max = 0, tl = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
    double ld = 0;
    for (int b = 0; b < nblk; ++b) {
      t0 = std::min(t0, L[b * 8 + 0]);
      t0max = std::max(t0max, L[b * 8 + 0]);
      tl = std::max(tl, L[b * 8 + 1]);
      t2 = std::max(t2, L[b * 8 + 2]);
      t3 = std::max(t3, L[b * 8 + 3]);
      t4 = std::max(t4, L[b * 8 + 4]);
      t5 = std::max(t5, L[b * 8 + 5]);
      ld += (double)(L[b * 8 + 2] - L[b * 8 + 0]);
    }
    span_start += (t0max - t0) * 0.01;
    land += (tl - t0) * 0.01;
    loop += (t2 - t0) * 0.01;
    park += (t3 - t0) * 0.01;
    issued += (t4 - t0) * 0.01;
    pbar += (t5 - t0) * 0.01;
    loopdur += ld / nblk * 0.01;
  }
  std::printf("{\"event_us\": %.2f, \"start_skew_us\": %.2f, \"last_landed_us\": %.2f, "
              "\"loop_done_us\": %.2f, \"mean_wg_loop_us\": %.2f, \"park_barrier_us\": %.2f, \"parked_us\": %.2f, "
              "\"stores_issued_us\": %.2f}\n",
              ev / iters, span_start / iters, land / iters, loop / iters, loopdur / iters,
              pbar / iters, park / iters, issued / iters);
  return 0;
}
