// strip_bench.hip -- standalone check + timing of the l4 strip correlation (csrc/corr_strip.hip)
// against the stream kernel (csrc/corr_stream.hip), no torch.  Config 2 l4: B=8, 32x96x112 fp32,
// Correlation(9,1,9,1,2).  Prints: v_permlane32_swap semantics check, max |strip - stream|,
// max |kernel - fp64 host| over a sample, and per-launch event times of both (buffer sets
// rotated past the Infinity Cache, launches back to back, the two kernels alternated).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/strip_bench tools/strip_bench.hip
//   tools/strip_bench [iters] [B] [H] [W]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../pwc-net_pytorch_amd/csrc/corr_stream.hip"
#include "../pwc-net_pytorch_amd/csrc/corr_strip.hip"
#include "../pwc-net_pytorch_amd/csrc/corr_mstrip16.hip"

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

// the stream kernel itself (corr_forward_stream now hands these shapes to the strip kernel)
static hipError_t stream_ref(const void* a, const void* b, void* o, int B, int C, int H, int W) {
  return W % 112 == 0 ? pwc::stream::pick<float, 2, 112>(a, b, o, B, C, H, W, 0, 32.f, 0)
                      : pwc::stream::pick<float, 2, 128>(a, b, o, B, C, H, W, 0, 32.f, 0);
}

// geometries the harness can time (PWC_DEBUG strip_geo=N; the library ships 4 = GeoL4 and
// 10 = GeoF, its default at W = 112)
using G5 = pwc::strip::Geo<32, 12, 56, 2, 2, 2>;
using G6 = pwc::strip::Geo<32, 12, 56, 2, 2, 1>;
using G7 = pwc::strip::Geo<32, 12, 56, 2, 4, 1>;
using G8 = pwc::strip::Geo<32, 12, 56, 2, 4, 2>;
using G9 = pwc::strip::Geo<32, 6, 56, 1, 2, 2>;
using G10 = pwc::strip::GeoF;
using G11 = pwc::strip::Geo<32, 6, 112, 2, 3, 1, true>;     // 2 steps of 3 rows, 12 compute waves
static int g_geo = 10;
template <class F>
static auto with_geo(F&& f) {
  switch (g_geo) {
    case 4: return f(pwc::strip::GeoL4{});
    case 6: return f(G6{});
    case 7: return f(G7{});
    case 8: return f(G8{});
    case 9: return f(G9{});
    case 10: return f(G10{});
    case 11: return f(G11{});
    case 5: return f(G5{});
    default: return f(G10{});
  }
}
static hipError_t strip_call(const void* a, const void* b, void* o, int B, int H, int W) {
  return with_geo([&](auto g) {
    return pwc::strip::launch<decltype(g)>(a, b, o, B, H, W, 32.f, 0);
  });
}

__global__ void swap_probe(unsigned* o) {
  const unsigned l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  o[l] = r[0];
  o[64 + l] = r[1];
}

// STRIP_PRODUCER: rewrite f2 (nontemporal 16-B stores, as the warp kernel writes x2_warp)
// right before each timed strip launch -- the bench step's order (warp, then correlation)
// (STRIP_PRODUCER=1 nt, 2 plain, 3 sc1, 4 sc0 sc1: the store cache policy of the producer)
typedef float pf4 __attribute__((ext_vector_type(4)));
template <int AUX>
__global__ void produce(const pf4* __restrict__ src, pf4* __restrict__ dst, unsigned n) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, (int)(n * 16), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(src[i < n ? i : 0], r, (int)(i < n ? i * 16 : 0x80000000u), 0, AUX);
}

// one dword per `stride` bytes of a buffer (STRIP_WARM); the sum goes to a sink so the loads stay
__global__ void touch_pages(const char* p, unsigned n, unsigned stride, unsigned* sink) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned v = *reinterpret_cast<const unsigned*>(p + (size_t)i * stride);
  if (v == 0x12345678u) sink[threadIdx.x] = v;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  const int B = argc > 2 ? std::atoi(argv[2]) : 8;
  const int H = argc > 3 ? std::atoi(argv[3]) : 96;
  const int W = argc > 4 ? std::atoi(argv[4]) : 112;
  const int C = 32;
  g_geo = pwc::debug_knob("strip_geo", 10);
  {
    unsigned* d;
    CK(hipMalloc(&d, 128 * 4));
    swap_probe<<<1, 64>>>(d);
    unsigned h[128];
    CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    std::printf("{\"swap\": \"lane0 r0=%u r1=%u; lane32 r0=%u r1=%u\"}\n", h[0], h[64], h[32],
                h[96]);
    CK(hipFree(d));
  }
  const size_t nin = (size_t)B * C * H * W, nout = (size_t)B * 81 * H * W;
  const size_t set_b = (2 * nin + nout) * 4;
  const char* ns_env = std::getenv("STRIP_SETS");  // rotating buffer sets (default: past 320 MiB)
  const int NS = ns_env ? std::max(1, std::atoi(ns_env)) : std::max(2, (int)((320ull << 20) / set_b) + 1);
  std::vector<float*> f1(NS), f2(NS), o1(NS), o2(NS);
  std::vector<float> h1(nin), h2(nin);
  uint32_t s = 12345;
  auto rnd = [&] {
    s = s * 1664525u + 1013904223u;
    return (float)((s >> 8) & 0xffff) / 32768.f - 1.f;
  };
  for (auto& v : h1) v = rnd();
  for (auto& v : h2) v = rnd();
  // probe mode (argv[5] = channel c0): f1 one-hot in channel c0, f2 = 1 + y * 1000 + x + c * 1e5
  // (exact in fp32) -> out * C names the f2 element each output read
  const int probe = argc > 5 ? std::atoi(argv[5]) : -1;
  if (probe >= 0) {
    for (size_t i = 0; i < nin; ++i) {
      const int x = (int)(i % W), y = (int)(i / W % H), c = (int)(i / ((size_t)W * H) % C);
      h1[i] = c == probe ? 1.f : 0.f;
      h2[i] = 1.f + y * 1000.f + x + c * 100000.f;
    }
  }
  for (int i = 0; i < NS; ++i) {
    CK(hipMalloc(&f1[i], nin * 4));
    CK(hipMalloc(&f2[i], nin * 4));
    CK(hipMalloc(&o1[i], nout * 4));
    CK(hipMalloc(&o2[i], nout * 4));
    CK(hipMemcpy(f1[i], h1.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(f2[i], h2.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemset(o1[i], 0xff, nout * 4));  // NaN: an unwritten output shows
    CK(hipMemset(o2[i], 0xff, nout * 4));
  }
  const bool strip_ok = pwc::corr_strip_accepts(f1[0], f2[0], o2[0], B, C, H, W, 2, 0, 0);
  std::printf("{\"shape\": [%d, %d, %d, %d], \"sets\": %d, \"strip_accepts\": %s}\n", B, C, H, W,
              NS, strip_ok ? "true" : "false");
  if (!strip_ok) return 1;
  CK(stream_ref(f1[0], f2[0], o1[0], B, C, H, W));
  CK(strip_call(f1[0], f2[0], o2[0], B, H, W));
  CK(hipDeviceSynchronize());
  std::vector<float> r1(nout), r2(nout);
  CK(hipMemcpy(r1.data(), o1[0], nout * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), o2[0], nout * 4, hipMemcpyDeviceToHost));
  double dmax = 0;
  size_t nbad = 0, first_bad = (size_t)-1;
  for (size_t i = 0; i < nout; ++i) {
    const double d = std::fabs((double)r1[i] - (double)r2[i]);
    if (!(d <= 1e-5)) {
      ++nbad;
      if (first_bad == (size_t)-1) first_bad = i;
    }
    if (d > dmax || d != d) dmax = d != d ? 1e30 : d;
  }
  // fp64 host reference on a sample
  double hmax1 = 0, hmax2 = 0;
  for (size_t i = 0; i < nout; i += 7919) {
    const int x = (int)(i % W), y = (int)(i / W % H), oc = (int)(i / ((size_t)W * H) % 81);
    const int n = (int)(i / ((size_t)W * H * 81));
    const int dy = 2 * (oc / 9 - 4), dx = 2 * (oc % 9 - 4);
    double acc = 0;
    if (y + dy >= 0 && y + dy < H && x + dx >= 0 && x + dx < W)
      for (int c = 0; c < C; ++c)
        acc += (double)h1[(((size_t)n * C + c) * H + y) * W + x] *
               h2[(((size_t)n * C + c) * H + y + dy) * W + x + dx];
    acc /= C;
    hmax1 = std::max(hmax1, std::fabs(acc - r1[i]));
    hmax2 = std::max(hmax2, std::fabs(acc - r2[i]) + (r2[i] != r2[i] ? 1e30 : 0));
  }
  if (nbad) {
    // where the differences are: by output parity row of the group (step = ph / 2), by tj, ti
    size_t by_ph[6] = {}, by_tj[9] = {}, by_ti[9] = {}, by_x[4] = {};
    for (size_t i = 0; i < nout; ++i) {
      const double d = std::fabs((double)r1[i] - (double)r2[i]);
      if (d <= 1e-5) continue;
      const int x = (int)(i % W), y = (int)(i / W % H), oc = (int)(i / ((size_t)W * H) % 81);
      by_ph[(y / 2) % 6]++;
      by_tj[oc / 9]++;
      by_ti[oc % 9]++;
      by_x[(x % 56) / 14]++;
    }
    std::printf("{\"bad_by_ph\": [%zu,%zu,%zu,%zu,%zu,%zu], \"bad_by_tj\": [", by_ph[0], by_ph[1],
                by_ph[2], by_ph[3], by_ph[4], by_ph[5]);
    for (int k = 0; k < 9; ++k) std::printf("%zu%s", by_tj[k], k < 8 ? "," : "], \"bad_by_ti\": [");
    for (int k = 0; k < 9; ++k) std::printf("%zu%s", by_ti[k], k < 8 ? "," : "], \"bad_by_xq\": [");
    std::printf("%zu,%zu,%zu,%zu]}\n", by_x[0], by_x[1], by_x[2], by_x[3]);
    const size_t i = first_bad;
    std::printf("{\"first_bad\": {\"n\": %zu, \"oc\": %zu, \"y\": %zu, \"x\": %zu, \"stream\": %g, "
                "\"strip\": %g}}\n",
                i / ((size_t)W * H * 81), i / ((size_t)W * H) % 81, i / W % H, i % W, r1[i],
                r2[i]);
  }
  if (probe >= 0) {
    const int pts[][4] = {{0, 40, 20, 40}, {0, 40, 20, 0}, {0, 44, 20, 80}, {0, 41, 30, 10},
                          {1, 40, 20, 44}, {0, 12, 4, 60}};  // n, oc, y, x
    for (auto& q : pts) {
      const size_t i = (((size_t)q[0] * 81 + q[1]) * H + q[2]) * W + q[3];
      std::printf("{\"probe\": [%d,%d,%d,%d], \"stream\": %.1f, \"strip\": %.1f}\n", q[0], q[1],
                  q[2], q[3], r1[i] * C, r2[i] * C);
    }
  }
  std::printf("{\"max_abs_strip_vs_stream\": %.3g, \"n_over_1e-5\": %zu, \"host_max_stream\": %.3g, "
              "\"host_max_strip\": %.3g}\n",
              dmax, nbad, hmax1, hmax2);
  std::vector<hipEvent_t> e0(2 * iters), e1(2 * iters);
  for (int i = 0; i < 2 * iters; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  for (int i = 0; i < 20; ++i) {
    CK(stream_ref(f1[i % NS], f2[i % NS], o1[i % NS], B, C, H, W));
    CK(strip_call(f1[i % NS], f2[i % NS], o2[i % NS], B, H, W));
  }
  CK(hipDeviceSynchronize());
  // A: stream x iters, then strip x iters (back to back within each kernel)
  for (int i = 0; i < iters; ++i) {
    pwc::g_e0 = e0[i];
    pwc::g_e1 = e1[i];
    CK(stream_ref(f1[i % NS], f2[i % NS], o1[i % NS], B, C, H, W));
  }
  // STRIP_WARM=stride (bytes): before each timed strip launch, a small kernel loads one dword per
  // stride of that launch's f1, f2 and output (address translations warm, < 2 % of the data
  // cached); the events bracket the strip kernel only
  const char* warm_env = std::getenv("STRIP_WARM");
  const long warm = warm_env ? std::atol(warm_env) : 0;
  unsigned* sink = nullptr;
  if (warm > 0) CK(hipMalloc(&sink, 4096 * 4));
  auto touch = [&](int k) {
    const float* bufs[3] = {f1[k], f2[k], o2[k]};
    const size_t bytes[3] = {nin * 4, nin * 4, nout * 4};
    for (int j = 0; j < 3; ++j) {
      const unsigned n = (unsigned)(bytes[j] / (size_t)warm);
      hipLaunchKernelGGL(touch_pages, dim3((n + 255) / 256), dim3(256), 0, 0,
                         reinterpret_cast<const char*>(bufs[j]), n, (unsigned)warm, sink);
    }
  };
  const char* prod_env = std::getenv("STRIP_PRODUCER");
  const int prod = prod_env ? std::atoi(prod_env) : 0;
  float* psrc = nullptr;
  if (prod) {
    CK(hipMalloc(&psrc, nin * 4));
    CK(hipMemcpy(psrc, h2.data(), nin * 4, hipMemcpyHostToDevice));
  }
  for (int i = 0; i < iters; ++i) {
    if (warm > 0) touch(i % NS);
    if (prod) {
      const dim3 g((unsigned)((nin / 4 + 255) / 256));
      const pf4* a = (const pf4*)psrc;
      pf4* d = (pf4*)f2[i % NS];
      const unsigned n4 = (unsigned)(nin / 4);
      if (prod == 2) hipLaunchKernelGGL(produce<0>, g, dim3(256), 0, 0, a, d, n4);
      else if (prod == 3) hipLaunchKernelGGL(produce<16>, g, dim3(256), 0, 0, a, d, n4);
      else if (prod == 4) hipLaunchKernelGGL(produce<17>, g, dim3(256), 0, 0, a, d, n4);
      else hipLaunchKernelGGL(produce<2>, g, dim3(256), 0, 0, a, d, n4);
    }
    pwc::g_e0 = e0[iters + i];
    pwc::g_e1 = e1[iters + i];
    CK(strip_call(f1[i % NS], f2[i % NS], o2[i % NS], B, H, W));
  }
  CK(hipDeviceSynchronize());
  double ta = 0, tb = 0;
  std::vector<double> vb;
  for (int i = 0; i < iters; ++i) {
    float ms;
    CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
    ta += ms * 1e3;
    CK(hipEventElapsedTime(&ms, e0[iters + i], e1[iters + i]));
    tb += ms * 1e3;
    vb.push_back(ms * 1e3);
  }
  std::sort(vb.begin(), vb.end());
#ifdef PWC_STRIP_CENSUS
  {
    // one more batch of launches with the census buffer armed: per launch, each stamp's
    // LATEST workgroup relative to the launch's earliest workgroup start, and the mean
    // per-workgroup span from its own start (us); quad A = wave 0, quad B = wave WPP
    const int nb = (int)with_geo([&](auto g) {
      return pwc::strip::grid_blocks<decltype(g)>(B, H, W);
    });
    const int nstep = with_geo([&](auto g) { return decltype(g)::NSTEP; }), CI = 50;
    unsigned long long* cen;
    CK(hipMalloc(&cen, (size_t)CI * nb * 64 * 8));
    CK(hipMemset(cen, 0, (size_t)CI * nb * 64 * 8));
    for (int i = 0; i < CI; ++i) {
      unsigned long long* p = cen + (size_t)i * nb * 64;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::strip::g_census), &p, sizeof(p)));
      CK(strip_call(f1[i % NS], f2[i % NS], o2[i % NS], B, H, W));
    }
    unsigned long long* np = nullptr;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::strip::g_census), &np, sizeof(np)));
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> c((size_t)CI * nb * 64);
    CK(hipMemcpy(c.data(), cen, c.size() * 8, hipMemcpyDeviceToHost));
    double mx[64] = {}, mean[64] = {}, skew = 0;
    for (int i = 0; i < CI; ++i) {
      const unsigned long long* L = c.data() + (size_t)i * nb * 64;
      unsigned long long t0 = ~0ull, t0max = 0;
      for (int b = 0; b < nb; ++b) {
        t0 = std::min(t0, L[b * 64]);
        t0max = std::max(t0max, L[b * 64]);
      }
      skew += (t0max - t0) * 0.01;
      for (int k = 1; k < 64; ++k) {
        unsigned long long m = 0;
        double sm = 0;
        for (int b = 0; b < nb; ++b) {
          const int base = k >= 32 ? 32 : 0;  // quad B and the loader: quad B's entry stamp
          m = std::max(m, L[b * 64 + k]);
          sm += L[b * 64 + k] ? (double)(L[b * 64 + k] - L[b * 64 + base]) : 0.0;
        }
        mx[k] += m ? (m - t0) * 0.01 : 0.0;
        mean[k] += sm / nb * 0.01;
      }
    }
    auto name = [&](int k) -> std::string {
      if (k == 1) return "first_data";
      if (k >= 2 && k < 2 + 3 * nstep) {
        const char* ph[3] = {"loop", "reduced", "stored"};
        return "s" + std::to_string((k - 2) / 3) + "_" + ph[(k - 2) % 3];
      }
      return "";
    };
    std::printf("{\"geometry\": %d, \"census_start_skew_us\": %.2f", g_geo, skew / CI);
    for (int k = 1; k < 32; ++k)
      if (!name(k).empty()) std::printf(", \"%s\": [%.2f, %.2f]", name(k).c_str(), mx[k] / CI, mean[k] / CI);
    const char* ld[3] = {"ld_group0", "ld_window", "ld_all"};
    for (int k = 0; k < 3; ++k)
      std::printf(", \"%s\": [%.2f, %.2f]", ld[k], mx[61 + k] / CI, mean[61 + k] / CI);
    std::printf(", \"quadB\": {");
    for (int k = 33; k < 32 + 2 + 3 * nstep; ++k)
      std::printf("%s\"%s\": %.2f", k > 33 ? ", " : "", name(k - 32).c_str(), mean[k] / CI);
    std::printf("}}  ([latest workgroup vs earliest start, mean per-workgroup span] us)\n");
  }
#endif
  const double bytes = (double)B * (2.0 * C * H * W + 81.0 * H * W) * 4;
  std::printf("{\"strip_geo\": %d, \"stream_us\": %.2f, \"strip_us\": %.2f, "
              "\"strip_median_us\": %.2f, \"strip_frac_8TBs\": %.3f, \"stream_frac_8TBs\": %.3f}\n",
              g_geo, ta / iters, tb / iters, vb[iters / 2],
              bytes / (tb / iters * 1e-6) / 8e12,
              bytes / (ta / iters * 1e-6) / 8e12);
  return 0;
}
