// cbench.hip — standalone timing harness for correlation forward kernel variants (no torch).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPWC_RING_ABLATION -DPWC_PAR_ABLATION \
//         -o tools/cbench tools/cbench.hip
//   tools/cbench [B C H W] [iters]
//
// Allocates rotating input/output sets (> 512 MiB in all, past the Infinity Cache), checks
// every variant against a naive one-thread-per-output kernel (same fp32 fma order over
// channels, so a correct variant matches bit for bit), and prints per-launch device time from
// hipExtLaunchKernel start/stop events, plus algorithmic GB/s and the fraction of 8 TB/s.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "corr_par.hip"
#include "../pwc-net_pytorch_amd/csrc/corr_ring.hip"
#include "../pwc-net_pytorch_amd/csrc/corr_pt.hip"
#include "../pwc-net_pytorch_amd/csrc/corr_grp.hip"
#include "../pwc-net_pytorch_amd/csrc/corr_small.hip"

namespace pwc {
hipEvent_t g_e0 = nullptr, g_e1 = nullptr;
void take_launch_events(hipEvent_t* a, hipEvent_t* b) {
  *a = g_e0;
  *b = g_e1;
  g_e0 = g_e1 = nullptr;
}
__global__ void red_k(const float* partial, float* out, size_t n, int nsplit, float div) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = partial[i];
  for (int k = 1; k < nsplit; ++k) s += partial[(size_t)k * n + i];
  out[i] = s / div;
}
hipError_t corr_reduce_splits_f32(const void* partial, void* out, size_t n, int nsplit,
                                  float divisor, float, hipStream_t stream) {
  hipLaunchKernelGGL(red_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const float*)partial, (float*)out, n, nsplit, divisor);
  return hipGetLastError();
}
}  // namespace pwc

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                   hipGetErrorString(e_));                                      \
      std::exit(2);                                                             \
    }                                                                           \
  } while (0)

// naive reference: cu:34-106 with k=1, s1=1, dr=4, s2=2, raster channels, zeros outside
__global__ void ref_corr(const float* f1, const float* f2, float* out, int B, int C, int H, int W,
                         int Ho, int Wo, int off, float divisor) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long tot = (long long)B * 81 * Ho * Wo;
  if (i >= tot) return;
  const int ox = i % Wo, oy = (i / Wo) % Ho, tc = (i / ((long long)Wo * Ho)) % 81;
  const int n = i / ((long long)Wo * Ho * 81);
  const int tj = tc / 9 - 4, ti = tc % 9 - 4;
  const int y1 = oy + off, x1 = ox + off, y2 = y1 + 2 * tj, x2 = x1 + 2 * ti;
  float acc = 0.f;
  for (int c = 0; c < C; ++c) {
    const float a = (y1 >= 0 && y1 < H && x1 >= 0 && x1 < W)
                        ? f1[(((size_t)n * C + c) * H + y1) * W + x1] : 0.f;
    const float b = (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W)
                        ? f2[(((size_t)n * C + c) * H + y2) * W + x2] : 0.f;
    acc = fmaf(a, b, acc);
  }
  out[i] = acc / divisor;
}

// HBM floor: read the two inputs once, write the output once (16 B per lane, grid-stride).
__global__ void floor_copy(const float4* __restrict__ a, const float4* __restrict__ b,
                           float4* __restrict__ o, long long n_in, long long n_out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += stride) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n_in) {
      const float4 x = a[i], y = b[i];
      v = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
    o[i] = v;
  }
}

__global__ void floor_read(const float4* __restrict__ a, const float4* __restrict__ b,
                           float4* __restrict__ o, long long n_in) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n_in; i += stride) {
    const float4 x = a[i], y = b[i];
    acc += x.x + y.x + x.y + y.y + x.z + y.z + x.w + y.w;
  }
  if (acc == 12345.f) o[0] = make_float4(acc, 0, 0, 0);
}

__global__ void floor_write(float4* __restrict__ o, long long n_out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += stride)
    o[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// ---- store-pattern probes: write the 81-channel output volume with each kernel's epilogue
// shape (values only; no loads) ----
// parA: tile 16 cols x 16 parity rows, lane (tj, r, s) writes 8 px x 9 ti as 18 float4
__global__ void st_par(float* out, int Ho, int Wo, int n_tr, int n_tx) {
  const int t = pwc::xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % n_tx, tr = (t / n_tx) % n_tr, p = (t / (n_tx * n_tr)) & 1,
            n = t / (n_tx * n_tr * 2);
  const int tj = threadIdx.x >> 5, r = (threadIdx.x >> 1) & 15, s = threadIdx.x & 1;
  const int oy = 2 * (tr * 16 + r) + p, ox = tx * 16 + 8 * s;
  if (oy >= Ho || ox >= Wo) return;
  const float v = (float)threadIdx.x;
  for (int ti = 0; ti < 9; ++ti) {
    float* o = out + (((size_t)n * 81 + tj * 9 + ti) * Ho + oy) * Wo + ox;
    *reinterpret_cast<float4*>(o) = make_float4(v, v, v, v);
    *reinterpret_cast<float4*>(o + 4) = make_float4(v, v, v, v);
  }
}
// full-width band of R rows: lane (tj, r, seg) writes 8 px x 9 ti
template <int R>
__global__ void st_band(float* out, int Ho, int Wo) {
  const int nb = (Ho + R - 1) / R;
  const int t = pwc::xcd_remap(blockIdx.x, gridDim.x);
  const int b = t % nb, n = t / nb;
  const int nseg = Wo / 8;
  const int lane = threadIdx.x;
  const int seg = lane % nseg, r = (lane / nseg) % R, tj = lane / (nseg * R);
  if (tj >= 9) return;
  const int oy = b * R + r, ox = 8 * seg;
  if (oy >= Ho) return;
  const float v = (float)threadIdx.x;
  for (int ti = 0; ti < 9; ++ti) {
    float* o = out + (((size_t)n * 81 + tj * 9 + ti) * Ho + oy) * Wo + ox;
    *reinterpret_cast<float4*>(o) = make_float4(v, v, v, v);
    *reinterpret_cast<float4*>(o + 4) = make_float4(v, v, v, v);
  }
}
// full-width band of R rows, ideal order: for each oc plane the WG writes its contiguous
// R*Wo span with consecutive lanes (what an LDS-transposed epilogue would issue)
template <int R>
__global__ void st_band_lin(float* out, int Ho, int Wo) {
  const int nb = (Ho + R - 1) / R;
  const int t = pwc::xcd_remap(blockIdx.x, gridDim.x);
  const int b = t % nb, n = t / nb;
  const int rows = min(R, Ho - b * R);
  const int nq = rows * Wo / 4;
  const float v = (float)threadIdx.x;
  for (int oc = 0; oc < 81; ++oc) {
    float4* o = reinterpret_cast<float4*>(out + (((size_t)n * 81 + oc) * Ho + b * R) * Wo);
    for (int i = threadIdx.x; i < nq; i += blockDim.x) o[i] = make_float4(v, v, v, v);
  }
}

// pt pattern: tile 16 cols x 24 parity rows, 448 threads, lane map of corr_pt.hip
template <bool CONTIG>
__global__ void st_pt(float* out, int Ho, int Wo, int n_tr, int n_tx) {
  const int t = pwc::xcd_remap(blockIdx.x, gridDim.x);
  const int tx = t % n_tx, tr = (t / n_tx) % n_tr, p = (t / (n_tx * n_tr)) & 1,
            n = t / (n_tx * n_tr * 2);
  int tj, r, s;
  bool valid = true;
  const int u = threadIdx.x;
  if (u < 288) { tj = u >> 5; r = (u >> 1) & 15; s = u & 1; }
  else {
    const int v = u - 288, pair = v >> 5, h = (v >> 4) & 1, i = (v >> 1) & 7;
    s = v & 1; tj = 2 * pair + h; r = 16 + (h ? ((i + 7) & 7) : i);
    if (tj > 8) { tj = 8; valid = false; }
  }
  const int oy = 2 * (tr * 24 + r) + p, ox = tx * 16 + 8 * s;
  if (!valid || oy >= Ho || ox >= Wo) return;
  const float v = (float)threadIdx.x;
  for (int ti = 0; ti < 9; ++ti) {
    float* o = out + (((size_t)n * 81 + tj * 9 + ti) * Ho + oy) * Wo + tx * 16;
    if (CONTIG) {  // instruction 1: lanes s=0,1 write px 0-3 / 4-7; instruction 2: 8-11 / 12-15
      *reinterpret_cast<float4*>(o + 4 * s) = make_float4(v, v, v, v);
      *reinterpret_cast<float4*>(o + 8 + 4 * s) = make_float4(v, v, v, v);
    } else {
      *reinterpret_cast<float4*>(o + 8 * s) = make_float4(v, v, v, v);
      *reinterpret_cast<float4*>(o + 8 * s + 4) = make_float4(v, v, v, v);
    }
  }
}

__global__ void fill_rand(float* p, size_t n, unsigned seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = ((x & 0xffffff) / 16777216.0f) * 2.f - 1.f;
}

struct Set {
  float *f1, *f2, *out;
};

int main(int argc, char** argv) {
  int B = 8, C = 32, H = 96, W = 112, iters = 50;
  if (argc >= 5) {
    B = atoi(argv[1]); C = atoi(argv[2]); H = atoi(argv[3]); W = atoi(argv[4]);
  }
  if (argc >= 6) iters = atoi(argv[5]);
  const char* only = std::getenv("ONLY");
  const int off = 0, Ho = H, Wo = W;
  const float divisor = (float)C;
  const size_t nin = (size_t)B * C * H * W, nout = (size_t)B * 81 * Ho * Wo;
  const double alg = (2.0 * nin + nout) * 4.0;
  int nsets = std::max(2, (int)std::ceil(600e6 / alg));
  if (std::getenv("NSETS")) nsets = atoi(std::getenv("NSETS"));
  std::vector<Set> sets(nsets);
  for (int s = 0; s < nsets; ++s) {
    CK(hipMalloc(&sets[s].f1, nin * 4));
    CK(hipMalloc(&sets[s].f2, nin * 4));
    CK(hipMalloc(&sets[s].out, nout * 4));
    fill_rand<<<(nin + 255) / 256, 256>>>(sets[s].f1, nin, 1234u + s);
    fill_rand<<<(nin + 255) / 256, 256>>>(sets[s].f2, nin, 777u + s);
  }
  float* ref;
  CK(hipMalloc(&ref, nout * 4));
  float* wsp;
  CK(hipMalloc(&wsp, nout * 4 * 16));
  ref_corr<<<(nout + 255) / 256, 256>>>(sets[0].f1, sets[0].f2, ref, B, C, H, W, Ho, Wo, off,
                                       divisor);
  CK(hipDeviceSynchronize());
  std::vector<float> href(nout), hout(nout);
  CK(hipMemcpy(href.data(), ref, nout * 4, hipMemcpyDeviceToHost));

  const int NEV = iters;
  std::vector<hipEvent_t> e0(NEV), e1(NEV);
  for (int i = 0; i < NEV; ++i) {
    CK(hipEventCreate(&e0[i]));
    CK(hipEventCreate(&e1[i]));
  }
  std::printf("shape B=%d C=%d H=%d W=%d  alg bytes %.0f  sets %d\n", B, C, H, W, alg, nsets);

  auto run = [&](const char* name, std::function<hipError_t(const Set&)> fn, bool check,
                 int ring_abl, int par_abl) {
    if (only && !strstr(name, only)) return;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::g_ablation), &ring_abl, sizeof(int)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::par::g_par_abl), &par_abl, sizeof(int)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::pt::g_pt_abl), &par_abl, sizeof(int)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pwc::sm::g_sm_abl), &par_abl, sizeof(int)));
    if (check) {
      CK(hipMemset(sets[0].out, 0xff, nout * 4));
      CK(fn(sets[0]));
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(hout.data(), sets[0].out, nout * 4, hipMemcpyDeviceToHost));
      double md = 0;
      size_t bad = 0;
      for (size_t i = 0; i < nout; ++i) {
        const double d = std::fabs((double)hout[i] - (double)href[i]);
        if (!(d <= 1e-6)) ++bad;
        if (d > md || d != d) md = d != d ? 1e30 : d;
      }
      std::printf("  %-28s check: max|d| %.3g  mismatches %zu\n", name, md, bad);
    }
    const int warm = std::getenv("WARM") ? atoi(std::getenv("WARM")) : 300;
    for (int w = 0; w < warm; ++w) CK(fn(sets[w % nsets]));
    CK(hipDeviceSynchronize());
    for (int i = 0; i < iters; ++i) {
      pwc::g_e0 = e0[i];
      pwc::g_e1 = e1[i];
      const bool wrap = false;  // (multi-kernel paths: the launcher times its main kernel)
      if (wrap) {
        pwc::g_e0 = pwc::g_e1 = nullptr;
        CK(hipEventRecord(e0[i], 0));
      }
      CK(fn(sets[i % nsets]));
      if (wrap) CK(hipEventRecord(e1[i], 0));
    }
    CK(hipDeviceSynchronize());
    std::vector<float> t(iters);
    double sum = 0;
    for (int i = 0; i < iters; ++i) {
      CK(hipEventElapsedTime(&t[i], e0[i], e1[i]));
      sum += t[i];
    }
    std::sort(t.begin(), t.end());
    const double avg = sum / iters * 1e3, med = t[iters / 2] * 1e3, mn = t[0] * 1e3;
    std::printf("%-30s avg %7.2f us  med %7.2f  min %7.2f   %7.1f GB/s  frac %.3f\n", name, avg,
                med, mn, alg / (avg * 1e-6) / 1e9, alg / (avg * 1e-6) / 8e12);
  };

  const long long nin4 = nin / 4, nout4 = nout / 4;
  run("floor_copy", [&](const Set& s) {
    hipExtLaunchKernelGGL(floor_copy, dim3(2048), dim3(256), 0, 0, pwc::g_e0, pwc::g_e1, 0,
                          (const float4*)s.f1, (const float4*)s.f2, (float4*)s.out, nin4, nout4);
    pwc::g_e0 = pwc::g_e1 = nullptr;
    return hipGetLastError();
  }, false, 0, 0);

  run("floor_read", [&](const Set& s) {
    hipExtLaunchKernelGGL(floor_read, dim3(2048), dim3(256), 0, 0, pwc::g_e0, pwc::g_e1, 0,
                          (const float4*)s.f1, (const float4*)s.f2, (float4*)s.out, nin4);
    pwc::g_e0 = pwc::g_e1 = nullptr;
    return hipGetLastError();
  }, false, 0, 0);
  run("floor_write", [&](const Set& s) {
    hipExtLaunchKernelGGL(floor_write, dim3(2048), dim3(256), 0, 0, pwc::g_e0, pwc::g_e1, 0,
                          (float4*)s.out, nout4);
    pwc::g_e0 = pwc::g_e1 = nullptr;
    return hipGetLastError();
  }, false, 0, 0);

  {
    const int n_tr = ((Ho + 1) / 2 + 15) / 16, n_tx = (Wo + 15) / 16;
    run("st_par", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_par, dim3(B * 2 * n_tr * n_tx), dim3(288), 0, 0, pwc::g_e0,
                            pwc::g_e1, 0, s.out, Ho, Wo, n_tr, n_tx);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    const int n_tr24 = ((Ho + 1) / 2 + 23) / 24;
    run("st_pt", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_pt<false>, dim3(B * 2 * n_tr24 * n_tx), dim3(448), 0, 0,
                            pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo, n_tr24, n_tx);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    run("st_pt_contig", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_pt<true>, dim3(B * 2 * n_tr24 * n_tx), dim3(448), 0, 0,
                            pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo, n_tr24, n_tx);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    run("st_pt_contig_lds", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_pt<true>, dim3(B * 2 * n_tr24 * n_tx), dim3(448), 150000, 0,
                            pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo, n_tr24, n_tx);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    const int nseg = Wo / 8;
    run("st_band3", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_band<3>, dim3(B * ((Ho + 2) / 3)), dim3((9 * 3 * nseg + 63) / 64 * 64),
                            0, 0, pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    run("st_band3_lin", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_band_lin<3>, dim3(B * ((Ho + 2) / 3)), dim3(384), 0, 0,
                            pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    run("st_band2_lin", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_band_lin<2>, dim3(B * ((Ho + 1) / 2)), dim3(256), 0, 0,
                            pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
    run("st_band6_lin", [&](const Set& s) {
      hipExtLaunchKernelGGL(st_band_lin<6>, dim3(B * ((Ho + 5) / 6)), dim3(512), 0, 0,
                            pwc::g_e0, pwc::g_e1, 0, s.out, Ho, Wo);
      pwc::g_e0 = pwc::g_e1 = nullptr;
      return hipGetLastError();
    }, false, 0, 0);
  }
  const char* ring_cfgs[] = {"N", "C"};
  for (const char* cfg : ring_cfgs) {
    setenv("PWC_RING_CFG", cfg, 1);
    // ring_cfg() caches on first call: only the first config is honoured per process
    static int once = 0;
    if (once++) break;
    for (int abl : {0, 1, 2, 4, 5, 6, 3}) {
      std::string nm = std::string("ring") + cfg + (abl ? "_abl" + std::to_string(abl) : "");
      run(nm.c_str(), [&](const Set& s) {
        return pwc::corr_forward_ring_f32(s.f1, s.f2, s.out, B, C, H, W, Ho, Wo, off, 4, 2, 0,
                                          divisor, 1, nullptr, 0);
      }, abl == 0, abl, 0);
    }
  }
  const char* par_env = std::getenv("PWC_PAR_CFG");
  for (int abl : {0, 1, 2, 4, 5, 6, 3}) {
    std::string nm = std::string("par") + (par_env ? par_env : "A") +
                     (abl ? "_abl" + std::to_string(abl) : "");
    run(nm.c_str(), [&](const Set& s) {
      return pwc::corr_forward_par_f32(s.f1, s.f2, s.out, B, C, H, W, Ho, Wo, off, 4, 2, 0,
                                       divisor, 0);
    }, abl == 0, 0, abl);
  }
  for (int abl : {0, 1, 2, 4, 7, 8}) {
    std::string nm = std::string("small") + (abl ? "_abl" + std::to_string(abl) : "");
    run(nm.c_str(), [&](const Set& s) {
      return pwc::corr_forward_small_f32(s.f1, s.f2, s.out, B, C, H, W, Ho, Wo, off, 4, 2, 0,
                                         divisor, 16, wsp, 0);
    }, abl == 0, 0, abl);
  }
  run("grp", [&](const Set& s) {
    return pwc::corr_forward_grp_f32(s.f1, s.f2, s.out, B, C, H, W, Ho, Wo, off, 4, 2, 0,
                                     divisor, 0);
  }, true, 0, 0);
  const char* pt_env = std::getenv("PWC_PT_K");
  for (int abl : {0, 1, 2, 4, 5, 6, 3}) {
    std::string nm = std::string("pt") + (pt_env ? pt_env : "auto") +
                     (abl ? "_abl" + std::to_string(abl) : "");
    run(nm.c_str(), [&](const Set& s) {
      return pwc::corr_forward_pt_f32(s.f1, s.f2, s.out, B, C, H, W, Ho, Wo, off, 4, 2, 0,
                                      divisor, 0, 0);
    }, abl == 0, 0, abl);
  }
  std::printf("done\n");
  return 0;
}
