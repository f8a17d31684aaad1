// capi.hip — the extern "C" boundary declared in include/pwc_hotpath.h.
//
// Argument checks mirror what the reference enforced or silently assumed
// (correlation_package/functions/correlation.py:17-18 contiguity asserts are done by the
// Python layer; correlation_cuda.c:20-42 shape math and fills; cu:361-368 launch check).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/pwc_hotpath.h"
#include "pwc_common.cuh"

namespace pwc {
template <typename T>
hipError_t corr_forward_t(const void*, const void*, void*, int, int, int, int, int, int, int,
                          int, int, int, int, int, float, void*, hipStream_t, int);
size_t corr_workspace_bytes(int B, int OC, int Ho, int Wo);
template <typename T>
hipError_t corr_backward_t(const void*, const void*, const void*, void*, void*, int, int, int,
                           int, int, int, int, int, int, int, int, int, float, hipStream_t,
                           int);
template <typename T>
hipError_t warp_forward_t(const void*, const void*, void*, int, int, int, int, hipStream_t);
template <typename T>
hipError_t warp_forward_group_t(const WarpProblem*, int, hipStream_t);
hipError_t warp_backward_f32(const void*, const void*, const void*, void*, void*, int, int, int,
                             int, hipStream_t);
size_t warp_backward_workspace_size(int B, int C, int H, int W);
hipError_t warp_backward_tiles_f32(const void*, const void*, const void*, void*, void*, int, int,
                                   int, int, void*, size_t, hipStream_t);
template <typename T>
hipError_t upsample_warp_forward_t(const void*, const void*, void*, void*, int, int, int, int,
                                   hipStream_t);
hipError_t corr_forward_rows_pair(const void*, const void*, void*, int, int, int, int,
                                  const void*, const void*, void*, int, int, int, int, float,
                                  float, hipStream_t);
hipError_t flow_up2_backward_f32(const void*, void*, int, int, int, hipStream_t);
hipError_t warp_corr_band_pair(const BandProblem& a, const BandProblem& b, float divisor_a,
                               float divisor_b, int dtype, hipStream_t stream);
hipError_t warp_corr_band(const void*, const void*, const void*, void*, void*, int, int, int, int,
                          float, int, int, hipStream_t);
}  // namespace pwc

namespace pwc {
// PWC_DEBUG="name=value,..." (pwc_common.cuh): read from the environment once, replaceable by
// pwc_set_debug() (tests / measurement tools); empty in production, where every knob returns
// its default without parsing anything.
std::string& debug_spec() {
  static std::string spec = [] {
    const char* e = std::getenv("PWC_DEBUG");
    return std::string(e ? e : "");
  }();
  return spec;
}

int debug_knob(const char* name, int def) {
  const std::string& spec = debug_spec();
  if (spec.empty()) return def;
  const size_t n = std::strlen(name);
  size_t pos = 0;
  while (pos < spec.size()) {
    size_t end = spec.find(',', pos);
    if (end == std::string::npos) end = spec.size();
    const std::string item = spec.substr(pos, end - pos);
    if (item.size() > n + 1 && item.compare(0, n, name) == 0 && item[n] == '=')
      return std::atoi(item.c_str() + n + 1);
    pos = end + 1;
  }
  return def;
}

hipError_t lds_limit(const void* kernel, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;  // (kernel, device) -> bytes set
  std::lock_guard<std::mutex> lock(mu);
  const auto it = done.find({kernel, dev});
  if (it != done.end() && it->second >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done[{kernel, dev}] = bytes;
  return e;
}

// output epilogue of the next correlation launch of this thread (pwc_corr_forward_into)
thread_local OutEpi g_epi = {0, 1.f};
OutEpi current_epi() { return g_epi; }

struct EpiScope {
  EpiScope(long long ostride, float slope) { g_epi = OutEpi{ostride, slope}; }
  ~EpiScope() { g_epi = OutEpi{0, 1.f}; }
};

// dst[n * ostride + i] = leaky(src[n * vol + i]) -- the fallback of pwc_corr_forward_into for
// configurations whose kernels write dense volumes only
template <typename T>
__global__ __launch_bounds__(256) void copy_strided_act(const T* __restrict__ src,
                                                        T* __restrict__ dst, size_t vol,
                                                        long long ostride, float slope,
                                                        size_t total) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < total;
       i += (size_t)gridDim.x * 256) {
    const size_t n = i / vol, e = i - n * vol;
    dst[n * (size_t)ostride + e] = from_f32<T>(epi_act(to_f32(src[i]), slope));
  }
}

thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
void take_launch_events(hipEvent_t* start, hipEvent_t* stop) {
  *start = g_ev_start;
  *stop = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
}
}  // namespace pwc

namespace {

thread_local char g_err[512] = "";

int fail(const char* fn, const char* msg) {
  std::snprintf(g_err, sizeof(g_err), "%s: %s", fn, msg);
  return 0;
}

int check_launch(const char* fn, hipError_t e) {
  if (e != hipSuccess) {
    std::snprintf(g_err, sizeof(g_err), "%s: launch failed: %s", fn, hipGetErrorString(e));
    return 0;
  }
  g_err[0] = '\0';
  return 1;
}

bool dims_ok(int B, int C, int H, int W) { return B >= 0 && C >= 0 && H >= 0 && W >= 0; }

// correlation_cuda.c:20-34
bool corr_shape(int H, int W, int pad, int k, int md, int s1, int s2, int* oc, int* oh,
                int* ow) {
  if (s1 <= 0 || s2 <= 0 || k < 0 || md < 0 || pad < 0) return false;
  const int kr = (k - 1) / 2;
  const int br = kr + md;
  const int pH = H + 2 * pad, pW = W + 2 * pad;
  const int dr = md / s2;
  *oc = (2 * dr + 1) * (2 * dr + 1);
  *oh = (int)std::ceil((float)(pH - 2 * br) / (float)s1);
  *ow = (int)std::ceil((float)(pW - 2 * br) / (float)s1);
  return true;
}

// Kernel-selection override for cross-checks (PWC_DEBUG setting corr_path, read once):
//   1: literal one-thread-per-output kernels only; 2: the register-tiled kernel (measurement)
int force_generic() { return pwc::debug_knob("corr_path", 0); }

}  // namespace

namespace pwc {
bool corr_strip_accepts(const void*, const void*, const void*, int, int, int, int, int, int, int);
bool corr_mstrip16_accepts(const void*, const void*, const void*, int, int, int, int, int, int,
                           int);
bool corr_bwd_strip_accepts(const void*, const void*, const void*, const void*, const void*, int,
                            int, int, int);
size_t warp_corr_bwd_small_workspace(int B, int C, int H, int W);
hipError_t warp_corr_bwd_small(const void* in1, const void* x2, const void* flow,
                               const void* x2w, const void* grad_corr, const void* grad_x2w,
                               void* grad_in1, void* grad_x2, void* grad_flow, int B, int C,
                               int H, int W, float divisor, void* ws, size_t ws_bytes,
                               void* counters, hipStream_t stream);
hipError_t add_inplace_f32(void* y, const void* x, size_t n, hipStream_t stream);
}  // namespace pwc

extern "C" {

int pwc_abi_version(void) { return 11; }

int pwc_corr_forward_plan(const void* in1, const void* in2, const void* out, int B, int C, int H,
                          int W, int pad_size, int kernel_size, int max_displacement, int stride1,
                          int stride2, int dtype) {
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W) ||
      !corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo) ||
      Ho <= 0 || Wo <= 0 || dtype < PWC_DTYPE_F32 || dtype > PWC_DTYPE_BF16)
    return -1;
  if (force_generic() != 0) return PWC_PLAN_OTHER;
  const int path = pwc::corr_forward_path(in1, in2, out, B, C, H, W, pad_size, kernel_size,
                                          max_displacement, stride1, stride2, pwc::kRaster,
                                          dtype);
  if (path == pwc::kPathBand) return PWC_PLAN_BAND;
  if (path == pwc::kPathRows) return PWC_PLAN_ROWS;
  if (path != pwc::kPathStream) return PWC_PLAN_OTHER;
  // the order of corr_forward_stream (corr_stream.hip)
  if (pwc::corr_mstrip16_accepts(in1, in2, out, B, C, H, W, stride2, dtype, pwc::kRaster))
    return PWC_PLAN_MSTRIP16;
  if (pwc::corr_strip_accepts(in1, in2, out, B, C, H, W, stride2, dtype, pwc::kRaster))
    return PWC_PLAN_STRIP;
  return PWC_PLAN_STREAM;
}

int pwc_corr_backward_plan(const void* in1, const void* in2, const void* grad_out,
                           const void* grad_in1, const void* grad_in2, int B, int C, int H, int W,
                           int pad_size, int kernel_size, int max_displacement, int stride1,
                           int stride2, int dtype) {
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W) || stride1 != 1 ||
      !corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo) ||
      Ho <= 0 || Wo <= 0 || dtype < PWC_DTYPE_F32 || dtype > PWC_DTYPE_BF16)
    return -1;
  // the model configuration's fp32 kernels (corr_backward_t, corr_bwd.hip)
  if (force_generic() != 0 || dtype != PWC_DTYPE_F32 || kernel_size != 1 || stride2 != 2 ||
      pad_size != max_displacement || (max_displacement != 8 && max_displacement != 9))
    return PWC_BWD_PLAN_OTHER;
  if (pwc::corr_bwd_strip_accepts(in1, in2, grad_out, grad_in1, grad_in2, B, C, H, W))
    return PWC_BWD_PLAN_STRIP;
  return pwc::debug_knob("bwd_rows", 1) != 0 ? PWC_BWD_PLAN_ROWS : PWC_BWD_PLAN_OTHER;
}

int pwc_set_debug(const char* spec) {
  pwc::debug_spec() = spec ? spec : "";
  return 1;
}

int pwc_time_next_corr(void* start_event, void* stop_event) {
  if ((start_event == nullptr) != (stop_event == nullptr))
    return fail("pwc_time_next_corr", "give both events or neither");
  pwc::g_ev_start = (hipEvent_t)start_event;
  pwc::g_ev_stop = (hipEvent_t)stop_event;
  return 1;
}

const char* pwc_last_error(void) { return g_err; }

int pwc_corr_output_shape(int H, int W, int pad_size, int kernel_size, int max_displacement,
                          int stride1, int stride2, int* out_channels, int* out_height,
                          int* out_width) {
  if (!out_channels || !out_height || !out_width)
    return fail("pwc_corr_output_shape", "null output pointer");
  if (!corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2,
                  out_channels, out_height, out_width))
    return fail("pwc_corr_output_shape", "invalid correlation parameters");
  if (*out_height <= 0 || *out_width <= 0)
    return fail("pwc_corr_output_shape", "empty correlation output");
  return 1;
}

static int corr_forward_impl(const char* fn, const void* in1, const void* in2, void* out, int B,
                             int C, int H, int W, int pad_size, int kernel_size,
                             int max_displacement, int stride1, int stride2, int dtype,
                             void* workspace, size_t workspace_bytes, void* stream) {
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (!corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo))
    return fail(fn, "invalid correlation parameters");
  if (Ho <= 0 || Wo <= 0) return fail(fn, "empty correlation output");
  if ((size_t)B * C * H * W && (!in1 || !in2 || !out)) return fail(fn, "null buffer");
  if (workspace && workspace_bytes < pwc::corr_workspace_bytes(B, OC, Ho, Wo))
    return fail(fn, "workspace smaller than pwc_corr_workspace_size()");
  const float divisor = (float)(kernel_size * kernel_size * C);  // cu:65 nelems
  hipStream_t s = (hipStream_t)stream;
  // pwc_time_next_corr: the main correlation kernel of every path launches with the armed
  // events (hipExtLaunchKernel: exact kernel start/stop, no extra stream packets)
  hipError_t e;
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::corr_forward_t<float>(in1, in2, out, B, C, H, W, Ho, Wo, pad_size, kernel_size,
                                     max_displacement, stride1, stride2, pwc::kRaster, divisor,
                                     workspace, s, force_generic());
      break;
    case PWC_DTYPE_F16:
      e = pwc::corr_forward_t<__half>(in1, in2, out, B, C, H, W, Ho, Wo, pad_size, kernel_size,
                                      max_displacement, stride1, stride2, pwc::kRaster,
                                      divisor, workspace, s, force_generic());
      break;
    case PWC_DTYPE_BF16:
      e = pwc::corr_forward_t<__hip_bfloat16>(in1, in2, out, B, C, H, W, Ho, Wo, pad_size,
                                              kernel_size, max_displacement, stride1, stride2,
                                              pwc::kRaster, divisor, workspace, s,
                                              force_generic());
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  pwc::g_ev_start = pwc::g_ev_stop = nullptr;  // one-shot, consumed or not
  return check_launch(fn, e);
}

size_t pwc_corr_forward_into_workspace_size(int B, int C, int H, int W, int pad_size,
                                            int kernel_size, int max_displacement, int stride1,
                                            int stride2, int dtype) {
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W) ||
      !corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo) ||
      Ho <= 0 || Wo <= 0)
    return 0;
  const size_t esz = dtype == PWC_DTYPE_F32 ? 4 : 2;
  return (size_t)B * OC * Ho * Wo * esz;
}

int pwc_corr_forward_into(const void* in1, const void* in2, void* out,
                          long long out_image_stride, float negative_slope, int B, int C, int H,
                          int W, int pad_size, int kernel_size, int max_displacement,
                          int stride1, int stride2, int corr_multiply, int dtype,
                          void* workspace, size_t workspace_bytes, void* stream) {
  (void)corr_multiply;  // ignored, as in the reference (cu)
  const char* fn = "pwc_corr_forward_into";
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (!corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo))
    return fail(fn, "invalid correlation parameters");
  if (Ho <= 0 || Wo <= 0) return fail(fn, "empty correlation output");
  const long long vol = (long long)OC * Ho * Wo;
  if (B > 1 && out_image_stride < vol) return fail(fn, "out_image_stride < OC*Ho*Wo");
  if (!(negative_slope == negative_slope)) return fail(fn, "negative_slope is NaN");
  if (B == 0) return check_launch(fn, hipSuccess);
  if (!in1 || !in2 || !out) return fail(fn, "null buffer");
  const long long ostride = out_image_stride > 0 ? out_image_stride : vol;
  const float divisor = (float)(kernel_size * kernel_size * C);  // cu:65 nelems
  hipStream_t s = (hipStream_t)stream;
  if (dtype != PWC_DTYPE_F32 && dtype != PWC_DTYPE_F16 && dtype != PWC_DTYPE_BF16)
    return fail(fn, "unsupported dtype");
  hipError_t e = hipErrorNotSupported;
  const long long epi_stride = ostride == vol ? 0 : ostride;
  if (dtype == PWC_DTYPE_F32 && force_generic() == 0) {  // kernels that write the slice directly
    pwc::EpiScope scope(epi_stride, negative_slope);
    e = pwc::corr_forward_t<float>(in1, in2, out, B, C, H, W, Ho, Wo, pad_size, kernel_size,
                                   max_displacement, stride1, stride2, pwc::kRaster, divisor,
                                   nullptr, s, 0);
  } else if (dtype == PWC_DTYPE_F16 && force_generic() == 0 && epi_stride % 8 == 0) {
    // fp16: the matrix-core strip, stream and row-band kernels write the slice with 16-B
    // stores of 8 halves, so an image stride that keeps them aligned (else: workspace + copy)
    pwc::EpiScope scope(epi_stride, negative_slope);
    e = pwc::corr_forward_t<__half>(in1, in2, out, B, C, H, W, Ho, Wo, pad_size, kernel_size,
                                    max_displacement, stride1, stride2, pwc::kRaster, divisor,
                                    nullptr, s, 0);
  }
  if (e != hipErrorNotSupported) return check_launch(fn, e);
  // dense volume in the workspace, then one strided copy applying the activation
  const size_t esz = dtype == PWC_DTYPE_F32 ? 4 : 2;
  if (!workspace || workspace_bytes < (size_t)B * vol * esz)
    return fail(fn, "workspace smaller than pwc_corr_forward_into_workspace_size()");
  if (!corr_forward_impl(fn, in1, in2, workspace, B, C, H, W, pad_size, kernel_size,
                         max_displacement, stride1, stride2, dtype, nullptr, 0, stream))
    return 0;
  const size_t total = (size_t)B * vol;
  const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 65536);
  switch (dtype) {
    case PWC_DTYPE_F32:
      hipLaunchKernelGGL(pwc::copy_strided_act<float>, dim3(blocks), dim3(256), 0, s,
                         (const float*)workspace, (float*)out, (size_t)vol, ostride,
                         negative_slope, total);
      break;
    case PWC_DTYPE_F16:
      hipLaunchKernelGGL(pwc::copy_strided_act<__half>, dim3(blocks), dim3(256), 0, s,
                         (const __half*)workspace, (__half*)out, (size_t)vol, ostride,
                         negative_slope, total);
      break;
    default:
      hipLaunchKernelGGL(pwc::copy_strided_act<__hip_bfloat16>, dim3(blocks), dim3(256), 0, s,
                         (const __hip_bfloat16*)workspace, (__hip_bfloat16*)out, (size_t)vol,
                         ostride, negative_slope, total);
  }
  return check_launch(fn, hipGetLastError());
}

size_t pwc_corr_workspace_size(int B, int C, int H, int W, int pad_size, int kernel_size,
                               int max_displacement, int stride1, int stride2) {
  int OC, Ho, Wo;
  (void)C;
  if (!dims_ok(B, C, H, W) ||
      !corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo) ||
      Ho <= 0 || Wo <= 0)
    return 0;
  return pwc::corr_workspace_bytes(B, OC, Ho, Wo);
}

int pwc_corr_forward(const void* in1, const void* in2, void* out, int B, int C, int H, int W,
                     int pad_size, int kernel_size, int max_displacement, int stride1,
                     int stride2, int corr_multiply, int dtype, void* stream) {
  (void)corr_multiply;  // ignored by the reference kernels as well
  return corr_forward_impl("pwc_corr_forward", in1, in2, out, B, C, H, W, pad_size,
                           kernel_size, max_displacement, stride1, stride2, dtype, nullptr, 0,
                           stream);
}

int pwc_corr_forward_ws(const void* in1, const void* in2, void* out, int B, int C, int H, int W,
                        int pad_size, int kernel_size, int max_displacement, int stride1,
                        int stride2, int corr_multiply, int dtype, void* workspace,
                        size_t workspace_bytes, void* stream) {
  (void)corr_multiply;
  return corr_forward_impl("pwc_corr_forward_ws", in1, in2, out, B, C, H, W, pad_size,
                           kernel_size, max_displacement, stride1, stride2, dtype, workspace,
                           workspace_bytes, stream);
}

int pwc_corr_backward(const void* in1, const void* in2, const void* grad_out, void* grad_in1,
                      void* grad_in2, int B, int C, int H, int W, int pad_size,
                      int kernel_size, int max_displacement, int stride1, int stride2,
                      int corr_multiply, int dtype, void* stream) {
  (void)corr_multiply;
  const char* fn = "pwc_corr_backward";
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (stride1 != 1)
    return fail(fn, "stride1 != 1 is undefined in the reference backward (cu:120-121)");
  if (!corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo))
    return fail(fn, "invalid correlation parameters");
  if (Ho <= 0 || Wo <= 0) return fail(fn, "empty correlation output");
  if ((size_t)B * C * H * W && (!in1 || !in2 || !grad_out || !grad_in1 || !grad_in2))
    return fail(fn, "null buffer");
  const float divisor = (float)(kernel_size * kernel_size * C);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::corr_backward_t<float>(in1, in2, grad_out, grad_in1, grad_in2, B, C, H, W, Ho,
                                      Wo, pad_size, kernel_size, max_displacement, stride1,
                                      stride2, pwc::kRaster, divisor, s, force_generic());
      break;
    case PWC_DTYPE_F16:
      e = pwc::corr_backward_t<__half>(in1, in2, grad_out, grad_in1, grad_in2, B, C, H, W, Ho,
                                       Wo, pad_size, kernel_size, max_displacement, stride1,
                                       stride2, pwc::kRaster, divisor, s, force_generic());
      break;
    case PWC_DTYPE_BF16:
      e = pwc::corr_backward_t<__hip_bfloat16>(in1, in2, grad_out, grad_in1, grad_in2, B, C, H,
                                               W, Ho, Wo, pad_size, kernel_size,
                                               max_displacement, stride1, stride2,
                                               pwc::kRaster, divisor, s, force_generic());
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  return check_launch(fn, e);
}

static int cost_volume_forward_impl(const char* fn, const void* src, const void* tgt, void* out,
                                    int B, int C, int H, int W, int search_range, int dtype,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (search_range < 0) return fail(fn, "negative search_range");
  if ((size_t)B * C * H * W && (!src || !tgt || !out)) return fail(fn, "null buffer");
  const int K = (2 * search_range + 1) * (2 * search_range + 1);
  if (workspace && workspace_bytes < pwc::corr_workspace_bytes(B, K, H, W))
    return fail(fn, "workspace smaller than pwc_cost_volume_workspace_size()");
  const float divisor = (float)K;  // modules.py:74 output / shape[1]
  const int sr = search_range;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  // CostVolumeLayer == Correlation(pad=sr, k=1, md=sr, s1=1, s2=1) with CVL channel order.
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::corr_forward_t<float>(src, tgt, out, B, C, H, W, H, W, sr, 1, sr, 1, 1,
                                     pwc::kCvl, divisor, workspace, s, force_generic());
      break;
    case PWC_DTYPE_F16:
      e = pwc::corr_forward_t<__half>(src, tgt, out, B, C, H, W, H, W, sr, 1, sr, 1, 1,
                                      pwc::kCvl, divisor, workspace, s, force_generic());
      break;
    case PWC_DTYPE_BF16:
      e = pwc::corr_forward_t<__hip_bfloat16>(src, tgt, out, B, C, H, W, H, W, sr, 1, sr, 1, 1,
                                              pwc::kCvl, divisor, workspace, s,
                                              force_generic());
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  return check_launch(fn, e);
}

size_t pwc_cost_volume_workspace_size(int B, int C, int H, int W, int search_range) {
  if (!dims_ok(B, C, H, W) || search_range < 0) return 0;
  const int K = (2 * search_range + 1) * (2 * search_range + 1);
  return pwc::corr_workspace_bytes(B, K, H, W);
}

int pwc_cost_volume_forward(const void* src, const void* tgt, void* out, int B, int C, int H,
                            int W, int search_range, int dtype, void* stream) {
  return cost_volume_forward_impl("pwc_cost_volume_forward", src, tgt, out, B, C, H, W,
                                  search_range, dtype, nullptr, 0, stream);
}

int pwc_cost_volume_forward_ws(const void* src, const void* tgt, void* out, int B, int C,
                               int H, int W, int search_range, int dtype, void* workspace,
                               size_t workspace_bytes, void* stream) {
  return cost_volume_forward_impl("pwc_cost_volume_forward_ws", src, tgt, out, B, C, H, W,
                                  search_range, dtype, workspace, workspace_bytes, stream);
}

int pwc_cost_volume_backward(const void* src, const void* tgt, const void* grad_out,
                             void* grad_src, void* grad_tgt, int B, int C, int H, int W,
                             int search_range, int dtype, void* stream) {
  const char* fn = "pwc_cost_volume_backward";
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (search_range < 0) return fail(fn, "negative search_range");
  if ((size_t)B * C * H * W && (!src || !tgt || !grad_out || !grad_src || !grad_tgt))
    return fail(fn, "null buffer");
  const int K = (2 * search_range + 1) * (2 * search_range + 1);
  const float divisor = (float)K;
  const int sr = search_range;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::corr_backward_t<float>(src, tgt, grad_out, grad_src, grad_tgt, B, C, H, W, H, W,
                                      sr, 1, sr, 1, 1, pwc::kCvl, divisor, s, force_generic());
      break;
    case PWC_DTYPE_F16:
      e = pwc::corr_backward_t<__half>(src, tgt, grad_out, grad_src, grad_tgt, B, C, H, W, H,
                                       W, sr, 1, sr, 1, 1, pwc::kCvl, divisor, s,
                                       force_generic());
      break;
    case PWC_DTYPE_BF16:
      e = pwc::corr_backward_t<__hip_bfloat16>(src, tgt, grad_out, grad_src, grad_tgt, B, C, H,
                                               W, H, W, sr, 1, sr, 1, 1, pwc::kCvl, divisor, s,
                                               force_generic());
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  return check_launch(fn, e);
}

int pwc_warp_forward(const void* x, const void* flow, void* out, int B, int C, int H, int W,
                     int dtype, void* stream) {
  const char* fn = "pwc_warp_forward";
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if ((size_t)B * C * H * W && (!x || !flow || !out)) return fail(fn, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::warp_forward_t<float>(x, flow, out, B, C, H, W, s);
      break;
    case PWC_DTYPE_F16:
      e = pwc::warp_forward_t<__half>(x, flow, out, B, C, H, W, s);
      break;
    case PWC_DTYPE_BF16:
      e = pwc::warp_forward_t<__hip_bfloat16>(x, flow, out, B, C, H, W, s);
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  return check_launch(fn, e);
}

int pwc_warp_forward_group(const pwc_warp_problem* problems, int count, int dtype,
                           void* stream) {
  const char* fn = "pwc_warp_forward_group";
  if (count < 0 || (count > 0 && !problems)) return fail(fn, "invalid problem list");
  static_assert(sizeof(pwc_warp_problem) == sizeof(pwc::WarpProblem), "problem layout");
  for (int i = 0; i < count; ++i) {
    const pwc_warp_problem& q = problems[i];
    if (!dims_ok(q.B, q.C, q.H, q.W)) return fail(fn, "negative dimension");
    if ((size_t)q.B * q.C * q.H * q.W && (!q.x || !q.flow || !q.out))
      return fail(fn, "null buffer");
  }
  const pwc::WarpProblem* p = reinterpret_cast<const pwc::WarpProblem*>(problems);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::warp_forward_group_t<float>(p, count, s);
      break;
    case PWC_DTYPE_F16:
      e = pwc::warp_forward_group_t<__half>(p, count, s);
      break;
    case PWC_DTYPE_BF16:
      e = pwc::warp_forward_group_t<__hip_bfloat16>(p, count, s);
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  return check_launch(fn, e);
}

int pwc_warp_backward(const void* x, const void* flow, const void* grad_out, void* grad_x,
                      void* grad_flow, int B, int C, int H, int W, int dtype, void* stream) {
  const char* fn = "pwc_warp_backward";
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (dtype != PWC_DTYPE_F32) return fail(fn, "backward is fp32 only");
  if ((size_t)B * H * W && (!x || !flow || !grad_out || !grad_x || !grad_flow))
    return fail(fn, "null buffer");
  return check_launch(fn, pwc::warp_backward_f32(x, flow, grad_out, grad_x, grad_flow, B, C, H,
                                                 W, (hipStream_t)stream));
}

size_t pwc_warp_backward_workspace_size(int B, int C, int H, int W, int dtype) {
  if (!dims_ok(B, C, H, W) || dtype != PWC_DTYPE_F32) return 0;
  return pwc::warp_backward_workspace_size(B, C, H, W);
}

int pwc_warp_backward_ws(const void* x, const void* flow, const void* grad_out, void* grad_x,
                         void* grad_flow, int B, int C, int H, int W, int dtype, void* workspace,
                         size_t workspace_bytes, void* stream) {
  const char* fn = "pwc_warp_backward_ws";
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (dtype != PWC_DTYPE_F32) return fail(fn, "backward is fp32 only");
  if ((size_t)B * H * W && (!x || !flow || !grad_out || !grad_x || !grad_flow))
    return fail(fn, "null buffer");
  if ((size_t)B * H * W == 0) return 1;
  const hipError_t e =
      pwc::warp_backward_tiles_f32(x, flow, grad_out, grad_x, grad_flow, B, C, H, W, workspace,
                                   workspace_bytes, (hipStream_t)stream);
  if (e != hipErrorNotSupported) return check_launch(fn, e);
  return check_launch(fn, pwc::warp_backward_f32(x, flow, grad_out, grad_x, grad_flow, B, C, H,
                                                 W, (hipStream_t)stream));
}

int pwc_upsample_warp_forward(const void* x2, const void* flow_coarse, void* flow_up,
                              void* x2_warp, int B, int C, int H, int W, int dtype,
                              void* stream) {
  const char* fn = "pwc_upsample_warp_forward";
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if ((H | W) & 1) return fail(fn, "H and W must be even (2x the coarse flow)");
  if ((size_t)B * H * W && (!flow_coarse || (C && (!x2 || !x2_warp))))
    return fail(fn, "null buffer");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case PWC_DTYPE_F32:
      e = pwc::upsample_warp_forward_t<float>(x2, flow_coarse, flow_up, x2_warp, B, C, H, W, s);
      break;
    case PWC_DTYPE_F16:
      e = pwc::upsample_warp_forward_t<__half>(x2, flow_coarse, flow_up, x2_warp, B, C, H, W, s);
      break;
    case PWC_DTYPE_BF16:
      e = pwc::upsample_warp_forward_t<__hip_bfloat16>(x2, flow_coarse, flow_up, x2_warp, B, C,
                                                       H, W, s);
      break;
    default:
      return fail(fn, "unsupported dtype");
  }
  return check_launch(fn, e);
}

int pwc_flow_upsample_backward(const void* grad_flow_up, void* grad_flow_coarse, int B, int H,
                               int W, int dtype, void* stream) {
  const char* fn = "pwc_flow_upsample_backward";
  if (!dims_ok(B, 2, H, W)) return fail(fn, "negative dimension");
  if ((H | W) & 1) return fail(fn, "H and W must be even (2x the coarse flow)");
  if (dtype != PWC_DTYPE_F32) return fail(fn, "backward is fp32 only");
  if ((size_t)B * H * W && (!grad_flow_up || !grad_flow_coarse)) return fail(fn, "null buffer");
  return check_launch(fn, pwc::flow_up2_backward_f32(grad_flow_up, grad_flow_coarse, B, H, W,
                                                     (hipStream_t)stream));
}

// ---- fused warp -> correlation (model.py:80-83 as one call) ----
// The fused kernel covers model.py:24's configuration (pad == md in {8, 9}, k 1, s1 1, s2 2)
// for fp32 wherever one band workgroup holds the level; everything else runs the warp kernel
// then the correlation kernels (x2_warp, or the workspace's tail when x2_warp is NULL, holds
// the warped features in between).
static bool warp_corr_fusable(int pad, int k, int md, int s1, int s2, int dtype) {
  return (dtype == PWC_DTYPE_F32 || dtype == PWC_DTYPE_F16) && k == 1 && s1 == 1 && s2 == 2 &&
         pad == md && (md == 8 || md == 9);
}

static int fused_disabled() { return pwc::debug_knob("fused", 1) == 0; }

static size_t elem_size(int dtype) { return dtype == PWC_DTYPE_F32 ? 4 : 2; }

size_t pwc_warp_corr_workspace_size(int B, int C, int H, int W, int pad_size, int kernel_size,
                                    int max_displacement, int stride1, int stride2, int dtype,
                                    int emit_warp) {
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W) || (dtype < 0 || dtype > 2) ||
      !corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo) ||
      Ho <= 0 || Wo <= 0)
    return 0;
  // the unfused fallback may run: split-channel partials + (without x2_warp) a warp buffer
  size_t ws = (pwc::corr_workspace_bytes(B, OC, Ho, Wo) + 255) & ~(size_t)255;
  if (!emit_warp) ws += (size_t)B * C * H * W * elem_size(dtype);
  return ws;
}

int pwc_warp_corr_forward(const void* in1, const void* x2, const void* flow, void* x2_warp,
                          void* out, int B, int C, int H, int W, int pad_size, int kernel_size,
                          int max_displacement, int stride1, int stride2, int corr_multiply,
                          int dtype, void* workspace, size_t workspace_bytes, void* stream) {
  (void)corr_multiply;
  const char* fn = "pwc_warp_corr_forward";
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (!corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo))
    return fail(fn, "invalid correlation parameters");
  if (Ho <= 0 || Wo <= 0) return fail(fn, "empty correlation output");
  if (dtype < 0 || dtype > 2) return fail(fn, "unsupported dtype");
  if ((size_t)B * C * H * W && (!in1 || !x2 || !flow || !out)) return fail(fn, "null buffer");
  const size_t need = pwc_warp_corr_workspace_size(B, C, H, W, pad_size, kernel_size,
                                                   max_displacement, stride1, stride2, dtype,
                                                   x2_warp != nullptr);
  hipStream_t s = (hipStream_t)stream;
  if (!fused_disabled() && warp_corr_fusable(pad_size, kernel_size, max_displacement, stride1,
                                             stride2, dtype)) {
    const hipError_t e = pwc::warp_corr_band(in1, x2, flow, x2_warp, out, B, C, H, W,
                                             (float)C, 1, dtype, s);
    if (e != hipErrorNotSupported) return check_launch(fn, e);
  }
  // two launches: warp into x2_warp (or the workspace tail), then the correlation
  void* warped = x2_warp;
  void* corr_ws = workspace;
  size_t corr_ws_bytes = workspace_bytes;
  if (!warped) {
    if (!workspace || workspace_bytes < need)
      return fail(fn, "x2_warp is NULL and the workspace is smaller than "
                      "pwc_warp_corr_workspace_size(..., emit_warp=0)");
    const size_t split = (pwc::corr_workspace_bytes(B, OC, Ho, Wo) + 255) & ~(size_t)255;
    warped = (char*)workspace + split;
    corr_ws_bytes = split;
    if (split == 0) corr_ws = nullptr;
  }
  if (!pwc_warp_forward(x2, flow, warped, B, C, H, W, dtype, stream)) return 0;
  return corr_forward_impl(fn, in1, warped, out, B, C, H, W, pad_size, kernel_size,
                           max_displacement, stride1, stride2, dtype, corr_ws, corr_ws_bytes,
                           stream);
}

int pwc_warp_corr_forward_group(const pwc_warp_corr_problem* problems, int count, int pad_size,
                                int kernel_size, int max_displacement, int stride1, int stride2,
                                int corr_multiply, int dtype, void* stream) {
  const char* fn = "pwc_warp_corr_forward_group";
  if (count < 0 || (count > 0 && !problems)) return fail(fn, "invalid problem list");
  // every problem is checked as pwc_warp_corr_forward checks it BEFORE any launch, so a bad
  // list never leaves work partly done (a NULL buffer would fault the pair kernel)
  if (dtype < 0 || dtype > 2) return fail(fn, "unsupported dtype");
  for (int i = 0; i < count; ++i) {
    const pwc_warp_corr_problem& q = problems[i];
    int OC, Ho, Wo;
    if (!dims_ok(q.B, q.C, q.H, q.W)) return fail(fn, "negative dimension");
    if (!corr_shape(q.H, q.W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC,
                    &Ho, &Wo))
      return fail(fn, "invalid correlation parameters");
    if (Ho <= 0 || Wo <= 0) return fail(fn, "empty correlation output");
    if ((size_t)q.B * q.C * q.H * q.W == 0) continue;
    if (!q.in1 || !q.x2 || !q.flow || !q.out) return fail(fn, "null buffer");
    if (!q.x2_warp) return fail(fn, "x2_warp is required");
  }
  // fused pairs first (in list order), then every problem left, one call each
  hipStream_t s = (hipStream_t)stream;
  std::vector<char> done((size_t)count, 0);
  if (!fused_disabled() && warp_corr_fusable(pad_size, kernel_size, max_displacement, stride1,
                                             stride2, dtype)) {
    int open = -1;
    for (int i = 0; i < count; ++i) {
      const pwc_warp_corr_problem& q = problems[i];
      if ((size_t)q.B * q.C * q.H * q.W == 0) continue;
      if (open < 0) {
        open = i;
        continue;
      }
      const pwc_warp_corr_problem& p = problems[open];
      const pwc::BandProblem a{p.in1, p.x2, p.flow, p.x2_warp, p.out, p.B, p.C, p.H, p.W};
      const pwc::BandProblem b{q.in1, q.x2, q.flow, q.x2_warp, q.out, q.B, q.C, q.H, q.W};
      const hipError_t e = pwc::warp_corr_band_pair(a, b, (float)p.C, (float)q.C, dtype, s);
      if (e == hipErrorNotSupported) {
        open = i;  // no pair with the open one: try the next problem against this one
        continue;
      }
      if (!check_launch(fn, e)) return 0;
      done[(size_t)open] = done[(size_t)i] = 1;
      open = -1;
    }
  }
  for (int i = 0; i < count; ++i) {
    if (done[(size_t)i]) continue;
    const pwc_warp_corr_problem& q = problems[i];
    if (!pwc_warp_corr_forward(q.in1, q.x2, q.flow, q.x2_warp, q.out, q.B, q.C, q.H, q.W,
                               pad_size, kernel_size, max_displacement, stride1, stride2,
                               corr_multiply, dtype, nullptr, 0, stream))
      return 0;
  }
  return 1;
}

// ---- the backward of one level (model.py:80-83) as one call ----
// model.py:24's configuration in fp32 on images one workgroup holds (l0 / l1): one launch
// (warp_corr_bwd.hip); otherwise the correlation backward into the workspace (d/dx2_warp), the
// incoming x2_warp gradient added, and the warp backward (its workspace after that buffer).
size_t pwc_warp_corr_backward_workspace_size(int B, int C, int H, int W, int pad_size,
                                             int kernel_size, int max_displacement, int stride1,
                                             int stride2, int dtype) {
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W) || dtype != PWC_DTYPE_F32 ||
      !corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo) ||
      Ho <= 0 || Wo <= 0)
    return 0;
  const size_t gw = ((size_t)B * C * H * W * sizeof(float) + 255) & ~(size_t)255;
  const size_t two = gw + pwc::warp_backward_workspace_size(B, C, H, W);
  size_t one = 0;
  if (warp_corr_fusable(pad_size, kernel_size, max_displacement, stride1, stride2, dtype))
    one = pwc::warp_corr_bwd_small_workspace(B, C, H, W);
  return one > two ? one : two;
}

int pwc_warp_corr_backward(const void* in1, const void* x2, const void* flow,
                           const void* x2_warp, const void* grad_corr, const void* grad_x2_warp,
                           void* grad_in1, void* grad_x2, void* grad_flow, int B, int C, int H,
                           int W, int pad_size, int kernel_size, int max_displacement,
                           int stride1, int stride2, int corr_multiply, int dtype,
                           void* workspace, size_t workspace_bytes, void* counters,
                           void* stream) {
  const char* fn = "pwc_warp_corr_backward";
  int OC, Ho, Wo;
  if (!dims_ok(B, C, H, W)) return fail(fn, "negative dimension");
  if (dtype != PWC_DTYPE_F32) return fail(fn, "backward is fp32 only");
  if (stride1 != 1) return fail(fn, "stride1 must be 1 (the reference backward is undefined)");
  if (!corr_shape(H, W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC, &Ho,
                  &Wo))
    return fail(fn, "invalid correlation parameters");
  if (Ho <= 0 || Wo <= 0) return fail(fn, "empty correlation output");
  if ((size_t)B * H * W == 0) return 1;
  if (!in1 || !x2 || !flow || !x2_warp || !grad_corr || !grad_in1 || !grad_x2 || !grad_flow)
    return fail(fn, "null buffer");
  const size_t need = pwc_warp_corr_backward_workspace_size(
      B, C, H, W, pad_size, kernel_size, max_displacement, stride1, stride2, dtype);
  if (!workspace || workspace_bytes < need)
    return fail(fn, "workspace smaller than pwc_warp_corr_backward_workspace_size()");
  hipStream_t s = (hipStream_t)stream;
  if (!fused_disabled() &&
      warp_corr_fusable(pad_size, kernel_size, max_displacement, stride1, stride2, dtype)) {
    const hipError_t e = pwc::warp_corr_bwd_small(
        in1, x2, flow, x2_warp, grad_corr, grad_x2_warp, grad_in1, grad_x2, grad_flow, B, C, H,
        W, (float)(kernel_size * kernel_size * C), workspace, workspace_bytes, counters, s);
    if (e != hipErrorNotSupported) return check_launch(fn, e);
  }
  // two launches (+ the x2_warp gradient): gw in the workspace head
  void* gw = workspace;
  const size_t gwb = ((size_t)B * C * H * W * sizeof(float) + 255) & ~(size_t)255;
  if (!pwc_corr_backward(in1, x2_warp, grad_corr, grad_in1, gw, B, C, H, W, pad_size,
                         kernel_size, max_displacement, stride1, stride2, corr_multiply, dtype,
                         stream))
    return 0;
  if (grad_x2_warp &&
      !check_launch(fn, pwc::add_inplace_f32(gw, grad_x2_warp, (size_t)B * C * H * W, s)))
    return 0;
  return pwc_warp_backward_ws(x2, flow, gw, grad_x2, grad_flow, B, C, H, W, dtype,
                              (char*)workspace + gwb, workspace_bytes - gwb, stream);
}

}  // extern "C"

// ---- grouped correlation (independent problems; the bench's l2 + l3) ----
// A problem the row-band kernel takes in a single call: model.py:24's configuration in fp32,
// rows too narrow for the stream kernel (W < 64), too many for the band kernel ((H+1)/2 > 6),
// 16-B aligned buffers (corr_fwd.hip's dispatch order: stream, band, rows).
// Two problems share a row-band launch only when the single-call dispatch would run each on
// the row-band kernel (the same predicate corr_forward_t dispatches by): then the paired result
// equals the single calls' bit for bit.
static bool rows_pairable(const pwc_corr_problem& q, int pad, int k, int md, int s1, int s2,
                          int dtype) {
  return dtype == PWC_DTYPE_F32 && force_generic() == 0 && (size_t)q.B * q.C * q.H * q.W > 0 &&
         pwc::corr_forward_path(q.in1, q.in2, q.out, q.B, q.C, q.H, q.W, pad, k, md, s1, s2,
                                pwc::kRaster, 0) == pwc::kPathRows;
}

int pwc_corr_forward_group(const pwc_corr_problem* problems, int count, int pad_size,
                           int kernel_size, int max_displacement, int stride1, int stride2,
                           int corr_multiply, int dtype, void* stream) {
  const char* fn = "pwc_corr_forward_group";
  if (count < 0 || (count > 0 && !problems)) return fail(fn, "invalid problem list");
  for (int i = 0; i < count; ++i) {
    const pwc_corr_problem& q = problems[i];
    int OC, Ho, Wo;
    if (!dims_ok(q.B, q.C, q.H, q.W)) return fail(fn, "negative dimension");
    if (!corr_shape(q.H, q.W, pad_size, kernel_size, max_displacement, stride1, stride2, &OC,
                    &Ho, &Wo))
      return fail(fn, "invalid correlation parameters");
    if ((size_t)q.B * q.C * q.H * q.W && (!q.in1 || !q.in2 || !q.out))
      return fail(fn, "null buffer");
  }
  hipStream_t s = (hipStream_t)stream;
  std::vector<char> done((size_t)count, 0);
  int open = -1;
  for (int i = 0; i < count; ++i) {
    const pwc_corr_problem& q = problems[i];
    if (!rows_pairable(q, pad_size, kernel_size, max_displacement, stride1, stride2, dtype))
      continue;
    if (open < 0) {
      open = i;
      continue;
    }
    const pwc_corr_problem& p = problems[open];
    const hipError_t e = pwc::corr_forward_rows_pair(
        p.in1, p.in2, p.out, p.B, p.C, p.H, p.W, q.in1, q.in2, q.out, q.B, q.C, q.H, q.W,
        (float)p.C, (float)q.C, s);
    if (e == hipErrorNotSupported) {
      open = i;
      continue;
    }
    if (!check_launch(fn, e)) return 0;
    done[(size_t)open] = done[(size_t)i] = 1;
    open = -1;
  }
  for (int i = 0; i < count; ++i) {
    if (done[(size_t)i]) continue;
    const pwc_corr_problem& q = problems[i];
    if (!pwc_corr_forward(q.in1, q.in2, q.out, q.B, q.C, q.H, q.W, pad_size, kernel_size,
                          max_displacement, stride1, stride2, corr_multiply, dtype, stream))
      return 0;
  }
  pwc::g_ev_start = pwc::g_ev_stop = nullptr;  // one-shot, consumed or not
  return 1;
}
