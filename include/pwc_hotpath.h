/*
 * pwc_hotpath.h — C ABI of the MI355X (gfx950) PWC-Net hot path:
 * cost-volume correlation, CostVolumeLayer-ordered cost volume and bilinear flow warp.
 *
 * Plain pointers and sizes only: no torch / THC types.  Every tensor is a caller-owned,
 * contiguous NCHW device buffer (hipMalloc'd or torch-allocated) of the element type named
 * by `dtype`.  `stream` is a hipStream_t (NULL = the legacy default stream).  All calls are
 * asynchronous on `stream`, perform no host synchronisation and no allocation, so they may
 * be captured into a hipGraph.
 *
 * Return value mirrors the reference launcher (correlation_cuda_kernel.cu:361-368):
 *   1 = kernels enqueued, 0 = error (argument check or launch failure); the message is then
 *   available from pwc_last_error() (thread-local).  The reference turned 0 into
 *   THError("aborting") (correlation_cuda.c:86-89); the Python layer raises RuntimeError.
 *
 * Reference interfaces replaced (paths relative to daigo0927/PWC-Net_pytorch):
 *   pwc_corr_output_shape  <- shape math of Correlation_forward_cuda, correlation_cuda.c:20-34
 *   pwc_corr_forward       <- Correlation_forward_cuda (correlation_cuda.c:11-93, declared
 *                             correlation_cuda.h:1-8) -> Correlation_forward_cuda_kernel
 *                             (correlation_cuda_kernel.h:5-38, .cu:296-369).  No rInput1/
 *                             rInput2 scratch: the NHWC transpose (cu:10-32) is not needed.
 *   pwc_corr_forward_into  <- model.py:83-84 (corr, optional leaky_relu_) feeding the cat of
 *                             model.py:89/91, as one call writing the cat buffer's slice
 *   pwc_corr_backward      <- Correlation_backward_cuda (correlation_cuda.c:95-180,
 *                             correlation_cuda.h:10-17) -> Correlation_backward_cuda_kernel
 *                             (correlation_cuda_kernel.h:40-88, .cu:371-473)
 *   pwc_cost_volume_forward/backward <- CostVolumeLayer.forward (modules.py:53-74) and its
 *                             autograd; there is no C interface in the reference (pure ATen).
 *   pwc_warp_forward/backward <- WarpingLayer.forward (modules.py:31-42) + get_grid
 *                             (utils.py:3-8) + F.grid_sample/grid_sampler_2d_backward with
 *                             torch-0.4 semantics (bilinear, zeros, align_corners=True).
 *   pwc_warp_corr_forward  <- the two calls of one pyramid level, model.py:80 (warp) + :83
 *                             (corr), as one entry point (fused kernel where it applies).
 *   pwc_warp_corr_backward <- their backward: Correlation_backward_cuda (correlation_cuda.c:
 *                             95-180) into x2_warp, then grid_sample's backward (modules.py:41),
 *                             as one entry point (one kernel at the coarse levels).
 *   pwc_upsample_warp_forward <- model.py:78 (F.upsample(flow, scale_factor=2,
 *                             mode='bilinear') * 2, torch-0.4 align_corners=False) + :80
 *                             (WarpingLayer) as one launch; pwc_flow_upsample_backward is the
 *                             adjoint of model.py:78 (ATen upsample_bilinear2d_backward * 2).
 */
#ifndef PWC_HOTPATH_H
#define PWC_HOTPATH_H

#if defined(__GNUC__) || defined(__clang__)
#define PWC_API __attribute__((visibility("default")))
#else
#define PWC_API
#endif

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types (`dtype` arguments).  Arithmetic is always fp32 accumulate. */
#define PWC_DTYPE_F32 0
#define PWC_DTYPE_F16 1
#define PWC_DTYPE_BF16 2

/* ABI version; bumped on any signature change (2: workspace entry points, 3: timing hook,
 * 4: fused warp -> correlation, 5: fused flow upsample -> warp, corr into a slice,
 * 6: pwc_set_debug, 7: grouped warp / warp -> correlation launches, 8: one-launch warp
 * backward with a workspace, 9: pwc_corr_forward_plan, 10: pwc_corr_backward_plan,
 * 11: pwc_warp_corr_backward). */
PWC_API int pwc_abi_version(void);

/* Which kernel family pwc_corr_forward would launch for these arguments (the same dispatch
 * predicates; no device call, no launch -- pointers are only inspected for alignment), for
 * tests and measurement tools.  Returns -1 for arguments pwc_corr_forward rejects.  Replaces
 * nothing in the reference (its launcher has one kernel, correlation_cuda_kernel.cu:348-359). */
#define PWC_PLAN_OTHER 0    /* parity tiles / whole-half / generic kernels (corr_fwd.hip) */
#define PWC_PLAN_STREAM 1   /* channel-streaming row bands (corr_stream.hip) */
#define PWC_PLAN_BAND 2     /* all-channel band (warp_corr.hip, l0/l1) */
#define PWC_PLAN_ROWS 3     /* row bands, channel chunks (corr_rows.hip, l2/l3) */
#define PWC_PLAN_STRIP 4    /* fp32 stepped column strips (corr_strip.hip, l4) */
#define PWC_PLAN_MSTRIP16 5 /* fp16 matrix-core strips (corr_mstrip16.hip) */
PWC_API int pwc_corr_forward_plan(const void* in1, const void* in2, const void* out, int B,
                                  int C, int H, int W, int pad_size, int kernel_size,
                                  int max_displacement, int stride1, int stride2, int dtype);

/* Which kernel family pwc_corr_backward would launch (same predicates; no device call), -1 for
 * arguments it rejects.  Replaces nothing in the reference (cu:417-473 launches two kernels). */
#define PWC_BWD_PLAN_OTHER 0 /* stencil / tiled / generic kernels (corr_bwd.hip) */
#define PWC_BWD_PLAN_ROWS 1  /* row bands with tj partials (corr_bwd_rows.hip; shapes it cannot
                                band fall back to the stencil kernels) */
#define PWC_BWD_PLAN_STRIP 2 /* displacement-row steps over resident rows (corr_bwd_strip.hip) */
PWC_API int pwc_corr_backward_plan(const void* in1, const void* in2, const void* grad_out,
                                   const void* grad_in1, const void* grad_in2, int B, int C,
                                   int H, int W, int pad_size, int kernel_size,
                                   int max_displacement, int stride1, int stride2, int dtype);

/* Measurement hook: the next correlation dispatch of the calling thread that runs the l4-class
 * LDS-DMA kernel is launched with hipExtLaunchKernel, recording `start_event` / `stop_event`
 * (hipEvent_t, timing enabled) at that kernel's start and end on its stream.  One-shot; pass
 * (NULL, NULL) to disarm.  Used by bench.py to time the dominant kernel live. */
PWC_API int pwc_time_next_corr(void* start_event, void* stop_event);

/* Measurement / test hook: replace the debug knob string (initially the PWC_DEBUG environment
 * variable; "name=value,name=value", integer values; NULL or "" = production defaults).  Knobs
 * only select among equivalent kernel variants (tests run every variant against the oracle)
 * or disable work for ablation timings; no knob is set in production.  Not thread-safe with
 * concurrent launches. */
PWC_API int pwc_set_debug(const char* spec);

/* Last error message of the calling thread ("" if none). */
PWC_API const char* pwc_last_error(void);

/* correlation_cuda.c:20-34: OC = ((md/s2)*2+1)^2, Ho = ceil((H+2pad-2(kr+md))/s1), Wo alike,
 * kr = (k-1)/2 (C truncation).  Returns 0 if the output would be empty. */
PWC_API int pwc_corr_output_shape(int H, int W, int pad_size, int kernel_size, int max_displacement,
                          int stride1, int stride2, int* out_channels, int* out_height,
                          int* out_width);

/* out[B][OC][Ho][Wo] = correlation of in1, in2 ([B][C][H][W]) exactly as
 * correlation_cuda_kernel.cu:34-106: channel tc = (tj+dr)*D + (ti+dr), value divided by
 * kernel_size^2 * C.  corr_multiply is accepted and ignored, as in the reference. */
PWC_API int pwc_corr_forward(const void* in1, const void* in2, void* out, int B, int C, int H, int W,
                     int pad_size, int kernel_size, int max_displacement, int stride1,
                     int stride2, int corr_multiply, int dtype, void* stream);

/* Same as pwc_corr_forward with a caller-owned device workspace of at least
 * pwc_corr_workspace_size() bytes.  For grids too small to fill the GPU (coarse pyramid
 * levels) the channel sum is split across workgroups into partial volumes in `workspace` and
 * reduced in a fixed order (deterministic).  A size of 0 means no workspace is used. */
PWC_API size_t pwc_corr_workspace_size(int B, int C, int H, int W, int pad_size, int kernel_size,
                               int max_displacement, int stride1, int stride2);
PWC_API int pwc_corr_forward_ws(const void* in1, const void* in2, void* out, int B, int C, int H,
                        int W, int pad_size, int kernel_size, int max_displacement,
                        int stride1, int stride2, int corr_multiply, int dtype,
                        void* workspace, size_t workspace_bytes, void* stream);

/* model.py:83-84 + :89/91: the correlation written straight into a caller's buffer slice --
 * image n's OC x Ho x Wo block starts at out + n * out_image_stride elements (e.g. the corr
 * channels of the cat([x1, corr, flow], 1) buffer: out = buf + C*H*W, stride (C+OC+2)*H*W) --
 * with every value passed through leaky_relu(negative_slope) (model.py:84's in-place
 * F.leaky_relu_ when args.corr_activation, slope 0.01; 1.0 = no activation, bit-identical to
 * pwc_corr_forward).  For model.py:24's configuration in fp32 the correlation kernels write
 * the slice themselves; other configurations compute the dense volume in `workspace` (at least
 * pwc_corr_forward_into_workspace_size() bytes; may be NULL when not needed) and copy it. */
PWC_API size_t pwc_corr_forward_into_workspace_size(int B, int C, int H, int W, int pad_size,
                                                    int kernel_size, int max_displacement,
                                                    int stride1, int stride2, int dtype);
PWC_API int pwc_corr_forward_into(const void* in1, const void* in2, void* out,
                                  long long out_image_stride, float negative_slope, int B, int C,
                                  int H, int W, int pad_size, int kernel_size,
                                  int max_displacement, int stride1, int stride2,
                                  int corr_multiply, int dtype, void* workspace,
                                  size_t workspace_bytes, void* stream);
/* grad_in1/grad_in2 ([B][C][H][W]) from grad_out ([B][OC][Ho][Wo]) exactly as
 * correlation_cuda_kernel.cu:108-290.  Requires stride1 == 1 (the reference backward is
 * undefined otherwise: it indexes gradInput with the strided coordinate).  Every element of
 * both gradients is written (no pre-zeroing needed). */
PWC_API int pwc_corr_backward(const void* in1, const void* in2, const void* grad_out, void* grad_in1,
                      void* grad_in2, int B, int C, int H, int W, int pad_size,
                      int kernel_size, int max_displacement, int stride1, int stride2,
                      int corr_multiply, int dtype, void* stream);

/* CostVolumeLayer (modules.py:53-74): out[B][(2sr+1)^2][H][W], channel order of
 * modules.py:58-72, value sum_c src*tgt(shifted) / (2sr+1)^2. */
PWC_API int pwc_cost_volume_forward(const void* src, const void* tgt, void* out, int B, int C, int H,
                            int W, int search_range, int dtype, void* stream);
PWC_API size_t pwc_cost_volume_workspace_size(int B, int C, int H, int W, int search_range);
PWC_API int pwc_cost_volume_forward_ws(const void* src, const void* tgt, void* out, int B, int C,
                               int H, int W, int search_range, int dtype, void* workspace,
                               size_t workspace_bytes, void* stream);
PWC_API int pwc_cost_volume_backward(const void* src, const void* tgt, const void* grad_out,
                             void* grad_src, void* grad_tgt, int B, int C, int H, int W,
                             int search_range, int dtype, void* stream);

/* WarpingLayer: out[b][c][y][x] = bilinear sample of x at (x + u, y + v) with the reference's
 * normalisation chain (flow / ((W-1)/2) + linspace(-1,1), align_corners=True), zeros outside.
 * flow is [B][2][H][W], channel 0 = u (horizontal), 1 = v (vertical), in pixels. */
PWC_API int pwc_warp_forward(const void* x, const void* flow, void* out, int B, int C, int H, int W,
                     int dtype, void* stream);
/* Several INDEPENDENT warps (e.g. the bench's synthetic pyramid levels, or the levels of
 * different batches in flight; inside one model forward each level's warp needs the previous
 * level's flow, so those are not a group) in one launch per 4 problems: the problems' grids are
 * laid end to end in one flat grid, so they share one launch gap and fill each other's tails.
 * Each problem's output equals a pwc_warp_forward call on it, bit for bit (same fmaf chain per
 * element; only the channels-per-thread grouping follows the largest problem).  Replaces a
 * sequence of WarpingLayer calls (modules.py:31-42); returns 1 on success. */
typedef struct {
  const void* x;
  const void* flow;
  void* out;
  int B, C, H, W;
} pwc_warp_problem;
PWC_API int pwc_warp_forward_group(const pwc_warp_problem* problems, int count, int dtype,
                                   void* stream);
/* Adjoint of pwc_warp_forward (ATen grid_sampler_2d_backward with the reference's grid chain).
 * grad_x: every element is written once (no memset, no atomics): per 8x32 tile of grad_x the
 * output pixels whose bilinear corners land in the tile are gathered in fixed order (a
 * counting sort in LDS), so the result is deterministic.  grad_flow: per pixel, element-wise;
 * only corners that fall outside the gather window of their tile (flows beyond ~8 px) are
 * added with fp32 atomics.  fp32 only. */
PWC_API int pwc_warp_backward(const void* x, const void* flow, const void* grad_out, void* grad_x,
                      void* grad_flow, int B, int C, int H, int W, int dtype, void* stream);
/* Same result with a caller-owned device workspace of at least
 * pwc_warp_backward_workspace_size() bytes (no initialisation needed).  On wide images
 * (W >= 56: the l3 / l4 levels) grad_x and grad_flow come from one tile kernel -- per 16x16 tile of
 * grad_x its output pixels' lists (fixed order) with x and grad_out streamed through LDS --
 * plus a small kernel that adds the channel groups' grad_flow partials (fixed order) and the
 * rare corners beyond the tiles' 8-pixel margins (fp32 atomics).  Other sizes, or a NULL /
 * short workspace, run pwc_warp_backward's kernels.  fp32 only. */
PWC_API size_t pwc_warp_backward_workspace_size(int B, int C, int H, int W, int dtype);
PWC_API int pwc_warp_backward_ws(const void* x, const void* flow, const void* grad_out,
                                 void* grad_x, void* grad_flow, int B, int C, int H, int W,
                                 int dtype, void* workspace, size_t workspace_bytes, void* stream);

/* model.py:78 + :80 in one launch: flow_up = bilinear x2 upsample of flow_coarse
 * ([B][2][H/2][W/2], ATen upsample_bilinear2d with align_corners=False -- torch 0.4's default)
 * times 2, then x2_warp = WarpingLayer(x2, flow_up) exactly as pwc_warp_forward on the stored
 * flow_up.  H, W = the size of x2 (even).  flow_up ([B][2][H][W]) may be NULL (not needed);
 * it is written otherwise (model.py:89/91 concatenates it). */
PWC_API int pwc_upsample_warp_forward(const void* x2, const void* flow_coarse, void* flow_up,
                                      void* x2_warp, int B, int C, int H, int W, int dtype,
                                      void* stream);
/* Adjoint of model.py:78: grad_flow_coarse ([B][2][H/2][W/2], written) from grad_flow_up
 * ([B][2][H][W]); fixed-order gather, no atomics.  fp32. */
PWC_API int pwc_flow_upsample_backward(const void* grad_flow_up, void* grad_flow_coarse, int B,
                                       int H, int W, int dtype, void* stream);
/* One pyramid level of model.py:80-83: x2_warp = WarpingLayer(x2, flow), then
 * out = Correlation(in1, x2_warp) exactly as pwc_warp_forward followed by pwc_corr_forward
 * (same values: x2_warp bit-identical, out within fp32 summation order).  x2_warp may be NULL
 * (not needed by the caller); it is written otherwise.  For model.py:24's configuration in
 * fp32 this is ONE kernel launch per level where the level fits (no warped-feature round trip
 * through HBM); other configurations run the two kernels.  `workspace` must hold
 * pwc_warp_corr_workspace_size(..., emit_warp = x2_warp != NULL) bytes; NULL is accepted when
 * x2_warp is given (the fallback then runs without channel splitting). */
PWC_API size_t pwc_warp_corr_workspace_size(int B, int C, int H, int W, int pad_size,
                                    int kernel_size, int max_displacement, int stride1,
                                    int stride2, int dtype, int emit_warp);
PWC_API int pwc_warp_corr_forward(const void* in1, const void* x2, const void* flow, void* x2_warp,
                          void* out, int B, int C, int H, int W, int pad_size,
                          int kernel_size, int max_displacement, int stride1, int stride2,
                          int corr_multiply, int dtype, void* workspace,
                          size_t workspace_bytes, void* stream);
/* Several INDEPENDENT warp -> correlation problems (e.g. the pyramid levels of different
 * batches in flight, or of the bench's synthetic levels; inside one forward of the model the
 * levels depend on each other and are not a group).  Each problem is one pwc_warp_corr_forward
 * call with x2_warp required (not NULL); problems of model.py:24's configuration in fp32 that
 * take the fused band kernel are paired into ONE launch whose two grids share the CUs
 * (the coarse levels' workgroups are latency-bound: 384x448 l0 + l1 run side by side), the
 * rest run one pwc_warp_corr_forward call each, without a workspace.  Values are those of
 * separate pwc_warp_corr_forward calls, bit for bit.  Returns 1 on success. */
typedef struct {
  const void* in1;
  const void* x2;
  const void* flow;
  void* x2_warp;
  void* out;
  int B, C, H, W;
} pwc_warp_corr_problem;
PWC_API int pwc_warp_corr_forward_group(const pwc_warp_corr_problem* problems, int count,
                                        int pad_size, int kernel_size, int max_displacement,
                                        int stride1, int stride2, int corr_multiply, int dtype,
                                        void* stream);

/* The backward of pwc_warp_corr_forward (WarpCorrelationFunction.backward): from grad_corr
 * ([B][OC][Ho][Wo]) and an optional gradient arriving on x2_warp itself (grad_x2_warp, NULL =
 * none) -> grad_in1 (d/dx1, as pwc_corr_backward's grad_in1), grad_x2 and grad_flow (the warp
 * backward, as pwc_warp_backward_ws, of d/dx2_warp + grad_x2_warp).  fp32, stride1 == 1.
 * `workspace`: at least pwc_warp_corr_backward_workspace_size() bytes.  `counters`: B uint32
 * in device memory, zero before the first call; every call leaves them zero (one set per
 * stream: concurrent calls must not share it); NULL selects the two-launch path.  For
 * model.py:24's configuration on images of <= 256 pixels with C % 4 == 0 (the l0 / l1 levels)
 * this is ONE kernel whose d/dx2_warp never leaves LDS; grad_flow then adds per-channel-group
 * partials in a fixed order (deterministic).  Elsewhere: pwc_corr_backward into the workspace,
 * the x2_warp gradient added, then pwc_warp_backward_ws. */
PWC_API size_t pwc_warp_corr_backward_workspace_size(int B, int C, int H, int W, int pad_size,
                                                     int kernel_size, int max_displacement,
                                                     int stride1, int stride2, int dtype);
PWC_API int pwc_warp_corr_backward(const void* in1, const void* x2, const void* flow,
                                   const void* x2_warp, const void* grad_corr,
                                   const void* grad_x2_warp, void* grad_in1, void* grad_x2,
                                   void* grad_flow, int B, int C, int H, int W, int pad_size,
                                   int kernel_size, int max_displacement, int stride1,
                                   int stride2, int corr_multiply, int dtype, void* workspace,
                                   size_t workspace_bytes, void* counters, void* stream);
/* Several INDEPENDENT correlations (e.g. the bench's synthetic pyramid levels, or the levels
 * of different batches in flight; inside one model forward each level's correlation needs that
 * level's warp, which needs the previous level's flow).  Each problem's output equals a
 * pwc_corr_forward call on it, bit for bit; problems of model.py:24's configuration in fp32
 * that take the row-band kernel (l2 + l3 at 384x448) are paired into ONE launch (one workgroup
 * per CU; the second grid fills the CUs the first leaves idle), the rest run one
 * pwc_corr_forward call each.  Replaces a sequence of Correlation calls
 * (correlation_cuda.c:36-90 per call); returns 1 on success. */
typedef struct {
  const void* in1;
  const void* in2;
  void* out;
  int B, C, H, W;
} pwc_corr_problem;
PWC_API int pwc_corr_forward_group(const pwc_corr_problem* problems, int count, int pad_size,
                                   int kernel_size, int max_displacement, int stride1,
                                   int stride2, int corr_multiply, int dtype, void* stream);
#ifdef __cplusplus
}
#endif
#endif /* PWC_HOTPATH_H */
