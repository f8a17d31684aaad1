"""Raw device ops over the C ABI plus their autograd Functions.

Each op takes contiguous NCHW tensors on a HIP device (fp32, fp16 or bf16 storage, fp32
arithmetic), allocates its outputs through the PyTorch caching allocator (caller-owned, as the
reference's ``input1.new()`` outputs, correlation_package/functions/correlation.py:28-30) and
enqueues the kernels on the current stream of the tensors' device.  Nothing synchronises.
"""
from __future__ import annotations

import ctypes

import torch
from torch.autograd import Function

from . import _lib


def _ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _check_inputs(what: str, *ts: torch.Tensor, dtypes=tuple(_lib.DTYPE_CODES)) -> None:
    dev = ts[0].device
    for t in ts:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{what}: expected tensors, got {type(t)}")
        if t.device.type != "cuda":
            raise RuntimeError(
                f"{what}: pwcnet_amd runs on HIP devices only (got a {t.device} tensor); "
                "there is no CPU implementation (the reference's correlation.c is a stub too)")
        if t.device != dev:
            raise RuntimeError(f"{what}: tensors on different devices ({t.device} vs {dev})")
        if t.dtype not in dtypes:
            raise TypeError(f"{what}: unsupported dtype {t.dtype}")
        if t.dtype != ts[0].dtype:
            raise TypeError(f"{what}: mixed dtypes {t.dtype} vs {ts[0].dtype}")
        if t.dim() != 4:
            raise ValueError(f"{what}: expected NCHW 4-d tensors, got shape {tuple(t.shape)}")


def _workspace(nbytes: int, device):
    """Split-channel scratch from the caching allocator (stream-ordered, graph-capturable)."""
    if nbytes == 0:
        return None, ctypes.c_void_p(0)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
    return ws, ctypes.c_void_p(ws.data_ptr())


def _i32(*vals) -> None:
    for v in vals:
        if not (-(2 ** 31) <= int(v) < 2 ** 31):
            raise ValueError(f"argument {v} does not fit the C ABI's int")


# ---------------------------------------------------------------------------------------
# correlation (correlation_package, cu:34-290)
# ---------------------------------------------------------------------------------------
def corr_forward(input1, input2, pad_size, kernel_size, max_displacement, stride1, stride2,
                 corr_multiply=1):
    _check_inputs("Correlation", input1, input2)
    if input1.shape != input2.shape:
        raise ValueError(f"Correlation: input shapes differ {tuple(input1.shape)} vs "
                         f"{tuple(input2.shape)}")
    B, C, H, W = input1.shape
    _i32(B, C, H, W, input1.numel())
    OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement, stride1,
                                        stride2)
    out = torch.empty((B, OC, Ho, Wo), dtype=input1.dtype, device=input1.device)
    if out.numel() == 0:
        return out
    lib = _lib.load()
    nws = lib.pwc_corr_workspace_size(B, C, H, W, pad_size, kernel_size, max_displacement,
                                      stride1, stride2)
    ws, wsp = _workspace(nws, input1.device)
    _lib.check(lib.pwc_corr_forward_ws(
        _ptr(input1), _ptr(input2), _ptr(out), B, C, H, W, pad_size, kernel_size,
        max_displacement, stride1, stride2, corr_multiply, _lib.DTYPE_CODES[input1.dtype],
        wsp, nws, _stream(input1.device)), "Correlation_forward")
    del ws  # the caching allocator keeps it stream-ordered until the kernels ran
    return out


def corr_backward(input1, input2, grad_output, pad_size, kernel_size, max_displacement, stride1,
                  stride2, corr_multiply=1):
    _check_inputs("Correlation backward", input1, input2, grad_output)
    B, C, H, W = input1.shape
    OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement, stride1,
                                        stride2)
    if tuple(grad_output.shape) != (B, OC, Ho, Wo):
        raise ValueError(f"Correlation backward: grad_output shape {tuple(grad_output.shape)} "
                         f"!= {(B, OC, Ho, Wo)}")
    grad_output = grad_output.contiguous()
    g1 = torch.empty_like(input1)
    g2 = torch.empty_like(input2)
    if g1.numel() == 0:
        return g1, g2
    _lib.check(_lib.load().pwc_corr_backward(
        _ptr(input1), _ptr(input2), _ptr(grad_output), _ptr(g1), _ptr(g2), B, C, H, W,
        pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply,
        _lib.DTYPE_CODES[input1.dtype], _stream(input1.device)), "Correlation_backward")
    return g1, g2


def corr_forward_into(input1, input2, out, pad_size, kernel_size, max_displacement, stride1,
                      stride2, corr_multiply=1, negative_slope=None):
    """Correlation written into ``out`` -- a (B, OC, Ho, Wo) view whose images may sit at any
    stride (e.g. ``buf[:, C:C+OC]`` of model.py:89/91's cat buffer) -- optionally through
    leaky_relu (model.py:84).  fp32 model.py:24 correlations are written by the kernels."""
    _check_inputs("Correlation into", input1, input2, out)
    B, C, H, W = input1.shape
    OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement, stride1,
                                        stride2)
    if tuple(out.shape) != (B, OC, Ho, Wo) or out.dtype != input1.dtype:
        raise ValueError(f"Correlation into: out {tuple(out.shape)} {out.dtype} != "
                         f"{(B, OC, Ho, Wo)} {input1.dtype}")
    if out.stride()[1:] != (Ho * Wo, Wo, 1) or (B > 1 and out.stride(0) < OC * Ho * Wo):
        raise ValueError("Correlation into: each image's block of `out` must be contiguous")
    _i32(B, C, H, W, input1.numel())
    input1, input2 = input1.contiguous(), input2.contiguous()
    lib = _lib.load()
    args = (B, C, H, W, pad_size, kernel_size, max_displacement, stride1, stride2)
    nbytes = lib.pwc_corr_forward_into_workspace_size(*args, _lib.DTYPE_CODES[input1.dtype])
    ws, wptr = _workspace(nbytes, input1.device)  # used only by the dense-then-copy fallback
    slope = 1.0 if negative_slope is None else float(negative_slope)
    _lib.check(lib.pwc_corr_forward_into(
        _ptr(input1), _ptr(input2), _ptr(out), out.stride(0), slope, *args, corr_multiply,
        _lib.DTYPE_CODES[input1.dtype], wptr, nbytes, _stream(input1.device)),
        "Correlation_forward_into")
    return out


class CorrelationCatFunction(Function):
    """cat([x1, act(corr(x1, x2_warp)), flow], 1) of model.py:83-91 with the correlation written
    into the cat buffer by the kernels (no separate volume, no copy of it)."""

    @staticmethod
    def forward(ctx, x1, x2_warp, flow, pad_size, kernel_size, max_displacement, stride1,
                stride2, negative_slope):
        x1, x2_warp, flow = x1.contiguous(), x2_warp.contiguous(), flow.contiguous()
        B, C, H, W = x1.shape
        OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement,
                                            stride1, stride2)
        if (Ho, Wo) != (H, W) or tuple(flow.shape[2:]) != (H, W):
            raise ValueError("CorrelationCat: the correlation must keep the feature size "
                             "(pad_size == max_displacement, kernel_size 1, stride1 1)")
        buf = torch.empty(B, C + OC + flow.shape[1], H, W, device=x1.device, dtype=x1.dtype)
        buf[:, :C].copy_(x1)
        buf[:, C + OC:].copy_(flow)
        with torch.cuda.device(x1.device):
            corr_forward_into(x1, x2_warp, buf[:, C:C + OC], pad_size, kernel_size,
                              max_displacement, stride1, stride2, 1, negative_slope)
        ctx.params = (pad_size, kernel_size, max_displacement, stride1, stride2, negative_slope,
                      C, OC)
        ctx.save_for_backward(x1, x2_warp, buf)
        return buf

    @staticmethod
    def backward(ctx, g):
        x1, x2_warp, buf = ctx.saved_tensors
        pad, k, md, s1, s2, slope, C, OC = ctx.params
        gcorr = g[:, C:C + OC]
        if slope is not None:  # in-place leaky_relu_: derivative from the result's sign
            gcorr = torch.where(buf[:, C:C + OC] > 0, gcorr, gcorr * slope)
        with torch.cuda.device(x1.device):
            g1, g2 = corr_backward(x1, x2_warp, gcorr.contiguous(), pad, k, md, s1, s2)
        return (g[:, :C] + g1, g2, g[:, C + OC:], None, None, None, None, None, None)


class CorrelationFunction(Function):
    """Drop-in for correlation_package/functions/correlation.py:7-56 (same signature and
    defaults, same contiguity asserts, backward returns (g1, g2) + (None,) * 6)."""

    @staticmethod
    def forward(ctx, input1, input2, pad_size=3, kernel_size=3, max_displacement=20, stride1=1,
                stride2=2, corr_multiply=1):
        assert input1.is_contiguous()
        assert input2.is_contiguous()
        ctx.save_for_backward(input1, input2)
        ctx.pad_size = pad_size
        ctx.kernel_size = kernel_size
        ctx.max_displacement = max_displacement
        ctx.stride1 = stride1
        ctx.stride2 = stride2
        ctx.corr_multiply = corr_multiply
        with torch.cuda.device(input1.device) if input1.is_cuda else _nullctx():
            return corr_forward(input1, input2, pad_size, kernel_size, max_displacement,
                                stride1, stride2, corr_multiply)

    @staticmethod
    def backward(ctx, grad_output):
        input1, input2 = ctx.saved_tensors
        with torch.cuda.device(input1.device):
            g1, g2 = corr_backward(input1, input2, grad_output, ctx.pad_size, ctx.kernel_size,
                                   ctx.max_displacement, ctx.stride1, ctx.stride2,
                                   ctx.corr_multiply)
        return (g1, g2) + (None,) * 6


# ---------------------------------------------------------------------------------------
# CostVolumeLayer (modules.py:45-74)
# ---------------------------------------------------------------------------------------
def cost_volume_forward(src, tgt, search_range):
    _check_inputs("CostVolumeLayer", src, tgt)
    if src.shape != tgt.shape:
        raise ValueError("CostVolumeLayer: src/tgt shapes differ")
    src, tgt = src.contiguous(), tgt.contiguous()
    B, C, H, W = src.shape
    K = (2 * search_range + 1) ** 2
    out = torch.empty((B, K, H, W), dtype=src.dtype, device=src.device)
    if out.numel() == 0:
        return out
    lib = _lib.load()
    nws = lib.pwc_cost_volume_workspace_size(B, C, H, W, search_range)
    ws, wsp = _workspace(nws, src.device)
    _lib.check(lib.pwc_cost_volume_forward_ws(
        _ptr(src), _ptr(tgt), _ptr(out), B, C, H, W, search_range, _lib.DTYPE_CODES[src.dtype],
        wsp, nws, _stream(src.device)), "CostVolumeLayer_forward")
    del ws
    return out


def cost_volume_backward(src, tgt, grad_output, search_range):
    _check_inputs("CostVolumeLayer backward", src, tgt, grad_output)
    B, C, H, W = src.shape
    grad_output = grad_output.contiguous()
    gs = torch.empty_like(src)
    gt = torch.empty_like(tgt)
    if gs.numel() == 0:
        return gs, gt
    _lib.check(_lib.load().pwc_cost_volume_backward(
        _ptr(src), _ptr(tgt), _ptr(grad_output), _ptr(gs), _ptr(gt), B, C, H, W, search_range,
        _lib.DTYPE_CODES[src.dtype], _stream(src.device)), "CostVolumeLayer_backward")
    return gs, gt


class CostVolumeFunction(Function):
    @staticmethod
    def forward(ctx, src, tgt, search_range):
        src, tgt = src.contiguous(), tgt.contiguous()
        ctx.save_for_backward(src, tgt)
        ctx.search_range = search_range
        with torch.cuda.device(src.device) if src.is_cuda else _nullctx():
            return cost_volume_forward(src, tgt, search_range)

    @staticmethod
    def backward(ctx, grad_output):
        src, tgt = ctx.saved_tensors
        with torch.cuda.device(src.device):
            gs, gt = cost_volume_backward(src, tgt, grad_output, ctx.search_range)
        return gs, gt, None


# ---------------------------------------------------------------------------------------
# WarpingLayer (modules.py:25-42)
# ---------------------------------------------------------------------------------------
def warp_forward(x, flow):
    _check_inputs("WarpingLayer", x, flow)
    B, C, H, W = x.shape
    if tuple(flow.shape) != (B, 2, H, W):
        raise ValueError(f"WarpingLayer: flow shape {tuple(flow.shape)} != {(B, 2, H, W)}")
    x, flow = x.contiguous(), flow.contiguous()
    out = torch.empty_like(x)
    if out.numel() == 0:
        return out
    _lib.check(_lib.load().pwc_warp_forward(_ptr(x), _ptr(flow), _ptr(out), B, C, H, W,
                                            _lib.DTYPE_CODES[x.dtype], _stream(x.device)),
               "WarpingLayer_forward")
    return out


def warp_forward_group(problems):
    """[x2_warp] for a list of INDEPENDENT (x, flow) problems -- ``warp_forward`` each, bit
    for bit, in one launch per 4 problems (pwc_warp_forward_group).  Inside one model forward
    each level's warp needs the previous level's flow, so those levels are not a group."""
    if not problems:
        return []
    items, dt = [], None
    for (x, flow) in problems:
        _check_inputs("WarpingLayer", x, flow)
        B, C, H, W = x.shape
        if tuple(flow.shape) != (B, 2, H, W):
            raise ValueError(f"WarpingLayer: flow shape {tuple(flow.shape)} != {(B, 2, H, W)}")
        if x.device != problems[0][0].device:
            raise ValueError("WarpingLayer group: problems on different devices")
        code = _lib.DTYPE_CODES[x.dtype]
        if dt is not None and code != dt:
            raise ValueError("WarpingLayer group: problems of different dtypes")
        dt = code
        _i32(B, C, H, W, x.numel())
        x, flow = x.contiguous(), flow.contiguous()
        items.append((x, flow, torch.empty_like(x)))
    arr = (_lib.WarpProblem * len(items))()
    for i, (x, f, o) in enumerate(items):
        B, C, H, W = x.shape
        arr[i] = _lib.WarpProblem(x.data_ptr(), f.data_ptr(), o.data_ptr(), B, C, H, W)
    _lib.check(_lib.load().pwc_warp_forward_group(arr, len(items), dt,
                                                  _stream(items[0][0].device)),
               "WarpingLayer_forward_group")
    return [o for (_, _, o) in items]


def corr_forward_group(problems, pad_size, kernel_size, max_displacement, stride1, stride2,
                       corr_multiply=1):
    """[corr] for a list of INDEPENDENT (input1, input2) problems -- ``corr_forward`` each,
    bit for bit; fp32 problems of model.py:24's configuration that take the row-band kernel
    (l2 + l3 at 384x448) are paired into one launch (pwc_corr_forward_group)."""
    if not problems:
        return []
    items, dt = [], None
    for (input1, input2) in problems:
        _check_inputs("Correlation", input1, input2)
        if input1.shape != input2.shape:
            raise ValueError(f"Correlation: input shapes differ {tuple(input1.shape)} vs "
                             f"{tuple(input2.shape)}")
        if input1.device != problems[0][0].device:
            raise ValueError("Correlation group: problems on different devices")
        code = _lib.DTYPE_CODES[input1.dtype]
        if dt is not None and code != dt:
            raise ValueError("Correlation group: problems of different dtypes")
        dt = code
        B, C, H, W = input1.shape
        _i32(B, C, H, W, input1.numel())
        input1, input2 = input1.contiguous(), input2.contiguous()
        OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement,
                                            stride1, stride2)
        out = torch.empty((B, OC, Ho, Wo), dtype=input1.dtype, device=input1.device)
        items.append((input1, input2, out))
    arr = (_lib.CorrProblem * len(items))()
    for i, (a, b, o) in enumerate(items):
        B, C, H, W = a.shape
        arr[i] = _lib.CorrProblem(a.data_ptr(), b.data_ptr(), o.data_ptr(), B, C, H, W)
    _lib.check(_lib.load().pwc_corr_forward_group(
        arr, len(items), pad_size, kernel_size, max_displacement, stride1, stride2,
        corr_multiply, dt, _stream(items[0][0].device)), "Correlation_forward_group")
    return [o for (_, _, o) in items]


def warp_backward(x, flow, grad_output):
    _check_inputs("WarpingLayer backward", x, flow, grad_output, dtypes=(torch.float32,))
    B, C, H, W = x.shape
    grad_output = grad_output.contiguous()
    gx = torch.empty_like(x)
    gf = torch.empty_like(flow)
    if gf.numel() == 0:
        return gx, gf
    lib = _lib.load()
    nws = lib.pwc_warp_backward_workspace_size(B, C, H, W, 0)
    ws, wsp = _workspace(nws, x.device)
    _lib.check(lib.pwc_warp_backward_ws(_ptr(x), _ptr(flow), _ptr(grad_output), _ptr(gx),
                                        _ptr(gf), B, C, H, W, 0, wsp, nws, _stream(x.device)),
               "WarpingLayer_backward")
    del ws
    return gx, gf


class WarpFunction(Function):
    @staticmethod
    def forward(ctx, x, flow):
        x, flow = x.contiguous(), flow.contiguous()
        ctx.save_for_backward(x, flow)
        with torch.cuda.device(x.device) if x.is_cuda else _nullctx():
            return warp_forward(x, flow)

    @staticmethod
    def backward(ctx, grad_output):
        x, flow = ctx.saved_tensors
        with torch.cuda.device(x.device):
            gx, gf = warp_backward(x, flow, grad_output)
        return gx, gf


# ---------------------------------------------------------------------------------------
# model.py:78 + :80: flow upsample (x2, bilinear, * 2) then warp, fused
# ---------------------------------------------------------------------------------------
def upsample_warp_forward(x2, flow_coarse, emit_flow=True):
    """(x2_warp, flow_up) with flow_up = F.upsample(flow_coarse, scale_factor=2,
    mode='bilinear') * 2 (torch 0.4: align_corners=False) and x2_warp = WarpingLayer(x2,
    flow_up): model.py:78 + :80 as one kernel launch.  ``emit_flow=False`` skips writing
    flow_up (returned as None)."""
    _check_inputs("UpsampleWarp", x2, flow_coarse)
    B, C, H, W = x2.shape
    if tuple(flow_coarse.shape) != (B, 2, H // 2, W // 2) or H % 2 or W % 2:
        raise ValueError(f"UpsampleWarp: flow shape {tuple(flow_coarse.shape)} is not "
                         f"{(B, 2, H // 2, W // 2)} (x2 {tuple(x2.shape)} must be 2x it)")
    if flow_coarse.dtype != x2.dtype:
        raise TypeError("UpsampleWarp: x2 and flow must share a dtype")
    _i32(B, C, H, W, x2.numel(), B * 2 * H * W)
    x2, flow_coarse = x2.contiguous(), flow_coarse.contiguous()
    out = torch.empty_like(x2)
    fup = torch.empty(B, 2, H, W, device=x2.device, dtype=x2.dtype) if emit_flow else None
    if B * H * W == 0:
        return out, fup
    _lib.check(_lib.load().pwc_upsample_warp_forward(
        _ptr(x2), _ptr(flow_coarse), _ptr(fup) if fup is not None else None, _ptr(out), B, C,
        H, W, _lib.DTYPE_CODES[x2.dtype], _stream(x2.device)), "UpsampleWarp_forward")
    return out, fup


def flow_upsample_backward(grad_flow_up):
    """Adjoint of model.py:78 (fp32): grad of the coarse flow from grad of flow_up."""
    _check_inputs("UpsampleWarp backward", grad_flow_up, dtypes=(torch.float32,))
    B, two, H, W = grad_flow_up.shape
    if two != 2 or H % 2 or W % 2:
        raise ValueError(f"flow upsample backward: bad shape {tuple(grad_flow_up.shape)}")
    grad_flow_up = grad_flow_up.contiguous()
    gc = torch.empty(B, 2, H // 2, W // 2, device=grad_flow_up.device, dtype=torch.float32)
    if gc.numel() == 0:
        return gc
    _lib.check(_lib.load().pwc_flow_upsample_backward(_ptr(grad_flow_up), _ptr(gc), B, H, W, 0,
                                                      _stream(grad_flow_up.device)),
               "UpsampleWarp_backward")
    return gc


class UpsampleWarpFunction(Function):
    @staticmethod
    def forward(ctx, x2, flow_coarse):
        x2, flow_coarse = x2.contiguous(), flow_coarse.contiguous()
        with torch.cuda.device(x2.device):
            out, fup = upsample_warp_forward(x2, flow_coarse)
        ctx.save_for_backward(x2, fup)
        return out, fup

    @staticmethod
    def backward(ctx, grad_out, grad_fup):
        x2, fup = ctx.saved_tensors
        with torch.cuda.device(x2.device):
            gx2, gflow = (warp_backward(x2, fup, grad_out) if grad_out is not None
                          else (None, torch.zeros_like(fup)))
            if grad_fup is not None:
                gflow = gflow + grad_fup
            gcoarse = flow_upsample_backward(gflow)
        return gx2, gcoarse


# ---------------------------------------------------------------------------------------
# one pyramid level of model.py:80-83: warp then correlation, fused
# ---------------------------------------------------------------------------------------
def warp_corr_forward(input1, x2, flow, pad_size, kernel_size, max_displacement, stride1,
                      stride2, corr_multiply=1, emit_warp=True):
    """(corr, x2_warp) = (Correlation(input1, WarpingLayer(x2, flow)), WarpingLayer(x2, flow)).

    Same values as ``warp_forward`` followed by ``corr_forward`` (x2_warp bit-identical); for
    model.py:24's configuration in fp32 the pair runs as one kernel launch per level.
    ``emit_warp=False`` skips writing x2_warp (returned as None)."""
    _check_inputs("WarpCorrelation", input1, x2, flow)
    if input1.shape != x2.shape:
        raise ValueError(f"WarpCorrelation: input shapes differ {tuple(input1.shape)} vs "
                         f"{tuple(x2.shape)}")
    B, C, H, W = input1.shape
    if tuple(flow.shape) != (B, 2, H, W):
        raise ValueError(f"WarpCorrelation: flow shape {tuple(flow.shape)} != {(B, 2, H, W)}")
    _i32(B, C, H, W, input1.numel())
    input1, x2, flow = input1.contiguous(), x2.contiguous(), flow.contiguous()
    OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement, stride1,
                                        stride2)
    out = torch.empty((B, OC, Ho, Wo), dtype=input1.dtype, device=input1.device)
    x2w = torch.empty_like(x2) if emit_warp else None
    if out.numel() == 0:
        return out, x2w
    lib = _lib.load()
    dt = _lib.DTYPE_CODES[input1.dtype]
    nws = lib.pwc_warp_corr_workspace_size(B, C, H, W, pad_size, kernel_size, max_displacement,
                                           stride1, stride2, dt, int(emit_warp))
    ws, wsp = _workspace(nws, input1.device)
    _lib.check(lib.pwc_warp_corr_forward(
        _ptr(input1), _ptr(x2), _ptr(flow), _ptr(x2w) if emit_warp else ctypes.c_void_p(0),
        _ptr(out), B, C, H, W, pad_size, kernel_size, max_displacement, stride1, stride2,
        corr_multiply, dt, wsp, nws, _stream(input1.device)), "WarpCorrelation_forward")
    del ws
    return out, x2w


def warp_corr_forward_group(problems, pad_size, kernel_size, max_displacement, stride1,
                            stride2, corr_multiply=1):
    """[(corr, x2_warp)] for a list of INDEPENDENT (input1, x2, flow) problems -- one
    ``warp_corr_forward`` each, bit for bit, but problems that take the fused band kernel are
    paired into one launch whose two grids share the CUs (pwc_warp_corr_forward_group).  Inside
    one model forward the pyramid levels depend on each other and are not a group."""
    if not problems:
        return []
    items, outs = [], []
    dt = None
    for (input1, x2, flow) in problems:
        _check_inputs("WarpCorrelation", input1, x2, flow)
        if input1.shape != x2.shape:
            raise ValueError(f"WarpCorrelation: input shapes differ {tuple(input1.shape)} vs "
                             f"{tuple(x2.shape)}")
        B, C, H, W = input1.shape
        if tuple(flow.shape) != (B, 2, H, W):
            raise ValueError(f"WarpCorrelation: flow shape {tuple(flow.shape)} != "
                             f"{(B, 2, H, W)}")
        if input1.device != problems[0][0].device:
            raise ValueError("WarpCorrelation group: problems on different devices")
        code = _lib.DTYPE_CODES[input1.dtype]
        if dt is not None and code != dt:
            raise ValueError("WarpCorrelation group: problems of different dtypes")
        dt = code
        _i32(B, C, H, W, input1.numel())
        input1, x2, flow = input1.contiguous(), x2.contiguous(), flow.contiguous()
        OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement,
                                            stride1, stride2)
        out = torch.empty((B, OC, Ho, Wo), dtype=input1.dtype, device=input1.device)
        x2w = torch.empty_like(x2)
        items.append((input1, x2, flow, x2w, out))
        outs.append((out, x2w))
    arr = (_lib.WarpCorrProblem * len(items))()
    for i, (a, b, f, w, o) in enumerate(items):
        B, C, H, W = a.shape
        arr[i] = _lib.WarpCorrProblem(a.data_ptr(), b.data_ptr(), f.data_ptr(), w.data_ptr(),
                                      o.data_ptr(), B, C, H, W)
    dev = items[0][0].device
    _lib.check(_lib.load().pwc_warp_corr_forward_group(
        arr, len(items), pad_size, kernel_size, max_displacement, stride1, stride2,
        corr_multiply, dt, _stream(dev)), "WarpCorrelation_forward_group")
    return outs


# Arrival counters of the one-launch level backward (pwc_warp_corr_backward): B uint32 per
# device, zeroed once here (outside any graph capture, so captured replays reuse them); every
# call leaves them zero.  One set per device: level backwards of one device must not run
# concurrently on two streams (autograd runs a device's backward on one stream).
_COUNTERS = {}


def _counters(B, device):
    c = _COUNTERS.get(device)
    if c is None or c.numel() < B:
        if torch.cuda.is_current_stream_capturing():
            return None  # not allocated inside a capture: the two-launch path runs instead
        c = torch.zeros(max(B, 64), dtype=torch.int32, device=device)
        _COUNTERS[device] = c
    return c


def warp_corr_backward(input1, x2, flow, x2_warp, grad_corr, pad_size, kernel_size,
                       max_displacement, stride1, stride2, corr_multiply=1, grad_x2_warp=None):
    """(grad_input1, grad_x2, grad_flow): the backward of ``warp_corr_forward`` --
    ``corr_backward(input1, x2_warp, grad_corr)`` then ``warp_backward(x2, flow, d/dx2_warp +
    grad_x2_warp)`` -- as one C call (pwc_warp_corr_backward; one kernel at the coarse levels of
    model.py:24's configuration, where d/dx2_warp never leaves LDS)."""
    _check_inputs("WarpCorrelation backward", input1, x2, flow, x2_warp, grad_corr,
                  dtypes=(torch.float32,))
    B, C, H, W = input1.shape
    if tuple(x2.shape) != (B, C, H, W) or tuple(x2_warp.shape) != (B, C, H, W):
        raise ValueError("WarpCorrelation backward: input shapes differ")
    if tuple(flow.shape) != (B, 2, H, W):
        raise ValueError(f"WarpCorrelation backward: flow shape {tuple(flow.shape)} != "
                         f"{(B, 2, H, W)}")
    OC, Ho, Wo = _lib.corr_output_shape(H, W, pad_size, kernel_size, max_displacement, stride1,
                                        stride2)
    if tuple(grad_corr.shape) != (B, OC, Ho, Wo):
        raise ValueError(f"WarpCorrelation backward: grad shape {tuple(grad_corr.shape)} != "
                         f"{(B, OC, Ho, Wo)}")
    if grad_x2_warp is not None:
        _check_inputs("WarpCorrelation backward", grad_x2_warp, dtypes=(torch.float32,))
        if tuple(grad_x2_warp.shape) != (B, C, H, W):
            raise ValueError("WarpCorrelation backward: grad_x2_warp shape differs")
        grad_x2_warp = grad_x2_warp.contiguous()
    _i32(B, C, H, W, input1.numel())
    input1, x2, flow = input1.contiguous(), x2.contiguous(), flow.contiguous()
    x2_warp, grad_corr = x2_warp.contiguous(), grad_corr.contiguous()
    g1 = torch.empty_like(input1)
    gx2 = torch.empty_like(x2)
    gfl = torch.empty_like(flow)
    if gfl.numel() == 0:
        return g1, gx2, gfl
    lib = _lib.load()
    nws = lib.pwc_warp_corr_backward_workspace_size(B, C, H, W, pad_size, kernel_size,
                                                    max_displacement, stride1, stride2, 0)
    ws, wsp = _workspace(nws, input1.device)
    cnt = _counters(B, input1.device)
    _lib.check(lib.pwc_warp_corr_backward(
        _ptr(input1), _ptr(x2), _ptr(flow), _ptr(x2_warp), _ptr(grad_corr),
        _ptr(grad_x2_warp) if grad_x2_warp is not None else ctypes.c_void_p(0),
        _ptr(g1), _ptr(gx2), _ptr(gfl), B, C, H, W, pad_size, kernel_size, max_displacement,
        stride1, stride2, corr_multiply, 0, wsp, nws,
        _ptr(cnt) if cnt is not None else ctypes.c_void_p(0), _stream(input1.device)),
        "WarpCorrelation_backward")
    del ws
    return g1, gx2, gfl


class WarpCorrelationFunction(Function):
    """autograd for model.py:80-83 as one op: outputs (corr, x2_warp).  Backward chains the
    reference's two backward passes -- correlation (cu:108-290) into the warped features, plus
    any gradient arriving on x2_warp itself, then grid_sample's -- as warp_corr_backward (one
    launch at the coarse levels)."""

    @staticmethod
    def forward(ctx, input1, x2, flow, pad_size=9, kernel_size=1, max_displacement=9,
                stride1=1, stride2=2, corr_multiply=1):
        with torch.cuda.device(input1.device) if input1.is_cuda else _nullctx():
            out, x2w = warp_corr_forward(input1, x2, flow, pad_size, kernel_size,
                                         max_displacement, stride1, stride2, corr_multiply)
        ctx.save_for_backward(input1, x2.contiguous(), flow.contiguous(), x2w)
        ctx.args = (pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply)
        return out, x2w

    @staticmethod
    def backward(ctx, grad_corr, grad_x2w):
        input1, x2, flow, x2w = ctx.saved_tensors
        with torch.cuda.device(input1.device):
            # unused outputs arrive as zeros (autograd materialises them); fp16 / bf16 storage
            # has no backward kernels (as corr_backward / warp_backward)
            g1, gx2, gflow = warp_corr_backward(input1, x2, flow, x2w, grad_corr, *ctx.args,
                                                grad_x2_warp=grad_x2w)
        return (g1, gx2, gflow) + (None,) * 6


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
