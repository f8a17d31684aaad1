"""torch.library registration of the hot-path ops (SURVEY.md §8b "Wrappers").

The reference exposed its CUDA correlation through a cffi extension plus an autograd.Function
(correlation_package/functions/correlation.py:7-56, _ext/correlation/__init__.py:6-15), which
graph capture tools cannot see into.  Here each op is a ``torch.library.custom_op`` in the
``pwcnet`` namespace -- an opaque node with a fake (meta) implementation for shape
propagation and a registered autograd formula -- so ``torch.compile`` / FX / ``torch.export``
trace ``Correlation``, ``WarpingLayer`` and ``CostVolumeLayer`` as single nodes:

    torch.ops.pwcnet.correlation(in1, in2, pad, k, md, s1, s2, mult)   cu:34-106
    torch.ops.pwcnet.correlation_backward(in1, in2, gO, pad, ...)      cu:108-290
    torch.ops.pwcnet.cost_volume(src, tgt, sr) / _backward             modules.py:53-74
    torch.ops.pwcnet.warp(x, flow) / warp_backward                     modules.py:31-42

The real implementations are the HIP kernels behind the C ABI (ops.py); there is no CPU
kernel, so calling these ops on CPU tensors raises, as the reference's CPU stubs did.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import ops as _ops

_NS = "pwcnet"


def _on(t: Tensor):
    """The tensor's HIP device as current device (CPU tensors fall through to ops.py, which
    raises: there is no CPU implementation)."""
    import contextlib
    return torch.cuda.device(t.device) if t.is_cuda else contextlib.nullcontext()


def corr_output_shape(H: int, W: int, pad: int, k: int, md: int, s1: int, s2: int):
    """correlation_cuda.c:20-34 (C semantics: truncating integer division, float ceil)."""
    import math
    kr = int((k - 1) / 2)
    br = kr + md
    dr = md // s2
    D = 2 * dr + 1
    Ho = int(math.ceil((H + 2 * pad - 2 * br) / float(s1)))
    Wo = int(math.ceil((W + 2 * pad - 2 * br) / float(s1)))
    return D * D, max(Ho, 0), max(Wo, 0)


# ---------------------------------------------------------------------------------------
# correlation
# ---------------------------------------------------------------------------------------
@torch.library.custom_op(f"{_NS}::correlation", mutates_args=())
def correlation(input1: Tensor, input2: Tensor, pad_size: int, kernel_size: int,
                max_displacement: int, stride1: int, stride2: int,
                corr_multiply: int) -> Tensor:
    with _on(input1):
        return _ops.corr_forward(input1, input2, pad_size, kernel_size, max_displacement,
                                 stride1, stride2, corr_multiply)


@correlation.register_fake
def _(input1, input2, pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply):
    B, _, H, W = input1.shape
    OC, Ho, Wo = corr_output_shape(H, W, pad_size, kernel_size, max_displacement, stride1,
                                   stride2)
    return input1.new_empty((B, OC, Ho, Wo))


@torch.library.custom_op(f"{_NS}::correlation_backward", mutates_args=())
def correlation_backward(input1: Tensor, input2: Tensor, grad_output: Tensor, pad_size: int,
                         kernel_size: int, max_displacement: int, stride1: int, stride2: int,
                         corr_multiply: int) -> Tuple[Tensor, Tensor]:
    with _on(input1):
        return _ops.corr_backward(input1, input2, grad_output, pad_size, kernel_size,
                                  max_displacement, stride1, stride2, corr_multiply)


@correlation_backward.register_fake
def _(input1, input2, grad_output, *args):
    return torch.empty_like(input1), torch.empty_like(input2)


def _corr_setup(ctx, inputs, output):
    input1, input2, *params = inputs
    ctx.save_for_backward(input1, input2)
    ctx.params = params


def _corr_bwd(ctx, grad):
    input1, input2 = ctx.saved_tensors
    g1, g2 = correlation_backward(input1, input2, grad.contiguous(), *ctx.params)
    return (g1, g2) + (None,) * 6


correlation.register_autograd(_corr_bwd, setup_context=_corr_setup)


# ---------------------------------------------------------------------------------------
# CostVolumeLayer
# ---------------------------------------------------------------------------------------
@torch.library.custom_op(f"{_NS}::cost_volume", mutates_args=())
def cost_volume(src: Tensor, tgt: Tensor, search_range: int) -> Tensor:
    with _on(src):
        return _ops.cost_volume_forward(src, tgt, search_range)


@cost_volume.register_fake
def _(src, tgt, search_range):
    B, _, H, W = src.shape
    return src.new_empty((B, (2 * search_range + 1) ** 2, H, W))


@torch.library.custom_op(f"{_NS}::cost_volume_backward", mutates_args=())
def cost_volume_backward(src: Tensor, tgt: Tensor, grad_output: Tensor,
                         search_range: int) -> Tuple[Tensor, Tensor]:
    with _on(src):
        return _ops.cost_volume_backward(src, tgt, grad_output, search_range)


@cost_volume_backward.register_fake
def _(src, tgt, grad_output, search_range):
    return torch.empty_like(src), torch.empty_like(tgt)


def _cvl_setup(ctx, inputs, output):
    src, tgt, sr = inputs
    ctx.save_for_backward(src, tgt)
    ctx.sr = sr


def _cvl_bwd(ctx, grad):
    src, tgt = ctx.saved_tensors
    gs, gt = cost_volume_backward(src, tgt, grad.contiguous(), ctx.sr)
    return gs, gt, None


cost_volume.register_autograd(_cvl_bwd, setup_context=_cvl_setup)


# ---------------------------------------------------------------------------------------
# WarpingLayer
# ---------------------------------------------------------------------------------------
@torch.library.custom_op(f"{_NS}::warp", mutates_args=())
def warp(x: Tensor, flow: Tensor) -> Tensor:
    with _on(x):
        return _ops.warp_forward(x, flow)


@warp.register_fake
def _(x, flow):
    return torch.empty_like(x)


@torch.library.custom_op(f"{_NS}::warp_backward", mutates_args=())
def warp_backward(x: Tensor, flow: Tensor, grad_output: Tensor) -> Tuple[Tensor, Tensor]:
    with _on(x):
        return _ops.warp_backward(x, flow, grad_output)


@warp_backward.register_fake
def _(x, flow, grad_output):
    return torch.empty_like(x), torch.empty_like(flow)


def _warp_setup(ctx, inputs, output):
    x, flow = inputs
    ctx.save_for_backward(x, flow)


def _warp_bwd(ctx, grad):
    x, flow = ctx.saved_tensors
    gx, gf = warp_backward(x, flow, grad.contiguous())
    return gx, gf


warp.register_autograd(_warp_bwd, setup_context=_warp_setup)
