"""nn.Module drop-ins for the reference's hot-path layers.

* ``Correlation``     — correlation_package/modules/correlation.py:6-27 (same ctor, no params)
* ``WarpingLayer``    — modules.py:25-42 (ctor takes the reference's ``args`` namespace)
* ``CostVolumeLayer`` — modules.py:45-74 (ctor reads ``args.search_range``)
* ``WarpCorrelation`` — model.py:80-83 (warp, then correlation) as one module / one launch
* ``get_grid``        — utils.py:3-8 (host-built normalised base grid, for API completeness;
  the HIP warp recomputes it in registers and never calls this)
"""
from __future__ import annotations

import torch
from torch import nn

from . import library as _library  # registers torch.ops.pwcnet.* (traceable single nodes)
from .ops import (CorrelationCatFunction, UpsampleWarpFunction, WarpCorrelationFunction)


class Correlation(nn.Module):
    """``Correlation(pad_size, kernel_size, max_displacement, stride1, stride2, corr_multiply)``.

    ``forward(input1, input2)`` -> B x ((md/s2)*2+1)^2 x Ho x Wo, values of
    correlation_cuda_kernel.cu:34-106 (divided by kernel_size^2 * C).  model.py:24 builds it
    as Correlation(pad_size=9, kernel_size=1, max_displacement=9, stride1=1, stride2=2).
    """

    def __init__(self, pad_size=0, kernel_size=0, max_displacement=0, stride1=1, stride2=2,
                 corr_multiply=1):
        super().__init__()
        self.pad_size = pad_size
        self.kernel_size = kernel_size
        self.max_displacement = max_displacement
        self.stride1 = stride1
        self.stride2 = stride2
        self.corr_multiply = corr_multiply

    def forward(self, input1, input2):
        # functions/correlation.py:17-18 asserts contiguity; the op (torch.ops.pwcnet.
        # correlation, autograd registered) is CorrelationFunction's traceable twin
        assert input1.is_contiguous()
        assert input2.is_contiguous()
        return _library.correlation(input1, input2, self.pad_size, self.kernel_size,
                                    self.max_displacement, self.stride1, self.stride2,
                                    self.corr_multiply)

    def extra_repr(self):
        return (f"pad_size={self.pad_size}, kernel_size={self.kernel_size}, "
                f"max_displacement={self.max_displacement}, stride1={self.stride1}, "
                f"stride2={self.stride2}")


class WarpingLayer(nn.Module):
    """Backward-warp ``x`` by ``flow`` (pixels; channel 0 horizontal, 1 vertical).

    Matches modules.py:31-42 under the reference's pinned torch 0.4 (grid_sample bilinear,
    zeros padding, align_corners=True).  ``args`` is kept for signature parity; the device is
    taken from the inputs.
    """

    def __init__(self, args=None):
        super().__init__()
        self.args = args

    def forward(self, x, flow):
        return _library.warp(x, flow)


class WarpCorrelation(nn.Module):
    """One pyramid level of model.py:80-83 in one call:

        x2_warp = self.warping_layer(x2, flow)      # model.py:80
        corr = self.corr(x1, x2_warp)               # model.py:83
    becomes
        corr, x2_warp = self.warp_corr(x1, x2, flow)

    Same ctor as ``Correlation`` (model.py:24's values by default).  Values equal the two
    reference layers applied in sequence; gradients flow to x1, x2 and flow.
    """

    def __init__(self, pad_size=9, kernel_size=1, max_displacement=9, stride1=1, stride2=2,
                 corr_multiply=1):
        super().__init__()
        self.pad_size = pad_size
        self.kernel_size = kernel_size
        self.max_displacement = max_displacement
        self.stride1 = stride1
        self.stride2 = stride2
        self.corr_multiply = corr_multiply

    def forward(self, x1, x2, flow):
        return WarpCorrelationFunction.apply(x1, x2, flow, self.pad_size, self.kernel_size,
                                             self.max_displacement, self.stride1, self.stride2,
                                             self.corr_multiply)


class CorrelationCat(nn.Module):
    """model.py:83-91 in one call:

        corr = self.corr(x1, x2_warp)                                  # model.py:83
        if args.corr_activation: F.leaky_relu_(corr)                   # model.py:84
        ... torch.cat([x1, corr, flow], dim = 1) ...                   # model.py:89/91
    becomes
        inp = self.corr_cat(x1, x2_warp, flow)

    The correlation kernels write straight into the concatenated buffer's corr channels
    (with the leaky_relu fused when ``corr_activation``); ctor as ``Correlation``."""

    def __init__(self, pad_size=9, kernel_size=1, max_displacement=9, stride1=1, stride2=2,
                 corr_multiply=1, corr_activation=False, negative_slope=0.01):
        super().__init__()
        self.params = (pad_size, kernel_size, max_displacement, stride1, stride2)
        self.negative_slope = negative_slope if corr_activation else None

    def forward(self, x1, x2_warp, flow):
        return CorrelationCatFunction.apply(x1, x2_warp, flow, *self.params,
                                            self.negative_slope)


class UpsampleWarp(nn.Module):
    """model.py:78 + :80 in one call:

        flow = F.upsample(flow, scale_factor=2, mode='bilinear') * 2     # model.py:78
        x2_warp = self.warping_layer(x2, flow)                            # model.py:80
    becomes
        x2_warp, flow = self.upsample_warp(x2, flow)

    torch 0.4's bilinear upsample (align_corners=False) and the WarpingLayer chain
    (align_corners=True grid_sample); gradients flow to x2 and the coarse flow.
    """

    def forward(self, x2, flow_coarse):
        return UpsampleWarpFunction.apply(x2, flow_coarse)


class CostVolumeLayer(nn.Module):
    """modules.py:45-74: (2*search_range+1)^2 channels in the reference's order, / K."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.search_range = args.search_range

    def forward(self, src, tgt):
        return _library.cost_volume(src, tgt, self.search_range)


def get_grid(x: torch.Tensor) -> torch.Tensor:
    """utils.py:3-8: B x 2 x H x W grid of linspace(-1, 1) (x then y)."""
    B, _, H, W = x.shape
    horiz = torch.linspace(-1.0, 1.0, W).view(1, 1, 1, W).expand(B, 1, H, W)
    vert = torch.linspace(-1.0, 1.0, H).view(1, 1, H, 1).expand(B, 1, H, W)
    return torch.cat([horiz, vert], 1)
