"""PWC-Net harness: model.py's ``Net`` driving the MI355X hot path through the drop-ins.

The conv networks (feature pyramid, flow estimators, context network) are plain PyTorch
(MIOpen on the GPU) and out of this project's scope; they are restated here with the
reference's module tree -- same submodule names, same construction order and the same init
loop (model.py:39-46) -- so a state_dict of the reference loads unchanged and the same
``torch.manual_seed`` yields the same weights.  What this module exists for is the per-level
loop of model.py:72-113, where the hot path runs:

    flow = F.upsample(flow, scale_factor=2, mode='bilinear') * 2     # model.py:78
    x2_warp = self.warping_layer(x2, flow)                            # model.py:80
    corr = self.corr(x1, x2_warp)                                     # model.py:83
    if args.corr_activation: F.leaky_relu_(corr)                      # model.py:84
    ... self.flow_estimators[l](torch.cat([x1, corr, flow], dim=1))  # model.py:89/91

``fused=False`` runs exactly those calls through the drop-in modules (WarpingLayer,
Correlation / CostVolumeLayer).  ``fused=True`` (default) runs the same values through the
fused forms: ``UpsampleWarp`` (model.py:78 + :80 in one launch) and, for the GPU
Correlation, ``CorrelationCat`` (model.py:83-91: the correlation written into the cat
buffer, leaky_relu fused).  Returns ``(flows, summaries)`` as model.py does.

Reference: model.py:11-115, modules.py:11-22 (conv), :77-99 (FeaturePyramidExtractor),
:102-128 (OpticalFlowEstimator), :131-160 (ContextNetwork); defaults main.py:42-81.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.nn.functional as F
from torch import nn

from .layers import (Correlation, CorrelationCat, CostVolumeLayer, UpsampleWarp,
                     WarpingLayer)


@dataclass
class NetArgs:
    """The reference's argparse defaults that Net reads (main.py:42-81)."""
    search_range: int = 4
    num_levels: int = 7
    lv_chs: list = field(default_factory=lambda: [16, 32, 64, 96, 128, 192])
    output_level: int = 4
    batch_norm: bool = False
    input_norm: bool = False
    rgb_max: float = 255.0
    residual: bool = False
    flow_norm: bool = False
    corr: str = "cost_volume"        # anything but 'CostVolumeLayer' -> Correlation (model.py:21)
    corr_activation: bool = False
    device: str = "cuda"


def conv(batch_norm, in_planes, out_planes, kernel_size=3, stride=1):
    """modules.py:11-22."""
    layers = [nn.Conv2d(in_planes, out_planes, kernel_size=kernel_size, stride=stride,
                        padding=(kernel_size - 1) // 2, bias=not batch_norm)]
    if batch_norm:
        layers.append(nn.BatchNorm2d(out_planes))
    layers.append(nn.LeakyReLU(0.1, inplace=True))
    return nn.Sequential(*layers)


class FeaturePyramidExtractor(nn.Module):
    """modules.py:77-99: num_levels-1 stride-2 stages; returns coarsest first."""

    def __init__(self, args):
        super().__init__()
        self.convs = []
        for l in range(args.num_levels - 1):
            layer = nn.Sequential(
                conv(args.batch_norm, 3 if l == 0 else args.lv_chs[l - 1], args.lv_chs[l],
                     stride=2),
                conv(args.batch_norm, args.lv_chs[l], args.lv_chs[l]))
            self.add_module(f"Feature(Lv{l + 1})", layer)
            self.convs.append(layer)

    def forward(self, x):
        pyramid = []
        for c in self.convs:
            x = c(x)
            pyramid.append(x)
        return pyramid[::-1]


class OpticalFlowEstimator(nn.Module):
    """modules.py:102-128."""

    def __init__(self, args, ch_in):
        super().__init__()
        self.args = args
        bn = args.batch_norm
        self.convs = nn.Sequential(conv(bn, ch_in, 128), conv(bn, 128, 128), conv(bn, 128, 96),
                                   conv(bn, 96, 64), conv(bn, 64, 32),
                                   nn.Conv2d(32, 2, kernel_size=3, stride=1, padding=1))

    def forward(self, x):
        if not self.args.flow_norm:
            return self.convs(x)
        out = torch.tanh(self.convs(x))
        scale = (x.size(3) - 1.0) / 2.0  # modules.py:123-124 scales both channels by width
        return out * scale


class ContextNetwork(nn.Module):
    """modules.py:131-160: dilated 3x3 stack (dilations 1, 2, 4, 8, 16, 1, 1)."""

    def __init__(self, args, ch_in):
        super().__init__()
        spec = [(ch_in, 128, 1), (128, 128, 2), (128, 128, 4), (128, 96, 8), (96, 64, 16),
                (64, 32, 1)]
        layers = []
        for cin, cout, d in spec:
            layers += [nn.Conv2d(cin, cout, 3, 1, padding=d, dilation=d),
                       nn.LeakyReLU(inplace=True)]
        layers.append(nn.Conv2d(32, 2, 3, 1, padding=1))
        self.convs = nn.Sequential(*layers)

    def forward(self, x):
        return self.convs(x)


class Net(nn.Module):
    """model.py:11-115 with the hot path on the MI355X drop-ins (see module docstring)."""

    def __init__(self, args: NetArgs):
        super().__init__()
        self.args = args
        self.feature_pyramid_extractor = FeaturePyramidExtractor(args)
        self.warping_layer = WarpingLayer(args)
        sr = args.search_range
        if args.corr == "CostVolumeLayer":
            self.corr = CostVolumeLayer(args)
        else:  # model.py:24
            self.corr = Correlation(pad_size=sr * 2 + 1, kernel_size=1,
                                    max_displacement=sr * 2 + 1, stride1=1, stride2=2,
                                    corr_multiply=1)
        self.upsample_warp = UpsampleWarp()
        self.corr_cat = CorrelationCat(pad_size=sr * 2 + 1, kernel_size=1,
                                       max_displacement=sr * 2 + 1, stride1=1, stride2=2,
                                       corr_activation=args.corr_activation)
        self.flow_estimators = []
        for l, ch in enumerate(args.lv_chs[::-1] + [3]):
            layer = OpticalFlowEstimator(args, ch + (sr * 2 + 1) ** 2 + 2)
            self.add_module(f"FlowEstimator(Lv{l})", layer)
            self.flow_estimators.append(layer)
        self.context_network = ContextNetwork(args, 3 + 2)
        # init (model.py:39-46): uniform bias, xavier-uniform weight, module order
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                if m.bias is not None:
                    nn.init.uniform_(m.bias)
                nn.init.xavier_uniform_(m.weight)

    def forward(self, x, fused: bool = True):
        args = self.args
        if args.input_norm:
            mean = x.contiguous().view(x.size()[:2] + (-1,)).mean(dim=-1)
            x = (x - mean.view(x.size()[:2] + (1, 1, 1))) / args.rgb_max
        x1_raw = x[:, :, 0].contiguous()
        x2_raw = x[:, :, 1].contiguous()
        x1_pyr = self.feature_pyramid_extractor(x1_raw) + [x1_raw]
        x2_pyr = self.feature_pyramid_extractor(x2_raw) + [x2_raw]
        cat_fused = fused and isinstance(self.corr, Correlation)

        flows, summaries = [], {"x2_warps": []}
        flow = None
        for l, (x1, x2) in enumerate(zip(x1_pyr, x2_pyr)):
            if l == 0:
                flow = x1.new_zeros((x1.size(0), 2, x1.size(2), x1.size(3)))
                x2_warp = self.warping_layer(x2, flow)                           # :80
            elif fused:
                x2_warp, flow = self.upsample_warp(x2, flow)                     # :78 + :80
            else:
                flow = F.interpolate(flow, scale_factor=2, mode="bilinear",
                                     align_corners=False) * 2                    # :78
                x2_warp = self.warping_layer(x2, flow)                           # :80
            if cat_fused:
                inp = self.corr_cat(x1, x2_warp, flow)                           # :83-91
            else:
                corr = self.corr(x1, x2_warp)                                    # :83
                if args.corr_activation:
                    F.leaky_relu_(corr)                                          # :84
                inp = torch.cat([x1, corr, flow], dim=1)                         # :89/91
            flow_coarse = self.flow_estimators[l](inp)
            if args.residual:
                flow_coarse = flow_coarse + flow
            summaries["x2_warps"].append(x2_warp.detach())
            if l == args.output_level:
                up = 2 ** (args.num_levels - args.output_level - 1)
                flow = F.interpolate(flow_coarse, scale_factor=up, mode="bilinear",
                                     align_corners=False) * up
                flow = flow + self.context_network(torch.cat([x1_pyr[-1], flow], dim=1))
                flows.append(flow)
                break
            flow = flow_coarse
            flows.append(flow)
        return flows, summaries
