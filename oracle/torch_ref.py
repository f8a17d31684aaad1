"""Pure-PyTorch (CPU) restatement of the reference's hot path — TEST INFRASTRUCTURE ONLY.

This is the reference's own CPU path (no correlation_package: ATen ops only), restated so
it can run where /root/reference does not exist (the GPU box):

* ``get_grid``      <- utils.py:3-8 (linspace grids, concatenated [horizontal, vertical])
* ``warp``          <- WarpingLayer.forward, modules.py:31-42 (flow / ((W-1)/2), grid_sample
                       with torch-0.4 semantics: bilinear, zeros, align_corners=True)
* ``cost_volume``   <- CostVolumeLayer.forward, modules.py:53-74 (81 shifted products summed
                       over channels, the reference's channel order, / (2 sr + 1)^2)
* ``correlation``   <- correlation_cuda_kernel.cu:34-106 for kernel_size 1, stride1 1 (the
                       GPU Correlation of model.py:24 and Corr4): shifted products / C
* ``upsample_flow`` <- model.py:78 (F.upsample(flow, scale_factor=2, mode='bilinear') * 2,
                       torch-0.4 default align_corners=False)

Pinned directly by tests/test_torch_ref_golden.py against every fixture gen_golden.py produced
from the reference's modules.py (cost_volume and warp forward + autograd backward, correlation
through the CVL identities, upsample_flow + warp), and end to end by tests/test_net_harness.py
(the reduced model.py Net).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
(and bench.py's explicit ``--device cpu`` launcher rehearsal) use it; the product path
(pwc-net_pytorch_amd/) never imports anything under oracle/.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def get_grid(x: torch.Tensor) -> torch.Tensor:
    """utils.py:3-8: (B, 2, H, W) of [linspace(-1,1,W)[x], linspace(-1,1,H)[y]]."""
    B, _, H, W = x.shape
    gx = torch.linspace(-1.0, 1.0, W, dtype=x.dtype).view(1, 1, 1, W).expand(B, 1, H, W)
    gy = torch.linspace(-1.0, 1.0, H, dtype=x.dtype).view(1, 1, H, 1).expand(B, 1, H, W)
    return torch.cat([gx, gy], 1)


def warp(x: torch.Tensor, flow: torch.Tensor) -> torch.Tensor:
    """modules.py:31-42 (pixel-unit flow -> normalised grid -> bilinear grid_sample)."""
    H, W = flow.shape[2], flow.shape[3]
    norm = torch.empty_like(flow)
    norm[:, 0] = flow[:, 0] / ((W - 1.0) / 2.0)
    norm[:, 1] = flow[:, 1] / ((H - 1.0) / 2.0)
    grid = (get_grid(x).to(x.device) + norm).permute(0, 2, 3, 1)
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def cvl_offsets(sr: int):
    """(dy, dx) of CostVolumeLayer's output channels in order (modules.py:58-72): channel k
    holds src[y, x] * tgt[y + dy, x + dx]."""
    offs = [(0, 0)]
    for i in range(1, sr + 1):
        offs += [(-i, 0), (i, 0), (0, -i), (0, i)]
        for j in range(1, sr + 1):
            offs += [(-i, -j), (i, j), (-i, j), (i, -j)]
    return offs


def _shifted_products(src, tgt, offsets, divisor):
    """out[:, k] = sum_c src * tgt shifted by offsets[k] (zeros outside) / divisor."""
    B, C, H, W = src.shape
    m = max(max(abs(dy), abs(dx)) for dy, dx in offsets)
    tp = F.pad(tgt, (m, m, m, m))
    out = src.new_empty((B, len(offsets), H, W))
    for k, (dy, dx) in enumerate(offsets):
        out[:, k] = (src * tp[:, :, m + dy:m + dy + H, m + dx:m + dx + W]).sum(1)
    return out / divisor


def cost_volume(src: torch.Tensor, tgt: torch.Tensor, sr: int = 4) -> torch.Tensor:
    """CostVolumeLayer(search_range=sr).forward (modules.py:53-74)."""
    return _shifted_products(src, tgt, cvl_offsets(sr), float((2 * sr + 1) ** 2))


def correlation(f1: torch.Tensor, f2: torch.Tensor, pad_size=9, kernel_size=1,
                max_displacement=9, stride1=1, stride2=2) -> torch.Tensor:
    """Correlation(pad, 1, md, 1, s2) of correlation_cuda_kernel.cu:34-106: channel
    (tj + dr) * D + (ti + dr) holds sum_c f1[y + off, x + off] * f2[y + off + tj s2,
    x + off + ti s2] / C, off = md - pad, zeros outside the image (cu:65,98-100)."""
    if kernel_size != 1 or stride1 != 1 or max_displacement != pad_size:
        raise NotImplementedError("torch_ref.correlation: k=1, s1=1, pad=md only")
    dr = max_displacement // stride2
    offsets = [(tj * stride2, ti * stride2) for tj in range(-dr, dr + 1)
               for ti in range(-dr, dr + 1)]
    return _shifted_products(f1, f2, offsets, float(f1.shape[1]))


def upsample_flow(flow: torch.Tensor) -> torch.Tensor:
    """model.py:78 with torch-0.4 semantics (align_corners=False)."""
    return F.interpolate(flow, scale_factor=2, mode="bilinear", align_corners=False) * 2


class RefWarpingLayer(torch.nn.Module):
    """nn.Module form of ``warp`` (drop-in for modules.WarpingLayer on CPU)."""

    def forward(self, x, flow):
        return warp(x, flow)


class RefCostVolumeLayer(torch.nn.Module):
    """nn.Module form of ``cost_volume`` (drop-in for modules.CostVolumeLayer on CPU)."""

    def __init__(self, search_range=4):
        super().__init__()
        self.search_range = search_range

    def forward(self, src, tgt):
        return cost_volume(src, tgt, self.search_range)


def reference_cpu_net(seed=0):
    """model.py's Net on the reference's CPU path (corr = CostVolumeLayer): the harness
    (pwcnet_amd/net.py, same module tree and init as model.py:11-46) with its hot-path layers
    swapped for this module's restatements; run it with ``fused=False``."""
    from pwcnet_amd.net import Net, NetArgs
    torch.manual_seed(seed)
    net = Net(NetArgs(corr="CostVolumeLayer", device="cpu"))
    net.warping_layer = RefWarpingLayer()
    net.corr = RefCostVolumeLayer(4)
    return net.eval()
