"""Generate the golden fixtures in tests/golden/ from the reference's own Python code.

Run in the build container (the only place /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

What is imported from the reference (read-only, /root/reference):
  * modules.CostVolumeLayer  (modules.py:45-74)   - pure-PyTorch cost volume
  * modules.WarpingLayer     (modules.py:25-42) + utils.get_grid (utils.py:3-8)

The reference pins torch==0.4.0 (requirements.txt:62) whose F.grid_sample behaved as
align_corners=True; modern torch defaults to False (3.26 max error on an identity warp).
So ``modules.F`` is pointed at a namespace whose ``grid_sample`` passes
``align_corners=True`` explicitly.  Nothing else of the reference is altered.

The reference CUDA correlation package cannot be built or imported here (torch.utils.ffi,
THC, nvcc); its values are pinned through the CostVolumeLayer fixtures: for k=1, s1=1
Correlation(pad=md=r, s2=1) * C == CVL(sr=r)[perm] * (2r+1)^2 and
Correlation(pad=md=9, s2=2) * C == CVL(sr=8)[perm, even offsets] * 289.

Every fixture holds float32 inputs (the reference's dtype), the reference's outputs,
a seeded upstream gradient and the reference's autograd gradients.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _load_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import modules as ref_modules  # noqa: E402  (reference modules.py)

    ref_modules.F = types.SimpleNamespace(
        grid_sample=lambda x, g: F.grid_sample(
            x, g, mode="bilinear", padding_mode="zeros", align_corners=True))
    return ref_modules


def _cvl_case(M, name, seed, B, C, H, W, sr):
    g = torch.Generator().manual_seed(seed)
    src = torch.randn(B, C, H, W, generator=g)
    tgt = torch.randn(B, C, H, W, generator=g)
    args = types.SimpleNamespace(search_range=sr, device="cpu")
    s = src.clone().requires_grad_(True)
    t = tgt.clone().requires_grad_(True)
    out = M.CostVolumeLayer(args)(s, t)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), src=src.numpy(), tgt=tgt.numpy(),
                        out=out.detach().numpy(), gout=gout.numpy(), gsrc=s.grad.numpy(),
                        gtgt=t.grad.numpy(), sr=np.int32(sr))
    print(name, tuple(out.shape))


def _warp_case(M, name, seed, B, C, H, W, flow_std, zero_flow=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, H, W, generator=g)
    if zero_flow:
        flow = torch.zeros(B, 2, H, W)
    else:
        flow = torch.randn(B, 2, H, W, generator=g) * flow_std
    args = types.SimpleNamespace(device="cpu")
    xs = x.clone().requires_grad_(True)
    fs = flow.clone().requires_grad_(True)
    out = M.WarpingLayer(args)(xs, fs)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x.numpy(), flow=flow.numpy(),
                        out=out.detach().numpy(), gout=gout.numpy(), gx=xs.grad.numpy(),
                        gflow=fs.grad.numpy())
    print(name, tuple(out.shape))


def _upwarp_case(M, name, seed, B, C, h, w, flow_std):
    """model.py:78 (F.upsample(flow, scale_factor=2, mode='bilinear') * 2, called as the
    reference calls it: torch 0.4's default is align_corners=False, as is modern torch's) then
    model.py:80 (the reference WarpingLayer); gradients wrt x2 and the coarse flow for seeded
    upstream gradients of x2_warp and of the upsampled flow (model.py:89/91 concatenates it)."""
    g = torch.Generator().manual_seed(seed)
    x2 = torch.randn(B, C, 2 * h, 2 * w, generator=g)
    flow = torch.randn(B, 2, h, w, generator=g) * flow_std
    args = types.SimpleNamespace(device="cpu")
    xs = x2.clone().requires_grad_(True)
    fs = flow.clone().requires_grad_(True)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        fup = F.upsample(fs, scale_factor=2, mode="bilinear") * 2
    out = M.WarpingLayer(args)(xs, fup)
    gout = torch.randn(out.shape, generator=g)
    gfup = torch.randn(fup.shape, generator=g)
    torch.autograd.backward([out, fup], [gout, gfup])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x2=x2.numpy(), flow=flow.numpy(),
                        out=out.detach().numpy(), flow_up=fup.detach().numpy(),
                        gout=gout.numpy(), gflow_up=gfup.numpy(), gx2=xs.grad.numpy(),
                        gflow=fs.grad.numpy())
    print(name, tuple(out.shape))


def main():
    M = _load_reference()
    # CostVolumeLayer sr=4 ("Corr4" pin) and sr=8 ("Corr9" pin), SURVEY §8c shapes.
    _cvl_case(M, "cvl_sr4_b2c8_12x14", 1, 2, 8, 12, 14, 4)
    _cvl_case(M, "cvl_sr4_b2c32_24x28", 2, 2, 32, 24, 28, 4)
    _cvl_case(M, "cvl_sr8_b2c8_12x14", 3, 2, 8, 12, 14, 8)
    _cvl_case(M, "cvl_sr8_b1c32_12x14", 4, 1, 32, 12, 14, 8)
    # true pyramid shapes at 384x448, B=1 (l0 192x6x7, l1 128x12x14)
    _cvl_case(M, "cvl_sr4_l0_b1c192_6x7", 5, 1, 192, 6, 7, 4)
    _cvl_case(M, "cvl_sr8_l0_b1c192_6x7", 6, 1, 192, 6, 7, 8)
    _cvl_case(M, "cvl_sr4_l1_b1c128_12x14", 7, 1, 128, 12, 14, 4)
    # warp: flows ~ N(0, 2^2) incl. out-of-bounds samples; a large-flow case; zero flow.
    _warp_case(M, "warp_b2c8_12x14", 11, 2, 8, 12, 14, 2.0)
    _warp_case(M, "warp_b2c32_24x28", 12, 2, 32, 24, 28, 2.0)
    _warp_case(M, "warp_b1c16_9x31_far", 13, 1, 16, 9, 31, 12.0)
    _warp_case(M, "warp_b1c4_6x7_zero", 14, 1, 4, 6, 7, 0.0, zero_flow=True)
    # flow upsample x2 (model.py:78) then warp (model.py:80): l0 -> l1 shape and a ragged one
    _upwarp_case(M, "upwarp_b2c8_6x7", 21, 2, 8, 6, 7, 1.5)
    _upwarp_case(M, "upwarp_b1c4_5x9_far", 22, 1, 4, 5, 9, 6.0)


if __name__ == "__main__":
    main()
