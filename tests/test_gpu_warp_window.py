"""The LDS-window forward warp (csrc/warp_fwd_win.hip, 16-bit storage) against the gather kernel
it replaces on large grids (warp_fwd_kernel, knob warp_win=0) -- bit for bit, fp16 / bf16 -- and
against the oracle (WarpingLayer, modules.py:31-42).  Flows beyond the 8-px window margin take
the global-gather branch: covered by the large-flow cases.  fp32 keeps the gather kernel (the
window measured no faster there, profiles/r06k_warp_fwd_window.txt)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from pwcnet_amd import _lib
from pwcnet_amd.ops import warp_forward

pytestmark = pytest.mark.gpu

DT = {"fp16": torch.float16, "bf16": torch.bfloat16}

# (B, C, H, W): config 2 l3 / l4 (56-px tiles), config-4 widths (64-px tiles), ragged edges
# (H not a multiple of the tile height, W a multiple of 8 but not of the tile width, images
# narrower than one tile), C not a multiple of the channel slice
SHAPES = [(8, 32, 96, 112), (8, 64, 48, 56), (2, 32, 112, 256), (2, 96, 28, 64),
          (1, 5, 40, 120), (2, 12, 33, 72), (1, 3, 130, 200), (2, 16, 20, 8), (1, 4, 9, 16)]


def _inputs(shape, scale, dtype, seed):
    B, C, H, W = shape
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(B, C, H, W, device="cuda", generator=g).to(DT[dtype])
    f = (torch.randn(B, 2, H, W, device="cuda", generator=g) * scale).to(DT[dtype])
    return x, f


def _warp(x, f, knobs):
    _lib.set_debug(knobs)
    try:
        return warp_forward(x, f)
    finally:
        _lib.set_debug("")


def _both(x, f):
    """(window kernel forced on every shape, gather kernel)."""
    return _warp(x, f, "warp_win=2"), _warp(x, f, "warp_win=0")


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("scale", [0.0, 2.0, 12.0])
def test_window_warp_bitwise_equals_gather_kernel(shape, scale, dtype):
    x, f = _inputs(shape, scale, dtype, seed=sum(shape) + int(scale))
    a, b = _both(x, f)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("wgs", [1, 256, 100000])
def test_window_warp_slicing_bitwise(wgs):
    """Channel slices of one chunk up to all chunks in one workgroup (knob warp_win_wgs)."""
    x, f = _inputs((2, 40, 40, 128), 3.0, "fp16", seed=wgs)
    a = _warp(x, f, f"warp_win=2,warp_win_wgs={wgs}")
    assert torch.equal(a.view(torch.int16), _warp(x, f, "warp_win=0").view(torch.int16))


def test_window_warp_default_dispatch():
    """Default choice: fp16 config-4 levels take the window kernel (same bits either way); the
    knob-free call equals the forced one."""
    x, f = _inputs((16, 32, 112, 256), 2.0, "fp16", seed=3)
    assert torch.equal(warp_forward(x, f).view(torch.int16),
                       _warp(x, f, "warp_win=2").view(torch.int16))


def test_window_warp_non_finite_flows():
    """NaN / inf / huge flows: the same output as the gather kernel (every such sample leaves the
    window and takes the global branch, where both kernels clamp and mask alike)."""
    x, f = _inputs((1, 8, 64, 128), 2.0, "fp16", seed=7)
    f[0, 0, 3, 5] = float("nan")
    f[0, 1, 10, 20] = float("inf")
    f[0, 0, 30, 40] = -60000.0
    f[0, 1, 50, 100] = float("-inf")
    a, b = _both(x, f)
    assert torch.equal(torch.nan_to_num(a.float(), nan=7.0), torch.nan_to_num(b.float(), nan=7.0))


@pytest.mark.parametrize("scale", [2.0, 20.0])
def test_window_warp_vs_oracle(scale):
    """fp16 storage: the oracle on the same fp16 values in fp64, within the output's rounding."""
    B, C, H, W = 2, 8, 48, 64
    rng = np.random.default_rng(11)
    x = rng.standard_normal((B, C, H, W)).astype(np.float16)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float16)
    out = _warp(torch.from_numpy(x).cuda(), torch.from_numpy(f).cuda(), "warp_win=2")
    ref = O.warp_forward(x.astype(np.float32), f.astype(np.float32))
    np.testing.assert_allclose(out.float().cpu().numpy(), ref, rtol=2e-3, atol=2e-3)
