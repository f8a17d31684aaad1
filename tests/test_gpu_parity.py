"""GPU parity: the HIP hot path (through the C ABI) against the CPU oracle and the reference's
golden fixtures.

Tolerances (BASELINE.json north_star: "within 1e-5 fp32"):
  * fp32 forward: |hip - oracle_f64| <= 1e-5 + 1e-5*|oracle| on unit-scale inputs
  * fp32 backward: 1e-4
  * fp16/bf16 storage: compared with the fp64 oracle on the *rounded* inputs; tolerance is the
    output rounding of the storage type (fp16 2e-3 rel, bf16 1.6e-2 rel) + 1e-4 abs.
"""
import glob
import os

import numpy as np
import pytest
import torch


def _seed(*parts):
    """Process-independent seed (str hashing is randomised per process; crc32 is not)."""
    import zlib
    return zlib.crc32(repr(parts).encode())

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CORR_CASES = [
    # (B, C, H, W, pad, k, md, s1, s2)  -- tiled kernels: k=1, s1=1, md/s2 == 4
    (2, 8, 12, 14, 9, 1, 9, 1, 2),      # Corr9 (model.py:24), tiny
    (2, 32, 24, 28, 9, 1, 9, 1, 2),
    (1, 192, 6, 7, 9, 1, 9, 1, 2),      # l0 shape at 384x448
    (1, 128, 12, 14, 9, 1, 9, 1, 2),    # l1
    (1, 96, 24, 28, 9, 1, 9, 1, 2),     # l2
    (1, 64, 48, 56, 9, 1, 9, 1, 2),     # l3
    (2, 32, 96, 112, 9, 1, 9, 1, 2),    # l4
    (2, 40, 47, 52, 9, 1, 9, 1, 2),     # row bands: odd H, W/2 % 4 != 0, C % 16 != 0
    (1, 20, 30, 36, 8, 1, 8, 1, 2),     # row bands, md = 8
    (1, 3, 17, 23, 9, 1, 9, 1, 2),      # ragged: W % 4 != 0, C % CC != 0
    (1, 5, 1, 1, 9, 1, 9, 1, 2),        # 1x1 image
    (2, 8, 12, 14, 4, 1, 4, 1, 1),      # Corr4
    (2, 32, 24, 28, 4, 1, 4, 1, 1),
    (1, 7, 19, 13, 4, 1, 4, 1, 1),      # ragged Corr4
    (1, 16, 20, 24, 0, 1, 4, 1, 1),     # pad < md: off = 4 (vector loads disabled), Ho=H-8
    (1, 16, 20, 24, 8, 1, 8, 1, 2),     # md=8, s2=2 -> dr=4, tiled with off=0
    (1, 16, 20, 24, 6, 1, 9, 1, 2),     # off = 3: misaligned tile origin
    # generic kernel
    (2, 8, 12, 14, 3, 3, 2, 1, 1),      # kernel_size 3
    (2, 8, 13, 15, 4, 1, 4, 2, 2),      # stride1 2
    (1, 8, 12, 14, 2, 1, 2, 1, 1),      # dr = 2
    (1, 8, 12, 14, 20, 1, 20, 1, 2),    # FlowNetC-style md=20, s2=2 (dr=10)
]


def _t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _rand(rng, *shape):
    return rng.standard_normal(shape).astype(np.float32)


@pytest.mark.parametrize("case", CORR_CASES, ids=lambda c: "B{}C{}_{}x{}_p{}k{}md{}s{}{}".format(*c))
def test_corr_forward_fp32(case):
    from pwcnet_amd.ops import corr_forward
    B, C, H, W, pad, k, md, s1, s2 = case
    rng = np.random.default_rng(_seed(case))
    a, b = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W)
    out = corr_forward(_t(a), _t(b), pad, k, md, s1, s2)
    torch.cuda.synchronize()
    ref = O.corr_forward(a, b, pad, k, md, s1, s2)
    assert tuple(out.shape) == ref.shape
    np.testing.assert_allclose(_np(out), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", [c for c in CORR_CASES if c[7] == 1],
                         ids=lambda c: "B{}C{}_{}x{}_p{}k{}md{}s{}{}".format(*c))
def test_corr_backward_fp32(case):
    from pwcnet_amd.ops import corr_backward
    B, C, H, W, pad, k, md, s1, s2 = case
    rng = np.random.default_rng(_seed(1, case))
    a, b = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W)
    OC, Ho, Wo = O.corr_output_shape(H, W, pad, k, md, s1, s2)
    g = _rand(rng, B, OC, Ho, Wo)
    g1, g2 = corr_backward(_t(a), _t(b), _t(g), pad, k, md, s1, s2)
    torch.cuda.synchronize()
    r1, r2 = O.corr_backward(a, b, g, pad, k, md, s1, s2)
    np.testing.assert_allclose(_np(g1), r1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(g2), r2, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype,rtol", [(torch.float16, 2e-3), (torch.bfloat16, 1.6e-2)])
@pytest.mark.parametrize("case", [(2, 32, 24, 28, 9, 1, 9, 1, 2), (1, 16, 17, 23, 4, 1, 4, 1, 1),
                                  (1, 8, 12, 14, 3, 3, 2, 1, 1)])
def test_corr_forward_low_precision(case, dtype, rtol):
    from pwcnet_amd.ops import corr_forward
    B, C, H, W, pad, k, md, s1, s2 = case
    rng = np.random.default_rng(7)
    a, b = _t(_rand(rng, B, C, H, W), dtype), _t(_rand(rng, B, C, H, W), dtype)
    out = corr_forward(a, b, pad, k, md, s1, s2)
    assert out.dtype == dtype
    ref = O.corr_forward(_np(a), _np(b), pad, k, md, s1, s2)
    np.testing.assert_allclose(_np(out), ref, rtol=rtol, atol=1e-4 + rtol * np.abs(ref).max())


def test_correlation_module_autograd_matches_oracle():
    """Correlation nn.Module + CorrelationFunction end to end (model.py:24 config)."""
    from correlation_package.modules.correlation import Correlation
    rng = np.random.default_rng(3)
    a, b = _rand(rng, 2, 16, 20, 24), _rand(rng, 2, 16, 20, 24)
    x1 = _t(a).requires_grad_(True)
    x2 = _t(b).requires_grad_(True)
    corr = Correlation(pad_size=9, kernel_size=1, max_displacement=9, stride1=1, stride2=2,
                       corr_multiply=1)
    out = corr(x1, x2)
    g = _rand(rng, *out.shape)
    out.backward(_t(g))
    np.testing.assert_allclose(_np(out), O.corr_forward(a, b, 9, 1, 9, 1, 2), rtol=1e-5,
                               atol=1e-5)
    r1, r2 = O.corr_backward(a, b, g, 9, 1, 9, 1, 2)
    np.testing.assert_allclose(_np(x1.grad), r1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(x2.grad), r2, rtol=1e-4, atol=1e-4)


def test_correlation_asserts_contiguous():
    from pwcnet_amd.ops import CorrelationFunction
    x = torch.randn(1, 8, 12, 14, device=DEV).transpose(2, 3)
    with pytest.raises(AssertionError):
        CorrelationFunction.apply(x, x, 9, 1, 9, 1, 2, 1)


def test_corr_empty_batch():
    from pwcnet_amd.ops import corr_forward
    x = torch.zeros(0, 8, 12, 14, device=DEV)
    assert tuple(corr_forward(x, x, 9, 1, 9, 1, 2).shape) == (0, 81, 12, 14)


# ---------------------------------------------------------------------------------------
# reference fixtures (outputs of the reference's own modules.py, tests/golden)
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "cvl_*.npz"))),
                         ids=os.path.basename)
def test_cost_volume_layer_vs_reference(path):
    import types
    from pwcnet_amd import CostVolumeLayer
    z = np.load(path)
    sr = int(z["sr"])
    layer = CostVolumeLayer(types.SimpleNamespace(search_range=sr, device=DEV))
    s = _t(z["src"]).requires_grad_(True)
    t = _t(z["tgt"]).requires_grad_(True)
    out = layer(s, t)
    out.backward(_t(z["gout"]))
    np.testing.assert_allclose(_np(out), z["out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(s.grad), z["gsrc"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(t.grad), z["gtgt"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "cvl_sr*.npz"))),
                         ids=os.path.basename)
def test_correlation_vs_reference_cvl(path):
    """Correlation (Corr4 / Corr9) against the reference CVL through the channel pin."""
    from pwcnet_amd.ops import corr_forward
    z = np.load(path)
    sr = int(z["sr"])
    C = z["src"].shape[1]
    K = (2 * sr + 1) ** 2
    pad, md, s2 = (4, 4, 1) if sr == 4 else (9, 9, 2)
    idx = O.corr_channel_from_cvl(sr, s2, md)
    out = corr_forward(_t(z["src"]), _t(z["tgt"]), pad, 1, md, 1, s2)
    np.testing.assert_allclose(_np(out) * C, z["out"][:, idx] * K, rtol=1e-5, atol=2e-5 * C)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "warp_*.npz"))),
                         ids=os.path.basename)
def test_warping_layer_vs_reference(path):
    from pwcnet_amd import WarpingLayer
    z = np.load(path)
    x = _t(z["x"]).requires_grad_(True)
    f = _t(z["flow"]).requires_grad_(True)
    out = WarpingLayer(None)(x, f)
    out.backward(_t(z["gout"]))
    np.testing.assert_allclose(_np(out), z["out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(x.grad), z["gx"], rtol=1e-4, atol=1e-4)
    # same fp32 chain as the reference: even the zero-flow (integer coordinate) case agrees
    np.testing.assert_allclose(_np(f.grad), z["gflow"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape", [(2, 32, 96, 112), (1, 192, 6, 7), (3, 5, 9, 31),
                                   (1, 16, 448 // 4, 1024 // 4)])
def test_warp_vs_oracle(shape):
    from pwcnet_amd.ops import warp_backward, warp_forward
    B, C, H, W = shape
    rng = np.random.default_rng(11)
    x = _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H, W)) * 3).astype(np.float32)
    out = warp_forward(_t(x), _t(f))
    np.testing.assert_allclose(_np(out), O.warp_forward(x, f), rtol=1e-5, atol=1e-5)
    g = _rand(rng, B, C, H, W)
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    rx, rf = O.warp_backward(x, f, g)
    np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)))


@pytest.mark.parametrize("scale", [0.0, 2.0, 7.5, 25.0])
@pytest.mark.parametrize("shape", [(8, 32, 96, 112), (8, 64, 48, 56), (2, 96, 24, 28),
                                   (2, 128, 12, 14), (2, 192, 6, 7), (1, 13, 37, 70),
                                   (1, 3, 9, 2), (3, 5, 17, 33)])
def test_warp_backward_one_launch_vs_oracle(shape, scale):
    """pwc_warp_backward_ws (16x16 grad_x tiles with 8-px margins and channel groups, then a
    small kernel for the groups' grad_flow partials and the far corners) against the float64
    oracle: zero flow, in-margin, around the margin and far beyond it; ragged tiles, W % 4 != 0,
    a 2-pixel-wide image; and against the multi-kernel path (PWC_DEBUG warp_bwd_tiles=0)."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = shape
    rng = np.random.default_rng(int(scale * 4) + 7 * H + W)
    x = _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    g = _rand(rng, B, C, H, W)
    _lib.set_debug("warp_bwd_tiles=2")  # the one-launch path at every size
    try:
        gx, gf = warp_backward(_t(x), _t(f), _t(g))
        _lib.set_debug("warp_bwd_tiles=0")
        gx0, gf0 = warp_backward(_t(x), _t(f), _t(g))
    finally:
        _lib.set_debug("")
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(gx), _np(gx0), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(gf), _np(gf0), rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)),
                               equal_nan=True)
    if x.size <= 2 * 96 * 24 * 28:
        rx, rf = O.warp_backward(x, f, g)
        np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)),
                                   equal_nan=True)


@pytest.mark.parametrize("scale", [2.0, 25.0])
@pytest.mark.parametrize("shape", [(2, 96, 24, 28), (8, 96, 24, 28), (1, 40, 12, 40),
                                   (1, 8, 12, 48), (1, 16, 12, 48), (1, 32, 12, 48), (1, 64, 10, 50)],
                         ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_warp_backward_whole_image_candidates(shape, scale):
    """Images of <= 768 pixels (l2): every pixel is a candidate of every grad_x tile, so there
    is no far-corner pass -- against the oracle (flows far beyond the 8-px margins included),
    repeatable bit for bit (no atomics left), and within fp32 summation order of the margin
    windows + far pass (PWC_DEBUG warp_bwd_whole=0).  One shape per instantiation."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = shape
    rng = np.random.default_rng(int(scale) * 3 + W)
    x, g = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    gx1, gf1 = warp_backward(_t(x), _t(f), _t(g))
    _lib.set_debug("warp_bwd_whole=0")
    try:
        gx0, gf0 = warp_backward(_t(x), _t(f), _t(g))
    finally:
        _lib.set_debug("")
    torch.cuda.synchronize()
    assert torch.equal(gx, gx1) and torch.equal(gf.nan_to_num(), gf1.nan_to_num())
    np.testing.assert_allclose(_np(gx), _np(gx0), rtol=1e-6, atol=1e-6)
    assert torch.equal(gf.nan_to_num(), gf0.nan_to_num())  # the same grad_flow code
    if x.size <= 2 * 96 * 24 * 28:
        rx, rf = O.warp_backward(x, f, g)
        np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)),
                                   equal_nan=True)


@pytest.mark.parametrize("scale", [2.0, 25.0])
def test_warp_backward_margin_windows_merged(scale):
    """Images over 768 pixels keep the 8-px margin windows and the far pass after the merged
    launch (here 8 x 32 tiles, two grad_flow channel groups): against the oracle."""
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = 1, 24, 30, 40
    rng = np.random.default_rng(int(scale) + 5)
    x, g = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    rx, rf = O.warp_backward(x, f, g)
    np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)),
                               equal_nan=True)


def test_warp_backward_one_launch_repeatable():
    """No far corners -> no atomics: two calls agree bit for bit (fixed list and group order)."""
    from pwcnet_amd.ops import warp_backward
    rng = np.random.default_rng(3)
    x, g = _rand(rng, 4, 32, 96, 112), _rand(rng, 4, 32, 96, 112)
    f = (rng.standard_normal((4, 2, 96, 112)) * 2).clip(-6, 6).astype(np.float32)
    a = warp_backward(_t(x), _t(f), _t(g))
    b = warp_backward(_t(x), _t(f), _t(g))
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("scale", [0.0, 6.0, 25.0])
def test_warp_backward_tiles_and_outliers(scale):
    # grad_x of the LDS-binned kernel (tiles of 8x32, candidate margin 8) + the corners left
    # to global atomics: zero flow, flows around the margin, and flows far beyond it; ragged
    # tile edges (37 x 70) and a channel count that is not a multiple of the chunk (13)
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = 2, 13, 37, 70
    rng = np.random.default_rng(17)
    x = _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    g = _rand(rng, B, C, H, W)
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    rx, rf = O.warp_backward(x, f, g)
    np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)))


@pytest.mark.parametrize("shape", [(2, 192, 6, 7), (2, 128, 12, 14), (2, 96, 24, 28)])
@pytest.mark.parametrize("scale", [0.0, 3.0, 25.0])
def test_warp_backward_small_images_one_launch(shape, scale):
    """l0 / l1-sized images fit one grad_x tile: grad_x lists and grad_flow run as one merged
    launch (warp_bwd_small); l2-sized grids run the tiles and grad_flow as one launch plus the
    far-corner pass (warp_bwd_merged + warp_bwd_far) -- against the oracle for zero, moderate
    and far (mostly out-of-image) flows, repeatable bit for bit when no far corner exists, and
    equal to the separate launches up to the summation order (l1 takes 16 x 16 tiles there,
    8 x 32 in two launches)."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = shape
    rng = np.random.default_rng(29)
    x, g = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    rx, rf = O.warp_backward(x, f, g)
    np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)))
    gx1, gf1 = warp_backward(_t(x), _t(f), _t(g))
    assert torch.equal(gf, gf1)
    if scale < 8:  # far corners go through atomics (ATen's order-free scatter)
        assert torch.equal(gx, gx1)
    _lib.set_debug("warp_bwd_small=0,warp_bwd_merge=0")
    try:
        gx2, gf2 = warp_backward(_t(x), _t(f), _t(g))
    finally:
        _lib.set_debug("")
    np.testing.assert_allclose(_np(gx), _np(gx2), rtol=1e-6, atol=1e-6)
    assert torch.equal(gf, gf2)  # same grad_flow code, same channel groups


@pytest.mark.parametrize("shape", [(2, 32, 96, 112), (2, 13, 37, 70)])
def test_warp_backward_converging_lists_repeatable(shape):
    """Flows pulling every pixel toward a few sinks (within the candidate margin, so no
    corner is left to atomics): tile pixels near a sink collect long lists from many sources
    and several waves.  grad_x / grad_flow match the oracle and repeat bit for bit (the
    per-wave slot counters fix the list order)."""
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = shape
    rng = np.random.default_rng(23)
    x, g = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W)
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    sy, sx = (yy // 12) * 12 + 6, (xx // 16) * 16 + 8  # one sink per 12 x 16 cell
    f = np.stack([np.clip(sx - xx, -6, 6) + 0.25, np.clip(sy - yy, -6, 6) - 0.5])
    f = np.broadcast_to(f, (B, 2, H, W)).astype(np.float32).copy()
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    rx, rf = O.warp_backward(x, f, g)
    np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)))
    for _ in range(2):
        gx2, gf2 = warp_backward(_t(x), _t(f), _t(g))
        assert torch.equal(gx, gx2) and torch.equal(gf, gf2)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "upwarp_*.npz"))),
                         ids=os.path.basename)
def test_upsample_warp_vs_reference(path):
    # model.py:78 + :80 as one launch (UpsampleWarp), reference fixtures incl. gradients
    from pwcnet_amd import UpsampleWarp
    z = np.load(path)
    x2 = _t(z["x2"]).requires_grad_(True)
    f = _t(z["flow"]).requires_grad_(True)
    out, fup = UpsampleWarp()(x2, f)
    torch.autograd.backward([out, fup], [_t(z["gout"]), _t(z["gflow_up"])])
    np.testing.assert_allclose(_np(fup), z["flow_up"], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(_np(out), z["out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(x2.grad), z["gx2"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(f.grad), z["gflow"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape", [(8, 32, 96, 112), (2, 128, 12, 14), (1, 3, 10, 18)])
def test_upsample_warp_vs_oracle(shape):
    # fused == flow upsample then warp (oracle), at the l4 size and small/ragged ones; the
    # warp of the stored flow_up is bit-identical to pwc_warp_forward on it
    from pwcnet_amd.ops import flow_upsample_backward, upsample_warp_forward, warp_forward
    B, C, H, W = shape
    rng = np.random.default_rng(23)
    x2 = _rand(rng, B, C, H, W)
    f = (rng.standard_normal((B, 2, H // 2, W // 2)) * 2).astype(np.float32)
    out, fup = upsample_warp_forward(_t(x2), _t(f))
    np.testing.assert_allclose(_np(fup), O.flow_upsample2(f), rtol=1e-6, atol=1e-5)
    # the warp is pinned on the flow it sampled with (the stored fp32 flow_up, as the reference
    # stores it): an fp64 flow_up moves samples near integer coordinates by ~1 fp32 ulp
    np.testing.assert_allclose(_np(out), O.warp_forward(x2, _np(fup)), rtol=1e-5, atol=1e-5)
    assert torch.equal(out, warp_forward(_t(x2), fup))
    out2, none = upsample_warp_forward(_t(x2), _t(f), emit_flow=False)
    assert none is None and torch.equal(out, out2)
    g = (rng.standard_normal((B, 2, H, W))).astype(np.float32)
    np.testing.assert_allclose(_np(flow_upsample_backward(_t(g))), O.flow_upsample2_backward(g),
                               rtol=1e-5, atol=1e-5)


def test_upsample_warp_fp16_and_shape_checks():
    from pwcnet_amd.ops import upsample_warp_forward
    rng = np.random.default_rng(29)
    x2 = _t(_rand(rng, 2, 16, 24, 28), torch.float16)
    f = _t(rng.standard_normal((2, 2, 12, 14)) * 2, torch.float16)
    out, fup = upsample_warp_forward(x2, f)
    rfup = O.flow_upsample2(_np(f))
    np.testing.assert_allclose(_np(fup), rfup, rtol=2e-3, atol=2e-3)
    # fp16 warps with the STORED (fp16-rounded) upsampled flow, like the reference would
    np.testing.assert_allclose(_np(out), O.warp_forward(_np(x2), _np(fup)), rtol=2e-3, atol=5e-3)
    with pytest.raises(ValueError):
        upsample_warp_forward(_t(_rand(rng, 1, 4, 11, 14)), _t(_rand(rng, 1, 2, 5, 7)))


@pytest.mark.parametrize("shape", [(2, 192, 6, 7), (2, 128, 12, 14), (2, 96, 24, 28),
                                   (2, 64, 48, 56), (2, 32, 96, 112)])
@pytest.mark.parametrize("slope", [None, 0.01])
def test_corr_forward_into_cat_slice(shape, slope):
    # model.py:83-91: the kernels write the corr channels of the cat buffer (with the fused
    # leaky_relu_); values equal corr_forward (+ F.leaky_relu) bit for bit, and nothing
    # outside the slice is touched
    from pwcnet_amd.ops import corr_forward, corr_forward_into
    B, C, H, W = shape
    rng = np.random.default_rng(31)
    x1, x2 = _t(_rand(rng, B, C, H, W)), _t(_rand(rng, B, C, H, W))
    buf = torch.full((B, C + 83, H, W), 7.25, device=DEV)
    corr_forward_into(x1, x2, buf[:, C:C + 81], 9, 1, 9, 1, 2, negative_slope=slope)
    ref = corr_forward(x1, x2, 9, 1, 9, 1, 2)
    if slope is not None:
        ref = torch.nn.functional.leaky_relu(ref, slope)
    assert torch.equal(buf[:, C:C + 81], ref)
    assert bool((buf[:, :C] == 7.25).all()) and bool((buf[:, C + 81:] == 7.25).all())


@pytest.mark.parametrize("case", [("fp16", 9, 2), ("fp32", 4, 1)])
def test_corr_forward_into_fallback(case):
    # configurations without slice-writing kernels: dense volume + strided copy
    from pwcnet_amd.ops import corr_forward, corr_forward_into
    dt, md, s2 = case
    dtype = torch.float16 if dt == "fp16" else torch.float32
    B, C, H, W = 2, 16, 12, 14
    rng = np.random.default_rng(37)
    x1, x2 = _t(_rand(rng, B, C, H, W), dtype), _t(_rand(rng, B, C, H, W), dtype)
    buf = torch.full((B, C + 83, H, W), -3.0, device=DEV, dtype=dtype)
    corr_forward_into(x1, x2, buf[:, C:C + 81], md, 1, md, 1, s2, negative_slope=0.1)
    ref = torch.nn.functional.leaky_relu(corr_forward(x1, x2, md, 1, md, 1, s2).float(), 0.1)
    np.testing.assert_allclose(_np(buf[:, C:C + 81]), _np(ref), rtol=2e-3, atol=1e-4)
    assert bool((buf[:, :C] == -3.0).all()) and bool((buf[:, C + 81:] == -3.0).all())


@pytest.mark.parametrize("act", [False, True])
def test_correlation_cat_autograd(act):
    from pwcnet_amd import Correlation, CorrelationCat
    B, C, H, W = 2, 32, 24, 28
    rng = np.random.default_rng(41)
    a, b, f = _rand(rng, B, C, H, W), _rand(rng, B, C, H, W), _rand(rng, B, 2, H, W)
    g = _t(_rand(rng, B, C + 83, H, W))
    x1, x2, fl = (_t(v).requires_grad_(True) for v in (a, b, f))
    out = CorrelationCat(corr_activation=act)(x1, x2, fl)
    out.backward(g)
    y1, y2, yf = (_t(v).requires_grad_(True) for v in (a, b, f))
    corr = Correlation(9, 1, 9, 1, 2)(y1, y2)
    if act:
        corr = torch.nn.functional.leaky_relu(corr, 0.01)
    ref = torch.cat([y1, corr, yf], 1)
    ref.backward(g)
    assert torch.equal(out.detach(), ref.detach())
    for u, v in ((x1, y1), (x2, y2), (fl, yf)):
        np.testing.assert_allclose(_np(u.grad), _np(v.grad), rtol=1e-5, atol=1e-6)


def test_warp_fp16():
    from pwcnet_amd.ops import warp_forward
    rng = np.random.default_rng(5)
    x = _t(_rand(rng, 2, 16, 24, 28), torch.float16)
    f = _t(rng.standard_normal((2, 2, 24, 28)) * 3, torch.float16)
    out = warp_forward(x, f)
    ref = O.warp_forward(_np(x), _np(f))
    np.testing.assert_allclose(_np(out), ref, rtol=2e-3, atol=5e-3)


LOW = [(torch.float16, 2e-3), (torch.bfloat16, 1.6e-2)]


@pytest.mark.parametrize("dtype,rtol", LOW, ids=["fp16", "bf16"])
def test_low_precision_warp_upsample_backward_into(dtype, rtol):
    """fp16 / bf16 storage through every op that takes it: warp (small and l4-sized images),
    upsample+warp, Correlation backward (Corr9 and the s2 = 1 shape) and the activated strided
    write of pwc_corr_forward_into -- against the oracle on the stored (rounded) inputs, fp32
    arithmetic, tolerance one storage ulp relative to the output's magnitude."""
    from pwcnet_amd.ops import (corr_backward, corr_forward, corr_forward_into,
                                upsample_warp_forward, warp_forward)

    def close(got, ref):
        got = _np(got)
        np.testing.assert_allclose(got, ref, rtol=rtol, atol=1e-4 + rtol * np.abs(ref).max())

    rng = np.random.default_rng(61)
    for shape in [(2, 16, 24, 28), (1, 16, 96, 112)]:
        x = _t(_rand(rng, *shape), dtype)
        f = _t(rng.standard_normal((shape[0], 2) + shape[2:]) * 3, dtype)
        close(warp_forward(x, f), O.warp_forward(_np(x), _np(f)))
    x2 = _t(_rand(rng, 2, 16, 24, 28), dtype)
    fc = _t(rng.standard_normal((2, 2, 12, 14)) * 2, dtype)
    out, fup = upsample_warp_forward(x2, fc)
    close(fup, O.flow_upsample2(_np(fc)))
    close(out, O.warp_forward(_np(x2), _np(fup)))
    for B, C, H, W, pad, k, md, s1, s2 in [(2, 32, 24, 28, 9, 1, 9, 1, 2),
                                           (1, 16, 17, 23, 4, 1, 4, 1, 1)]:
        a, b = _t(_rand(rng, B, C, H, W), dtype), _t(_rand(rng, B, C, H, W), dtype)
        OC, Ho, Wo = O.corr_output_shape(H, W, pad, k, md, s1, s2)
        g = _t(_rand(rng, B, OC, Ho, Wo), dtype)
        g1, g2 = corr_backward(a, b, g, pad, k, md, s1, s2)
        assert g1.dtype == dtype and g2.dtype == dtype
        r1, r2 = O.corr_backward(_np(a), _np(b), _np(g), pad, k, md, s1, s2)
        close(g1, r1)
        close(g2, r2)
    a, b = _t(_rand(rng, 2, 16, 12, 14), dtype), _t(_rand(rng, 2, 16, 12, 14), dtype)
    buf = torch.full((2, 16 + 83, 12, 14), -3.0, device=DEV, dtype=dtype)
    corr_forward_into(a, b, buf[:, 16:97], 9, 1, 9, 1, 2, negative_slope=0.1)
    ref = torch.nn.functional.leaky_relu(corr_forward(a, b, 9, 1, 9, 1, 2).float(), 0.1)
    close(buf[:, 16:97], _np(ref))
    assert bool((buf[:, :16] == -3.0).all()) and bool((buf[:, 97:] == -3.0).all())


@pytest.mark.parametrize("case", [(1, 512, 6, 7), (2, 448, 5, 9)],
                         ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_corr_forward_wide_small_levels_channel_split(case):
    """Small images with too many channels for the band kernel's LDS (and rows that are not
    16-B aligned): the whole-parity-half kernel with channel slices into the workspace and its
    fixed-order reduce (corr_small.hip) -- oracle parity and bitwise repeatability."""
    from pwcnet_amd.ops import corr_forward
    B, C, H, W = case
    rng = np.random.default_rng(67)
    a, b = _t(_rand(rng, B, C, H, W)), _t(_rand(rng, B, C, H, W))
    out = corr_forward(a, b, 9, 1, 9, 1, 2)
    np.testing.assert_allclose(_np(out), O.corr_forward(_np(a), _np(b), 9, 1, 9, 1, 2),
                               rtol=1e-5, atol=1e-5)
    assert torch.equal(out, corr_forward(a, b, 9, 1, 9, 1, 2))


# ---------------------------------------------------------------------------------------
# full BASELINE sizes: size-independent properties + full oracle compare (seconds on CPU)
# ---------------------------------------------------------------------------------------
def test_level2_full_size_corr9_b8():
    """Config 2 l4 ('level 2'): B=8, 32x96x112, Corr9 — full compare with the oracle."""
    from pwcnet_amd.ops import corr_forward
    rng = np.random.default_rng(2024)
    a, b = _rand(rng, 8, 32, 96, 112), _rand(rng, 8, 32, 96, 112)
    out = _np(corr_forward(_t(a), _t(b), 9, 1, 9, 1, 2))
    np.testing.assert_allclose(out, O.corr_forward(a, b, 9, 1, 9, 1, 2), rtol=1e-5, atol=1e-5)


def test_correlation_properties_sintel_fp16():
    """Config 4 l4 (B=16, 32x112x256, fp16): symmetry property
    corr(a, b)[tc] at x == corr(b, a)[mirror tc] at x + d (size-independent check),
    plus a full oracle compare on two images of the batch."""
    from pwcnet_amd.ops import corr_forward
    rng = np.random.default_rng(99)
    a = _t(_rand(rng, 16, 32, 112, 256), torch.float16)
    b = _t(_rand(rng, 16, 32, 112, 256), torch.float16)
    ab = corr_forward(a, b, 9, 1, 9, 1, 2).float()
    ba = corr_forward(b, a, 9, 1, 9, 1, 2).float()
    # displacement (dy,dx)=(2,2): channel (tj=1,ti=1) -> 6*9+... raster tc=(1+4)*9+(1+4)=50,
    # mirror (-1,-1) -> tc=(3)*9+3=30: ab[50][y][x] == ba[30][y+2][x+2]
    torch.testing.assert_close(ab[:, 50, :-2, :-2], ba[:, 30, 2:, 2:], rtol=0, atol=2e-3)
    ref = O.corr_forward(_np(a[:2]), _np(b[:2]), 9, 1, 9, 1, 2)
    np.testing.assert_allclose(_np(ab[:2]), ref, rtol=2e-3, atol=2e-3)


def test_layers_reject_cpu_tensors():
    from pwcnet_amd.ops import corr_forward
    with pytest.raises(RuntimeError):
        corr_forward(torch.zeros(1, 2, 3, 3), torch.zeros(1, 2, 3, 3), 9, 1, 9, 1, 2)


@pytest.mark.parametrize("case", [(1, 192, 6, 7), (2, 128, 12, 14), (2, 96, 24, 28),
                                  (1, 64, 48, 56)])
def test_corr_forward_with_and_without_workspace(case):
    """pwc_corr_forward (single pass over C) and pwc_corr_forward_ws (channel split into a
    caller workspace + fixed-order reduce) both match the oracle; the split result is
    deterministic across calls."""
    import ctypes
    from pwcnet_amd import _lib
    B, C, H, W = case
    rng = np.random.default_rng(21)
    a, b = _t(_rand(rng, B, C, H, W)), _t(_rand(rng, B, C, H, W))
    lib = _lib.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ref = O.corr_forward(_np(a), _np(b), 9, 1, 9, 1, 2)
    out0 = torch.empty(B, 81, H, W, device=DEV)
    _lib.check(lib.pwc_corr_forward(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                    ctypes.c_void_p(out0.data_ptr()), B, C, H, W, 9, 1, 9, 1, 2,
                                    1, 0, stream), "t")
    nws = lib.pwc_corr_workspace_size(B, C, H, W, 9, 1, 9, 1, 2)
    assert nws > 0  # these grids are small enough to split
    ws = torch.empty(nws, dtype=torch.uint8, device=DEV)
    outs = []
    for _ in range(2):
        o = torch.empty(B, 81, H, W, device=DEV)
        _lib.check(lib.pwc_corr_forward_ws(
            ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
            ctypes.c_void_p(o.data_ptr()), B, C, H, W, 9, 1, 9, 1, 2, 1, 0,
            ctypes.c_void_p(ws.data_ptr()), nws, stream), "t")
        outs.append(o)
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(out0), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(outs[0]), ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(outs[0], outs[1])
    # undersized workspace is an error, not a silent fallback
    with pytest.raises(RuntimeError, match="workspace"):
        _lib.check(lib.pwc_corr_forward_ws(
            ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
            ctypes.c_void_p(outs[0].data_ptr()), B, C, H, W, 9, 1, 9, 1, 2, 1, 0,
            ctypes.c_void_p(ws.data_ptr()), nws - 4, stream), "t")


@pytest.mark.parametrize("cfg", [(9, 1, 9, 1, 2), (4, 1, 4, 1, 1)], ids=["corr9", "corr4"])
@pytest.mark.parametrize("shape", [(1, 1, 1, 1), (2, 3, 1, 9), (1, 5, 9, 1), (3, 1, 5, 5),
                                   (1, 2, 2, 3), (0, 4, 6, 7)],
                         ids=lambda s: "x".join(map(str, s)))
def test_correlation_degenerate_shapes(shape, cfg):
    """Single-pixel, single-row / single-column images, one channel and an empty batch through
    the default dispatch, forward and backward, against the oracle (every displacement but
    (0, 0) of a 1 x 1 image falls in the zero padding)."""
    from pwcnet_amd.ops import corr_backward, corr_forward
    rng = np.random.default_rng(_seed("degenerate", shape, cfg))
    a, b = _rand(rng, *shape), _rand(rng, *shape)
    out = corr_forward(_t(a), _t(b), *cfg)
    torch.cuda.synchronize()
    assert tuple(out.shape) == (shape[0], 81, shape[2], shape[3])
    if shape[0] == 0:
        return
    np.testing.assert_allclose(_np(out), O.corr_forward(a, b, *cfg), rtol=1e-5, atol=1e-6)
    g = _rand(rng, *out.shape)
    g1, g2 = corr_backward(_t(a), _t(b), _t(g), *cfg)
    torch.cuda.synchronize()
    r1, r2 = O.corr_backward(a, b, g, *cfg)
    np.testing.assert_allclose(_np(g1), r1, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(_np(g2), r2, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("shape", [(1, 1, 2, 2), (2, 3, 2, 9), (1, 4, 9, 2), (0, 4, 6, 7)],
                         ids=lambda s: "x".join(map(str, s)))
def test_warp_degenerate_shapes(shape):
    """2-pixel-wide / 2-row images (the smallest the reference's (size - 1) / 2 normalisation
    allows), one channel and an empty batch: warp forward and backward against the oracle,
    flows reaching past every border."""
    from pwcnet_amd.ops import warp_backward, warp_forward
    B, C, H, W = shape
    rng = np.random.default_rng(_seed("warp-degenerate", shape))
    x = _rand(rng, *shape)
    f = (rng.standard_normal((B, 2, H, W)) * 1.5).astype(np.float32)
    out = warp_forward(_t(x), _t(f))
    torch.cuda.synchronize()
    assert tuple(out.shape) == shape
    if B == 0:
        return
    np.testing.assert_allclose(_np(out), O.warp_forward(x, f), rtol=1e-5, atol=1e-6)
    g = _rand(rng, *shape)
    gx, gf = warp_backward(_t(x), _t(f), _t(g))
    torch.cuda.synchronize()
    rx, rf = O.warp_backward(x, f, g)
    np.testing.assert_allclose(_np(gx), rx, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(_np(gf), rf, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("level", [0, 1, 2, 3, 4])
def test_full_size_homogeneity_config2(level):
    """Config 2 (B = 8, 384x448) at every level, fp32: corr(2a, b) == 2 corr(a, b) and
    warp(2x, f) == 2 warp(x, f) bit for bit (a power-of-two scale is exact through every product,
    sum and the /C) -- a size-independent check of the default kernels at full size."""
    from bench import level_shapes
    from pwcnet_amd.ops import corr_forward, warp_forward
    C, H, W = level_shapes(384, 448)[level]
    rng = np.random.default_rng(_seed("homog", level))
    a, b = _t(_rand(rng, 8, C, H, W)), _t(_rand(rng, 8, C, H, W))
    f = _t((rng.standard_normal((8, 2, H, W)) * 2).astype(np.float32))
    assert torch.equal(corr_forward(2 * a, b, 9, 1, 9, 1, 2), 2 * corr_forward(a, b, 9, 1, 9, 1, 2))
    assert torch.equal(warp_forward(2 * a, f), 2 * warp_forward(a, f))


@pytest.mark.parametrize("level", [2, 3, 4])
def test_full_size_adjoint_config5(level):
    """Config 5 (B = 8, 384x448) at l2-l4: the backward kernels are the adjoints of the forward
    ones -- <corr(a, b), g> = <a, dL/da> = <b, dL/db> and <warp(x, f), g> = <x, dL/dx> (both
    maps are linear in the argument), in float64 sums over the full tensors."""
    from bench import level_shapes
    from pwcnet_amd.ops import corr_backward, corr_forward, warp_backward, warp_forward
    C, H, W = level_shapes(384, 448)[level]
    rng = np.random.default_rng(_seed("adjoint", level))
    a, b = _t(_rand(rng, 8, C, H, W)), _t(_rand(rng, 8, C, H, W))
    g = _t(_rand(rng, 8, 81, H, W))
    f = _t((rng.standard_normal((8, 2, H, W)) * 2).astype(np.float32))
    gw = _t(_rand(rng, 8, C, H, W))
    out = corr_forward(a, b, 9, 1, 9, 1, 2)
    g1, g2 = corr_backward(a, b, g, 9, 1, 9, 1, 2)
    w = warp_forward(a, f)
    gx, _ = warp_backward(a, f, gw)
    torch.cuda.synchronize()

    def dot(x, y):
        return float((x.double() * y.double()).sum())
    lhs = dot(out, g)
    for rhs in (dot(a, g1), dot(b, g2)):
        assert abs(lhs - rhs) <= 1e-5 * (abs(lhs) + float((out.double().abs() * g.double().abs()).sum())), (lhs, rhs)
    lw, rw = dot(w, gw), dot(a, gx)
    assert abs(lw - rw) <= 1e-5 * float((w.double().abs() * gw.double().abs()).sum()), (lw, rw)


@pytest.mark.parametrize("level", [0, 1, 2, 3, 4])
def test_full_size_homogeneity_config4_and_fused(level):
    """Config 4 (B = 16, 448x1024, fp16 storage) at every level: corr(2a, b) == 2 corr(a, b)
    and warp(2x, f) == 2 warp(x, f) bit for bit wherever the output is a normal fp16 number
    (fp32 arithmetic, one fp16 rounding of an exactly doubled value; where the undoubled output
    is subnormal its rounding quantum does not scale, so there the two may differ by one 2^-24
    step; inputs carry no subnormals); and the fused warp + correlation (model.py:80-83) of
    config 2's level in fp32 bit for bit."""
    from bench import level_shapes
    from pwcnet_amd.ops import corr_forward, warp_corr_forward, warp_forward
    C, H, W = level_shapes(448, 1024)[level]
    rng = np.random.default_rng(_seed("homog16", level))
    def no_subnormals(v):  # inputs without fp16 subnormals: the check is about output rounding
        return np.where(np.abs(v) < 2.0 ** -12, 0.0, v).astype(np.float32)
    a = _t(no_subnormals(_rand(rng, 16, C, H, W)), torch.float16)
    b = _t(no_subnormals(_rand(rng, 16, C, H, W)), torch.float16)
    f = _t((rng.standard_normal((16, 2, H, W)) * 2).astype(np.float32), torch.float16)

    def same_but_subnormals(x, y):
        x, y = x.float(), y.float()
        normal = y.abs() > 2.0 ** -13  # y = 2 * (a normal fp16 value above the smallest)
        assert torch.equal(x[normal], y[normal])
        assert float((x - y).abs().max()) <= 2.0 ** -24
    same_but_subnormals(corr_forward(2 * a, b, 9, 1, 9, 1, 2), 2 * corr_forward(a, b, 9, 1, 9, 1, 2))
    same_but_subnormals(warp_forward(2 * a, f), 2 * warp_forward(a, f))
    C2, H2, W2 = level_shapes(384, 448)[level]
    x1, x2 = _t(_rand(rng, 8, C2, H2, W2)), _t(_rand(rng, 8, C2, H2, W2))
    f2 = _t((rng.standard_normal((8, 2, H2, W2)) * 2).astype(np.float32))
    c1, w1 = warp_corr_forward(x1, 2 * x2, f2, 9, 1, 9, 1, 2)
    c0, w0 = warp_corr_forward(x1, x2, f2, 9, 1, 9, 1, 2)
    assert torch.equal(c1, 2 * c0) and torch.equal(w1, 2 * w0)
