"""BASELINE config 4 (Sintel shape 448x1024, fp16 storage) and the stride-1 correlations at
full size, through the C ABI, against the fp64 oracle.

fp16: the reference has no fp16 path (correlation_cuda_kernel.cu:5 is fp32 only); the oracle
runs on the fp16-rounded inputs and the tolerance is the fp16 output rounding (2e-3 relative
to the volume's max) -- SURVEY §8d config 4.  Shapes at 448x1024 (SURVEY §8 notation):
l0 192x7x16, l1 128x14x32, l2 96x28x64, l3 64x56x128, l4 32x112x256, plus the north star's
192x224x32 stress shape (C=32, 192x224, not a pyramid level)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
SINTEL = [(2, 192, 7, 16), (2, 128, 14, 32), (2, 96, 28, 64), (2, 64, 56, 128),
          (2, 32, 112, 256)]


def _h(rng, *shape, scale=1.0):
    return torch.from_numpy((rng.standard_normal(shape) * scale).astype(np.float32)).to(
        DEV, torch.float16)


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _close_rel(out, ref, rtol):
    err = np.abs(out - ref).max() / (np.abs(ref).max() + 1e-12)
    assert err <= rtol, f"max error {err:.2e} (relative to the max) > {rtol}"


@pytest.mark.parametrize("shape", SINTEL, ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_sintel_levels_fp16_corr9(shape):
    from pwcnet_amd.ops import corr_forward
    rng = np.random.default_rng(40 + shape[2])
    a, b = _h(rng, *shape), _h(rng, *shape)
    out = corr_forward(a, b, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    assert out.dtype == torch.float16 and tuple(out.shape) == (shape[0], 81) + shape[2:]
    _close_rel(_np(out), O.corr_forward(_np(a), _np(b), 9, 1, 9, 1, 2), 2e-3)


@pytest.mark.parametrize("shape", SINTEL[2:], ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_sintel_levels_fp16_warp(shape):
    from pwcnet_amd.ops import warp_forward
    rng = np.random.default_rng(50 + shape[2])
    x = _h(rng, *shape)
    f = _h(rng, shape[0], 2, shape[2], shape[3], scale=3.0)
    out = warp_forward(x, f)
    torch.cuda.synchronize()
    _close_rel(_np(out), O.warp_forward(_np(x), _np(f)), 2e-3)


def test_stress_192x224x32_fp16():
    """The north star's 192x224x32 correlation stress shape (labelled separately from the true
    level 2 = 112x256x32)."""
    from pwcnet_amd.ops import corr_forward
    rng = np.random.default_rng(77)
    a, b = _h(rng, 2, 32, 192, 224), _h(rng, 2, 32, 192, 224)
    out = corr_forward(a, b, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    _close_rel(_np(out), O.corr_forward(_np(a), _np(b), 9, 1, 9, 1, 2), 2e-3)


def test_stress_192x224x32_fp16_b16_matrix_cores():
    """The stress shape at the batch bench.py's `stress_192x224x32` line times (B = 16): the
    matrix-core strip kernel (two column strips, 128 + 96 px, the second one partial); images 0
    and 15 against the oracle."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward
    assert _lib.corr_forward_plan(16, 32, 192, 224, 9, 1, 9, 1, 2, 1) == "mstrip16"
    rng = np.random.default_rng(79)
    a, b = _h(rng, 16, 32, 192, 224), _h(rng, 16, 32, 192, 224)
    out = corr_forward(a, b, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    pick = [0, 15]
    _close_rel(_np(out[pick]), O.corr_forward(_np(a[pick]), _np(b[pick]), 9, 1, 9, 1, 2), 2e-3)


def test_stress_192x224x32_fp32():
    from pwcnet_amd.ops import corr_forward
    rng = np.random.default_rng(78)
    a = rng.standard_normal((2, 32, 192, 224)).astype(np.float32)
    b = rng.standard_normal((2, 32, 192, 224)).astype(np.float32)
    out = corr_forward(torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV), 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(out), O.corr_forward(a, b, 9, 1, 9, 1, 2), rtol=1e-5,
                               atol=1e-5)


@pytest.mark.parametrize("sr_cfg", ["corr4", "cvl"])
def test_stride1_full_size_l4_b8(sr_cfg):
    """Corr4 = Correlation(4, 1, 4, 1, 1) (the north star's literal d = 4) and CostVolumeLayer
    (sr = 4, modules.py:53-74) at config 2's l4 size (B=8, 32x96x112), fp32, full compare."""
    from pwcnet_amd.ops import corr_forward, cost_volume_forward
    rng = np.random.default_rng(88)
    a = rng.standard_normal((8, 32, 96, 112)).astype(np.float32)
    b = rng.standard_normal((8, 32, 96, 112)).astype(np.float32)
    ta, tb = torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV)
    if sr_cfg == "corr4":
        out, ref = corr_forward(ta, tb, 4, 1, 4, 1, 1), O.corr_forward(a, b, 4, 1, 4, 1, 1)
    else:
        out, ref = cost_volume_forward(ta, tb, 4), O.cvl_forward(a, b, 4)
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(out), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape,md,s2", [((8, 32, 112, 256), 9, 2), ((16, 64, 56, 128), 9, 2),
                                         ((8, 32, 112, 256), 4, 1), ((16, 32, 55, 128), 9, 2),
                                         ((12, 16, 54, 128), 4, 1)],
                         ids=["l4_corr9", "l3_corr9", "l4_corr4", "rows4_odd_h_tail",
                              "rows4_corr4_tail"])
def test_sintel_stream_fp16_channel_pairs(shape, md, s2):
    """Config-4 batch sizes that reach the stream kernel: its fp16 channel-pair form (loader
    interleaves channels c, c+1 into half2 dwords; v_dot2_f32_f16, fp32 sums) against the
    oracle.  The smaller grids take 4-row bands (l3; odd H and bands cut short at the image's
    last rows)."""
    from pwcnet_amd.ops import corr_forward
    rng = np.random.default_rng(60 + shape[2] + md)
    a, b = _h(rng, *shape), _h(rng, *shape)
    out = corr_forward(a, b, md, 1, md, 1, s2)
    torch.cuda.synchronize()
    ref = O.corr_forward(_np(a), _np(b), md, 1, md, 1, s2)
    _close_rel(_np(out), ref, 2e-3)


@pytest.mark.parametrize("shape", SINTEL[:2] + [(2, 192, 6, 7), (2, 128, 12, 14), (1, 24, 13, 15)],
                         ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_fused_band_fp16_coarse_levels(shape):
    """fp16 WarpCorrelation at the coarse levels runs as ONE band launch (model.py:80-83): its
    x2_warp equals the fp16 warp kernel's bit for bit (same fmaf chain, same rounding), the
    correlation reads x2_warp as stored (rounded to fp16, as the two-launch path does), and the
    volume matches the two-launch path (PWC_DEBUG fused=0) and the oracle on the fp16-rounded
    warp within the fp16 output rounding."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import warp_corr_forward, warp_forward
    B, C, H, W = shape
    rng = np.random.default_rng(60 + H)
    a, b = _h(rng, *shape), _h(rng, *shape)
    f = _h(rng, B, 2, H, W, scale=2.0)
    out, x2w = warp_corr_forward(a, b, f, 9, 1, 9, 1, 2)
    _lib.set_debug("fused=0")
    try:
        out2, x2w2 = warp_corr_forward(a, b, f, 9, 1, 9, 1, 2)
    finally:
        _lib.set_debug("")
    torch.cuda.synchronize()
    assert out.dtype == torch.float16 and x2w.dtype == torch.float16
    assert torch.equal(x2w, warp_forward(b, f)) and torch.equal(x2w, x2w2)
    _close_rel(_np(out), _np(out2), 2e-3)
    _close_rel(_np(out), O.corr_forward(_np(a), _np(x2w), 9, 1, 9, 1, 2), 2e-3)


def test_fused_band_fp16_group_pair_equals_single_calls():
    """Config 4's l0 + l1 as one paired launch (pwc_warp_corr_forward_group) equal their
    single-level fused calls bit for bit."""
    from pwcnet_amd.ops import warp_corr_forward, warp_corr_forward_group
    rng = np.random.default_rng(71)
    probs = []
    for (B, C, H, W) in SINTEL[:2]:
        probs.append((_h(rng, 4, C, H, W), _h(rng, 4, C, H, W), _h(rng, 4, 2, H, W, scale=2.0)))
    grouped = warp_corr_forward_group(probs, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    for (a, b, f), (c, w) in zip(probs, grouped):
        c1, w1 = warp_corr_forward(a, b, f, 9, 1, 9, 1, 2)
        assert torch.equal(c, c1) and torch.equal(w, w1)


# Stride 1 (Correlation(4, 1, 4, 1, 1) and CostVolumeLayer sr = 4) on the matrix cores
# (corr_mstrip16.hip, S1 geometries): config-4 l4 / l3 at B = 16, an odd height (a chunk cut
# short), a width that is not a multiple of the 128-px strip (partial second strip), both channel
# orders; against the oracle on the fp16 inputs within the fp16 output rounding, and against the
# VALU stream kernel (knob mstrip16_s1=0).
S1_CASES = [("corr4", (16, 32, 112, 256)), ("cvl", (16, 32, 112, 256)), ("corr4", (16, 64, 56, 128)),
            ("cvl", (16, 64, 56, 128)), ("corr4", (16, 96, 28, 64)), ("cvl", (16, 96, 28, 64)),
            ("corr4", (16, 32, 111, 256)), ("corr4", (24, 32, 56, 200))]


@pytest.mark.parametrize("cfg,shape", S1_CASES, ids=lambda v: v if isinstance(v, str) else "x".join(map(str, v)))
def test_stride1_matrix_cores_vs_oracle(cfg, shape):
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward, cost_volume_forward
    B, C, H, W = shape
    assert _lib.corr_forward_plan(B, C, H, W, 4, 1, 4, 1, 1, dtype=1) == "mstrip16"
    rng = np.random.default_rng(90 + H + W + C)
    a, b = _h(rng, *shape), _h(rng, *shape)

    def run():
        return corr_forward(a, b, 4, 1, 4, 1, 1) if cfg == "corr4" else cost_volume_forward(a, b, 4)
    out = run()
    torch.cuda.synchronize()
    an, bn = _np(a), _np(b)
    ref = O.corr_forward(an, bn, 4, 1, 4, 1, 1) if cfg == "corr4" else O.cvl_forward(an, bn, 4)
    _close_rel(_np(out), ref, 2e-3)
    _lib.set_debug("mstrip16_s1=0")
    try:
        alt = run()
    finally:
        _lib.set_debug("")
    torch.cuda.synchronize()
    err = float((out.float() - alt.float()).abs().max()) / float(alt.float().abs().max())
    assert err <= 2e-3, err
