"""CPU: pin the oracle (oracle/pwc_oracle.c) against the reference's own outputs.

Fixtures in tests/golden/ come from /root/reference/modules.py (CostVolumeLayer, WarpingLayer
with torch-0.4 align_corners=True semantics) via tests/golden/gen_golden.py.  The reference
computes in fp32, the oracle in fp64: tolerances are fp32-rounding sized.

The CUDA Correlation cannot run here; it is pinned through the CVL fixtures
(SURVEY.md §8c): Corr(pad=md=4,s2=1)*C == CVL(sr=4)[perm]*81 and
Corr(pad=md=9,s2=2)*C == CVL(sr=8)[perm, even offsets]*289, forward and backward.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O

CVL = sorted(glob.glob(os.path.join(GOLDEN, "cvl_*.npz")))
WARP = sorted(glob.glob(os.path.join(GOLDEN, "warp_*.npz")))


def _close(a, b, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


@pytest.mark.parametrize("path", CVL, ids=os.path.basename)
def test_cvl_forward_backward_vs_reference(path):
    z = np.load(path)
    sr = int(z["sr"])
    _close(O.cvl_forward(z["src"], z["tgt"], sr), z["out"])
    gs, gt = O.cvl_backward(z["src"], z["tgt"], z["gout"], sr)
    _close(gs, z["gsrc"], atol=1e-5)
    _close(gt, z["gtgt"], atol=1e-5)


@pytest.mark.parametrize("path", CVL, ids=os.path.basename)
def test_correlation_pinned_by_cvl(path):
    z = np.load(path)
    sr = int(z["sr"])
    src, tgt = z["src"], z["tgt"]
    C = src.shape[1]
    K = (2 * sr + 1) ** 2
    if sr == 4:  # Corr4 = Correlation(4, 1, 4, 1, 1)
        pad = md = 4
        s2 = 1
    elif sr == 8:  # Corr9 = Correlation(9, 1, 9, 1, 2): model.py:24 at search_range=4
        pad = md = 9
        s2 = 2
    else:
        pytest.skip("no correlation counterpart")
    idx = O.corr_channel_from_cvl(sr, s2, md)
    corr = O.corr_forward(src, tgt, pad, 1, md, 1, s2)
    _close(corr * C, z["out"][:, idx] * K, atol=1e-5)
    # backward: d/d(in) of sum(corr * G) == CVL grads with upstream grad scattered to idx
    G = np.random.default_rng(0).standard_normal(corr.shape)
    g1, g2 = O.corr_backward(src, tgt, G, pad, 1, md, 1, s2)
    Gc = np.zeros(z["out"].shape)
    Gc[:, idx] = G * K / C
    e1, e2 = O.cvl_backward(src, tgt, Gc, sr)
    _close(g1, e1, atol=1e-9)
    _close(g2, e2, atol=1e-9)


@pytest.mark.parametrize("path", WARP, ids=os.path.basename)
def test_warp_vs_reference(path):
    z = np.load(path)
    _close(O.warp_forward(z["x"], z["flow"]), z["out"], atol=2e-5)
    gx, gf = O.warp_backward(z["x"], z["flow"], z["gout"])
    _close(gx, z["gx"], atol=2e-5)
    # the oracle restates the reference's fp32 grid chain, so even zero flow (every sample on
    # an integer coordinate, one-sided derivative) picks the reference's side
    _close(gf, z["gflow"], rtol=1e-4, atol=1e-4)


def test_corr_shape_math():
    # correlation_cuda.c:20-34
    assert O.corr_output_shape(96, 112, 9, 1, 9, 1, 2) == (81, 96, 112)
    assert O.corr_output_shape(96, 112, 4, 1, 4, 1, 1) == (81, 96, 112)
    assert O.corr_output_shape(20, 30, 0, 1, 4, 1, 1) == (81, 12, 22)
    # k=3 -> kr=1, br=3: Ho = ceil((20+6-6)/2) = 10, Wo = ceil((30+6-6)/2) = 15
    assert O.corr_output_shape(20, 30, 3, 3, 2, 2, 1) == (25, 10, 15)
    assert O.corr_output_shape(21, 31, 3, 3, 2, 2, 1) == (25, 11, 16)  # ceil(10.5)


UPWARP = sorted(glob.glob(os.path.join(GOLDEN, "upwarp_*.npz")))


@pytest.mark.parametrize("path", UPWARP, ids=os.path.basename)
def test_upsample_warp_vs_reference(path):
    # model.py:78 (F.upsample x2, align_corners=False, * 2) + :80 (WarpingLayer), reference run
    z = np.load(path)
    out, fup = O.upsample_warp_forward(z["x2"], z["flow"])
    np.testing.assert_allclose(fup, z["flow_up"], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(out, z["out"], rtol=1e-5, atol=1e-5)
    gx, gf = O.upsample_warp_backward(z["x2"], z["flow"], z["gout"], z["gflow_up"])
    np.testing.assert_allclose(gx, z["gx2"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(gf, z["gflow"], rtol=1e-4, atol=1e-4)


def test_flow_upsample_adjoint():
    # <up(f), g> == <f, up^T(g)>: the backward is the exact adjoint of the forward
    rng = np.random.default_rng(3)
    f = rng.standard_normal((2, 2, 5, 7))
    g = rng.standard_normal((2, 2, 10, 14))
    lhs = float((O.flow_upsample2(f) * g).sum())
    rhs = float((f * O.flow_upsample2_backward(g)).sum())
    assert abs(lhs - rhs) <= 1e-9 * max(1.0, abs(lhs))
