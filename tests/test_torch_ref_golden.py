"""CPU: pin oracle/torch_ref.py (the pure-PyTorch CPU path behind bench.py's cpu_baseline,
the Net-harness CPU reference and the ``--device cpu`` stand-in op) directly against the
reference's own outputs in tests/golden/ (gen_golden.py imported /root/reference to make them).

* ``cost_volume``   vs every CVL fixture, forward and autograd backward (modules.py:53-74).
* ``correlation``   (Corr4 = Correlation(4,1,4,1,1), Corr9 = Correlation(9,1,9,1,2) of
  model.py:24) through the CVL identities of SURVEY.md §8c: Corr*C == CVL[perm]*K, forward
  and backward (correlation_cuda_kernel.cu:34-290 semantics).
* ``warp``          vs every warp fixture, forward and autograd backward incl. d/dflow
  (modules.py:31-42, utils.py:3-8, torch-0.4 align_corners=True).
* ``upsample_flow`` + ``warp`` vs the upsample->warp fixtures (model.py:78-80).

All in fp32, as the reference computed them: tolerances are fp32-rounding sized.
"""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle as O
from oracle import torch_ref as R

CVL = sorted(glob.glob(os.path.join(GOLDEN, "cvl_*.npz")))
WARP = sorted(glob.glob(os.path.join(GOLDEN, "warp_*.npz")))
UPWARP = sorted(glob.glob(os.path.join(GOLDEN, "upwarp_*.npz")))


def _t(a, grad=False):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).requires_grad_(grad)


def _close(a, b, rtol=1e-5, atol=1e-5):
    a = a.detach().double().numpy() if isinstance(a, torch.Tensor) else a
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


@pytest.mark.parametrize("path", CVL, ids=os.path.basename)
def test_torch_ref_cost_volume_vs_reference(path):
    z = np.load(path)
    sr = int(z["sr"])
    src, tgt = _t(z["src"], True), _t(z["tgt"], True)
    out = R.cost_volume(src, tgt, sr)
    assert out.shape == z["out"].shape
    _close(out, z["out"])
    out.backward(_t(z["gout"]))
    _close(src.grad, z["gsrc"], atol=2e-5)
    _close(tgt.grad, z["gtgt"], atol=2e-5)


@pytest.mark.parametrize("path", CVL, ids=os.path.basename)
def test_torch_ref_correlation_pinned_by_cvl(path):
    z = np.load(path)
    sr = int(z["sr"])
    if sr == 4:
        pad = md = 4
        s2 = 1
    elif sr == 8:
        pad = md = 9
        s2 = 2
    else:
        pytest.skip("no correlation counterpart")
    C = z["src"].shape[1]
    K = (2 * sr + 1) ** 2
    idx = O.corr_channel_from_cvl(sr, s2, md)
    f1, f2 = _t(z["src"], True), _t(z["tgt"], True)
    corr = R.correlation(f1, f2, pad, 1, md, 1, s2)
    assert corr.shape == (z["src"].shape[0], 81) + z["src"].shape[2:]
    _close(corr * C, z["out"][:, idx] * K, atol=2e-5)
    # backward: sum(corr * G) pulls back to the CVL gradient of G scattered onto idx
    G = np.random.default_rng(1).standard_normal(tuple(corr.shape)).astype(np.float32)
    corr.backward(_t(G))
    Gc = np.zeros(z["out"].shape)
    Gc[:, idx] = G * K / C
    e1, e2 = O.cvl_backward(z["src"], z["tgt"], Gc, sr)
    _close(f1.grad, e1, atol=2e-5)
    _close(f2.grad, e2, atol=2e-5)


@pytest.mark.parametrize("path", WARP, ids=os.path.basename)
def test_torch_ref_warp_vs_reference(path):
    z = np.load(path)
    x, flow = _t(z["x"], True), _t(z["flow"], True)
    out = R.warp(x, flow)
    _close(out, z["out"], atol=2e-5)
    out.backward(_t(z["gout"]))
    _close(x.grad, z["gx"], atol=2e-5)
    _close(flow.grad, z["gflow"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("path", UPWARP, ids=os.path.basename)
def test_torch_ref_upsample_warp_vs_reference(path):
    z = np.load(path)
    x2, flow = _t(z["x2"], True), _t(z["flow"], True)
    fup = R.upsample_flow(flow)
    _close(fup, z["flow_up"], rtol=1e-6, atol=1e-5)
    out = R.warp(x2, fup)
    _close(out, z["out"])
    torch.autograd.backward([out, fup], [_t(z["gout"]), _t(z["gflow_up"])])
    _close(x2.grad, z["gx2"], rtol=1e-4, atol=1e-4)
    _close(flow.grad, z["gflow"], rtol=1e-4, atol=1e-4)


def test_torch_ref_get_grid_is_utils_py():
    # utils.py:3-8: channel 0 = linspace(-1, 1, W) along x, channel 1 = linspace(-1, 1, H)
    x = torch.zeros(2, 3, 5, 7)
    g = R.get_grid(x)
    assert g.shape == (2, 2, 5, 7)
    # torch.linspace, as utils.py calls it (its fp32 values differ from numpy's in the last ulp)
    assert torch.equal(g[1, 0, 3], torch.linspace(-1.0, 1.0, 7))
    assert torch.equal(g[0, 1, :, 4], torch.linspace(-1.0, 1.0, 5))
    np.testing.assert_allclose(g[1, 0, 3].numpy(), np.linspace(-1, 1, 7), atol=1e-7)


def test_torch_ref_modules_match_functions():
    rng = np.random.default_rng(5)
    src = _t(rng.standard_normal((1, 8, 6, 7)))
    tgt = _t(rng.standard_normal((1, 8, 6, 7)))
    flow = _t(rng.standard_normal((1, 2, 6, 7)) * 2)
    assert torch.equal(R.RefCostVolumeLayer(4)(src, tgt), R.cost_volume(src, tgt, 4))
    assert torch.equal(R.RefWarpingLayer()(tgt, flow), R.warp(tgt, flow))
