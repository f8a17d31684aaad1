"""Config 5 (BASELINE.json: training step, B=8 384x448): tools/train_bench.py's own step
functions -- the dependency-order headline and the grouped-forward mode, exactly the calls it
times -- against the C oracle (oracle/pwc_oracle.c: correlation_cuda_kernel.cu:34-290 and
ATen's grid_sampler_2d forward/backward, float64) on the same inputs.

The oracle recomputes pairs 0 and 7 of the batch at every level (pairs are independent, so a
sub-batch is the same arithmetic); every output -- volume, d/dx1, d/dx2, d/dflow -- must be
within 1e-4 of it (max |gpu - oracle| / (1 + |oracle|), fp32 against float64).
"""
import importlib.util
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

_spec = importlib.util.spec_from_file_location("train_bench",
                                               os.path.join(ROOT, "tools", "train_bench.py"))
TB = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(TB)

PAIRS = [0, 7]
TOL = 1e-4


def _oracle_level(lv, pairs):
    from oracle import oracle as O
    sel = lambda t: t[pairs].detach().double().cpu().numpy()  # noqa: E731
    x1, x2, fl, gc = sel(lv["x1"]), sel(lv["x2"]), sel(lv["fl"]), sel(lv["gc"])
    x2w = O.warp_forward(x2, fl)
    corr = O.corr_forward(x1, x2w, 9, 1, 9, 1, 2)
    g1, g2w = O.corr_backward(x1, x2w, gc, 9, 1, 9, 1, 2)
    gx2, gfl = O.warp_backward(x2, fl, g2w)
    return dict(corr=corr, g1=g1, gx2=gx2, gfl=gfl)


def _rel(a, b):
    a = a.detach().double().cpu().numpy()
    assert a.shape == b.shape and np.isfinite(a).all()
    return float((np.abs(a - b) / (1 + np.abs(b))).max())


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["dependency", "grouped"])
def test_config5_train_step_matches_oracle(mode):
    dev = torch.device("cuda:0")
    shapes = TB.bench.level_shapes(384, 448)
    s = TB.make_set(8, shapes, dev, torch.Generator(device=dev).manual_seed(11))
    fn = TB.step_dependency if mode == "dependency" else TB.step_grouped
    fn(s, {0, 1})
    torch.cuda.synchronize()
    for l, lv in enumerate(s):
        ref = _oracle_level(lv, PAIRS)
        for k in TB.OUTPUTS:
            err = _rel(lv[k][PAIRS], ref[k])
            assert err <= TOL, f"{mode} l{l} {k}: {err:.2e} > {TOL}"


@pytest.mark.gpu
def test_train_bench_self_check_and_kernel_table():
    args = TB.parse_args(["--steps", "3", "--warmup", "2", "--batch", "2"])
    out = TB.run(args)
    assert out["checks"]["self_check"]["ok"], out["checks"]
    assert out["grouped"]["self_check"]["ok"], out["grouped"]
    ops = {(r["level"], r["op"]) for r in out["kernels"]}
    assert (4, "corr_fwd") in ops and (4, "corr_bwd") in ops and (4, "warp_bwd") in ops
    assert (0, "warp_corr_fwd") in ops
    assert all(r["us"] > 0 and r["frac_8TBs"] > 0 for r in out["kernels"])
