"""The Net harness (pwcnet_amd/net.py) against a reduced end-to-end run of the reference's own
model.py (tests/golden/net_cvl_128x128.npz, gen_golden.py: Net with corr='CostVolumeLayer',
reference defaults, 128x128, weights from torch.manual_seed(0)).

CPU: the harness builds the same weights (per-parameter sums) and, with its hot-path layers
swapped for the torch-CPU restatement (oracle/torch_ref.py), reproduces the reference's flows.
GPU: the same harness on the HIP drop-ins (CostVolumeLayer, WarpingLayer and the fused
UpsampleWarp) reproduces them too; with model.py:24's GPU Correlation the fused forms
(UpsampleWarp + CorrelationCat) equal the plain drop-in sequence."""
import os
import warnings

import numpy as np
import pytest
import torch
from torch import nn

from conftest import GOLDEN
from oracle import torch_ref as T
from pwcnet_amd.net import Net, NetArgs

FIX = os.path.join(GOLDEN, "net_cvl_128x128.npz")


_RefWarp = T.RefWarpingLayer


def _RefCVL():
    return T.RefCostVolumeLayer(4)


class _RefCorr9(nn.Module):
    def forward(self, a, b):
        return T.correlation(a, b, 9, 1, 9, 1, 2)


def _net(corr="CostVolumeLayer"):
    torch.manual_seed(0)
    return Net(NetArgs(corr=corr))


def _flows(z):
    return [z[f"flow{i}"] for i in range(int(z["n_flows"]))]


def _check_flows(got, ref, rtol):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        g = g.detach().double().cpu().numpy()
        assert g.shape == r.shape
        err = np.abs(g - r).max() / (np.abs(r).max() + 1e-12)
        assert err <= rtol, f"flow {r.shape}: relative error {err:.2e} > {rtol}"


def test_harness_builds_the_reference_weights():
    z = np.load(FIX)
    net = _net()
    names = [k for k, _ in net.named_parameters()]
    assert names == list(z["param_names"])  # same module tree => state_dicts interchange
    sums = np.array([float(p.double().sum()) for p in net.parameters()])
    np.testing.assert_allclose(sums, z["param_sums"], rtol=1e-12, atol=1e-9)


def test_harness_cpu_restatement_matches_reference_flows():
    z = np.load(FIX)
    net = _net()
    net.warping_layer = _RefWarp()
    net.corr = _RefCVL()
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        flows, summ = net(torch.from_numpy(z["x"]), fused=False)
    _check_flows(flows, _flows(z), 1e-4)  # ulp-level sum-order differences, amplified by convs
    for i, w in enumerate(summ["x2_warps"]):  # sampled at the (ulp-perturbed) upstream flows
        np.testing.assert_allclose(w.numpy(), z[f"x2_warp{i}"], rtol=0,
                                   atol=1e-4 * np.abs(z[f"x2_warp{i}"]).max())


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
def test_harness_hip_cvl_matches_reference_flows(fused):
    z = np.load(FIX)
    net = _net().cuda()
    with torch.no_grad():
        flows, summ = net(torch.from_numpy(z["x"]).cuda(), fused=fused)
    torch.cuda.synchronize()
    # convolutions run on MIOpen (not part of this project): fp32 tolerance relative to max
    _check_flows(flows, _flows(z), 2e-4)
    assert len(summ["x2_warps"]) == 5


@pytest.mark.gpu
def test_harness_hip_correlation_fused_equals_plain_and_cpu():
    z = np.load(FIX)
    x = torch.from_numpy(z["x"])
    net = _net(corr="cost_volume").cuda()  # model.py:24's Correlation(9, 1, 9, 1, 2)
    with torch.no_grad():
        f_plain, _ = net(x.cuda(), fused=False)
        f_fused, _ = net(x.cuda(), fused=True)
    torch.cuda.synchronize()
    _check_flows(f_fused, [f.double().cpu().numpy() for f in f_plain], 1e-4)
    cpu = _net(corr="cost_volume")
    cpu.warping_layer = _RefWarp()
    cpu.corr = _RefCorr9()
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        f_cpu, _ = cpu(x, fused=False)
    _check_flows(f_plain, [f.double().numpy() for f in f_cpu], 2e-4)
