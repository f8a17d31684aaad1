"""The `pred` harness (tools/pred.py; main.py:310-362, flow_utils.py:15-21,114-149).

CPU: the centre crop is main.py:321-327's StaticCenterCrop (it reproduces the committed config-1
crops of example/1.png, 2.png from their known offsets), the input stacking is model.py:48-56's
B x 3 x 2 x H x W, and the outputs round-trip (.flo via load_flow, the PNG is vis_flow's image).
GPU: config 1's workload -- the example pair at 384x448 -- runs through the HIP drop-ins and
its flows match the reference's CPU path (oracle/torch_ref.reference_cpu_net: CostVolumeLayer +
grid_sample, same seed) within the Net-harness tolerance; the end-to-end tool writes both files.
"""
import importlib.util
import os
import warnings

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT

_spec = importlib.util.spec_from_file_location("pred", os.path.join(ROOT, "tools", "pred.py"))
pred = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(pred)


def test_center_crop_is_static_center_crop():
    img = np.arange(436 * 1024 * 3, dtype=np.int64).reshape(436, 1024, 3)
    c = pred.center_crop(img, (384, 448))
    assert c.shape == (384, 448, 3)
    # main.py:327: rows (436-384)//2 = 26 .. 410, columns (1024-448)//2 = 288 .. 736
    np.testing.assert_array_equal(c, img[26:410, 288:736])
    with pytest.raises(ValueError):
        pred.center_crop(img, (500, 448))


def test_example_pair_and_input_layout():
    frames = pred.read_pair(None, (384, 448))
    assert [f.shape for f in frames] == [(384, 448, 3)] * 2
    x = pred.to_input(frames)
    assert x.shape == (1, 3, 2, 384, 448) and x.dtype == np.float32
    # model.py:55-56: frame k = x[:, :, k]
    np.testing.assert_array_equal(x[0, :, 1], frames[1].transpose(2, 0, 1))
    # a smaller crop of the crops keeps the centre
    small = pred.read_pair(None, (64, 96))
    np.testing.assert_array_equal(small[0], frames[0][160:224, 176:272])


def test_outputs_round_trip(tmp_path):
    from PIL import Image
    from pwcnet_amd.flow_io import load_flow, vis_flow
    rng = np.random.default_rng(0)
    flow = (rng.standard_normal((20, 24, 2)) * 3).astype(np.float32)
    png = pred.write_outputs(flow, str(tmp_path / "sub" / "f.flo"))
    np.testing.assert_array_equal(load_flow(str(tmp_path / "sub" / "f.flo")), flow)
    np.testing.assert_array_equal(np.array(Image.open(png)), vis_flow(flow))


def _check_flows(got, ref, rtol):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        g = g.detach().double().cpu().numpy()
        r = r.detach().double().cpu().numpy()
        assert g.shape == r.shape
        err = np.abs(g - r).max() / (np.abs(r).max() + 1e-12)
        assert err <= rtol, f"flow {r.shape}: relative error {err:.2e} > {rtol}"


@pytest.mark.gpu
def test_config1_pair_on_hip_matches_cpu_reference_path():
    from oracle import torch_ref as T
    x = pred.to_input(pred.read_pair(None, (384, 448)))

    class A:
        corr, load, seed = "CostVolumeLayer", None, 0

    net = pred.build_net(A, "cuda")
    flow, flows = pred.predict(net, x, "cuda")
    torch.cuda.synchronize()
    assert flow.shape == (384, 448, 2) and np.isfinite(flow).all()
    cpu = T.reference_cpu_net(seed=0)
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref, _ = cpu(torch.from_numpy(x), fused=False)
    # convolutions run on MIOpen: the Net-harness tolerance (fp32, relative to the max)
    _check_flows(flows, ref, 2e-4)


@pytest.mark.gpu
def test_pred_tool_end_to_end(tmp_path):
    from pwcnet_amd.flow_io import load_flow
    out = str(tmp_path / "example.flo")
    pred.main(["--output", out])
    flow = load_flow(out)
    assert flow.shape == (384, 448, 2) and np.isfinite(flow).all()
    assert os.path.getsize(os.path.splitext(out)[0] + ".png") > 0
