"""CPU: .flo I/O and flow visualisation (pwcnet_amd.flow_io, restating flow_utils.py).

The reference module imports cv2 at import time (absent here), so vis_flow is checked by
known answers of the Middlebury colour coding, not against the reference run: parity
unpinned for vis_flow; load/save follow the published .flo layout byte for byte."""
import os
import struct

import numpy as np
import pytest

from pwcnet_amd.flow_io import flow_to_hwc, load_flow, save_flow, vis_flow


def test_flo_round_trip_and_layout(tmp_path):
    rng = np.random.default_rng(0)
    flow = rng.standard_normal((5, 7, 2)).astype(np.float32)
    p = tmp_path / "a.flo"
    save_flow(str(p), flow)
    raw = p.read_bytes()
    assert len(raw) == 12 + 5 * 7 * 2 * 4
    magic, w, h = struct.unpack("<fii", raw[:12])
    assert (magic, w, h) == (202021.25, 7, 5)
    assert np.frombuffer(raw[12:], np.float32).tolist() == flow.ravel().tolist()
    back = load_flow(str(p))
    assert back.dtype == np.float32 and back.shape == (5, 7, 2)
    assert np.array_equal(back, flow)


def test_flo_bad_magic_returns_none(tmp_path):
    p = tmp_path / "b.flo"
    p.write_bytes(struct.pack("<fii", 1.0, 2, 2) + b"\0" * 32)
    assert load_flow(str(p)) is None


def test_flow_to_hwc():
    a = np.arange(2 * 2 * 3 * 4, dtype=np.float32).reshape(2, 2, 3, 4)
    out = flow_to_hwc(a)
    assert len(out) == 2 and out[1].shape == (3, 4, 2)
    assert out[1][2, 3, 1] == a[1, 1, 2, 3]


def test_vis_flow_known_answers():
    flow = np.zeros((2, 3, 2), np.float32)
    flow[0, 0] = (1.0, 0.0)   # max radius: saturated colour
    flow[0, 1] = (-1.0, 0.0)
    flow[1, 2] = (0.0, 0.0)   # zero flow: white
    img = vis_flow(flow)
    assert img.shape == (2, 3, 3) and img.dtype == np.uint8
    assert img[1, 2].tolist() == [255, 255, 255]
    # Middlebury wheel at angle atan2(-v, -u): +u (right) is the wheel's first entry (pure
    # red), -u sits opposite (cyan/blue side)
    assert img[0, 0].tolist() == [255, 0, 0]
    assert img[0, 1][2] > img[0, 1][0]
    # unknown flow (> 1e9) is zeroed and the input array is left untouched
    f2 = flow.copy()
    f2[0, 2] = (2e9, 0.0)
    img2 = vis_flow(f2)
    assert f2[0, 2, 0] == 2e9
    assert np.array_equal(img2, img)


def test_vis_flow_matches_reference_fixture():
    """flow_utils.vis_flow run in the build container (cv2 stubbed; gen_golden.py) on a flow
    with unknown (> 1e9) entries and a zero vector: identical uint8 image."""
    import os
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "visflow_20x24.npz"))
    img = vis_flow(z["flow"])
    assert img.dtype == np.uint8 and img.shape == z["img"].shape
    np.testing.assert_array_equal(img, z["img"])
