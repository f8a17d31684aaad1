"""Optical-flow file I/O and visualisation for the `pred` harness.

Restates daigo0927/PWC-Net_pytorch flow_utils.py (numpy only; the reference module imports cv2
at the top, which is absent here, so it is not importable):

  load_flow(path)  <- flow_utils.py:5-13   Middlebury .flo: float32 magic 202021.25, int32 width,
                                           int32 height, then H*W*2 float32 (u, v interleaved);
                                           returns an H x W x 2 float32 array, or None when the
                                           magic does not match (the reference's behaviour)
  save_flow(path, flow) <- flow_utils.py:15-21  the same layout, flow as H x W x 2 float32
  vis_flow(flow)   <- flow_utils.py:114-149 (+ makeColorwheel :28-77, computeColor :80-111):
                                           Middlebury colour coding, H x W x 3 uint8 (RGB)

One deliberate difference: the reference's vis_flow zeroes unknown flow (> 1e9) and NaNs *in
the caller's array* (u, v are views of `flow`); this one works on a copy.
"""
from __future__ import annotations

import sys

import numpy as np

__all__ = ["load_flow", "save_flow", "vis_flow", "flow_to_hwc"]

_MAGIC = 202021.25


def load_flow(path):
    with open(path, "rb") as f:
        magic = np.fromfile(f, np.float32, count=1)
        if magic.size != 1 or float(magic[0]) != _MAGIC:
            return None
        w = int(np.fromfile(f, np.int32, count=1)[0])
        h = int(np.fromfile(f, np.int32, count=1)[0])
        data = np.fromfile(f, np.float32, count=h * w * 2)
        if data.size != h * w * 2:
            raise ValueError(f"{path}: truncated .flo ({data.size} of {h * w * 2} values)")
        return data.reshape(h, w, 2)


def save_flow(path, flow):
    flow = np.ascontiguousarray(flow, dtype=np.float32)
    if flow.ndim != 3 or flow.shape[2] != 2:
        raise ValueError(f"save_flow: expected H x W x 2, got {flow.shape}")
    h, w = flow.shape[:2]
    with open(path, "wb") as f:
        np.array([_MAGIC], np.float32).tofile(f)
        np.array([w], np.int32).tofile(f)
        np.array([h], np.int32).tofile(f)
        flow.tofile(f)


def flow_to_hwc(flow):
    """B x 2 x H x W or 2 x H x W tensor/array (the network's layout) -> H x W x 2 numpy
    (per image), the layout load_flow / save_flow / vis_flow use (main.py:267-287)."""
    a = flow.detach().cpu().numpy() if hasattr(flow, "detach") else np.asarray(flow)
    if a.ndim == 4:
        return [np.ascontiguousarray(x.transpose(1, 2, 0)) for x in a]
    return np.ascontiguousarray(a.transpose(1, 2, 0))


def _colorwheel():
    RY, YG, GC, CB, BM, MR = 15, 6, 4, 11, 13, 6
    wheel = np.zeros([RY + YG + GC + CB + BM + MR, 3])
    col = 0
    wheel[0:RY, 0] = 255
    wheel[0:RY, 1] = np.floor(255 * np.arange(0, RY, 1) / RY)
    col += RY
    wheel[col:col + YG, 0] = 255 - np.floor(255 * np.arange(0, YG, 1) / YG)
    wheel[col:col + YG, 1] = 255
    col += YG
    wheel[col:col + GC, 1] = 255
    wheel[col:col + GC, 2] = np.floor(255 * np.arange(0, GC, 1) / GC)
    col += GC
    wheel[col:col + CB, 1] = 255 - np.floor(255 * np.arange(0, CB, 1) / CB)
    wheel[col:col + CB, 2] = 255
    col += CB
    wheel[col:col + BM, 2] = 255
    wheel[col:col + BM, 0] = np.floor(255 * np.arange(0, BM, 1) / BM)
    col += BM
    wheel[col:col + MR, 2] = 255 - np.floor(255 * np.arange(0, MR, 1) / MR)
    wheel[col:col + MR, 0] = 255
    return wheel


def _compute_color(u, v):
    wheel = _colorwheel()
    bad = np.isnan(u) | np.isnan(v)
    u[bad] = 0
    v[bad] = 0
    ncols = wheel.shape[0]
    radius = np.sqrt(u ** 2 + v ** 2)
    a = np.arctan2(-v, -u) / np.pi
    fk = (a + 1) / 2 * (ncols - 1)
    k0 = fk.astype(np.uint8)
    k1 = k0 + 1
    k1[k1 == ncols] = 0
    f = fk - k0
    img = np.empty([k1.shape[0], k1.shape[1], 3])
    for i in range(wheel.shape[1]):
        col0 = wheel[:, i][k0] / 255
        col1 = wheel[:, i][k1] / 255
        col = (1 - f) * col0 + f * col1
        idx = radius <= 1
        col[idx] = 1 - radius[idx] * (1 - col[idx])  # saturation grows with radius
        col[~idx] *= 0.75  # out of range
        img[:, :, 2 - i] = np.floor(255 * col).astype(np.uint8)
    return img.astype(np.uint8)


def vis_flow(flow):
    """H x W x 2 flow -> H x W x 3 uint8 Middlebury colour image (RGB channel order)."""
    eps = sys.float_info.epsilon
    u = np.array(flow[:, :, 0], dtype=np.float64 if flow.dtype == np.float64 else np.float32)
    v = np.array(flow[:, :, 1], dtype=u.dtype)
    big = (u > 1e9) | (v > 1e9)  # UNKNOWN_FLOW_THRESH
    u[big] = 0
    v[big] = 0
    rad = np.sqrt(u * u + v * v)
    maxrad = max(-1, np.amax(rad))
    u = u / (maxrad + eps)
    v = v / (maxrad + eps)
    return _compute_color(u, v)[:, :, [2, 1, 0]]
