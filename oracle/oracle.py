"""CPU oracle for the PWC-Net correlation / warp hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker (or the timed CPU baseline), never as the
thing measured or shipped.  The product path (``pwc-net_pytorch_amd/``) never imports it.

numpy in / numpy out.  The C restatement lives in ``oracle/pwc_oracle.c``; each function
here names the reference lines it follows (see that file's header).  ``dtype=np.float64``
(default) is the parity oracle; ``np.float32`` is the fp32 CPU port timed by bench.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "build")
_LIBS: dict = {}


def build() -> None:
    """Compile both oracle libraries (gcc; see oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _lib(dtype) -> ctypes.CDLL:
    key = np.dtype(dtype).name
    if key not in ("float64", "float32"):
        raise TypeError(f"oracle supports float64/float32, got {key}")
    if key in _LIBS:
        return _LIBS[key]
    path = os.path.join(_BUILD, "liboracle_f64.so" if key == "float64" else "liboracle_f32.so")
    if not os.path.exists(path):
        build()
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    I = ctypes.c_int
    lib.oracle_corr_forward.argtypes = [P, P, P] + [I] * 9
    lib.oracle_corr_backward.argtypes = [P, P, P, P, P] + [I] * 9
    lib.oracle_warp_forward.argtypes = [P, P, P] + [I] * 4
    lib.oracle_warp_backward.argtypes = [P, P, P, P, P] + [I] * 4
    lib.oracle_cvl_forward.argtypes = [P, P, P] + [I] * 5
    lib.oracle_cvl_backward.argtypes = [P, P, P, P, P] + [I] * 5
    lib.oracle_corr_output_shape.argtypes = [I] * 7 + [ctypes.POINTER(I)] * 3
    lib.oracle_cvl_offsets.argtypes = [I, ctypes.POINTER(I), ctypes.POINTER(I)]
    lib.oracle_num_threads.restype = I
    lib.oracle_set_num_threads.argtypes = [I]
    _LIBS[key] = lib
    return lib


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def set_num_threads(n: int, dtype=np.float64) -> None:
    _lib(dtype).oracle_set_num_threads(int(n))


def num_threads(dtype=np.float64) -> int:
    return int(_lib(dtype).oracle_num_threads())


def corr_output_shape(H, W, pad, k, md, s1, s2):
    """correlation_cuda.c:20-34 -> (OC, Ho, Wo)."""
    lib = _lib(np.float64)
    oc, oh, ow = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib.oracle_corr_output_shape(H, W, pad, k, md, s1, s2, ctypes.byref(oc), ctypes.byref(oh),
                                 ctypes.byref(ow))
    return oc.value, oh.value, ow.value


def corr_forward(in1, in2, pad, k, md, s1, s2, dtype=np.float64):
    """correlation_cuda_kernel.cu:34-106 (values), correlation_cuda.c:20-34 (shape)."""
    a, b = _c(in1, dtype), _c(in2, dtype)
    B, C, H, W = a.shape
    assert b.shape == a.shape
    OC, Ho, Wo = corr_output_shape(H, W, pad, k, md, s1, s2)
    out = np.zeros((B, OC, Ho, Wo), dtype=dtype)
    _lib(dtype).oracle_corr_forward(_p(a), _p(b), _p(out), B, C, H, W, pad, k, md, s1, s2)
    return out


def corr_backward(in1, in2, gout, pad, k, md, s1, s2, dtype=np.float64):
    """correlation_cuda_kernel.cu:108-290; defined by the reference only for stride1 == 1."""
    if s1 != 1:
        raise ValueError("reference correlation backward is only defined for stride1 == 1")
    a, b = _c(in1, dtype), _c(in2, dtype)
    B, C, H, W = a.shape
    OC, Ho, Wo = corr_output_shape(H, W, pad, k, md, s1, s2)
    g = _c(gout, dtype)
    assert g.shape == (B, OC, Ho, Wo), (g.shape, (B, OC, Ho, Wo))
    g1 = np.zeros_like(a)
    g2 = np.zeros_like(b)
    _lib(dtype).oracle_corr_backward(_p(a), _p(b), _p(g), _p(g1), _p(g2), B, C, H, W, pad, k,
                                     md, s1, s2)
    return g1, g2


def warp_forward(x, flow, dtype=np.float64):
    """modules.py:31-42 + utils.py:3-8 with torch-0.4 grid_sample (align_corners=True)."""
    a, f = _c(x, dtype), _c(flow, dtype)
    B, C, H, W = a.shape
    assert f.shape == (B, 2, H, W)
    out = np.zeros_like(a)
    _lib(dtype).oracle_warp_forward(_p(a), _p(f), _p(out), B, C, H, W)
    return out


def warp_backward(x, flow, gout, dtype=np.float64):
    """Gradients of warp_forward wrt x and flow (ATen grid_sampler_2d_backward formulas)."""
    a, f, g = _c(x, dtype), _c(flow, dtype), _c(gout, dtype)
    B, C, H, W = a.shape
    gx = np.zeros_like(a)
    gf = np.zeros_like(f)
    _lib(dtype).oracle_warp_backward(_p(a), _p(f), _p(g), _p(gx), _p(gf), B, C, H, W)
    return gx, gf


def _up2_taps(n_out, n_in):
    """ATen upsample_bilinear2d source taps along one axis for a x2 upsample with
    align_corners=False (area_pixel_compute_source_index: 0.5*(d+0.5)-0.5 clamped at 0;
    i1 = i0 + (i0 < n_in-1); lambda1 = src - i0) -- torch 0.4's F.upsample default, used by
    model.py:78."""
    d = np.arange(n_out, dtype=np.float64)
    src = np.maximum(0.5 * (d + 0.5) - 0.5, 0.0)
    i0 = src.astype(np.int64)
    i1 = i0 + (i0 < n_in - 1)
    l1 = src - i0
    return i0, i1, 1.0 - l1, l1


def flow_upsample2(flow, dtype=np.float64):
    """model.py:78: F.upsample(flow, scale_factor=2, mode='bilinear') * 2 (numpy)."""
    f = _c(flow, dtype)
    B, two, h, w = f.shape
    y0, y1, ly0, ly1 = _up2_taps(2 * h, h)
    x0, x1, lx0, lx1 = _up2_taps(2 * w, w)
    ly0, ly1 = ly0[:, None], ly1[:, None]
    top = lx0 * f[:, :, y0][:, :, :, x0] + lx1 * f[:, :, y0][:, :, :, x1]
    bot = lx0 * f[:, :, y1][:, :, :, x0] + lx1 * f[:, :, y1][:, :, :, x1]
    return ((ly0 * top + ly1 * bot) * 2).astype(dtype)


def flow_upsample2_backward(grad_up, dtype=np.float64):
    """Adjoint of flow_upsample2 (ATen upsample_bilinear2d_backward scatter, times 2)."""
    g = _c(grad_up, dtype) * 2
    B, two, H, W = g.shape
    h, w = H // 2, W // 2
    y0, y1, ly0, ly1 = _up2_taps(H, h)
    x0, x1, lx0, lx1 = _up2_taps(W, w)
    out = np.zeros((B, two, h, w), dtype)
    for oy in range(H):
        for (yy, wy) in ((y0[oy], ly0[oy]), (y1[oy], ly1[oy])):
            for (xx, wx) in ((x0, lx0), (x1, lx1)):
                np.add.at(out, (slice(None), slice(None), yy, xx), g[:, :, oy, :] * (wy * wx))
    return out


def upsample_warp_forward(x2, flow_coarse, dtype=np.float64):
    """model.py:78 + :80: (x2_warp, flow_up)."""
    fup = flow_upsample2(flow_coarse, dtype)
    return warp_forward(x2, fup, dtype), fup


def upsample_warp_backward(x2, flow_coarse, gout, gflow_up=None, dtype=np.float64):
    """Gradients of upsample_warp_forward wrt x2 and the coarse flow for upstream gradients of
    x2_warp (gout) and of flow_up (gflow_up, optional)."""
    fup = flow_upsample2(flow_coarse, dtype)
    gx, gf = warp_backward(x2, fup, gout, dtype)
    if gflow_up is not None:
        gf = gf + _c(gflow_up, dtype)
    return gx, flow_upsample2_backward(gf, dtype)


def cvl_offsets(sr):
    """(dy, dx) of each CostVolumeLayer channel, modules.py:58-72."""
    K = (2 * sr + 1) ** 2
    dy = (ctypes.c_int * K)()
    dx = (ctypes.c_int * K)()
    _lib(np.float64).oracle_cvl_offsets(sr, dy, dx)
    return list(dy), list(dx)


def cvl_forward(src, tgt, sr, dtype=np.float64):
    """CostVolumeLayer.forward, modules.py:53-74."""
    a, b = _c(src, dtype), _c(tgt, dtype)
    B, C, H, W = a.shape
    K = (2 * sr + 1) ** 2
    out = np.zeros((B, K, H, W), dtype=dtype)
    _lib(dtype).oracle_cvl_forward(_p(a), _p(b), _p(out), B, C, H, W, sr)
    return out


def cvl_backward(src, tgt, gout, sr, dtype=np.float64):
    """Autograd of CostVolumeLayer.forward."""
    a, b, g = _c(src, dtype), _c(tgt, dtype), _c(gout, dtype)
    B, C, H, W = a.shape
    ga = np.zeros_like(a)
    gb = np.zeros_like(b)
    _lib(dtype).oracle_cvl_backward(_p(a), _p(b), _p(g), _p(ga), _p(gb), B, C, H, W, sr)
    return ga, gb


def corr_channel_from_cvl(sr: int, s2: int = 1, md: int | None = None):
    """Permutation mapping Correlation (raster) channels to CostVolumeLayer channels.

    Correlation(pad=md, k=1, md, s1=1, s2) channel tc = (tj+dr)*D + (ti+dr) holds the
    displacement (dy, dx) = (tj*s2, ti*s2) (cu:74-78, 98).  Returns idx such that
    corr[:, tc] * C == cvl[:, idx[tc]] * K for the CVL with search range ``sr``.
    """
    if md is None:
        md = sr
    dr = md // s2
    D = 2 * dr + 1
    dys, dxs = cvl_offsets(sr)
    lut = {(dy, dx): k for k, (dy, dx) in enumerate(zip(dys, dxs))}
    idx = []
    for tc in range(D * D):
        tj, ti = tc // D - dr, tc % D - dr
        idx.append(lut[(tj * s2, ti * s2)])
    return idx
