"""GPU parity of the fused warp -> correlation path (model.py:80-83 as one call,
``pwc_warp_corr_forward`` / ``WarpCorrelation``) against the CPU oracle chain
``oracle.warp_forward`` -> ``oracle.corr_forward`` (fp64) and against the unfused HIP kernels.

Tolerances: corr 1e-5 abs + 1e-5 rel (BASELINE.json north_star), gradients 1e-4 (config 5);
x2_warp must be BIT-identical to ``pwc_warp_forward`` (same sample chain, same blend order).
"""
import os

import numpy as np
import pytest
import torch


def _seed(*parts):
    """Process-independent seed (str hashing is randomised per process; crc32 is not)."""
    import zlib
    return zlib.crc32(repr(parts).encode())

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (B, C, H, W): the pyramid levels at 384x448 (model.py:72 order, l0..l4), ragged shapes
LEVELS = [(2, 192, 6, 7), (2, 128, 12, 14), (2, 96, 24, 28), (1, 64, 48, 56), (1, 32, 96, 112)]
RAGGED = [(1, 8, 5, 3), (2, 16, 7, 9), (1, 24, 13, 15), (1, 12, 2, 2), (1, 40, 11, 30),
          (3, 3, 9, 4)]
# band configurations (R parity rows, T displacement rows per workgroup[, channel groups])
CFGS = ["", "3,1", "2,3", "3,3", "3,1,1", "2,3,5"]


def _t(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _inputs(seed, B, C, H, W, flow_sigma=2.0):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((B, C, H, W)).astype(np.float32)
    b = rng.standard_normal((B, C, H, W)).astype(np.float32)
    f = (rng.standard_normal((B, 2, H, W)) * flow_sigma).astype(np.float32)
    return a, b, f


@pytest.fixture
def band_cfg(request):
    """Band kernel configuration "R,T[,G]" through the library's debug knobs (pwc_set_debug:
    band_r, band_t, band_g); "" = the per-level default."""
    from pwcnet_amd import _lib
    spec = ""
    if request.param:
        parts = request.param.split(",")
        spec = ",".join(f"band_{k}={v}" for k, v in zip("rtg", parts))
    _lib.set_debug(spec)
    yield request.param
    _lib.set_debug("")


def _check(a, b, f, out, x2w, md=9):
    wref = O.warp_forward(b, f)
    cref = O.corr_forward(a, wref, md, 1, md, 1, 2)
    np.testing.assert_allclose(_np(out), cref, rtol=1e-5, atol=1e-5)
    if x2w is not None:
        np.testing.assert_allclose(_np(x2w), wref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape", LEVELS + RAGGED, ids=lambda s: "B{}C{}_{}x{}".format(*s))
@pytest.mark.parametrize("band_cfg", CFGS, indirect=True, ids=lambda c: "cfg" + (c or "auto"))
def test_fused_vs_oracle(shape, band_cfg):
    from pwcnet_amd.ops import warp_corr_forward, warp_forward
    B, C, H, W = shape
    a, b, f = _inputs(_seed(shape, band_cfg), *shape)
    out, x2w = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    _check(a, b, f, out, x2w)
    # x2_warp bit-identical to the standalone warp kernel
    ref_w = warp_forward(_t(b), _t(f))
    assert torch.equal(x2w, ref_w)


@pytest.mark.parametrize("shape", [(8, 192, 6, 7), (8, 128, 12, 14), (8, 96, 24, 28)],
                         ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_fused_full_batch_levels(shape):
    """BASELINE config 2's batch (B=8) at the coarse levels, flows up to far out of the image."""
    from pwcnet_amd.ops import warp_corr_forward
    a, b, f = _inputs(11, *shape, flow_sigma=4.0)
    out, x2w = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    _check(a, b, f, out, x2w)


def test_fused_matches_unfused_and_emit_flag():
    from pwcnet_amd.ops import corr_forward, warp_corr_forward, warp_forward
    a, b, f = _inputs(5, 2, 96, 24, 28)
    out, x2w = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2)
    out2, none = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2, emit_warp=False)
    assert none is None
    assert torch.equal(out, out2)  # same kernel, same order: bitwise
    ref = corr_forward(_t(a), warp_forward(_t(b), _t(f)), 9, 1, 9, 1, 2)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_fused_deterministic():
    from pwcnet_amd.ops import warp_corr_forward
    a, b, f = _inputs(6, 4, 128, 12, 14)
    o1, w1 = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2)
    o2, w2 = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2)
    assert torch.equal(o1, o2) and torch.equal(w1, w2)


def test_fused_zero_flow_is_plain_correlation():
    """model.py:75-76: level 0 runs with flow = 0, i.e. x2_warp == x2 (align_corners=True)."""
    from pwcnet_amd.ops import corr_forward, warp_corr_forward
    a, b, _ = _inputs(8, 2, 192, 6, 7)
    f = np.zeros((2, 2, 6, 7), np.float32)
    out, x2w = warp_corr_forward(_t(a), _t(b), _t(f), 9, 1, 9, 1, 2)
    torch.testing.assert_close(x2w, _t(b), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(out, corr_forward(_t(a), _t(b), 9, 1, 9, 1, 2), rtol=1e-5,
                               atol=1e-5)


@pytest.mark.parametrize("md", [8, 9])
def test_fused_md8(md):
    from pwcnet_amd.ops import warp_corr_forward
    a, b, f = _inputs(9, 2, 32, 12, 14)
    out, x2w = warp_corr_forward(_t(a), _t(b), _t(f), md, 1, md, 1, 2)
    torch.cuda.synchronize()
    _check(a, b, f, out, x2w, md=md)


@pytest.mark.parametrize("params", [(4, 1, 4, 1, 1), (9, 1, 9, 1, 2), (3, 3, 2, 1, 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_fused_fallback_configs(params, dtype):
    """Configurations the band kernel does not cover run warp + correlation; the result equals
    the two ops called separately (bitwise: same kernels).  model.py:24's configuration takes
    the band kernel in fp32 and fp16 (another summation order: within 1e-5, or the fp16 output
    rounding); x2_warp is bit-identical either way."""
    from pwcnet_amd.ops import corr_forward, warp_corr_forward, warp_forward
    a, b, f = _inputs(10, 2, 16, 20, 24)
    A, Bt, F = _t(a, dtype), _t(b, dtype), _t(f, dtype)
    for emit in (True, False):
        out, x2w = warp_corr_forward(A, Bt, F, *params, emit_warp=emit)
        w = warp_forward(Bt, F)
        ref = corr_forward(A, w, *params)
        if dtype == torch.float32 and params == (9, 1, 9, 1, 2):
            torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
        elif params == (9, 1, 9, 1, 2):
            err = (out.float() - ref.float()).abs().max() / ref.float().abs().max()
            assert float(err) <= 2e-3
        else:
            assert torch.equal(out, ref)
        if emit:
            assert torch.equal(x2w, w)


def test_fused_empty_batch():
    from pwcnet_amd.ops import warp_corr_forward
    x = torch.zeros(0, 8, 12, 14, device=DEV)
    fl = torch.zeros(0, 2, 12, 14, device=DEV)
    out, x2w = warp_corr_forward(x, x, fl, 9, 1, 9, 1, 2)
    assert tuple(out.shape) == (0, 81, 12, 14) and tuple(x2w.shape) == (0, 8, 12, 14)


def test_warp_correlation_module_autograd():
    """WarpCorrelation (model.py:80-83 in one module): forward and gradients to x1, x2, flow
    against the oracle chain (corr backward into the warped features, then warp backward),
    with a gradient also arriving on x2_warp (as when summaries feed a loss)."""
    import pwcnet_amd
    a, b, f = _inputs(12, 2, 32, 12, 14)
    x1 = _t(a).requires_grad_(True)
    x2 = _t(b).requires_grad_(True)
    fl = _t(f).requires_grad_(True)
    layer = pwcnet_amd.WarpCorrelation(pad_size=9, kernel_size=1, max_displacement=9,
                                       stride1=1, stride2=2, corr_multiply=1)
    out, x2w = layer(x1, x2, fl)
    rng = np.random.default_rng(13)
    g = rng.standard_normal(out.shape).astype(np.float32)
    gw_extra = rng.standard_normal(x2w.shape).astype(np.float32)
    torch.autograd.backward([out, x2w], [_t(g), _t(gw_extra)])
    wref = O.warp_forward(b, f)
    np.testing.assert_allclose(_np(out), O.corr_forward(a, wref, 9, 1, 9, 1, 2), rtol=1e-5,
                               atol=1e-5)
    g1, gw = O.corr_backward(a, wref, g, 9, 1, 9, 1, 2)
    gx2, gfl = O.warp_backward(b, f, gw + gw_extra)
    np.testing.assert_allclose(_np(x1.grad), g1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(x2.grad), gx2, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(fl.grad), gfl, rtol=1e-4, atol=1e-4)  # config 5


# grouped launches: lists of independent problems (pwc_warp_corr_forward_group)
GROUPS = [
    [(8, 192, 6, 7), (8, 128, 12, 14)],                  # the bench's l0 + l1: one paired launch
    [(8, 128, 12, 14), (8, 192, 6, 7)],                  # the other order
    [(2, 192, 6, 7), (3, 128, 12, 14), (2, 96, 24, 28)],  # a pair + an unfused level
    [(1, 24, 13, 15), (2, 16, 7, 9), (0, 8, 6, 7), (1, 40, 11, 30)],  # ragged, an empty batch
    [(2, 192, 6, 7)],                                   # a single problem
]


@pytest.mark.parametrize("group", GROUPS, ids=lambda g: "+".join("B{}C{}_{}x{}".format(*s)
                                                                 for s in g))
def test_fused_group_matches_single_calls(group):
    """Each problem of a group equals its own warp_corr_forward call bit for bit (the paired
    kernel runs the same workgroup body), and the oracle within the north-star tolerance."""
    from pwcnet_amd.ops import warp_corr_forward, warp_corr_forward_group
    data = [_inputs(_seed("group", i, s), *s) for i, s in enumerate(group)]
    probs = [(_t(a), _t(b), _t(f)) for (a, b, f) in data]
    outs = warp_corr_forward_group(probs, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    assert len(outs) == len(group)
    for (a, b, f), (x1, x2, fl), (out, x2w) in zip(data, probs, outs):
        ref_o, ref_w = warp_corr_forward(x1, x2, fl, 9, 1, 9, 1, 2)
        assert torch.equal(out, ref_o) and torch.equal(x2w, ref_w)
        if a.shape[0] > 0 and a.shape[1] * a.shape[2] * a.shape[3] <= 192 * 12 * 14:
            _check(a, b, f, out, x2w)


def test_fused_group_pair_disabled_is_identical():
    """The pair kernel against the one-launch-per-problem path of the same entry point."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import warp_corr_forward_group
    data = [_inputs(21 + i, *s) for i, s in enumerate(GROUPS[0])]
    probs = [(_t(a), _t(b), _t(f)) for (a, b, f) in data]
    o1 = warp_corr_forward_group(probs, 9, 1, 9, 1, 2)
    _lib.set_debug("band_pair=0")
    try:
        o2 = warp_corr_forward_group(probs, 9, 1, 9, 1, 2)
    finally:
        _lib.set_debug("")
    for (p, q), (r, s) in zip(o1, o2):
        assert torch.equal(p, r) and torch.equal(q, s)


# grouped warps: lists of independent (x, flow) problems (pwc_warp_forward_group)
WARP_GROUPS = [
    [(8, 96, 24, 28), (8, 64, 48, 56), (8, 32, 96, 112)],  # the bench's l2 + l3 + l4
    [(2, 32, 96, 112), (2, 96, 24, 28)],                   # largest first
    [(1, 8, 5, 3), (2, 16, 7, 9), (0, 8, 6, 7), (1, 40, 11, 30), (3, 3, 9, 4),
     (1, 12, 2, 2)],                                       # ragged, an empty batch, 2 launches
    [(2, 192, 6, 7)],                                      # a single problem
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16], ids=["fp32", "fp16"])
@pytest.mark.parametrize("group", WARP_GROUPS, ids=lambda g: "+".join(
    "B{}C{}_{}x{}".format(*s) for s in g))
def test_warp_group_matches_single_calls(group, dtype):
    """Each problem of a grouped warp launch equals its own warp_forward call bit for bit
    (same fmaf chain per element), and the oracle at 1e-5 (fp32; fp16 storage at 2e-3)."""
    from pwcnet_amd.ops import warp_forward, warp_forward_group
    data = [_inputs(_seed("wgroup", i, s), *s) for i, s in enumerate(group)]
    probs = [(_t(b, dtype), _t(f, dtype)) for (_, b, f) in data]
    outs = warp_forward_group(probs)
    torch.cuda.synchronize()
    assert len(outs) == len(group)
    for (_, b, f), (x, fl), out in zip(data, probs, outs):
        assert torch.equal(out, warp_forward(x, fl))
        if b.shape[0] > 0 and b.size <= 2 * 96 * 24 * 28:
            ref = O.warp_forward(_np(x), _np(fl))
            tol = 1e-5 if dtype == torch.float32 else 2e-3
            np.testing.assert_allclose(_np(out), ref, rtol=tol, atol=tol)


# grouped correlations (pwc_corr_forward_group): the row-band pair and the one-by-one rest
CORR_GROUPS = [
    [(8, 96, 24, 28), (8, 64, 48, 56)],                  # the bench's l2 + l3: one paired launch
    [(8, 64, 48, 56), (8, 96, 24, 28)],                  # the other order
    [(2, 192, 6, 7), (2, 96, 24, 28), (1, 32, 96, 112), (2, 64, 48, 56)],  # band, pair, stream
    [(1, 24, 13, 15), (0, 8, 6, 7), (2, 96, 24, 28)],    # ragged, an empty batch, one rows level
]


@pytest.mark.parametrize("group", CORR_GROUPS, ids=lambda g: "+".join(
    "B{}C{}_{}x{}".format(*s) for s in g))
def test_corr_group_matches_single_calls(group):
    """Each problem of a grouped correlation equals its own corr_forward call bit for bit (the
    pair kernel runs the row-band workgroup body on the same plan), and the oracle at 1e-5."""
    import ctypes
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward_group
    data = [_inputs(_seed("cgroup", i, s), *s) for i, s in enumerate(group)]
    probs = [(_t(a), _t(b)) for (a, b, _) in data]
    outs = corr_forward_group(probs, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    assert len(outs) == len(group)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for (a, b, _), (x1, x2), out in zip(data, probs, outs):
        ref = torch.empty_like(out)
        if ref.numel():  # the single call the group promises to equal: pwc_corr_forward
            B, C, H, W = x1.shape
            assert _lib.load().pwc_corr_forward(
                ctypes.c_void_p(x1.data_ptr()), ctypes.c_void_p(x2.data_ptr()),
                ctypes.c_void_p(ref.data_ptr()), B, C, H, W, 9, 1, 9, 1, 2, 1, 0, stream) == 1
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        if a.shape[0] > 0 and a.size <= 2 * 96 * 24 * 28:
            cref = O.corr_forward(a, b, 9, 1, 9, 1, 2)
            np.testing.assert_allclose(_np(out), cref, rtol=1e-5, atol=1e-5)


def test_corr_group_pair_disabled_is_identical():
    """The pair kernel against the one-call-per-problem path of the same entry point."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward_group
    data = [_inputs(31 + i, *s) for i, s in enumerate(CORR_GROUPS[0])]
    probs = [(_t(a), _t(b)) for (a, b, _) in data]
    o1 = corr_forward_group(probs, 9, 1, 9, 1, 2)
    _lib.set_debug("rows_pair=0")
    try:
        o2 = corr_forward_group(probs, 9, 1, 9, 1, 2)
    finally:
        _lib.set_debug("")
    for p, q in zip(o1, o2):
        assert torch.equal(p, q)
