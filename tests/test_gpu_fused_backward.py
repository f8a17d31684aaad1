"""GPU parity of the level backward as one call (``pwc_warp_corr_backward`` /
``WarpCorrelationFunction.backward``): d/dx1, d/dx2 and d/dflow of model.py:80-83 against the
float64 oracle chain ``oracle.corr_backward`` (into x2_warp) -> ``oracle.warp_backward``
(correlation_cuda_kernel.cu:108-290, then ATen grid_sampler_2d_backward semantics), and against
the two-launch HIP path (PWC_DEBUG warp_corr_bwd=0).

Tolerance: 1e-4 (BASELINE config 5).  The one-launch kernel covers images of <= 256 pixels with
C % 4 == 0 (the l0 / l1 levels); every other shape here exercises the two-launch path.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (B, C, H, W): one launch (l0, l1, a 16-B-copy shape, tiny images) and two launches (256
# pixels: LDS; l2 and other larger images; C % 4 != 0; 99 pixels not a multiple of 4 past the
# scalar-copy limit)
SHAPES = [(2, 192, 6, 7), (2, 128, 12, 14), (3, 16, 8, 10), (1, 8, 5, 3), (2, 4, 2, 3),
          (1, 12, 16, 16), (2, 96, 24, 28), (1, 8, 20, 20), (1, 4, 17, 20), (1, 6, 7, 9),
          (1, 8, 9, 11), (1, 4, 32, 24)]


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, torch.float32)


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _case(seed, B, C, H, W, scale):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((B, C, H, W)).astype(np.float32)
    b = rng.standard_normal((B, C, H, W)).astype(np.float32)
    f = (rng.standard_normal((B, 2, H, W)) * scale).astype(np.float32)
    g = rng.standard_normal((B, 81, H, W)).astype(np.float32)
    e = rng.standard_normal((B, C, H, W)).astype(np.float32)
    return a, b, f, g, e


def _oracle(a, b, f, g, e, md=9):
    w = O.warp_forward(b, f)
    g1, gw = O.corr_backward(a, w, g, md, 1, md, 1, 2)
    if e is not None:
        gw = gw + e
    gx2, gfl = O.warp_backward(b, f, gw)
    return g1, gx2, gfl


@pytest.mark.parametrize("extra", [False, True], ids=["no_gx2w", "gx2w"])
@pytest.mark.parametrize("scale", [0.0, 2.0, 25.0])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_warp_corr_backward_vs_oracle(shape, scale, extra):
    """Zero flow, N(0, 2^2)-px flows and flows mostly out of the image; with and without a
    gradient arriving on x2_warp."""
    from pwcnet_amd.ops import warp_corr_backward, warp_forward
    B, C, H, W = shape
    a, b, f, g, e = _case(int(scale * 10) + 7 * H + W + C, B, C, H, W, scale)
    x2w = warp_forward(_t(b), _t(f))
    g1, gx2, gfl = warp_corr_backward(_t(a), _t(b), _t(f), x2w, _t(g), 9, 1, 9, 1, 2,
                                      grad_x2_warp=_t(e) if extra else None)
    torch.cuda.synchronize()
    r1, rx2, rfl = _oracle(a, b, f, g, e if extra else None)
    np.testing.assert_allclose(_np(g1), r1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gx2), rx2, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gfl), rfl, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)))


# one shape per instantiation of the one-launch kernel (16-B / scalar gO copy class x channel
# quads per workgroup): (V4, loads, quads)
INSTANTIATIONS = [(1, 16, 8, 8), (1, 8, 8, 8), (1, 4, 8, 8), (1, 8, 10, 12), (2, 128, 12, 14),
                  (1, 12, 12, 16), (2, 192, 6, 7), (1, 8, 5, 3), (2, 4, 2, 3), (1, 16, 7, 7),
                  (1, 8, 5, 13), (1, 4, 7, 7)]


@pytest.mark.parametrize("shape", INSTANTIATIONS, ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_warp_corr_backward_instantiations(shape):
    """Every instantiation the one-launch dispatch can reach, against the oracle chain."""
    from pwcnet_amd.ops import warp_corr_backward, warp_forward
    B, C, H, W = shape
    a, b, f, g, e = _case(3 * H + W + C, B, C, H, W, 2.0)
    g1, gx2, gfl = warp_corr_backward(_t(a), _t(b), _t(f), warp_forward(_t(b), _t(f)), _t(g),
                                      9, 1, 9, 1, 2, grad_x2_warp=_t(e))
    r1, rx2, rfl = _oracle(a, b, f, g, e)
    np.testing.assert_allclose(_np(g1), r1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gx2), rx2, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gfl), rfl, rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(C)))


@pytest.mark.parametrize("shape", [(8, 192, 6, 7), (8, 128, 12, 14), (3, 16, 8, 10)],
                         ids=lambda s: "B{}C{}_{}x{}".format(*s))
def test_warp_corr_backward_one_launch_vs_two(shape):
    """The one-launch kernel against the two-launch path at config 5's l0 / l1 (B = 8): equal
    within 1e-5 (the correlation gradients and grad_flow's channel split sum in other orders),
    repeatable bit for bit, and the arrival counters are zero again after every call."""
    from pwcnet_amd import _lib
    from pwcnet_amd import ops
    B, C, H, W = shape
    a, b, f, g, e = _case(5 + C, B, C, H, W, 2.0)
    args = (_t(a), _t(b), _t(f), ops.warp_forward(_t(b), _t(f)), _t(g), 9, 1, 9, 1, 2)
    one = ops.warp_corr_backward(*args, grad_x2_warp=_t(e))
    again = ops.warp_corr_backward(*args, grad_x2_warp=_t(e))
    torch.cuda.synchronize()
    cnt = ops._COUNTERS[args[0].device]
    assert int(cnt.abs().sum()) == 0
    _lib.set_debug("warp_corr_bwd=0")
    try:
        two = ops.warp_corr_backward(*args, grad_x2_warp=_t(e))
        torch.cuda.synchronize()
    finally:
        _lib.set_debug("")
    for x, y, z in zip(one, again, two):
        assert torch.equal(x, y)
        torch.testing.assert_close(x, z, rtol=1e-5, atol=1e-5 * max(1.0, np.sqrt(C)))


def test_warp_corr_backward_md8():
    """pad = md = 8 (same displacement grid as md 9 with stride2 2)."""
    from pwcnet_amd.ops import warp_corr_backward, warp_forward
    a, b, f, g, e = _case(31, 2, 64, 12, 14, 2.0)
    g1, gx2, gfl = warp_corr_backward(_t(a), _t(b), _t(f), warp_forward(_t(b), _t(f)), _t(g),
                                      8, 1, 8, 1, 2)
    r1, rx2, rfl = _oracle(a, b, f, g, None, md=8)
    np.testing.assert_allclose(_np(g1), r1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gx2), rx2, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(gfl), rfl, rtol=1e-4, atol=1e-4 * 8)


def test_warp_correlation_module_one_launch_backward():
    """WarpCorrelation's autograd at config 5's l1 shape runs the one-launch backward and
    matches the oracle chain (gradient also on x2_warp)."""
    import pwcnet_amd
    a, b, f, g, e = _case(12, 2, 128, 12, 14, 2.0)
    x1 = _t(a).requires_grad_(True)
    x2 = _t(b).requires_grad_(True)
    fl = _t(f).requires_grad_(True)
    layer = pwcnet_amd.WarpCorrelation(pad_size=9, kernel_size=1, max_displacement=9,
                                       stride1=1, stride2=2, corr_multiply=1)
    out, x2w = layer(x1, x2, fl)
    torch.autograd.backward([out, x2w], [_t(g), _t(e)])
    r1, rx2, rfl = _oracle(a, b, f, g, e)
    np.testing.assert_allclose(_np(x1.grad), r1, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(x2.grad), rx2, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(fl.grad), rfl, rtol=1e-4, atol=1e-4 * 12)


def test_warp_corr_backward_rejects():
    from pwcnet_amd.ops import warp_corr_backward
    x = torch.randn(1, 8, 6, 7, device=DEV)
    fl = torch.zeros(1, 2, 6, 7, device=DEV)
    g = torch.randn(1, 81, 6, 7, device=DEV)
    with pytest.raises(ValueError):
        warp_corr_backward(x, x, fl, x, g[:, :80], 9, 1, 9, 1, 2)
    with pytest.raises(RuntimeError):  # stride1 2: the reference backward is undefined
        warp_corr_backward(x, x, fl, x, torch.randn(1, 81, 3, 4, device=DEV), 9, 1, 9, 2, 2)
