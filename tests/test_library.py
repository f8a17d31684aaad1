"""torch.library registration (pwcnet_amd/library.py; SURVEY §8b "Wrappers"): the drop-in
layers are single traceable nodes with shape propagation (CPU) and correct values and
gradients through torch.compile / opcheck (GPU)."""
import pytest
import torch

import pwcnet_amd
from pwcnet_amd import library as L


def test_ops_registered():
    for name in ("correlation", "correlation_backward", "cost_volume", "cost_volume_backward",
                 "warp", "warp_backward"):
        assert hasattr(torch.ops.pwcnet, name)


@pytest.mark.parametrize("args,expect", [
    ((96, 112, 9, 1, 9, 1, 2), (81, 96, 112)),     # model.py:24 at l4
    ((96, 112, 4, 1, 4, 1, 1), (81, 96, 112)),     # Corr4
    ((24, 28, 20, 3, 20, 2, 2), (441, 11, 13)),    # reference defaults k=3, md=20, s1=2
    ((6, 7, 0, 0, 0, 1, 2), (1, 6, 7)),            # Correlation() ctor defaults, k=0
])
def test_shape_math_matches_capi(args, expect):
    from pwcnet_amd import _lib
    assert L.corr_output_shape(*args) == expect
    assert _lib.corr_output_shape(*args) == expect  # the C ABI's correlation_cuda.c:20-34


def test_fake_tensor_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        a = torch.empty(8, 32, 96, 112)
        f = torch.empty(8, 2, 96, 112)
        assert torch.ops.pwcnet.correlation(a, a, 9, 1, 9, 1, 2, 1).shape == (8, 81, 96, 112)
        assert torch.ops.pwcnet.cost_volume(a, a, 4).shape == (8, 81, 96, 112)
        assert torch.ops.pwcnet.warp(a, f).shape == a.shape
        g1, g2 = torch.ops.pwcnet.correlation_backward(a, a, torch.empty(8, 81, 96, 112),
                                                       9, 1, 9, 1, 2, 1)
        assert g1.shape == a.shape and g2.shape == a.shape


def test_fx_trace_sees_one_node_per_layer():
    corr = pwcnet_amd.Correlation(9, 1, 9, 1, 2, 1)
    warp = pwcnet_amd.WarpingLayer(None)

    def level(x1, x2, flow):  # model.py:80 + :83
        return corr(x1, warp(x2, flow))

    from torch.fx.experimental.proxy_tensor import make_fx
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        a, f = torch.empty(2, 16, 12, 14), torch.empty(2, 2, 12, 14)
        gm = make_fx(level)(a, a, f)
    targets = [str(n.target) for n in gm.graph.nodes if n.op == "call_function"]
    assert targets == ["pwcnet.warp.default", "pwcnet.correlation.default"]


def test_cpu_tensors_raise_like_the_reference_stub():
    a = torch.randn(1, 4, 6, 7)
    with pytest.raises(RuntimeError, match="HIP devices only"):
        pwcnet_amd.Correlation(9, 1, 9, 1, 2, 1)(a, a)


@pytest.mark.gpu
def test_opcheck_and_compile():
    torch.manual_seed(0)
    a = torch.randn(2, 16, 12, 14, device="cuda", requires_grad=True)
    b = torch.randn(2, 16, 12, 14, device="cuda", requires_grad=True)
    f = (torch.randn(2, 2, 12, 14, device="cuda") * 2).requires_grad_(True)
    torch.library.opcheck(torch.ops.pwcnet.correlation.default, (a, b, 9, 1, 9, 1, 2, 1),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    torch.library.opcheck(torch.ops.pwcnet.warp.default, (a, f),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    corr = pwcnet_amd.Correlation(9, 1, 9, 1, 2, 1)
    warp = pwcnet_amd.WarpingLayer(None)

    def level(x1, x2, flow):
        return corr(x1, warp(x2, flow))

    eager = level(a, b, f)
    comp = torch.compile(level, backend="aot_eager", fullgraph=True)(a, b, f)
    assert torch.equal(eager, comp)
    g = torch.randn_like(eager)
    ge = torch.autograd.grad(eager, (a, b, f), g)
    gc = torch.autograd.grad(comp, (a, b, f), g)
    for x, y in zip(ge, gc):
        assert torch.equal(x, y)
