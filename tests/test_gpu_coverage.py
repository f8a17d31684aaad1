"""Every kernel instantiation the default dispatch can reach, at the shapes that reach it, against
the fp64 oracle (through the C ABI).  The shapes come from tools/coverage_sweep.py (round 4): it
runs every op over the pyramid shapes of 384x448 and 448x1024 at B in {1, 2, 3, 4, 8, 12, 16},
fp32 / fp16 / bf16, under a kernel trace and names the smallest call that reached each
instantiation; the cases below are the ones the rest of the suite did not already reach
(profiles/r03i_kernel_coverage.txt's unhit list), plus targeted shapes for variants that only
non-pyramid shapes reach, and the new strip kernel's edge cases (corr_strip.hip).

Reference semantics: correlation_cuda_kernel.cu:34-106 (forward), :108-290 (backward);
modules.py:31-42 (warp = grid_sample, align_corners=True).  fp32 forward within 1e-5, backward
1e-4; fp16 / bf16 storage within the output rounding, against the oracle on the
rounded inputs."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = {torch.float32: (1e-5, 1e-5), torch.float16: (2e-3, 1e-4), torch.bfloat16: (1.6e-2, 1e-4)}


def _seed(*parts):
    import zlib
    return zlib.crc32(repr(parts).encode())


def _rand(shape, dtype, *key, scale=1.0):
    rng = np.random.default_rng(_seed(*key))
    a = (rng.standard_normal(shape) * scale).astype(np.float32)
    t = torch.from_numpy(a).to(DEV, dtype)
    return t, t.detach().double().cpu().numpy()


def _np(t):
    return t.detach().double().cpu().numpy()


def _check(out, ref, dtype, bwd=False):
    rtol, atol = TOL[dtype]
    if dtype == torch.float32:
        if bwd:
            rtol = atol = 1e-4
        np.testing.assert_allclose(_np(out), ref, rtol=rtol, atol=atol)
    else:  # storage rounding relative to the volume's max
        err = np.abs(_np(out) - ref).max() / (np.abs(ref).max() + 1e-12)
        assert err <= rtol, f"max error {err:.2e} (relative to the max) > {rtol}"


CFG = {"corr9": (9, 1, 9, 1, 2), "corr4": (4, 1, 4, 1, 1)}
FWD = [
    # (cfg, dtype, shape, what the sweep named)
    ("corr9", torch.float32, (8, 32, 54, 128), "corr_fwd_pt<PtTile<1,4,5>>"),
    ("corr9", torch.float32, (4, 32, 54, 128), "corr_fwd_pt<PtTile<2,2,12>>"),
    ("corr9", torch.float32, (16, 96, 28, 64), "corr_fwd_rows<float,2,768,2,8>"),
    ("corr9", torch.float32, (16, 32, 28, 56), "corr_fwd_rows<float,2,768,2,6>"),
    ("corr9", torch.float32, (2, 96, 24, 48), "corr_fwd_rows<float,1,768,2,8>"),
    ("corr9", torch.float32, (12, 32, 54, 128), "stream<float,2,3,128> (128-px tiles)"),
    ("corr4", torch.float32, (12, 32, 54, 128), "stream<float,1,3,128>"),
    ("corr9", torch.float32, (4, 32, 112, 256), "448x1024 l4, B=4: stream 128-px tiles"),
    ("corr9", torch.float32, (4, 64, 56, 128), "448x1024 l3, B=4: stream 128-px tiles"),
    ("corr4", torch.float32, (4, 32, 112, 256), "448x1024 l4 Corr4, B=4"),
    ("corr4", torch.float32, (4, 64, 56, 128), "448x1024 l3 Corr4, B=4"),
    ("corr9", torch.float32, (8, 48, 96, 112), "stream<float,2,3,112> (C != 32: not the strip)"),
    ("corr9", torch.float16, (16, 32, 96, 112), "384x448 l4 fp16 B=16: stream<half,2,3,112>"),
    ("corr9", torch.float16, (4, 32, 192, 224), "stream<half,2,3,112>"),
    ("corr4", torch.float16, (4, 32, 192, 224), "stream<half,1,3,112>"),
    ("corr4", torch.float16, (2, 32, 192, 224), "stream<half,1,4,112>"),
    # the strip kernel (corr_strip.hip), full-row geometry at W = 112 (GeoF: two task groups,
    # shared channel-row halos): the smallest batch it takes, a partial last row group (H = 90:
    # 45 parity rows in groups of 6), an odd height (parity rows 48 / 47); the 56-px strips
    # (GeoL4) at W = 224: four strips per row
    ("corr9", torch.float32, (6, 32, 96, 112), "strip full rows, B=6"),
    ("corr9", torch.float32, (8, 32, 90, 112), "strip full rows, partial row group"),
    ("corr9", torch.float32, (8, 32, 95, 112), "strip full rows, odd height"),
    ("corr9", torch.float32, (4, 32, 192, 224), "strip, 4 strips per row"),
    # its C = 64 whole-row geometry at W = 56 (GeoF3, config 2 l3): the shape, the smallest
    # batch, a partial last row group (H = 46: 23 parity rows in groups of 3), an odd height
    ("corr9", torch.float32, (8, 64, 48, 56), "strip C=64 whole rows (config 2 l3)"),
    ("corr9", torch.float32, (6, 64, 48, 56), "strip C=64, B=6"),
    ("corr9", torch.float32, (8, 64, 46, 56), "strip C=64, partial row group"),
    ("corr9", torch.float32, (8, 64, 47, 56), "strip C=64, odd height"),
    # C = 96 at W = 28 (GeoF2, config 2 l2: one parity row per workgroup, channel quarters):
    # the shape and an odd height (parity rows 12 / 11)
    ("corr9", torch.float32, (8, 96, 24, 28), "strip C=96 quarters (config 2 l2)"),
    ("corr9", torch.float32, (8, 96, 23, 28), "strip C=96, odd height"),
    # the matrix-core fp16 strip kernel (corr_mstrip16.hip): its smallest batch at Sintel l4, a
    # partial last chunk (50 parity rows in chunks of 14) with a partial last strip (W = 200),
    # and an odd height (parity rows 50 / 49)
    ("corr9", torch.float16, (12, 32, 112, 256), "mstrip16, B=12"),
    ("corr9", torch.float16, (16, 32, 100, 200), "mstrip16, partial chunk and strip"),
    ("corr9", torch.float16, (24, 32, 99, 128), "mstrip16, odd height"),
    # its C = 64 geometry (config-4 l3: 64-px strips, 7-row chunks, K = 64 as two MFMAs): the
    # Sintel l3 shape, a partial last chunk with a partial strip, an odd height
    ("corr9", torch.float16, (16, 64, 56, 128), "mstrip16 l3 geometry"),
    ("corr9", torch.float16, (16, 64, 50, 96), "mstrip16 l3, partial chunk and strip"),
    ("corr9", torch.float16, (16, 64, 55, 128), "mstrip16 l3, odd height"),
    # its C = 96 geometry (config-4 l2: 32-px strips, 4-row chunks, K = 96 as three MFMAs,
    # rows of 24 halves): the Sintel l2 shape, partial chunk and strip, odd height
    ("corr9", torch.float16, (16, 96, 28, 64), "mstrip16 l2 geometry"),
    ("corr9", torch.float16, (16, 96, 26, 56), "mstrip16 l2, partial chunk and strip"),
    ("corr9", torch.float16, (16, 96, 27, 64), "mstrip16 l2, odd height"),
]


@pytest.mark.parametrize("cfg,dtype,shape,what", FWD,
                         ids=[f"{c}-{str(d)[6:]}-{'x'.join(map(str, s))}" for c, d, s, _ in FWD])
def test_corr_forward_reached_instantiations(cfg, dtype, shape, what):
    from pwcnet_amd.ops import corr_forward
    a, an = _rand(shape, dtype, "fa", cfg, shape)
    b, bn = _rand(shape, dtype, "fb", cfg, shape)
    out = corr_forward(a, b, *CFG[cfg])
    torch.cuda.synchronize()
    _check(out, O.corr_forward(an, bn, *CFG[cfg]), dtype)


@pytest.mark.parametrize("shape", [(8, 32, 96, 112), (8, 32, 91, 112)], ids=["l4", "odd"])
def test_strip_56px_geometry_at_w112(shape):
    """The 56-px strip geometry (GeoL4) at config 2's width, selected by the knob strip_geo=4
    (the full-row geometry is the default there): equal to the oracle, and to the default
    geometry bit for bit (same per-element fp32 order of the channel sum)."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward
    a, an = _rand(shape, torch.float32, "g4a", shape)
    b, bn = _rand(shape, torch.float32, "g4b", shape)
    ref = corr_forward(a, b, 9, 1, 9, 1, 2)
    _lib.set_debug("strip_geo=4")
    try:
        out = corr_forward(a, b, 9, 1, 9, 1, 2)
        torch.cuda.synchronize()
    finally:
        _lib.set_debug("")
    _check(out, O.corr_forward(an, bn, 9, 1, 9, 1, 2), torch.float32)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("shape", [(8, 32, 96, 112), (8, 64, 48, 56), (8, 96, 24, 28)],
                         ids=["l4", "l3", "l2"])
def test_corr_md8_forward_strip_vs_oracle(shape):
    """Correlation(8, 1, 8, 1, 2) (pad == md == 8: the same 81 displacements and output shape
    as model.py's md = 9) takes the strip kernels too; checked against the oracle."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward
    B, C, H, W = shape
    cfg = (8, 1, 8, 1, 2)
    assert _lib.corr_forward_plan(B, C, H, W, *cfg) == "strip"
    a, an = _rand(shape, torch.float32, "m8a", shape)
    b, bn = _rand(shape, torch.float32, "m8b", shape)
    out = corr_forward(a, b, *cfg)
    torch.cuda.synchronize()
    _check(out, O.corr_forward(an, bn, *cfg), torch.float32)


@pytest.mark.parametrize("shape", [(1, 32, 96, 112), (2, 64, 47, 56), (1, 96, 24, 28)],
                         ids=["l4", "l3_odd", "l2"])
def test_corr_md8_backward_strip_vs_oracle(shape):
    """The strip backward (corr_bwd_strip.hip) at pad == md == 8 (its plan accepts md 8 and 9),
    both gradients against the oracle."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_backward
    B, C, H, W = shape
    cfg = (8, 1, 8, 1, 2)
    _lib.set_debug("bwd_strip=2")  # small batches: the strip kernel regardless of grid size
    try:
        assert _lib.corr_backward_plan(B, C, H, W, *cfg) == "strip"
        a, an = _rand(shape, torch.float32, "m8ba", shape)
        b, bn = _rand(shape, torch.float32, "m8bb", shape)
        g, gn = _rand((B, 81, H, W), torch.float32, "m8bg", shape)
        g1, g2 = corr_backward(a, b, g, *cfg)
        torch.cuda.synchronize()
    finally:
        _lib.set_debug("")
    r1, r2 = O.corr_backward(an, bn, gn, *cfg)
    _check(g1, r1, torch.float32, bwd=True)
    _check(g2, r2, torch.float32, bwd=True)


@pytest.mark.parametrize("shape", [(4, 32, 112, 256), (4, 64, 56, 128)], ids=["l4", "l3"])
def test_cost_volume_448x1024_b4(shape):
    """CostVolumeLayer (modules.py:53-74) at 448x1024 l3 / l4 with B = 4 (stream 128-px tiles,
    CVL channel order)."""
    from pwcnet_amd.ops import cost_volume_forward
    a, an = _rand(shape, torch.float32, "ca", shape)
    b, bn = _rand(shape, torch.float32, "cb", shape)
    out = cost_volume_forward(a, b, 4)
    torch.cuda.synchronize()
    _check(out, O.cvl_forward(an, bn, 4), torch.float32)


@pytest.mark.parametrize("shape,knob", [((8, 96, 24, 28), "strip_l2=0"),
                                        ((8, 64, 48, 56), "strip_l3=0"),
                                        ((8, 32, 96, 112), "strip_geo=4")], ids=["l2", "l3", "l4"])
def test_strip_full_rows_after_other_kernels(shape, knob):
    """The whole-row strip geometries read each channel row's right halo from the next channel
    row's zero pad: a read issued before that pad's DMA group landed returns whatever LDS held
    (a round-5 bug at C = 64, caught only with other kernels' data left in LDS).  Each round
    runs the reference-path kernel (knob) on unrelated data first, then the default on fresh
    inputs, against the oracle."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward
    for it in range(4):
        z, _ = _rand(shape, torch.float32, "junk", it, shape, scale=50.0)
        _lib.set_debug(knob)
        try:
            corr_forward(z, z, 9, 1, 9, 1, 2)
        finally:
            _lib.set_debug("")
        a, an = _rand(shape, torch.float32, "sa", it, shape)
        b, bn = _rand(shape, torch.float32, "sb", it, shape)
        out = corr_forward(a, b, 9, 1, 9, 1, 2)
        torch.cuda.synchronize()
        _check(out, O.corr_forward(an, bn, 9, 1, 9, 1, 2), torch.float32)


@pytest.mark.parametrize("shape,knob", [((8, 64, 48, 56), "strip_l3=0"),
                                        ((8, 96, 24, 28), "strip_l2=0"),
                                        ((8, 32, 96, 112), "strip_geo=4")],
                         ids=["l3", "l2", "l4"])
def test_strip_c64_into_cat_slice_leaky(shape, knob):
    """model.py:83-84 + :89/91 at config 2's l3 / l2 / l4 (C = 64 / 96 / 32, B = 8) through the
    strip kernel's whole-row geometries: the cat slice with leaky_relu(0.01) fused; the other
    kernel's volume (knob: row band; the 56-px strips at l4) against the oracle too."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_forward, corr_forward_into
    B, C, H, W = shape
    a, an = _rand((B, C, H, W), torch.float32, "l3a", C)
    b, bn = _rand((B, C, H, W), torch.float32, "l3b", C)
    cat = torch.full((B, C + 81 + 2, H, W), 7.0, device=DEV)
    corr_forward_into(a, b, cat[:, C:C + 81], 9, 1, 9, 1, 2, negative_slope=0.01)
    plain = corr_forward(a, b, 9, 1, 9, 1, 2)
    _lib.set_debug(knob)
    try:
        rows = corr_forward(a, b, 9, 1, 9, 1, 2)
        torch.cuda.synchronize()
    finally:
        _lib.set_debug("")
    ref = O.corr_forward(an, bn, 9, 1, 9, 1, 2)
    np.testing.assert_allclose(_np(plain), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(rows), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(cat[:, C:C + 81]), np.where(ref > 0, ref, ref * 0.01),
                               rtol=1e-5, atol=1e-5)
    assert bool((cat[:, :C] == 7.0).all()) and bool((cat[:, C + 81:] == 7.0).all())


def test_strip_into_cat_slice_leaky():
    """model.py:83-84 + :89/91 at config 2's l4 through the strip kernel: the volume written into
    the cat buffer's slice with leaky_relu(0.01) fused, the rest of the buffer untouched."""
    from pwcnet_amd.ops import corr_forward_into
    B, C, H, W = 8, 32, 96, 112
    a, an = _rand((B, C, H, W), torch.float32, "ia")
    b, bn = _rand((B, C, H, W), torch.float32, "ib")
    cat = torch.full((B, C + 81 + 2, H, W), 7.0, device=DEV)
    corr_forward_into(a, b, cat[:, C:C + 81], 9, 1, 9, 1, 2, negative_slope=0.01)
    torch.cuda.synchronize()
    ref = O.corr_forward(an, bn, 9, 1, 9, 1, 2)
    ref = np.where(ref > 0, ref, ref * 0.01)
    np.testing.assert_allclose(_np(cat[:, C:C + 81]), ref, rtol=1e-5, atol=1e-5)
    assert bool((cat[:, :C] == 7.0).all()) and bool((cat[:, C + 81:] == 7.0).all())


def test_mstrip16_into_cat_slice_leaky():
    """model.py:83-84 + :89/91 at config 4's l4 (fp16): the matrix-core strip kernel writes the
    cat buffer's slice itself with leaky_relu(0.1) fused (its strided, activated epilogue); the
    rest of the buffer untouched."""
    from pwcnet_amd.ops import corr_forward_into
    B, C, H, W = 12, 32, 112, 256
    a, an = _rand((B, C, H, W), torch.float16, "ma")
    b, bn = _rand((B, C, H, W), torch.float16, "mb")
    cat = torch.full((B, C + 81 + 2, H, W), 7.0, device=DEV, dtype=torch.float16)
    corr_forward_into(a, b, cat[:, C:C + 81], 9, 1, 9, 1, 2, negative_slope=0.1)
    torch.cuda.synchronize()
    ref = O.corr_forward(an, bn, 9, 1, 9, 1, 2)
    ref = np.where(ref > 0, ref, ref * 0.1)
    _check(cat[:, C:C + 81], ref, torch.float16)
    assert bool((cat[:, :C] == 7.0).all()) and bool((cat[:, C + 81:] == 7.0).all())


@pytest.mark.parametrize("shape,extra", [((16, 64, 56, 128), 2), ((16, 96, 28, 64), 2),
                                         ((4, 32, 112, 256), 3), ((16, 128, 14, 32), 2)])
def test_fp16_into_cat_slice_strides(shape, extra):
    """fp16 pwc_corr_forward_into at config 4's l3 / l2 (matrix-core strip, C = 64 / 96
    geometries), l4 and l1 (row bands): the kernels write the slice directly with their fused
    epilogue (image stride (C + 81 + extra) H W halves; these kernels need W % 8 == 0, so the
    stride is always a multiple of the 8-half store).  Values against the oracle on the fp16
    inputs, leaky_relu(0.01), the rest of the buffer untouched."""
    from pwcnet_amd.ops import corr_forward_into
    B, C, H, W = shape
    a, an = _rand((B, C, H, W), torch.float16, "sa")
    b, bn = _rand((B, C, H, W), torch.float16, "sb")
    cat = torch.full((B, C + 81 + extra, H, W), 7.0, device=DEV, dtype=torch.float16)
    corr_forward_into(a, b, cat[:, C:C + 81], 9, 1, 9, 1, 2, negative_slope=0.01)
    torch.cuda.synchronize()
    ref = O.corr_forward(an, bn, 9, 1, 9, 1, 2)
    ref = np.where(ref > 0, ref, ref * 0.01)
    _check(cat[:, C:C + 81], ref, torch.float16)
    assert bool((cat[:, :C] == 7.0).all()) and bool((cat[:, C + 81:] == 7.0).all())


BWD = [
    ("corr9", torch.float32, (1, 32, 112, 256), "corr_bwd_rows<true,8,8>"),
    ("corr9", torch.float32, (1, 8, 12, 254), "corr_bwd_rows<false,2,8> (dword path, wide)"),
]


@pytest.mark.parametrize("cfg,dtype,shape,what", BWD, ids=[w.split(" ")[0] for *_, w in BWD])
def test_corr_backward_reached_instantiations(cfg, dtype, shape, what):
    from pwcnet_amd.ops import corr_backward
    B, C, H, W = shape
    a, an = _rand(shape, dtype, "ba", shape)
    b, bn = _rand(shape, dtype, "bb", shape)
    g, gn = _rand((B, 81, H, W), dtype, "bg", shape)
    g1, g2 = corr_backward(a, b, g, *CFG[cfg])
    torch.cuda.synchronize()
    r1, r2 = O.corr_backward(an, bn, gn, *CFG[cfg])
    _check(g1, r1, dtype, bwd=True)
    _check(g2, r2, dtype, bwd=True)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_corr_backward_generic_low_precision(dtype):
    """kernel_size 3 (the reference's non-adjoint k > 1 backward, cu:108-290) in fp16 / bf16
    storage: corr_bwd_generic<half / bf16>."""
    from pwcnet_amd.ops import corr_backward, corr_forward
    cfg = (3, 3, 2, 1, 1)
    a, an = _rand((2, 8, 12, 14), dtype, "ga", dtype)
    b, bn = _rand((2, 8, 12, 14), dtype, "gb", dtype)
    out = corr_forward(a, b, *cfg)
    g, gn = _rand(tuple(out.shape), dtype, "gg", dtype)
    g1, g2 = corr_backward(a, b, g, *cfg)
    torch.cuda.synchronize()
    r1, r2 = O.corr_backward(an, bn, gn, *cfg)
    _check(g1, r1, dtype)
    _check(g2, r2, dtype)


@pytest.mark.parametrize("shape,what", [((16, 96, 28, 48), "warp_bwd_flow<8,4>"),
                                        ((1, 16, 48, 48), "warp_bwd_merged<16,16,6,8,2>")],
                         ids=["flow_ng4", "merged_ng2"])
def test_warp_backward_reached_instantiations(shape, what):
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = shape
    x, xn = _rand(shape, torch.float32, "wx", shape)
    f, fn = _rand((B, 2, H, W), torch.float32, "wf", shape, scale=2.0)
    g, gn = _rand(shape, torch.float32, "wg", shape)
    gx, gf = warp_backward(x, f, g)
    torch.cuda.synchronize()
    rx, rf = O.warp_backward(xn, fn, gn)
    _check(gx, rx, torch.float32, bwd=True)
    _check(gf, rf, torch.float32, bwd=True)


def test_warp_bf16_wide_grid():
    """bf16 warp on a large grid: warp_fwd_kernel<bf16, 2, 4> (four 2-channel groups per
    thread)."""
    from pwcnet_amd.ops import warp_forward
    shape = (3, 32, 54, 128)
    x, xn = _rand(shape, torch.bfloat16, "bx")
    f, fn = _rand((3, 2, 54, 128), torch.bfloat16, "bf", scale=2.0)
    out = warp_forward(x, f)
    torch.cuda.synchronize()
    _check(out, O.warp_forward(xn, fn), torch.bfloat16)


@pytest.mark.parametrize("B", [1, 2])
def test_warp_group_bf16(B):
    """pwc_warp_forward_group in bf16 (l2..l4 of 384x448): warp_fwd_group<bf16, 4, 1> at B = 1,
    <bf16, 2, 4> at B = 2 -- bit-identical to the single calls, within bf16 rounding of the
    oracle."""
    from pwcnet_amd.ops import warp_forward, warp_forward_group
    probs, refs = [], []
    for (C, h, w) in [(96, 24, 28), (64, 48, 56), (32, 96, 112)]:
        x, xn = _rand((B, C, h, w), torch.bfloat16, "gx", B, C)
        f, fn = _rand((B, 2, h, w), torch.bfloat16, "gf", B, C, scale=2.0)
        probs.append((x, f))
        refs.append(O.warp_forward(xn, fn))
    outs = warp_forward_group(probs)
    torch.cuda.synchronize()
    for (x, f), o, r in zip(probs, outs, refs):
        assert torch.equal(o, warp_forward(x, f))
        _check(o, r, torch.bfloat16)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16], ids=["fp32", "fp16"])
@pytest.mark.parametrize("order", ["l0l1", "l1l0"])
def test_band_pair_both_orders(dtype, order):
    """pwc_warp_corr_forward_group on (l0, l1) and (l1, l0) of 384x448: both orders of the band
    pair kernel (warp_corr_band_pair<T, 3,1,2,3> / <T, 2,3,3,1>), bit-identical to single calls
    and within tolerance of the oracle on the warped x2."""
    from pwcnet_amd.ops import warp_corr_forward, warp_corr_forward_group
    shapes = [(1, 192, 6, 7), (1, 128, 12, 14)]
    if order == "l1l0":
        shapes = shapes[::-1]
    probs = []
    for s in shapes:
        a, _ = _rand(s, dtype, "pa", s)
        x2, _ = _rand(s, dtype, "px", s)
        f, _ = _rand((s[0], 2, s[2], s[3]), dtype, "pf", s, scale=2.0)
        probs.append((a, x2, f))
    outs = warp_corr_forward_group(probs, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    for (a, x2, f), (corr, x2w) in zip(probs, outs):
        c1, w1 = warp_corr_forward(a, x2, f, 9, 1, 9, 1, 2)
        assert torch.equal(corr, c1) and torch.equal(x2w, w1)
        _check(corr, O.corr_forward(_np(a), _np(x2w), 9, 1, 9, 1, 2), dtype)


def test_warp_backward_short_workspace_falls_back():
    """pwc_warp_backward_ws with a workspace shorter than pwc_warp_backward_workspace_size: the
    tile path declines and the multi-kernel path runs -- same gradients as the default (full
    workspace) call within fp32 summation order, both against the oracle."""
    import ctypes
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import warp_backward
    B, C, H, W = 2, 32, 96, 112
    x, xn = _rand((B, C, H, W), torch.float32, "sx")
    f, fn = _rand((B, 2, H, W), torch.float32, "sf", scale=2.0)
    g, gn = _rand((B, C, H, W), torch.float32, "sg")
    lib = _lib.load()
    assert lib.pwc_warp_backward_workspace_size(B, C, H, W, 0) > 64
    ws = torch.empty(64, dtype=torch.uint8, device=DEV)
    gx = torch.empty_like(x)
    gf = torch.empty_like(f)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(lib.pwc_warp_backward_ws(p(x), p(f), p(g), p(gx), p(gf), B, C, H, W, 0, p(ws), 64,
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "short workspace")
    dx, df = warp_backward(x, f, g)
    torch.cuda.synchronize()
    rx, rf = O.warp_backward(xn, fn, gn)
    for out, ref in ((gx, rx), (gf, rf), (dx, rx), (df, rf)):
        _check(out, ref, torch.float32, bwd=True)
    torch.testing.assert_close(gx, dx, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gf, df, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", ["aligned", "odd_offset", "odd_total"])
def test_warp_fp16_alignment(case):
    """fp16 warp (modules.py:31-42) on an aligned tensor, a tensor whose storage starts 2 bytes
    past an aligned address (bit-identical to the aligned copy) and an odd element count, within
    fp16 rounding of the oracle; flows reach past every border (N(0, 6^2) px)."""
    from pwcnet_amd.ops import warp_forward
    shape = (1, 3, 5, 7) if case == "odd_total" else (2, 8, 20, 36)
    x, xn = _rand(shape, torch.float16, "px", case)
    f, fn = _rand((shape[0], 2) + shape[2:], torch.float16, "pf", case, scale=6.0)
    if case == "odd_offset":  # same values, storage starting 2 bytes past an aligned address
        buf = torch.empty(x.numel() + 1, device=DEV, dtype=torch.float16)
        xv = buf[1:].view(shape)
        xv.copy_(x)
        out = warp_forward(xv, f)
    else:
        out = warp_forward(x, f)
    torch.cuda.synchronize()
    _check(out, O.warp_forward(xn, fn), torch.float16)
    if case == "odd_offset":
        assert torch.equal(out, warp_forward(x, f))


# corr_bwd_strip.hip (config 5's l4 / l3 / l2 backward): whole batches at the geometries' shapes,
# odd heights (the odd-row parity has a band fewer / a short band), a height below one band,
# batch 1 (knob bwd_strip=2: the plan sends grids below 192 workgroups to the row-band kernel);
# against the oracle, and repeatable bit for bit.
BWD_STRIP = [(1, 32, 96, 112), (2, 32, 95, 112), (1, 32, 6, 112), (1, 32, 14, 112),
             (2, 64, 48, 56), (1, 64, 47, 56), (3, 64, 10, 56),
             (2, 96, 24, 28), (1, 96, 23, 28), (1, 96, 3, 28)]


@pytest.mark.parametrize("shape", BWD_STRIP, ids=lambda s: "x".join(map(str, s)))
def test_corr_backward_strip_vs_oracle(shape):
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_backward
    B, C, H, W = shape
    assert _lib.corr_backward_plan(B, C, H, W, *CFG["corr9"]) == "rows"  # below 192 workgroups
    _lib.set_debug("bwd_strip=2")
    try:
        assert _lib.corr_backward_plan(B, C, H, W, *CFG["corr9"]) == "strip"
        a, an = _rand(shape, torch.float32, "sba", shape)
        b, bn = _rand(shape, torch.float32, "sbb", shape)
        g, gn = _rand((B, 81, H, W), torch.float32, "sbg", shape)
        g1, g2 = corr_backward(a, b, g, *CFG["corr9"])
        h1, h2 = corr_backward(a, b, g, *CFG["corr9"])
        torch.cuda.synchronize()
    finally:
        _lib.set_debug("")
    r1, r2 = O.corr_backward(an, bn, gn, *CFG["corr9"])
    _check(g1, r1, torch.float32, bwd=True)
    _check(g2, r2, torch.float32, bwd=True)
    assert torch.equal(g1, h1) and torch.equal(g2, h2)


@pytest.mark.parametrize("level", [2, 3, 4])
def test_corr_backward_strip_full_batch_vs_rows(level):
    """BASELINE config 5 (B = 8, 384x448) at l2 / l3 / l4: the strip backward against the
    row-band kernel (knob bwd_strip=0) on the same inputs, within fp32 summation-order
    differences."""
    from pwcnet_amd import _lib
    from pwcnet_amd.ops import corr_backward
    C, H, W = {2: (96, 24, 28), 3: (64, 48, 56), 4: (32, 96, 112)}[level]
    shape = (8, C, H, W)
    a, _ = _rand(shape, torch.float32, "fba", level)
    b, _ = _rand(shape, torch.float32, "fbb", level)
    g, _ = _rand((8, 81, H, W), torch.float32, "fbg", level)
    g1, g2 = corr_backward(a, b, g, *CFG["corr9"])
    _lib.set_debug("bwd_strip=0")
    try:
        r1, r2 = corr_backward(a, b, g, *CFG["corr9"])
    finally:
        _lib.set_debug("")
    torch.cuda.synchronize()
    for x, y in ((g1, r1), (g2, r2)):
        err = float((x - y).abs().max()) / float(y.abs().max())
        assert err < 1e-5, err


def test_missing_library_fails_loudly_on_gpu(tmp_path):
    """On the GPU too: with the HIP library absent, an op on device tensors raises
    HipLibraryMissing instead of running anything else (no eager / oracle fallback)."""
    import os
    import subprocess
    import sys
    code = (
        "import torch, pwcnet_amd\n"
        "from pwcnet_amd import _lib\n"
        "from pwcnet_amd.ops import corr_forward, warp_forward\n"
        "a, f = torch.zeros(1, 4, 6, 8, device='cuda'), torch.zeros(1, 2, 6, 8, device='cuda')\n"
        "for fn in (lambda: corr_forward(a, a, 9, 1, 9, 1, 2), lambda: warp_forward(a, f)):\n"
        "    try:\n"
        "        fn()\n"
        "    except _lib.HipLibraryMissing as e:\n"
        "        print('raised:', e)\n")
    env = dict(os.environ, PWC_HOTPATH_LIB=str(tmp_path / "absent.so"))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(root, "pwc-net_pytorch_amd"), root,
                                         env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("raised:") == 2 and "not built" in r.stdout, r.stdout
