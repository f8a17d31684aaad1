"""CPU: the C-ABI library loads, exports every symbol include/*.h declares, and its host-side
argument checks behave (no GPU compute is issued by any call here)."""
import ctypes
import glob
import os
import re
import types

import pytest
import torch

from conftest import ROOT


def _declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"PWC_API\s+[\w\s\*]+?\b(pwc_\w+)\s*\(", src))
    return names


def test_header_declares_expected_api():
    names = _declared_symbols()
    assert {"pwc_corr_forward", "pwc_corr_backward", "pwc_warp_forward", "pwc_warp_backward",
            "pwc_cost_volume_forward", "pwc_cost_volume_backward", "pwc_corr_output_shape",
            "pwc_last_error", "pwc_abi_version"} <= names


def test_library_exports_every_declared_symbol():
    from pwcnet_amd import _lib
    lib = _lib.load()
    for name in _declared_symbols():
        assert hasattr(lib, name), name
        assert name in _lib.SYMBOLS, f"{name} not typed in _lib.SYMBOLS"
    assert lib.pwc_abi_version() == _lib.ABI_VERSION


def test_library_is_gfx950_code_object():
    from pwcnet_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_output_shape_matches_reference_shape_math():
    from oracle import oracle as O
    from pwcnet_amd import _lib
    for args in [(96, 112, 9, 1, 9, 1, 2), (96, 112, 4, 1, 4, 1, 1), (20, 30, 0, 1, 4, 1, 1),
                 (20, 30, 3, 3, 2, 2, 1), (21, 31, 3, 3, 2, 2, 1), (1, 1, 9, 1, 9, 1, 2),
                 (384, 448, 20, 1, 20, 1, 2)]:
        assert _lib.corr_output_shape(*args) == O.corr_output_shape(*args)


def test_error_paths_return_zero_with_message():
    from pwcnet_amd import _lib
    lib = _lib.load()
    null = ctypes.c_void_p(0)
    one = ctypes.c_void_p(16)
    # unsupported dtype: rejected before any HIP call
    assert lib.pwc_corr_forward(one, one, one, 1, 1, 4, 4, 9, 1, 9, 1, 2, 1, 7, null) == 0
    assert b"dtype" in lib.pwc_last_error()
    # null buffers
    assert lib.pwc_warp_forward(null, null, null, 1, 1, 4, 4, 0, null) == 0
    assert b"null" in lib.pwc_last_error()
    # reference backward is undefined for stride1 != 1
    assert lib.pwc_corr_backward(one, one, one, one, one, 1, 1, 8, 8, 4, 1, 4, 2, 1, 1, 0,
                                 null) == 0
    assert b"stride1" in lib.pwc_last_error()
    # empty output (pad too small for the displacement)
    assert lib.pwc_corr_forward(one, one, one, 1, 1, 4, 4, 0, 1, 9, 1, 2, 1, 0, null) == 0
    assert b"empty" in lib.pwc_last_error()
    # warp backward is fp32 only
    assert lib.pwc_warp_backward(one, one, one, one, one, 1, 1, 4, 4, 1, null) == 0
    # ABI 8's workspace form: the same checks, and no workspace asked for where the tile path
    # declines (narrow images) or for a bad dtype / negative dims
    assert lib.pwc_warp_backward_ws(one, one, one, one, one, 1, 1, 4, 4, 1, null, 0, null) == 0
    assert b"fp32 only" in lib.pwc_last_error()
    assert lib.pwc_warp_backward_ws(null, null, null, null, null, 1, 1, 4, 4, 0, null, 0,
                                    null) == 0
    assert b"null" in lib.pwc_last_error()
    assert lib.pwc_warp_backward_ws(one, one, one, one, one, 1, 1, -4, 4, 0, null, 0, null) == 0
    assert b"negative" in lib.pwc_last_error()
    assert lib.pwc_warp_backward_workspace_size(8, 32, 96, 112, 1) == 0      # fp16
    assert lib.pwc_warp_backward_workspace_size(8, 32, -96, 112, 0) == 0     # negative dim
    assert lib.pwc_warp_backward_workspace_size(8, 96, 24, 28, 0) == 0       # l2: multi-kernel
    assert lib.pwc_warp_backward_workspace_size(8, 64, 48, 56, 0) > 0        # l3: tile path
    assert lib.pwc_warp_backward_workspace_size(8, 32, 96, 112, 0) > 0       # l4: tile path
    with pytest.raises(RuntimeError, match="aborting"):
        _lib.check(0, "x")


def test_layers_fail_loudly_on_cpu_tensors():
    """No CPU fallback: the product path refuses host tensors."""
    import pwcnet_amd
    x = torch.zeros(1, 4, 8, 8)
    f = torch.zeros(1, 2, 8, 8)
    with pytest.raises(RuntimeError, match="HIP"):
        pwcnet_amd.Correlation(9, 1, 9, 1, 2)(x, x)
    with pytest.raises(RuntimeError, match="HIP"):
        pwcnet_amd.WarpingLayer(None)(x, f)
    with pytest.raises(RuntimeError, match="HIP"):
        pwcnet_amd.CostVolumeLayer(types.SimpleNamespace(search_range=4))(x, x)


def test_correlation_module_signature_matches_reference():
    import inspect
    from correlation_package.modules.correlation import Correlation
    from correlation_package.functions.correlation import CorrelationFunction
    sig = inspect.signature(Correlation.__init__)
    assert [p for p in sig.parameters][1:] == ["pad_size", "kernel_size", "max_displacement",
                                                "stride1", "stride2", "corr_multiply"]
    assert [sig.parameters[p].default for p in list(sig.parameters)[1:]] == [0, 0, 0, 1, 2, 1]
    fsig = inspect.signature(CorrelationFunction.forward)
    assert [fsig.parameters[p].default for p in list(fsig.parameters)[3:]] == [3, 3, 20, 1, 2, 1]
    c = Correlation(pad_size=9, kernel_size=1, max_displacement=9, stride1=1, stride2=2)
    assert len(list(c.parameters())) == 0 and len(list(c.buffers())) == 0


def test_cvl_channel_formula_matches_reference_order():
    """csrc/pwc_common.cuh cvl_channel() restated in Python vs the oracle's modules.py order."""
    from oracle import oracle as O

    def cvl_channel(dy, dx, sr):
        if dy == 0 and dx == 0:
            return 0
        if dx == 0:
            i = abs(dy)
            return 1 + (i - 1) * (4 + 4 * sr) + (0 if dy < 0 else 1)
        if dy == 0:
            i = abs(dx)
            return 1 + (i - 1) * (4 + 4 * sr) + (2 if dx < 0 else 3)
        i, j = abs(dy), abs(dx)
        base = 1 + (i - 1) * (4 + 4 * sr) + 4 + (j - 1) * 4
        if dy < 0 and dx < 0:
            return base
        if dy > 0 and dx > 0:
            return base + 1
        return base + 2 if dy < 0 else base + 3

    for sr in (1, 2, 3, 4, 8):
        dys, dxs = O.cvl_offsets(sr)
        for k, (dy, dx) in enumerate(zip(dys, dxs)):
            assert cvl_channel(dy, dx, sr) == k, (sr, dy, dx, k)


def test_group_entry_host_checks():
    """pwc_warp_corr_forward_group rejects a bad list before any launch: negative count,
    a NULL list, a problem without x2_warp, invalid correlation parameters."""
    from pwcnet_amd import _lib
    lib = _lib.load()
    P = _lib.WarpCorrProblem
    assert lib.pwc_warp_corr_forward_group(None, -1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    assert b"invalid problem list" in lib.pwc_last_error()
    assert lib.pwc_warp_corr_forward_group(None, 1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    arr = (P * 1)(P(1, 1, 1, None, 1, 1, 4, 6, 7))
    assert lib.pwc_warp_corr_forward_group(arr, 1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    assert b"x2_warp is required" in lib.pwc_last_error()
    arr = (P * 1)(P(1, 1, 1, 1, 1, -1, 4, 6, 7))
    assert lib.pwc_warp_corr_forward_group(arr, 1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    assert b"negative dimension" in lib.pwc_last_error()
    arr = (P * 1)(P(1, 1, 1, 1, 1, 1, 4, 6, 7))
    assert lib.pwc_warp_corr_forward_group(arr, 1, 9, 1, 9, 1, 0, 1, 0, None) == 0
    assert b"invalid correlation parameters" in lib.pwc_last_error()
    # a NULL input in a pairable l0 + l1 list is rejected before the pair kernel launches
    # (pwc_warp_corr_forward's own check, repeated up front)
    l0 = P(1, 1, 1, 1, 1, 8, 192, 6, 7)
    for bad in ((None, 1, 1, 1, 1), (1, None, 1, 1, 1), (1, 1, None, 1, 1), (1, 1, 1, 1, None)):
        l1 = P(*bad, 8, 128, 12, 14)
        arr = (P * 2)(l0, l1)
        assert lib.pwc_warp_corr_forward_group(arr, 2, 9, 1, 9, 1, 2, 1, 0, None) == 0
        assert b"null buffer" in lib.pwc_last_error()
    arr = (P * 2)(l0, P(1, 1, 1, 1, 1, 8, 128, 12, 14))
    assert lib.pwc_warp_corr_forward_group(arr, 2, 9, 1, 9, 1, 2, 1, 7, None) == 0
    assert b"unsupported dtype" in lib.pwc_last_error()
    # an empty list is a no-op
    assert lib.pwc_warp_corr_forward_group(None, 0, 9, 1, 9, 1, 2, 1, 0, None) == 1


def test_warp_group_entry_host_checks():
    """pwc_warp_forward_group rejects a bad list before any launch: negative count, a NULL
    list, a negative dimension, a NULL buffer, an unknown dtype; an empty list is a no-op."""
    from pwcnet_amd import _lib
    lib = _lib.load()
    P = _lib.WarpProblem
    assert lib.pwc_warp_forward_group(None, -1, 0, None) == 0
    assert b"invalid problem list" in lib.pwc_last_error()
    assert lib.pwc_warp_forward_group(None, 1, 0, None) == 0
    arr = (P * 1)(P(1, 1, 1, -1, 4, 6, 7))
    assert lib.pwc_warp_forward_group(arr, 1, 0, None) == 0
    assert b"negative dimension" in lib.pwc_last_error()
    arr = (P * 1)(P(1, 1, None, 1, 4, 6, 7))
    assert lib.pwc_warp_forward_group(arr, 1, 0, None) == 0
    assert b"null buffer" in lib.pwc_last_error()
    arr = (P * 1)(P(1, 1, 1, 0, 4, 6, 7))  # empty batch: nothing to launch
    assert lib.pwc_warp_forward_group(arr, 1, 7, None) == 0
    assert b"unsupported dtype" in lib.pwc_last_error()
    assert lib.pwc_warp_forward_group(None, 0, 0, None) == 1
    assert lib.pwc_warp_forward_group(arr, 1, 0, None) == 1


def test_corr_group_entry_host_checks():
    """pwc_corr_forward_group rejects a bad list before any launch: negative count, a NULL
    list, a negative dimension, a NULL buffer, invalid correlation parameters."""
    from pwcnet_amd import _lib
    lib = _lib.load()
    P = _lib.CorrProblem
    assert lib.pwc_corr_forward_group(None, -1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    assert b"invalid problem list" in lib.pwc_last_error()
    assert lib.pwc_corr_forward_group(None, 1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    arr = (P * 1)(P(1, 1, 1, -1, 4, 6, 7))
    assert lib.pwc_corr_forward_group(arr, 1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    assert b"negative dimension" in lib.pwc_last_error()
    arr = (P * 1)(P(1, None, 1, 1, 4, 6, 7))
    assert lib.pwc_corr_forward_group(arr, 1, 9, 1, 9, 1, 2, 1, 0, None) == 0
    assert b"null buffer" in lib.pwc_last_error()
    arr = (P * 1)(P(1, 1, 1, 1, 4, 6, 7))
    assert lib.pwc_corr_forward_group(arr, 1, 9, 1, 9, 1, 0, 1, 0, None) == 0
    assert b"invalid correlation parameters" in lib.pwc_last_error()
    assert lib.pwc_corr_forward_group(None, 0, 9, 1, 9, 1, 2, 1, 0, None) == 1


def test_corr_forward_plan_routes_and_declines():
    """pwc_corr_forward_plan runs the dispatch predicates on the host: the config-2 / config-4
    levels reach their kernels, and grids the 32-bit-addressed strip kernels cannot address
    (an 81-plane output >= 2^31 bytes) fall through to the size_t stream kernel."""
    from pwcnet_amd import _lib
    plan = _lib.corr_forward_plan
    c9 = (9, 1, 9, 1, 2)
    assert plan(8, 32, 96, 112, *c9) == "strip"                # config 2 l4
    assert plan(8, 64, 48, 56, *c9) == "strip"                 # config 2 l3 (C = 64 rows)
    assert plan(8, 96, 24, 28, *c9) == "strip"                 # config 2 l2 (C = 96 quarters)
    assert plan(6, 96, 24, 28, *c9) == "rows"                  # 144 workgroups: row bands
    assert plan(8, 192, 6, 7, *c9) == "band"                   # config 2 l0
    assert plan(16, 32, 112, 256, *c9, dtype=1) == "mstrip16"  # config 4 l4
    assert plan(16, 64, 56, 128, *c9, dtype=1) == "mstrip16"   # config 4 l3
    assert plan(8, 32, 96, 112, 4, 1, 4, 1, 1) == "stream"     # Corr4 at l4
    assert plan(16, 32, 112, 256, 4, 1, 4, 1, 1, dtype=1) == "mstrip16"  # Corr4 fp16 config-4 l4
    assert plan(16, 64, 56, 128, 4, 1, 4, 1, 1, dtype=1) == "mstrip16"   # ... l3
    assert plan(16, 96, 28, 64, 4, 1, 4, 1, 1, dtype=1) == "mstrip16"    # ... l2
    assert plan(8, 32, 112, 256, 4, 1, 4, 1, 1, dtype=1) == "stream"     # 128 workgroups
    # H*W = 8.4 M px: input 1.07 GB (< 2^31, the strip would accept it), output 2.7 GB
    assert plan(1, 32, 3000, 2800, *c9) == "stream"
    assert plan(1, 32, 3000, 2800, *c9, dtype=1) == "mstrip16"  # fp16 output 1.36 GB < 2^31
    assert plan(1, 32, 5000, 2800, *c9, dtype=1) == "stream"    # fp16 output 2.27 GB
    assert plan(8, 32, 96, 112, *c9, ptrs=(0x1004, 0x2000, 0x3000)) != "strip"  # unaligned
    assert plan(8, 32, 96, 112, 9, 1, 9, 1, 2, dtype=7) == -1
    assert plan(8, 32, 96, 112, 9, 1, 9, 0, 2) == -1


def test_corr_backward_plan_routes_and_declines():
    """pwc_corr_backward_plan: config 5's l4 / l3 / l2 backward reach the displacement-row
    strip kernel, the other levels the row-band kernel, other configurations and dtypes the
    stencil kernels; rejected arguments -1."""
    from pwcnet_amd import _lib
    plan = _lib.corr_backward_plan
    c9 = (9, 1, 9, 1, 2)
    assert plan(8, 32, 96, 112, *c9) == "strip"   # config 5 l4
    assert plan(8, 64, 48, 56, *c9) == "strip"    # config 5 l3
    assert plan(1, 32, 7, 112, *c9) == "rows"     # 8 workgroups: the row-band kernel
    assert plan(4, 32, 96, 112, *c9) == "strip"   # 256 workgroups
    assert plan(2, 32, 96, 112, *c9) == "rows"    # 128: below 192
    assert plan(4, 64, 48, 56, *c9) == "rows"     # 128 at l3
    assert plan(4, 96, 24, 28, *c9) == "rows"     # 96 at l2
    assert plan(8, 96, 24, 28, *c9) == "strip"    # l2
    assert plan(8, 96, 24, 30, *c9) == "rows"     # l2-like, another width
    assert plan(8, 192, 6, 7, *c9) == "rows"      # l0
    assert plan(8, 32, 96, 112, 8, 1, 8, 1, 2) == "strip"  # pad = md = 8
    assert plan(8, 32, 96, 112, 4, 1, 4, 1, 1) == "other"  # Corr4
    assert plan(8, 32, 96, 112, *c9, dtype=1) == "other"   # fp16 storage
    assert plan(8, 32, 96, 112, *c9, ptrs=(0x1000, 0x2000, 0x3004, 0x4000, 0x5000)) == "rows"
    assert plan(8, 32, 96, 112, 9, 1, 9, 2, 2) == -1       # stride1 != 1: undefined backward
    assert plan(8, 32, 96, 112, *c9, dtype=5) == -1


def test_missing_library_fails_loudly(tmp_path):
    """No silent fallback: with the HIP library absent, loading it raises HipLibraryMissing, and
    an op on CPU tensors raises too (the product path has no CPU or oracle route)."""
    import subprocess
    import sys
    code = (
        "import torch, pwcnet_amd\n"
        "from pwcnet_amd import _lib\n"
        "from pwcnet_amd.ops import corr_forward, warp_forward\n"
        "a, f = torch.zeros(1, 4, 6, 7), torch.zeros(1, 2, 6, 7)\n"
        "try:\n"
        "    _lib.load()\n"
        "except _lib.HipLibraryMissing as e:\n"
        "    print('missing:', e)\n"
        "for fn in (lambda: corr_forward(a, a, 9, 1, 9, 1, 2), lambda: warp_forward(a, f)):\n"
        "    try:\n"
        "        fn()\n"
        "    except RuntimeError as e:\n"
        "        print('raised:', e)\n")
    env = dict(os.environ, PWC_HOTPATH_LIB=str(tmp_path / "absent.so"))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(root, "pwc-net_pytorch_amd"), root,
                                         env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "missing:" in r.stdout and "not built" in r.stdout, r.stdout
    assert r.stdout.count("raised:") == 2 and "HIP devices only" in r.stdout, r.stdout
