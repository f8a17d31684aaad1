"""ctypes binding of the C ABI in include/pwc_hotpath.h (libpwc_hotpath.so, gfx950).

The library is built in-tree (``make -C pwc-net_pytorch_amd/csrc`` or
``__graft_entry__.build()``).  There is no CPU fallback: if the library is missing or a
tensor is not on a HIP device every entry point raises.  ctypes releases the GIL around each
call, as the reference's cffi wrapper did (correlation_package/_ext/correlation/__init__.py).

``torch`` is imported first so that the HIP runtime torch ships is the one that satisfies the
library's ``libamdhip64.so.7`` dependency (one runtime per process; torch's streams are then
valid handles for the library).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

# PWC_HOTPATH_LIB overrides the library path (diagnostic builds, e.g. tools/ ablations).
LIB_PATH = os.environ.get("PWC_HOTPATH_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libpwc_hotpath.so")

DTYPE_CODES = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}

# Every symbol the header declares: (name, restype, argtypes).
_P = ctypes.c_void_p
_I = ctypes.c_int
_Z = ctypes.c_size_t
_IP = ctypes.POINTER(ctypes.c_int)


class WarpCorrProblem(ctypes.Structure):
    """pwc_warp_corr_problem (include/pwc_hotpath.h)."""
    _fields_ = [("in1", _P), ("x2", _P), ("flow", _P), ("x2_warp", _P), ("out", _P),
                ("B", _I), ("C", _I), ("H", _I), ("W", _I)]


class WarpProblem(ctypes.Structure):
    """pwc_warp_problem (include/pwc_hotpath.h)."""
    _fields_ = [("x", _P), ("flow", _P), ("out", _P), ("B", _I), ("C", _I), ("H", _I),
                ("W", _I)]


class CorrProblem(ctypes.Structure):
    """pwc_corr_problem (include/pwc_hotpath.h)."""
    _fields_ = [("in1", _P), ("in2", _P), ("out", _P), ("B", _I), ("C", _I), ("H", _I),
                ("W", _I)]


SYMBOLS = {
    "pwc_abi_version": (_I, []),
    "pwc_corr_forward_plan": (_I, [_P, _P, _P] + [_I] * 10),
    "pwc_corr_backward_plan": (_I, [_P] * 5 + [_I] * 10),
    "pwc_last_error": (ctypes.c_char_p, []),
    "pwc_time_next_corr": (_I, [_P, _P]),
    "pwc_set_debug": (_I, [ctypes.c_char_p]),
    "pwc_corr_output_shape": (_I, [_I] * 7 + [_IP] * 3),
    "pwc_corr_forward": (_I, [_P, _P, _P] + [_I] * 11 + [_P]),
    "pwc_corr_workspace_size": (_Z, [_I] * 9),
    "pwc_corr_forward_ws": (_I, [_P, _P, _P] + [_I] * 11 + [_P, _Z, _P]),
    "pwc_corr_backward": (_I, [_P, _P, _P, _P, _P] + [_I] * 11 + [_P]),
    "pwc_cost_volume_forward": (_I, [_P, _P, _P] + [_I] * 6 + [_P]),
    "pwc_cost_volume_workspace_size": (_Z, [_I] * 5),
    "pwc_cost_volume_forward_ws": (_I, [_P, _P, _P] + [_I] * 6 + [_P, _Z, _P]),
    "pwc_cost_volume_backward": (_I, [_P, _P, _P, _P, _P] + [_I] * 6 + [_P]),
    "pwc_warp_forward": (_I, [_P, _P, _P] + [_I] * 5 + [_P]),
    "pwc_warp_backward": (_I, [_P, _P, _P, _P, _P] + [_I] * 5 + [_P]),
    "pwc_warp_backward_workspace_size": (_Z, [_I] * 5),
    "pwc_warp_backward_ws": (_I, [_P, _P, _P, _P, _P] + [_I] * 5 + [_P, _Z, _P]),
    "pwc_warp_corr_workspace_size": (_Z, [_I] * 11),
    "pwc_warp_corr_forward": (_I, [_P] * 5 + [_I] * 11 + [_P, _Z, _P]),
    "pwc_warp_corr_forward_group": (_I, [ctypes.POINTER(WarpCorrProblem)] + [_I] * 8 + [_P]),
    "pwc_warp_corr_backward_workspace_size": (_Z, [_I] * 10),
    "pwc_warp_corr_backward": (_I, [_P] * 9 + [_I] * 11 + [_P, _Z, _P, _P]),
    "pwc_corr_forward_group": (_I, [ctypes.POINTER(CorrProblem)] + [_I] * 8 + [_P]),
    "pwc_warp_forward_group": (_I, [ctypes.POINTER(WarpProblem), _I, _I, _P]),
    "pwc_upsample_warp_forward": (_I, [_P] * 4 + [_I] * 5 + [_P]),
    "pwc_flow_upsample_backward": (_I, [_P, _P] + [_I] * 4 + [_P]),
    "pwc_corr_forward_into_workspace_size": (_Z, [_I] * 10),
    "pwc_corr_forward_into": (_I, [_P, _P, _P, ctypes.c_longlong, ctypes.c_float] + [_I] * 11
                              + [_P, _Z, _P]),
}
ABI_VERSION = 11

_lock = threading.Lock()
_lib = None


class HipLibraryMissing(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and type the hot-path library; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HipLibraryMissing(
                f"pwcnet_amd: HIP library not built ({LIB_PATH}); run "
                "`make -C pwc-net_pytorch_amd/csrc` or `python -c 'import __graft_entry__ as g; "
                "g.build()'`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SYMBOLS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.pwc_abi_version()
        if v != ABI_VERSION:
            raise HipLibraryMissing(f"pwcnet_amd: ABI version {v} != expected {ABI_VERSION}")
        _lib = lib
    return _lib


def check(ret: int, what: str) -> None:
    """Reference: a 0 return became THError("aborting") (correlation_cuda.c:86-89)."""
    if ret != 1:
        msg = load().pwc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} aborting: {msg}")


def corr_output_shape(H, W, pad, k, md, s1, s2):
    oc, oh, ow = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(load().pwc_corr_output_shape(H, W, pad, k, md, s1, s2, ctypes.byref(oc),
                                       ctypes.byref(oh), ctypes.byref(ow)),
          "Correlation")
    return oc.value, oh.value, ow.value


PLAN_NAMES = {0: "other", 1: "stream", 2: "band", 3: "rows", 4: "strip", 5: "mstrip16"}


def corr_forward_plan(B, C, H, W, pad, k, md, s1, s2, dtype=0, ptrs=(0x1000, 0x2000, 0x3000)):
    """Kernel family pwc_corr_forward would launch (pwc_corr_forward_plan; no device call)."""
    r = load().pwc_corr_forward_plan(*ptrs, B, C, H, W, pad, k, md, s1, s2, dtype)
    return PLAN_NAMES.get(r, r)


BWD_PLAN_NAMES = {0: "other", 1: "rows", 2: "strip"}


def corr_backward_plan(B, C, H, W, pad, k, md, s1, s2, dtype=0,
                       ptrs=(0x1000, 0x2000, 0x3000, 0x4000, 0x5000)):
    """Kernel family pwc_corr_backward would launch (pwc_corr_backward_plan; no device call)."""
    r = load().pwc_corr_backward_plan(*ptrs, B, C, H, W, pad, k, md, s1, s2, dtype)
    return BWD_PLAN_NAMES.get(r, r)


def set_debug(spec: str = "") -> None:
    """Measurement / test hook (pwc_set_debug): knobs as "name=value,...", "" = defaults."""
    check(load().pwc_set_debug(spec.encode()), "pwc_set_debug")
