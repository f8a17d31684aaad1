#!/usr/bin/env python3
"""Phase census of the displacement-row correlation backward (csrc/corr_bwd_strip.hip) at one
config-5 level: needs a census build of the library,

    UNIT=corr_bwd_strip DEFS=-DPWC_BSTRIP_CENSUS bash tools/build_variant.sh abl/cen
    PWC_HOTPATH_LIB=abl/cen/libpwc_hotpath.so python tools/bstrip_census.py --level 4

Per workgroup, s_memrealtime stamps (100 MHz, 10 ns) of: entry, the barriers B_0 .. B_8, the
last FMA, the stores issued (compute wave 0), and the loaders' prologue landing.  Prints, per
round of workgroups (by entry time), the median / max of each stamp relative to the
workgroup's entry, and the launch span."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import corr_backward  # noqa: E402

NAMES = ["entry"] + [f"B{u}" for u in range(9)] + ["fma_done", "stored", "rows0", "gO0"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    lib = _lib.load()
    fn = lib.pwc_debug_bstrip_census
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    C, H, W = bench.level_shapes(384, 448)[args.level]
    B = args.batch
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    a = torch.randn(B, C, H, W, device=dev, generator=g)
    b = torch.randn(B, C, H, W, device=dev, generator=g)
    go = torch.randn(B, 81, H, W, device=dev, generator=g)
    for _ in range(5):
        corr_backward(a, b, go, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    fn(None, 0)
    torch.cuda.synchronize()
    corr_backward(a, b, go, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    n = 8192 * 16
    buf = (ctypes.c_ulonglong * n)()
    assert fn(ctypes.addressof(buf), n)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 16).astype(np.int64)
    blk = np.nonzero(st[:, 0] != 0)[0]
    st = st[blk]
    t0 = st[:, 0].min()
    entry = st[:, 0] - t0
    out = {"level": args.level, "wgs": int(len(st)), "span_us": float((st[:, 11].max() - t0) / 100)}
    # entry by hardware XCD (blockIdx % 8) and by the remapped half (first / second gradient)
    out["entry_by_xcd_us"] = [round(float(np.median(entry[blk % 8 == x])) / 100, 2) for x in range(8)]
    q = np.quantile(entry, [0, 0.125, 0.25, 0.375, 0.5, 0.625, 0.75, 0.875, 1]) / 100
    out["entry_quantiles_us"] = [round(float(v), 2) for v in q]
    # rounds: workgroups entering within the first 2 us of the launch vs later
    first = entry < 200
    for name, sel in (("round0", first), ("round1", ~first)):
        if sel.sum() == 0:
            continue
        rel = (st[sel] - st[sel][:, :1]) / 100.0
        d = {"wgs": int(sel.sum()), "entry_abs": [float(np.median(entry[sel]) / 100),
                                                  float(entry[sel].max() / 100)]}
        for k, nm in enumerate(NAMES):
            if k == 0:
                continue
            col = rel[:, k]
            col = col[st[sel][:, k] != 0]
            if len(col):
                d[nm] = [round(float(np.median(col)), 2), round(float(col.max()), 2)]
        out[name] = d
    print(json.dumps(out))


if __name__ == "__main__":
    main()
