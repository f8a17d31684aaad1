#!/usr/bin/env python3
"""Phase census of the correlation-backward row-band kernel (csrc/corr_bwd_rows.hip) at one
level: per-workgroup s_memrealtime stamps (100 MHz).  Stamps are read relative to each
workgroup's own entry (the XCDs' clocks differ by ~2 us) and, for the entry itself, relative to
the earliest entry of the same XCD (blockIdx % 8).  Workgroups are split into dispatch rounds
by entry time.

    make -C pwc-net_pytorch_amd/csrc -B CENSUS=1 && python tools/bwd_phases.py --level 4
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import corr_backward  # noqa: E402

NAMES = {1: "chunk0_staged", 2: "chunk0_computed", 3: "last_staged", 4: "last_computed",
         5: "stores_issued"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=4)
    ap.add_argument("--knobs", default="")
    args = ap.parse_args()
    C, h, w = bench.level_shapes(384, 448)[args.level]
    B, dev = 8, torch.device("cuda:0")
    x1 = torch.randn(B, C, h, w, device=dev)
    x2 = torch.randn(B, C, h, w, device=dev)
    go = torch.randn(B, 81, h, w, device=dev)
    lib = _lib.load()
    lib.pwc_debug_bwd_census.restype = ctypes.c_int
    lib.pwc_debug_bwd_census.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _lib.set_debug(",".join(k for k in ("bwd_census=1", args.knobs) if k))
    for _ in range(3):
        corr_backward(x1, x2, go, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    lib.pwc_debug_bwd_census(None, 0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    corr_backward(x1, x2, go, 9, 1, 9, 1, 2)
    b.record()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.pwc_debug_bwd_census(buf.ctypes.data, buf.size) == 1
    _lib.set_debug("")
    t = buf.reshape(4096, 8).astype(np.int64)
    ids = np.nonzero(t[:, 0] > 0)[0]
    if len(ids) == 0:
        sys.exit("no census stamps: build the library with `make CENSUS=1` first")
    t = t[ids]
    xcd = ids % 8
    entry = np.zeros(len(t))
    for x in range(8):
        m = xcd == x
        if m.any():
            entry[m] = (t[m, 0] - t[m, 0].min()) / 100.0
    rel = np.where(t > 0, (t - t[:, [0]]) / 100.0, np.nan)
    out = dict(level=args.level, wgs=int(len(t)), event_us=round(a.elapsed_time(b) * 1e3, 2),
               knobs=args.knobs)
    # rounds: a gap > 2 us in the sorted entry times of one XCD starts a new round
    rnd = np.zeros(len(t), int)
    for x in range(8):
        m = np.nonzero(xcd == x)[0]
        order = m[np.argsort(entry[m])]
        r = 0
        for i in range(1, len(order)):
            if entry[order[i]] - entry[order[i - 1]] > 2.0:
                r += 1
            rnd[order[i]] = r
    for r in range(rnd.max() + 1):
        m = rnd == r
        row = {"wgs": int(m.sum()), "entry": [round(float(np.median(entry[m])), 2),
                                              round(float(entry[m].max()), 2)]}
        for k, n in NAMES.items():
            col = rel[m, k]
            if not np.isnan(col).all():
                row[n] = [round(float(np.nanmedian(col)), 2), round(float(np.nanmax(col)), 2)]
        out[f"round{r}"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
