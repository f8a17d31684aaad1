#!/usr/bin/env python3
"""Phase timeline of the fused band kernel (warp_corr.hip) from in-kernel s_memrealtime stamps.

    PWC_DEBUG=band_r=3,band_t=1 python tools/band_phases.py --level 0

Prints, over the workgroups of one launch: entry-time spread, and per phase (clear+f1 issue,
staging, compute, reduce, epilogue) the median / max duration, in microseconds (100 MHz clock).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)
os.environ["PWC_DEBUG"] = ",".join(
    x for x in (os.environ.get("PWC_DEBUG", ""), "band_abl=256") if x)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import warp_corr_forward  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=0)
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    C, h, w = bench.level_shapes(384, 448)[args.level]
    B = args.batch
    dev = torch.device("cuda:0")
    x1 = torch.randn(B, C, h, w, device=dev)
    x2 = torch.randn(B, C, h, w, device=dev)
    fl = torch.randn(B, 2, h, w, device=dev) * 2
    lib = _lib.load()
    lib.pwc_debug_band_times.restype = ctypes.c_int
    lib.pwc_debug_band_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        warp_corr_forward(x1, x2, fl, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    zero = np.zeros(4096 * 8, np.uint64)
    lib.pwc_debug_band_reset.argtypes = []
    lib.pwc_debug_band_reset()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    warp_corr_forward(x1, x2, fl, 9, 1, 9, 1, 2)
    b.record()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.pwc_debug_band_times(buf.ctypes.data, buf.size) == 1
    full = buf.reshape(4096, 8).astype(np.int64)
    full = full[full[:, 0] > 0]
    t = full[:, :6]
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0  # us
    ph = np.diff(rel, axis=1)
    names = ["clear+f1issue", "staging", "compute", "reduce", "epilogue"]
    out = dict(level=args.level, cfg=os.environ.get("PWC_DEBUG", ""), wgs=int(len(t)),
               event_us=round(a.elapsed_time(b) * 1e3, 2),
               entry_spread_us=round(float(rel[:, 0].max()), 2),
               last_end_us=round(float(rel[:, 5].max()), 2))
    we = (full[:, 6] - full[:, 0]) / 100.0
    wb = (full[:, 7] - full[:, 0]) / 100.0
    out["last_wave_entry_after_wave0"] = [round(float(np.median(we)), 2), round(float(we.max()), 2)]
    out["last_wave_at_barrier1"] = [round(float(np.median(wb)), 2), round(float(wb.max()), 2)]
    for i, n in enumerate(names):
        out[n] = [round(float(np.median(ph[:, i])), 2), round(float(ph[:, i].max()), 2)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
