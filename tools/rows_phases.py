#!/usr/bin/env python3
"""Phase census of the row-band correlation kernel (csrc/corr_rows.hip) at one level:
per-workgroup s_memrealtime stamps (100 MHz) -> [median, max] us after the first entry.

    python tools/rows_phases.py --level 3
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd")); sys.path.insert(0, ROOT)
import numpy as np
import torch
import bench
from pwcnet_amd import _lib
from pwcnet_amd.ops import corr_forward

NAMES = {0: "entry", 1: "chunk0_staged", 3: "chunk1_staged", 4: "compute_done",
         5: "partials_in_lds", 6: "stores_issued"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=3)
    ap.add_argument("--knobs", default="")
    args = ap.parse_args()
    C, h, w = bench.level_shapes(384, 448)[args.level]
    B, dev = 8, torch.device("cuda:0")
    x1 = torch.randn(B, C, h, w, device=dev)
    x2 = torch.randn(B, C, h, w, device=dev)
    lib = _lib.load()
    lib.pwc_debug_rows_census.restype = ctypes.c_int
    lib.pwc_debug_rows_census.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _lib.set_debug(",".join(k for k in ("rows_census=1", args.knobs) if k))
    for _ in range(3):
        corr_forward(x1, x2, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    lib.pwc_debug_rows_census(None, 0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    corr_forward(x1, x2, 9, 1, 9, 1, 2)
    b.record()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.pwc_debug_rows_census(buf.ctypes.data, buf.size) == 1
    _lib.set_debug("")
    t = buf.reshape(4096, 8).astype(np.int64)
    t = t[t[:, 0] > 0]
    rel = np.where(t > 0, (t - t[:, 0].min()) / 100.0, np.nan)
    out = dict(level=args.level, wgs=int(len(t)), event_us=round(a.elapsed_time(b) * 1e3, 2))
    for k, n in NAMES.items():
        col = rel[:, k]
        if not np.isnan(col).all():
            out[n] = [round(float(np.nanmedian(col)), 2), round(float(np.nanmax(col)), 2)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
