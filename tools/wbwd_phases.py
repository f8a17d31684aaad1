#!/usr/bin/env python3
"""Phase census of the one-launch warp backward tile kernel (csrc/warp_bwd.hip) at one level:
per-workgroup s_memrealtime stamps (100 MHz) -> median / max of each phase, in us.

    python tools/wbwd_phases.py --level 4
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd")); sys.path.insert(0, ROOT)
import numpy as np
import torch
import bench
from pwcnet_amd import _lib
from pwcnet_amd.ops import warp_backward


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=4)
    ap.add_argument("--knobs", default="")
    ap.add_argument("--census", type=int, default=1,
                    help="census knob: 1 = marks; | 2 no loads, | 4 no grad_x, | 8 no grad_x stores")
    args = ap.parse_args()
    C, h, w = bench.level_shapes(384, 448)[args.level]
    B, dev = 8, torch.device("cuda:0")
    x = torch.randn(B, C, h, w, device=dev)
    g = torch.randn(B, C, h, w, device=dev)
    fl = torch.randn(B, 2, h, w, device=dev) * 2
    lib = _lib.load()
    lib.pwc_debug_wbwd_census.restype = ctypes.c_int
    lib.pwc_debug_wbwd_census.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _lib.set_debug(",".join(k for k in (f"warp_bwd_census={args.census}", args.knobs) if k))
    for _ in range(3):
        warp_backward(x, fl, g)
    torch.cuda.synchronize()
    lib.pwc_debug_wbwd_census(None, 0)
    warp_backward(x, fl, g)
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 16, np.uint64)
    assert lib.pwc_debug_wbwd_census(buf.ctypes.data, buf.size) == 1
    _lib.set_debug("")
    t = buf.reshape(4096, 16).astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    rel = np.where(t > 0, (t - t0) / 100.0, np.nan)
    out = dict(level=args.level, census=args.census, wgs=int(len(t)), entry=[round(float(np.nanmedian(rel[:, 0])), 2),
                                                         round(float(np.nanmax(rel[:, 0])), 2)])
    names = {1: "lists", 2: "own", 15: "chunks_done"}
    names.update({3 + i: f"chunk{i}" for i in range(12)})
    if args.census & 16:  # sub-phases of chunks 2 and 3 (warp_bwd_tile's WB_SUB marks)
        sub = ["entry", "bar1", "bar2", "issued", "gx_stored", "own_done"]
        names.update({3 + 6 * c + j: f"c{2 + c}_{sub[j]}" for c in range(2) for j in range(6)})
    for k in [1, 2] + list(range(3, 15)) + [15]:
        col = rel[:, k] - rel[:, 0]
        if np.isnan(col).all():
            continue
        out[names[k]] = [round(float(np.nanmedian(col)), 2), round(float(np.nanmax(col)), 2)]
    out["last_end"] = round(float(np.nanmax(rel[:, 15])), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
