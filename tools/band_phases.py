#!/usr/bin/env python3
"""Phase census of the fused warp + correlation band kernel (csrc/warp_corr.hip) at config 2's
l0 / l1: knob band_abl=256 makes thread 0 of every workgroup stamp s_memrealtime (100 MHz) at
entry (0), after the LDS clear (1), after the staging barrier (2), after the FMA loop (3), after
the partial sums are parked (4) and at the end (5).  Prints, in us, the median / max of each
stamp relative to the workgroup's entry, the entry spread and the last end.

    python tools/band_phases.py --level 1
"""
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
from pwcnet_amd.ops import warp_corr_forward  # noqa: E402

NAMES = ["entry", "cleared", "staged", "fma_done", "parked", "end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--knobs", default="")
    ap.add_argument("--chain", type=int, default=1)
    args = ap.parse_args()
    C, H, W = bench.level_shapes(384, 448)[args.level]
    B, dev = args.batch, torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    x1 = torch.randn(B, C, H, W, device=dev, generator=g)
    x2 = torch.randn(B, C, H, W, device=dev, generator=g)
    fl = torch.randn(B, 2, H, W, device=dev, generator=g) * 2
    lib = _lib.load()
    lib.pwc_debug_band_times.restype = ctypes.c_int
    lib.pwc_debug_band_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.pwc_debug_band_reset.restype = ctypes.c_int
    _lib.set_debug(",".join(k for k in (args.knobs or "band_abl=256",) if k))
    for _ in range(5):
        warp_corr_forward(x1, x2, fl, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    lib.pwc_debug_band_reset()
    # --chain N: the stamped launch is the last of N back to back (every workgroup rewrites its
    # stamps), so it starts behind a running kernel as in the bench, not on an idle GPU
    for _ in range(args.chain):
        warp_corr_forward(x1, x2, fl, 9, 1, 9, 1, 2)
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.pwc_debug_band_times(buf.ctypes.data, buf.size) == 1
    _lib.set_debug("")
    t = buf.reshape(4096, 8).astype(np.int64)
    blk = np.nonzero(t[:, 0] > 0)[0]
    t = t[blk]
    t0 = t[:, 0].min()
    ent = (t[:, 0] - t0) / 100.0
    # entry against the block index (dispatch order) and by hardware XCD (blockIdx % 8)
    order = np.argsort(blk)
    q = len(blk) // 4
    print(json.dumps({"entry_by_block_quarter_us": [round(float(np.median(ent[order[i * q:(i + 1) * q]])), 2)
                                                     for i in range(4)],
                      "entry_by_xcd_us": [round(float(np.median(ent[blk % 8 == x])), 2)
                                          for x in range(8)],
                      "entry_first_16_blocks_us": [round(float(v), 2) for v in ent[order[:16]]]}))
    out = dict(level=args.level, wgs=int(len(t)),
               entry_spread_us=round(float((t[:, 0].max() - t0) / 100), 2),
               last_end_us=round(float((t[:, 5].max() - t0) / 100), 2))
    for k in range(1, 6):
        col = (t[:, k] - t[:, 0]) / 100.0
        out[NAMES[k]] = [round(float(np.median(col)), 2), round(float(col.max()), 2)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
