#!/usr/bin/env python3
"""Kernel-variant sweep: for each PWC_DEBUG knob string, the op's output is compared with the
default path's (itself parity-tested against the oracle) and timed (kbench.timeit).

    python tools/variants.py --op corr --level 4 --knobs "stream_cfg=3;stream_cfg=4"
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import bench  # noqa: E402
from kbench import timeit  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import (corr_backward, corr_forward, warp_backward,  # noqa: E402
                            warp_corr_forward, warp_forward)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="corr")
    ap.add_argument("--level", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=448)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--knobs", default="")
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--flow-scale", type=float, default=2.0)
    args = ap.parse_args()
    dt = torch.float32 if args.dtype == "fp32" else torch.float16
    esz = 4 if dt == torch.float32 else 2
    dev = torch.device("cuda:0")
    C, h, w = bench.level_shapes(args.height, args.width)[args.level]
    B = args.batch
    per = (3 * C * h * w + 83 * h * w) * B * esz
    n = max(2, int(2 * 256 * 2 ** 20 / per) + 1)
    g = torch.Generator(device=dev).manual_seed(7)
    sets = [dict(x1=torch.randn(B, C, h, w, device=dev, generator=g).to(dt),
                 x2=torch.randn(B, C, h, w, device=dev, generator=g).to(dt),
                 fl=(torch.randn(B, 2, h, w, device=dev, generator=g) * args.flow_scale).to(dt),
                 go=torch.randn(B, 81, h, w, device=dev, generator=g).to(dt),
                 gw=torch.randn(B, C, h, w, device=dev, generator=g).to(dt))
            for _ in range(n)]
    ops = {
        "corr": (lambda s: corr_forward(s["x1"], s["x2"], 9, 1, 9, 1, 2),
                 bench.corr_bytes_per_pair(C, h, w, esz) * B),
        "corr4": (lambda s: corr_forward(s["x1"], s["x2"], 4, 1, 4, 1, 1),
                  bench.corr_bytes_per_pair(C, h, w, esz) * B),
        "warp": (lambda s: warp_forward(s["x2"], s["fl"]), (2 * C * h * w + 2 * h * w) * B * esz),
        "corr_bwd": (lambda s: corr_backward(s["x1"], s["x2"], s["go"], 9, 1, 9, 1, 2),
                     (4 * C * h * w + 81 * h * w) * B * esz),
        "warp_corr": (lambda s: warp_corr_forward(s["x1"], s["x2"], s["fl"], 9, 1, 9, 1, 2),
                      (3 * C * h * w + 2 * h * w + 81 * h * w) * B * esz),
        "warp_bwd": (lambda s: warp_backward(s["x2"], s["fl"], s["gw"]),
                     (3 * C * h * w + 4 * h * w) * B * esz),
    }
    fn, nbytes = ops[args.op]
    _lib.set_debug("")
    ref = fn(sets[0])
    ref = [r.clone() for r in ref] if isinstance(ref, tuple) else [ref.clone()]
    for knob in [""] + [k for k in args.knobs.split(";") if k]:
        _lib.set_debug(knob)
        out = fn(sets[0])
        out = list(out) if isinstance(out, tuple) else [out]
        diffs = [float(((a.float() - b.float()).abs() / (1 + b.float().abs())).max())
                 for a, b in zip(out, ref)]
        diff = max(diffs)
        out = [o.clone() for o in out]
        rep = [fn(sets[0]) for _ in range(3)]
        same = all(torch.equal(a, b) for r in rep
                   for a, b in zip(list(r) if isinstance(r, tuple) else [r], out))
        med, mn = timeit(fn, sets, args.iters)
        print(json.dumps(dict(op=args.op, level=args.level, dtype=args.dtype, knob=knob or "default",
                              us=round(med, 2), min_us=round(mn, 2),
                              gbs=round(nbytes / (med * 1e-6) / 1e9, 1), max_rel_diff=diff, diffs=diffs,
                              repeatable=same)),
              flush=True)
    _lib.set_debug("")


if __name__ == "__main__":
    main()
