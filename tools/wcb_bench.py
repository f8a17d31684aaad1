#!/usr/bin/env python3
"""Level backward of config 5's l0 / l1 / l2 (B = 8): the one-launch
warp_corr_backward against the two-launch path (corr_backward + warp_backward), each timed as
20 back-to-back calls replayed from one hipGraph (event-timed, us per call), for the knob
settings given (PWC_DEBUG syntax; "-" = defaults).

    python tools/wcb_bench.py [- wcb_abl=1 warp_corr_bwd=0 ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import warp_corr_backward, warp_forward  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / reps * 1e3)
    return best


def main():
    knobs = sys.argv[1:] or ["-"]
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(3)
    B = 8
    for l, (C, h, w) in enumerate(bench.level_shapes(384, 448)[:3]):
        x1 = torch.randn(B, C, h, w, device=dev, generator=gen)
        x2 = torch.randn(B, C, h, w, device=dev, generator=gen)
        fl = torch.randn(B, 2, h, w, device=dev, generator=gen) * 2
        gc = torch.randn(B, 81, h, w, device=dev, generator=gen)
        x2w = warp_forward(x2, fl)
        for k in knobs:
            _lib.set_debug("" if k == "-" else k)
            us = timed(lambda: warp_corr_backward(x1, x2, fl, x2w, gc, **bench.CORR_ARGS))
            _lib.set_debug("")
            print(json.dumps(dict(level=l, shape=[B, C, h, w], knobs=k, us=round(us, 2))),
                  flush=True)


if __name__ == "__main__":
    main()
