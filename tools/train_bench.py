#!/usr/bin/env python3
"""Training-step timing of the hot path (BASELINE.json config 5: B=8 384x448, 1 GPU).

One step = for every correlated level l0..l4 (model.py:72-113): forward warp (modules.py:31-42)
+ Correlation (model.py:24), then the backward of both for an upstream gradient of the cost
volume: Correlation backward (correlation_cuda_kernel.cu:108-290 -> d/dx1, d/dx2_warp), then
WarpingLayer backward (ATen grid_sampler_2d_backward semantics -> d/dx2, d/dflow).  Each step
is one hipGraph replay; inputs rotate past the Infinity Cache.  Prints one JSON line.

    python tools/train_bench.py [--steps 100] [--warmup 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd.ops import (corr_backward, corr_forward, corr_forward_group,  # noqa: E402
                            warp_backward, warp_corr_forward, warp_corr_forward_group,
                            warp_forward, warp_forward_group)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100)  # ~28 ms: clocks settle
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=448)
    ap.add_argument("--fused-levels", default="0,1",
                    help="levels whose forward runs as one WarpCorrelation launch (as bench.py)")
    ap.add_argument("--group", default="on", choices=["on", "off"],
                    help="forward as bench.py's grouped launches (the levels' inputs are "
                         "independent here): fused l0+l1 pair, one warp group, the row-band "
                         "correlation pair; off = one call per level")
    args = ap.parse_args()
    fused = {int(v) for v in args.fused_levels.split(",") if v.strip()}
    dev = torch.device("cuda:0")
    B = args.batch
    shapes = bench.level_shapes(args.height, args.width)
    per = sum((4 * C * h * w + 4 * h * w + 2 * 81 * h * w) * B * 4 for C, h, w in shapes)
    nsets = max(2, int(2 * 256 * 2 ** 20 / per) + 1)
    gen = torch.Generator(device=dev).manual_seed(7)
    sets = []
    for _ in range(nsets):
        s = []
        for C, h, w in shapes:
            s.append(dict(x1=torch.randn(B, C, h, w, device=dev, generator=gen),
                          x2=torch.randn(B, C, h, w, device=dev, generator=gen),
                          fl=torch.randn(B, 2, h, w, device=dev, generator=gen) * 2.0,
                          gc=torch.randn(B, 81, h, w, device=dev, generator=gen)))
        sets.append(s)

    def forward_grouped(s):
        last = len(s) - 1
        fl = sorted(l for l in fused if l < last)
        for l, (c, w) in zip(fl, warp_corr_forward_group(
                [(s[l]["x1"], s[l]["x2"], s[l]["fl"]) for l in fl], **bench.CORR_ARGS)):
            s[l]["corr"], s[l]["x2w"] = c, w
        wl = [l for l in range(last, -1, -1) if l == last or l not in fused]
        for l, w in zip(wl, warp_forward_group([(s[l]["x2"], s[l]["fl"]) for l in wl])):
            s[l]["x2w"] = w
        cl = [l for l in wl if l != last]
        for l, c in zip(cl, corr_forward_group([(s[l]["x1"], s[l]["x2w"]) for l in cl],
                                               **bench.CORR_ARGS)):
            s[l]["corr"] = c
        s[last]["corr"] = corr_forward(s[last]["x1"], s[last]["x2w"], **bench.CORR_ARGS)
        for lv in s:
            g1, g2w = corr_backward(lv["x1"], lv["x2w"], lv["gc"], **bench.CORR_ARGS)
            lv["g1"] = g1
            lv["gx2"], lv["gfl"] = warp_backward(lv["x2"], lv["fl"], g2w)

    def one(s):
        if args.group == "on":
            forward_grouped(s)
            return
        for l, lv in enumerate(s):
            if l in fused:  # model.py:80-83 as one WarpCorrelation launch (emits x2_warp too)
                lv["corr"], x2w = warp_corr_forward(lv["x1"], lv["x2"], lv["fl"],
                                                    **bench.CORR_ARGS)
            else:
                x2w = warp_forward(lv["x2"], lv["fl"])
                lv["corr"] = corr_forward(lv["x1"], x2w, **bench.CORR_ARGS)
            g1, g2w = corr_backward(lv["x1"], x2w, lv["gc"], **bench.CORR_ARGS)
            lv["g1"] = g1
            lv["gx2"], lv["gfl"] = warp_backward(lv["x2"], lv["fl"], g2w)

    for s in sets:
        one(s)
    torch.cuda.synchronize()
    graphs = []
    pool = torch.cuda.graph_pool_handle()
    for i in range(nsets):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            one(sets[i])
        graphs.append(g)
    for i in range(args.warmup):
        graphs[i % nsets].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        graphs[i % nsets].replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({
        "metric": "image-pairs/sec (training step of the hot path, 384x448: warp + Correlation "
                  "forward and backward at l0-l4)",
        "value": round(B * args.steps / el, 2), "unit": "image-pairs/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 5), "dtype": "fp32",
        "data": "synthetic (randn features and cost-volume gradients, N(0,2^2) flows)",
        "config": {"workload": "BASELINE config 5: B=8 384x448 training step of the hot path",
                   "batch": B, "levels": [list(x) for x in shapes], "graph": True,
                   "fused_levels": sorted(fused), "grouped": args.group == "on",
                   "buffer_sets": nsets}}), flush=True)


if __name__ == "__main__":
    main()
