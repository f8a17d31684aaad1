#!/usr/bin/env python3
"""Per-kernel timing of the hot path (HIP events, rotating buffers past the Infinity Cache).

    python tools/kbench.py [--batch 8] [--height 384] [--width 448] [--iters 50]

Prints one JSON line per (level, op) with the mean device time and algorithmic GB/s.  The
kernel path can be forced with PWC_DEBUG=corr_path=1|2 (generic | register-tiled).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd.ops import (corr_backward, corr_forward, warp_backward, warp_corr_forward,  # noqa
                            warp_forward)


def timeit(fn, sets, iters):
    """Mean device time per launch over `iters` back-to-back launches (rotating buffer sets),
    captured into one hipGraph and replayed between two events, 5 times; returns (median-of-5,
    min-of-5) in microseconds.  The graph removes host launch cost (Python + ctypes + the
    allocator), which otherwise exceeds the device time of the small levels; the GPU's own
    inter-kernel gap stays in."""
    for s in sets:
        fn(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(sets[i % len(sets)])
    g.replay()
    torch.cuda.synchronize()
    res = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / iters)
    res.sort()
    return res[2], res[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=448)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--backward", action="store_true")
    ap.add_argument("--levels", default="0,1,2,3,4")
    ap.add_argument("--ops", default="corr,warp,fused")
    ap.add_argument("--tag", default="")
    ap.add_argument("--flow-scale", type=float, default=2.0, help="flows ~ N(0, scale^2) px")
    ap.add_argument("--sets", type=int, default=0, help="buffer sets (0 = past the MALL)")
    args = ap.parse_args()
    dt = torch.float32 if args.dtype == "fp32" else torch.float16
    esz = 4 if dt == torch.float32 else 2
    dev = torch.device("cuda:0")
    B = args.batch
    path = os.environ.get("PWC_DEBUG", "default")
    levels = [int(v) for v in args.levels.split(",")]
    for l, (C, h, w) in enumerate(bench.level_shapes(args.height, args.width)):
        if l not in levels:
            continue
        per = (3 * C * h * w + 83 * h * w) * B * esz
        n = args.sets or max(2, int(2 * 256 * 2 ** 20 / per) + 1)
        g = torch.Generator(device=dev).manual_seed(l)
        sets = [dict(x1=torch.randn(B, C, h, w, device=dev, generator=g).to(dt),
                     x2=torch.randn(B, C, h, w, device=dev, generator=g).to(dt),
                     fl=(torch.randn(B, 2, h, w, device=dev, generator=g) * args.flow_scale).to(dt))
                for _ in range(n)]
        ops = args.ops.split(",")
        cb = bench.corr_bytes_per_pair(C, h, w, esz) * B
        if "corr" in ops:
            med, mean = timeit(lambda s: corr_forward(s["x1"], s["x2"], 9, 1, 9, 1, 2), sets,
                               args.iters)
            print(json.dumps(dict(level=l, op="corr_fwd", path=path, shape=[B, C, h, w],
                                  us=round(med, 2), min_us=round(mean, 2),
                                  gbs=round(cb / (med * 1e-6) / 1e9, 1), tag=args.tag)))
        # stride-1 correlations (Corr4 = Correlation(4,1,4,1,1), CostVolumeLayer sr=4):
        # same algorithmic bytes as Corr9 (81 output channels)
        if "corr4" in ops:
            med, mean = timeit(lambda s: corr_forward(s["x1"], s["x2"], 4, 1, 4, 1, 1), sets,
                               args.iters)
            print(json.dumps(dict(level=l, op="corr4_fwd", shape=[B, C, h, w],
                                  us=round(med, 2), min_us=round(mean, 2),
                                  gbs=round(cb / (med * 1e-6) / 1e9, 1), tag=args.tag)))
        if "cvl" in ops:
            from pwcnet_amd.ops import cost_volume_forward
            med, mean = timeit(lambda s: cost_volume_forward(s["x1"], s["x2"], 4), sets,
                               args.iters)
            print(json.dumps(dict(level=l, op="cvl_fwd", shape=[B, C, h, w],
                                  us=round(med, 2), min_us=round(mean, 2),
                                  gbs=round(cb / (med * 1e-6) / 1e9, 1), tag=args.tag)))
        wb = (2 * C * h * w + 2 * h * w) * B * esz
        if "warp" in ops:
            med, mean = timeit(lambda s: warp_forward(s["x2"], s["fl"]), sets, args.iters)
            print(json.dumps(dict(level=l, op="warp_fwd", shape=[B, C, h, w], us=round(med, 2),
                                  min_us=round(mean, 2), gbs=round(wb / (med * 1e-6) / 1e9, 1),
                                  tag=args.tag)))
        if "fused" in ops:
            # one level of model.py:80-83 (x2_warp emitted): bytes = read x1, x2, flow, write
            # x2_warp and the volume
            fb = (3 * C * h * w + 2 * h * w + 81 * h * w) * B * esz
            med, mean = timeit(lambda s: warp_corr_forward(s["x1"], s["x2"], s["fl"], 9, 1, 9,
                                                           1, 2), sets, args.iters)
            print(json.dumps(dict(level=l, op="warp_corr", shape=[B, C, h, w],
                                  band=os.environ.get("PWC_DEBUG", ""), us=round(med, 2),
                                  min_us=round(mean, 2), gbs=round(fb / (med * 1e-6) / 1e9, 1),
                                  tag=args.tag)))
        if "seq" in ops:
            # the bench step's order at one level: the warp, then the correlation on its output
            # (two launches; seq_us - warp_fwd us = the correlation behind a warp)
            med, mean = timeit(lambda s: corr_forward(s["x1"], warp_forward(s["x2"], s["fl"]), 9,
                                                      1, 9, 1, 2), sets, args.iters)
            print(json.dumps(dict(level=l, op="warp_then_corr", shape=[B, C, h, w],
                                  us=round(med, 2), min_us=round(mean, 2), tag=args.tag)))
        if "upwarp" in ops and h % 2 == 0 and w % 2 == 0:
            # model.py:78 + :80: fused flow upsample -> warp (flow_up emitted) against the
            # unfused ATen upsample * 2 followed by the warp kernel
            from pwcnet_amd.ops import upsample_warp_forward
            import torch.nn.functional as F
            for s in sets:
                s["fc"] = s["fl"][:, :, ::2, ::2].contiguous()
            med, mean = timeit(lambda s: upsample_warp_forward(s["x2"], s["fc"]), sets,
                               args.iters)
            med2, _ = timeit(lambda s: warp_forward(s["x2"], F.interpolate(
                s["fc"], scale_factor=2, mode="bilinear", align_corners=False) * 2), sets,
                args.iters)
            print(json.dumps(dict(level=l, op="upsample_warp", shape=[B, C, h, w],
                                  us=round(med, 2), unfused_us=round(med2, 2), tag=args.tag)))
        if args.backward and dt == torch.float32:
            go = torch.randn(B, 81, h, w, device=dev)
            med, mean = timeit(lambda s: corr_backward(s["x1"], s["x2"], go, 9, 1, 9, 1, 2),
                               sets, args.iters)
            print(json.dumps(dict(level=l, op="corr_bwd", shape=[B, C, h, w],
                                  us=round(med, 2), min_us=round(mean, 2), tag=args.tag)))
            gw = torch.randn(B, C, h, w, device=dev)
            med, mean = timeit(lambda s: warp_backward(s["x2"], s["fl"], gw), sets, args.iters)
            print(json.dumps(dict(level=l, op="warp_bwd", shape=[B, C, h, w],
                                  us=round(med, 2), min_us=round(mean, 2), tag=args.tag)))


if __name__ == "__main__":
    main()
