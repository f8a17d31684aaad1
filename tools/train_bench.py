#!/usr/bin/env python3
"""Training-step timing of the hot path (BASELINE.json config 5: B=8 384x448, 1 GPU).

One step = for every correlated level l0..l4 (model.py:72-113): forward warp (modules.py:31-42)
+ Correlation (model.py:24), then the backward of both for an upstream gradient of the cost
volume: Correlation backward (correlation_cuda_kernel.cu:108-290 -> d/dx1, d/dx2_warp), then
WarpingLayer backward (ATen grid_sampler_2d_backward semantics -> d/dx2, d/dflow).  The fused
levels (--fused-levels, default l0 and l1) run the pair as WarpCorrelation: one forward launch
and one backward call (warp_corr_backward; WarpCorrelationFunction.backward).  Each step is one
hipGraph replay; inputs rotate past the Infinity Cache.

Headline ("value"): DEPENDENCY order -- level after level, each level's forward then its
backward, nothing batched across levels.  The "grouped" object times the same step with the
independent synthetic levels' forwards batched into group launches (l0+l1 band pair, one
warp group, the l2+l3 correlation pair): labelled, not the headline.

Checks (after timing): every output of one set (volume, d/dx1, d/dx2, d/dflow at each level)
is poisoned with NaN, the captured graph replayed, and compared with a fresh eager
computation in dependency order -- a kernel the graph skipped leaves NaN behind.
"kernels": per-op roofline lines at each level (forward warp / correlation / fused
warp+correlation, correlation backward, warp backward; one op may be several kernels):
algorithmic bytes / mean duration of 20 back-to-back launches replayed from one hipGraph
(event-timed; includes the graph's inter-kernel gaps, so small ops read low).

    python tools/train_bench.py [--steps 100] [--warmup 100] [--grouped-mode off]
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
                            warp_backward, warp_corr_backward, warp_corr_forward,
                            warp_corr_forward_group,
                            warp_forward, warp_forward_group)

OUTPUTS = ("corr", "g1", "gx2", "gfl")


def make_set(B, shapes, dev, gen):
    """One buffer set: per level x1, x2 (C channels), flow, and the upstream cost-volume
    gradient gc (81 channels)."""
    s = []
    for C, h, w in shapes:
        s.append(dict(x1=torch.randn(B, C, h, w, device=dev, generator=gen),
                      x2=torch.randn(B, C, h, w, device=dev, generator=gen),
                      fl=torch.randn(B, 2, h, w, device=dev, generator=gen) * 2.0,
                      gc=torch.randn(B, 81, h, w, device=dev, generator=gen)))
    return s


def backward_level(lv, x2w, fused):
    """The level's backward: fused levels (the forward was one WarpCorrelation launch) as ONE
    warp_corr_backward call (WarpCorrelationFunction.backward), the others as the correlation
    backward then the warp backward."""
    if fused:
        lv["g1"], lv["gx2"], lv["gfl"] = warp_corr_backward(lv["x1"], lv["x2"], lv["fl"], x2w,
                                                            lv["gc"], **bench.CORR_ARGS)
        return
    lv["g1"], g2w = corr_backward(lv["x1"], x2w, lv["gc"], **bench.CORR_ARGS)
    lv["gx2"], lv["gfl"] = warp_backward(lv["x2"], lv["fl"], g2w)


def step_dependency(s, fused):
    """Level after level: forward (fused levels as one WarpCorrelation launch that also emits
    x2_warp), then that level's backward."""
    for l, lv in enumerate(s):
        fl = l in fused and l < len(s) - 1
        if fl:
            lv["corr"], x2w = warp_corr_forward(lv["x1"], lv["x2"], lv["fl"], **bench.CORR_ARGS)
        else:
            x2w = warp_forward(lv["x2"], lv["fl"])
            lv["corr"] = corr_forward(lv["x1"], x2w, **bench.CORR_ARGS)
        backward_level(lv, x2w, fl)


def step_grouped(s, fused):
    """The forwards of the (independent) levels batched into group launches, then every
    level's backward."""
    last = len(s) - 1
    fl = sorted(l for l in fused if l < last)
    x2w = {}
    for l, (c, w) in zip(fl, warp_corr_forward_group(
            [(s[l]["x1"], s[l]["x2"], s[l]["fl"]) for l in fl], **bench.CORR_ARGS)):
        s[l]["corr"], x2w[l] = c, w
    wl = [l for l in range(last, -1, -1) if l == last or l not in fused]
    for l, w in zip(wl, warp_forward_group([(s[l]["x2"], s[l]["fl"]) for l in wl])):
        x2w[l] = w
    cl = [l for l in wl if l != last]
    for l, c in zip(cl, corr_forward_group([(s[l]["x1"], x2w[l]) for l in cl],
                                           **bench.CORR_ARGS)):
        s[l]["corr"] = c
    s[last]["corr"] = corr_forward(s[last]["x1"], x2w[last], **bench.CORR_ARGS)
    for l, lv in enumerate(s):
        backward_level(lv, x2w[l], l in fl)


def fresh(s):
    """Unfused eager recomputation of every output (the self-check's reference)."""
    out = []
    for lv in s:
        x2w = warp_forward(lv["x2"], lv["fl"])
        c = corr_forward(lv["x1"], x2w, **bench.CORR_ARGS)
        g1, g2w = corr_backward(lv["x1"], x2w, lv["gc"], **bench.CORR_ARGS)
        gx2, gfl = warp_backward(lv["x2"], lv["fl"], g2w)
        out.append(dict(corr=c, g1=g1, gx2=gx2, gfl=gfl))
    return out


def max_rel_diff(s, ref):
    """Per output name, the max over levels of bench._diff (NaN positions must match)."""
    return {k: max(bench._diff(lv[k], r[k]) for lv, r in zip(s, ref)) for k in OUTPUTS}


def op_table(s, fused, reps=20):
    """Per-op roofline lines (event-timed, `reps` back-to-back launches of one op)."""
    rows = []
    last = len(s) - 1

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()  # `reps` launches of the op in one graph: no host overhead
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / reps * 1e3  # us

    for l, lv in enumerate(s):
        B, C, h, w = lv["x1"].shape
        hw4 = B * h * w * 4
        x2w = warp_forward(lv["x2"], lv["fl"])
        _, g2w = corr_backward(lv["x1"], x2w, lv["gc"], **bench.CORR_ARGS)
        ops = []
        if l in fused and l < last:
            ops.append(("warp_corr_fwd", (3 * C + 2 + 81) * hw4,
                        lambda: warp_corr_forward(lv["x1"], lv["x2"], lv["fl"],
                                                  **bench.CORR_ARGS)))
        else:
            ops.append(("warp_fwd", (2 * C + 2) * hw4, lambda: warp_forward(lv["x2"], lv["fl"])))
            ops.append(("corr_fwd", (2 * C + 81) * hw4,
                        lambda: corr_forward(lv["x1"], x2w, **bench.CORR_ARGS)))
        if l in fused and l < last:
            # reads x1, x2, x2_warp, 81 gradient planes, the flow; writes g1, gx2, grad_flow
            ops.append(("warp_corr_bwd", (5 * C + 81 + 4) * hw4,
                        lambda: warp_corr_backward(lv["x1"], lv["x2"], lv["fl"], x2w, lv["gc"],
                                                   **bench.CORR_ARGS)))
        else:
            ops.append(("corr_bwd", (4 * C + 81) * hw4,
                        lambda: corr_backward(lv["x1"], x2w, lv["gc"], **bench.CORR_ARGS)))
            ops.append(("warp_bwd", (3 * C + 4) * hw4,
                        lambda: warp_backward(lv["x2"], lv["fl"], g2w)))
        for name, nbytes, fn in ops:
            us = timed(fn)
            gbs = nbytes / (us * 1e-6) / 1e9
            rows.append({"level": l, "op": name, "shape": [B, C, h, w], "us": round(us, 2),
                         "algorithmic_bytes": nbytes, "GB/s": round(gbs, 1),
                         "frac_8TBs": round(gbs / bench.HBM_PEAK_GBS, 3)})
    return rows


def run(args, dev=None):
    fused = {int(v) for v in args.fused_levels.split(",") if v.strip()}
    dev = dev or torch.device("cuda:0")
    B = args.batch
    shapes = bench.level_shapes(args.height, args.width)
    per = sum((4 * C * h * w + 4 * h * w + 2 * 81 * h * w) * B * 4 for C, h, w in shapes)
    nsets = max(2, int(2 * 256 * 2 ** 20 / per) + 1)
    gen = torch.Generator(device=dev).manual_seed(7)
    sets = [make_set(B, shapes, dev, gen) for _ in range(nsets)]
    modes = [("dependency", step_dependency)]
    if args.grouped_mode == "on":
        modes.append(("grouped", step_grouped))
    results = {}
    for name, fn in modes:
        for s in sets:
            fn(s, fused)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        graphs, outs = [], []
        for s in sets:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                fn(s, fused)
            graphs.append(g)
            outs.append({k: [lv[k] for lv in s] for k in OUTPUTS})  # the graph's outputs
        for i in range(args.warmup):
            graphs[i % nsets].replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            graphs[i % nsets].replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # self-check: poison the graph's outputs of one set, replay, compare with fresh eager
        k = (args.steps - 1) % nsets
        for key in OUTPUTS:
            for t in outs[k][key]:
                t.fill_(float("nan"))
        graphs[k].replay()
        torch.cuda.synchronize()
        got = [{key: outs[k][key][l] for key in OUTPUTS} for l in range(len(shapes))]
        diff = max_rel_diff(got, fresh(sets[k]))
        results[name] = {"value": round(B * args.steps / el, 2),
                         "ms_per_step": round(el / args.steps * 1e3, 5),
                         "self_check": {"ok": all(d <= 1e-4 for d in diff.values()),
                                        "max_rel_diff": diff}}
        del graphs
    head = results["dependency"]
    out = {
        "metric": "image-pairs/sec (training step of the hot path, 384x448: warp + Correlation "
                  "forward and backward at l0-l4)",
        "value": head["value"], "unit": "image-pairs/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
        "higher_is_better": True, "dtype": "fp32",
        "data": "synthetic (randn features and cost-volume gradients, N(0,2^2) flows)",
        "config": {"workload": "BASELINE config 5: B=8 384x448 training step of the hot path",
                   "batch": B, "levels": [list(x) for x in shapes], "graph": True,
                   "fused_levels": sorted(fused),
                   "order": "dependency (level after level, forward then backward)",
                   "buffer_sets": nsets},
        "checks": {"self_check": head["self_check"]},
    }
    if "grouped" in results:
        out["grouped"] = dict(results["grouped"], mode="grouped (NOT the headline: the levels' "
                              "forwards batched into group launches)")
    if not args.no_kernels:
        out["kernels"] = op_table(sets[0], fused)
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100)  # ~28 ms: clocks settle
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=448)
    ap.add_argument("--fused-levels", default="0,1",
                    help="levels whose forward runs as one WarpCorrelation launch (as bench.py)")
    ap.add_argument("--grouped-mode", default="on", choices=["on", "off"],
                    help="also time the grouped-forward step (reported as 'grouped')")
    ap.add_argument("--no-kernels", action="store_true", help="skip the per-op roofline table")
    return ap.parse_args(argv)


def main(argv=None):
    out = run(parse_args(argv))
    print(json.dumps(out), flush=True)
    ok = out["checks"]["self_check"]["ok"] and out.get("grouped", {}).get(
        "self_check", {"ok": True})["ok"]
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
