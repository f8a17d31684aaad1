#!/usr/bin/env python3
"""Which shape reaches which kernel instantiation: runs a list of candidate calls of every op
(fp32 / fp16 / bf16, Corr9 / Corr4 / CostVolumeLayer, forward / backward, warp, upsample-warp,
fused and grouped forms) at the pyramid shapes of 384x448 and 448x1024 and other batch sizes,
one call each, with a marker kernel (torch.cuda._sleep) before every call.  Run it under
``rocprofv3 --kernel-trace`` and give the trace to ``--attribute``: every pwc:: kernel is
credited to the call whose marker precedes it, and the report lists, per instantiation of
libpwc_hotpath.so, the first (smallest) call that reached it -- the shapes the GPU tests need.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cov -o run -- \
        python tools/coverage_sweep.py --run > gpurun_out/cov_cases.json
    python tools/coverage_sweep.py --attribute gpurun_out/cov/.../run_kernel_trace.csv \
        gpurun_out/cov_cases.json
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

L384 = [(192, 6, 7), (128, 12, 14), (96, 24, 28), (64, 48, 56), (32, 96, 112)]
L1024 = [(192, 7, 16), (128, 14, 32), (96, 28, 64), (64, 56, 128), (32, 112, 256)]
EXTRA = [(32, 192, 224), (16, 13, 15), (24, 13, 15), (64, 55, 128), (32, 54, 128)]
CFG = {"corr9": (9, 1, 9, 1, 2), "corr4": (4, 1, 4, 1, 1)}


def cases():
    out = []
    for dt in ("fp32", "fp16", "bf16"):
        for B in (1, 2, 3, 4, 8, 12, 16):
            for (C, h, w) in L384 + L1024 + EXTRA:
                if B * C * h * w > 16 * 32 * 112 * 256:
                    continue
                for cfg in ("corr9", "corr4", "cvl"):
                    out.append(dict(op="corr_fwd", dt=dt, cfg=cfg, shape=[B, C, h, w]))
                    if B in (1, 2, 8, 16):
                        out.append(dict(op="corr_bwd", dt=dt, cfg=cfg, shape=[B, C, h, w]))
                out.append(dict(op="warp_fwd", dt=dt, shape=[B, C, h, w]))
                if B in (1, 2, 8, 16):
                    out.append(dict(op="warp_bwd", dt=dt, shape=[B, C, h, w]))
                    out.append(dict(op="upwarp", dt=dt, shape=[B, C, h, w]))
                    out.append(dict(op="warp_corr", dt=dt, shape=[B, C, h, w]))
                    out.append(dict(op="corr_into", dt=dt, shape=[B, C, h, w]))
        for B in (1, 2, 8, 16):
            for lv in (L384, L1024):
                out.append(dict(op="band_group", dt=dt, shapes=[[B] + list(s) for s in lv[:2]]))
                out.append(dict(op="warp_group", dt=dt, shapes=[[B] + list(s) for s in lv[2:]]))
                out.append(dict(op="corr_group", dt=dt, shapes=[[B] + list(s) for s in lv[2:4]]))
    return out


def run_one(c, torch, ops, dev):
    dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[c["dt"]]
    g = torch.Generator(device=dev).manual_seed(1)

    def r(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(dt)

    op = c["op"]
    if op in ("band_group", "warp_group", "corr_group"):
        probs = []
        for (B, C, h, w) in c["shapes"]:
            probs.append((r(B, C, h, w), r(B, C, h, w), r(B, 2, h, w, scale=2.0)))
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)
        if op == "band_group":
            ops.warp_corr_forward_group(probs, *CFG["corr9"])
        elif op == "warp_group":
            ops.warp_forward_group([(b, f) for (_, b, f) in probs])
        else:
            ops.corr_forward_group([(a, b) for (a, b, _) in probs], *CFG["corr9"])
        torch.cuda.synchronize()
        return
    B, C, h, w = c["shape"]
    a, b, f = r(B, C, h, w), r(B, C, h, w), r(B, 2, h, w, scale=2.0)
    cfg = c.get("cfg")
    go = None
    if op == "corr_bwd":
        go = r(B, 81, h, w)
    if op == "warp_bwd":
        go = r(B, C, h, w)
    if op == "upwarp":
        f = r(B, 2, (h + 1) // 2, (w + 1) // 2, scale=2.0)
    if op == "corr_into":
        cat = torch.empty(B, C + 81 + 2, h, w, device=dev, dtype=dt)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    if op == "corr_fwd":
        if cfg == "cvl":
            ops.cost_volume_forward(a, b, 4)
        else:
            ops.corr_forward(a, b, *CFG[cfg])
    elif op == "corr_bwd":
        if cfg == "cvl":
            ops.cost_volume_backward(a, b, go, 4)
        else:
            ops.corr_backward(a, b, go, *CFG[cfg])
    elif op == "warp_fwd":
        ops.warp_forward(b, f)
    elif op == "warp_bwd":
        ops.warp_backward(b, f, go)
    elif op == "upwarp":
        ops.upsample_warp_forward(b, f)
    elif op == "warp_corr":
        ops.warp_corr_forward(a, b, f, *CFG["corr9"])
    elif op == "corr_into":
        ops.corr_forward_into(a, b, cat[:, C:C + 81], *CFG["corr9"])
    torch.cuda.synchronize()


def run(args):
    import torch
    from pwcnet_amd import ops
    dev = torch.device("cuda")
    done = []
    for c in cases():
        try:
            run_one(c, torch, ops, dev)
            c["ok"] = True
        except (RuntimeError, ValueError, TypeError) as e:  # declined shapes are fine
            c["ok"] = False
            c["err"] = str(e)[:120]
            torch.cuda.synchronize()
            torch.cuda._sleep(1000)  # keep the marker count aligned with the case list
            torch.cuda.synchronize()
        done.append(c)
    json.dump(done, sys.stdout)


def attribute(args):
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cs = json.load(open(args.cases))
    # marker k -> case: a declined call (its op raised after its marker) left a second marker
    owner = []
    for i, c in enumerate(cs):
        owner += [i] * (1 if c.get("ok") else 2)
    idx = -1
    hits = {}
    for r in rows:
        n = r["Kernel_Name"]
        if "spin_kernel" in n:
            idx += 1
            continue
        if "pwc::" not in n or idx < 0:
            continue
        n = n[5:] if n.startswith("void ") else n
        base = n.split("(")[0]
        c = cs[owner[idx]] if idx < len(owner) else {"op": "?"}
        hits.setdefault(base, []).append(c)
    print(f"# {idx + 1} markers for {len(cs)} cases ({len(owner)} expected)")
    for k in sorted(hits):
        def size(c):
            sh = c.get("shape") or [v for s in c.get("shapes") for v in s]
            p = 1
            for v in sh:
                p *= v
            return p
        first = min(hits[k], key=size)
        print(json.dumps({"kernel": k, "calls": len(hits[k]),
                          "smallest": {kk: first.get(kk) for kk in ("op", "dt", "cfg", "shape",
                                                                    "shapes")}}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--attribute", nargs=2, metavar=("TRACE", "CASES"))
    a = ap.parse_args()
    if a.run:
        run(a)
    elif a.attribute:
        a.trace, a.cases = a.attribute
        attribute(a)


if __name__ == "__main__":
    main()
