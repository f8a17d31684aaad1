#!/usr/bin/env python3
"""Is the bench step host-bound?  Per mode: host seconds to ISSUE N steps (no sync) against the
GPU seconds of the same N steps (issue + sync).  Modes: graph-eager (bench default), graph-all,
eager (direct C-ABI calls)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    shapes = bench.level_shapes(384, 448)
    gen = torch.Generator(device=dev).manual_seed(1)
    sets = [bench.random_set(shapes, 8, dev, torch.float32, gen) for _ in range(8)]
    p = bench.HipPass(dev, torch.float32, {0, 1})
    for s in sets:
        p.bind(s)
        p.full(s)
    torch.cuda.synchronize()
    pool = torch.cuda.graph_pool_handle()
    g_pre, g_all = [], []
    for s in sets:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            p.pre(s)
        g_pre.append(g)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            p.pre(s)
            p.corr_l4(s)
        g_all.append(g)
    torch.cuda.synchronize()
    N = 400
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(N + 40)]
    for a, b in evs:
        a.record()
        b.record()
    torch.cuda.synchronize()

    def eager_ev(i, every):
        p.pre(sets[i % 8])
        p.corr_l4(sets[i % 8], evs[i] if i % every == 0 else None)

    modes = {
        "graph-eager": lambda i: (g_pre[i % 8].replay(), p.corr_l4(sets[i % 8])),
        "graph-eager+ev": lambda i: (g_pre[i % 8].replay(), p.corr_l4(sets[i % 8], evs[i])),
        "graph-all": lambda i: g_all[i % 8].replay(),
        "eager": lambda i: p.full(sets[i % 8]),
        "eager+ev": lambda i: eager_ev(i, 1),
        "eager+ev/10": lambda i: eager_ev(i, 10),
    }
    for name, fn in modes.items():
        for i in range(20):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(N):
            fn(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ms = [a.elapsed_time(b) for a, b in evs[:N:10]] if "ev" in name else []
        kern = f"  l4 corr {1e3 * sum(ms) / len(ms):6.2f} us" if ms else ""
        print(f"{name:15s} host issue {1e6 * (t1 - t0) / N:7.2f} us/step   wall {1e6 * (t2 - t0) / N:7.2f} us/step{kern}",
              flush=True)


if __name__ == "__main__":
    main()
