#!/usr/bin/env python3
"""Probe (diagnostic): can kernel timing events live inside a captured hipGraph?

  a) torch external timing events recorded during capture around the l4 correlation;
  b) hipExtLaunchKernel start/stop events (pwc_time_next_corr) armed during capture;
  c) step time of one graph holding the whole pass vs graph + direct l4 launch.
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import corr_forward, warp_forward  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
B = 8
shapes = bench.level_shapes(384, 448)
gen = torch.Generator(device=dev).manual_seed(0)
s = bench.make_set(shapes, B, dev, torch.float32, gen)
stream = torch.cuda.current_stream(dev)
C4, h4, w4 = shapes[-1]


def corr_l4(x2w):
    ok = lib.pwc_corr_forward(ctypes.c_void_p(s[-1]["x1"].data_ptr()),
                              ctypes.c_void_p(x2w.data_ptr()),
                              ctypes.c_void_p(s[-1]["corr"].data_ptr()), B, C4, h4, w4,
                              9, 1, 9, 1, 2, 1, 0, ctypes.c_void_p(stream.cuda_stream))
    _lib.check(ok, "corr_l4")


def pre():
    for lv in s[:-1]:
        w = warp_forward(lv["x2"], lv["flow"])
        lv["corr"] = corr_forward(lv["x1"], w, **bench.CORR_ARGS)
    return warp_forward(s[-1]["x2"], s[-1]["flow"])


corr_l4(pre())
torch.cuda.synchronize()

# a) external events in capture
try:
    e0 = torch.cuda.Event(enable_timing=True, external=True)
    e1 = torch.cuda.Event(enable_timing=True, external=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        w = pre()
        e0.record()
        corr_l4(w)
        e1.record()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        g.replay()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    print("a) external events in graph: l4 corr us", sorted(ts)[len(ts) // 2], flush=True)
except Exception as ex:  # noqa: BLE001
    print("a) failed:", repr(ex), flush=True)

# b) hipExtLaunchKernel events armed during capture
try:
    f0 = torch.cuda.Event(enable_timing=True)
    f1 = torch.cuda.Event(enable_timing=True)
    f0.record()
    f1.record()
    torch.cuda.synchronize()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        w = pre()
        _lib.check(lib.pwc_time_next_corr(ctypes.c_void_p(f0.cuda_event),
                                          ctypes.c_void_p(f1.cuda_event)), "arm")
        corr_l4(w)
    g2.replay()
    torch.cuda.synchronize()
    print("b) ext-launch events in graph: l4 corr us", f0.elapsed_time(f1) * 1e3, flush=True)
except Exception as ex:  # noqa: BLE001
    print("b) failed:", repr(ex), flush=True)

# c) step times
g3 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g3):
    corr_l4(pre())
g4 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g4):
    w4_ = pre()
for name, fn in [("one graph", lambda: g3.replay()),
                 ("graph + direct l4", lambda: (g4.replay(), corr_l4(w4_)))]:
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    print(f"c) {name}: {(time.perf_counter() - t) / 200 * 1e6:.1f} us/step", flush=True)
