#!/usr/bin/env python3
"""Benchmark of the PWC-Net hot path on MI355X (BASELINE.json config 2 / config 3).

One step = one pass of the hot path over one batch of synthetic 384x448 image pairs: for every
pyramid level the reference's forward visits (model.py:72-113 at output_level=4: l0..l4 =
192x6x7, 128x12x14, 96x24x28, 64x48x56, 32x96x112 at 384x448), the WarpingLayer
(modules.py:31-42) warps the second image's features by the level's flow and the
Correlation of model.py:24 (pad 9, k 1, md 9, s1 1, s2 2: 81 channels) correlates them with
the first image's features.  Per GPU the batch is 8 pairs (config 2); with --gpus N every
rank processes its own 8 pairs (config 3: 64 pairs over 8 GPUs), no collective on the data
path ("scaling": "weak").

Launch: ``bench.py --gpus N`` with N > 1 and no torch.distributed environment starts N ranks
itself (a ``torch.distributed.run`` child, before this process touches the GPU) and exits
with its status; under an outer launcher ``--gpus`` must equal WORLD_SIZE.  At N > 1 rank 0
broadcasts the Net harness's weights (pwcnet_amd/net.py; SURVEY §8e's startup broadcast) and
every rank checks it received them.

Timed region: every step launches warp + correlation at l0..l3 and the l4 warp as direct
C-ABI calls on buffers bound once per set (the ctypes arguments are built once, so a launch
costs one foreign call), then the l4 correlation -- the dominant kernel, priced for the
roofline -- through the C ABI with hipExtLaunchKernel start/stop events (pwc_time_next_corr),
so that kernel's duration is measured live in every timed step on the stream it runs on.  On
ROCm this 8-kernel step runs faster as plain launches than replayed from a hipGraph (which
also makes the event-armed launch dearer), so graphs are comparison modes:
``--timing graph-eager`` replays a per-set graph of l0..l3 and the l4 warp before the same
event-armed launch; ``--timing graph-all`` captures the whole step in one graph, without
kernel events (HIP refuses external event-record nodes in a capture).
Order: the headline ``value`` runs the levels in DEPENDENCY order -- l0, l1, ..., l4, each
level's warp before its correlation (l0 and l1 as one fused WarpCorrelation launch each), no
launch batching work of different levels -- because in the network (model.py:72-113) level
l+1's warp needs level l's flow.  The ``grouped`` object then times the same step with the
independent synthetic levels batched into group launches (l0+l1 band pair, l2/l3/l4 warps,
l2+l3 correlations): a labelled upper bound for batching across independent pairs, not the
headline.
Inputs rotate over enough buffer sets (> 2x the 256 MiB Infinity Cache) that each step reads
them from HBM.  After timing, a replay self-check re-runs one step with every output poisoned
(NaN) and compares all five levels bit for bit with a fresh eager computation, and a shard
check compares per-pair checksums of every rank with rank 0's recomputation of the whole
global batch (all_gather) -- a step that skipped a kernel, or a rank that computed the wrong
pairs, fails the run.

cpu_baseline (rank 0, N=1 only): the reference's pure-PyTorch CPU path restated
(oracle/torch_ref.py: WarpingLayer = grid_sample(align_corners=True) + CostVolumeLayer, the
reference's CPU correlation) over the same pyramid shapes, on every host thread torch is
given; ``cpu_baseline_port`` is the fp32 C port of the GPU semantics (Corr9), labelled.

``--device cpu`` (gloo) is a launcher rehearsal for the tests: the same launcher, sharding,
broadcast and shard check with a torch-CPU stand-in for the per-shard op (not the product).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pwc-net_pytorch_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# reference defaults (main.py:42-81): lv_chs, num_levels=7, output_level=4, search_range=4
LV_CHS = [16, 32, 64, 96, 128, 192]
NUM_LEVELS = 7
OUTPUT_LEVEL = 4
SEARCH_RANGE = 4
CORR_ARGS = dict(pad_size=2 * SEARCH_RANGE + 1, kernel_size=1,
                 max_displacement=2 * SEARCH_RANGE + 1, stride1=1, stride2=2)  # model.py:24
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PAIR_SEED = 20240601   # synthetic pair g of the checked set is seeded PAIR_SEED + g
# the l4-sized correlation kernels (csrc/corr_strip.hip for fp32 C = 32, corr_stream.hip else)
L4_KERNEL_RE = "corr_fwd_(m?strip|stream)"
CORR4_ARGS = dict(pad_size=SEARCH_RANGE, kernel_size=1, max_displacement=SEARCH_RANGE,
                  stride1=1, stride2=1)  # the north star's literal "d=4": displacements -4..4


def level_shapes(H, W):
    """(C, h, w) of the correlated levels l = 0..output_level (model.py:72)."""
    chs = LV_CHS[::-1]
    out = []
    for l in range(OUTPUT_LEVEL + 1):
        s = 2 ** (NUM_LEVELS - 1 - l)
        out.append((chs[l], H // s, W // s))
    return out


def corr_bytes_per_pair(C, h, w, elem=4):
    """(2*C*H*W + 81*H*W) * sizeof -- read f1, read warped f2, write volume."""
    return (2 * C * h * w + 81 * h * w) * elem


# ---------------------------------------------------------------------------------------
# launcher
# ---------------------------------------------------------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default 300 on the GPU, about 30 ms at config 2: "
                         "clocks and caches settle; 2 for --device cpu)")
    ap.add_argument("--batch", type=int, default=8, help="pairs per GPU")
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=448)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp16"])
    ap.add_argument("--sets", type=int, default=0, help="rotating buffer sets (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-net-forward", action="store_true",
                    help="skip the labelled end-to-end Net forward object (N=1 only)")
    ap.add_argument("--no-corr4", action="store_true",
                    help="skip the labelled Correlation(4,1,4,1,1) roofline object (N=1 only)")
    ap.add_argument("--no-graph", action="store_true", help="same as --timing eager")
    ap.add_argument("--timing", default="eager", choices=["eager", "graph-eager", "graph-all"],
                    help="eager (default): every kernel a direct C-ABI launch on pre-built "
                         "arguments, the l4 correlation event-armed; graph-eager: per-set graphs "
                         "of l0..l3 + the l4 warp, then the event-armed l4 correlation; "
                         "graph-all (comparison only): the whole step in one graph, no kernel "
                         "events")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = launcher rehearsal over gloo with a torch-CPU stand-in op")
    ap.add_argument("--fused-levels", default="0,1",
                    help="levels run as one fused warp->correlation launch (WarpCorrelation)")
    ap.add_argument("--grouped-mode", default="on", choices=["on", "off"],
                    help="after the headline (dependency order: one level after the other, "
                         "as model.py:72-113 runs them), time the same step with independent "
                         "levels batched into group launches (--group / --corr-group / "
                         "--warp-group below) and report it as the separate 'grouped' object")
    ap.add_argument("--group", default="on", choices=["on", "off"],
                    help="grouped mode: issue the fused levels as one group "
                         "(pwc_warp_corr_forward_group: the bench's levels take independent "
                         "inputs, so l0 + l1 share one launch); off = one call per level")
    ap.add_argument("--corr-group", default="on", choices=["on", "off"],
                    help="grouped mode: the unfused levels' correlations below l4 (l2, l3) as one "
                         "pwc_corr_forward_group launch (independent inputs); off = one call "
                         "per level")
    ap.add_argument("--group-order", default="desc", choices=["asc", "desc"],
                    help="problem order inside the warp / correlation groups: asc = l2 first, "
                         "desc = the largest level's workgroups dispatched first")
    ap.add_argument("--warp-group", default="on", choices=["on", "off"],
                    help="grouped mode: the unfused levels' warps (l2, l3, l4) as one pwc_warp_forward_group "
                         "launch ahead of their correlations (independent inputs); off = one "
                         "warp call per level")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r05_l4corr_pmc.json"),
                    help="committed PMC summary used when the live passes cannot run")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 PMC passes for roofline.traffic")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 on GPUs: nccl (= RCCL, the production path) or gloo (rehearsal: "
                         "the collectives run on CPU copies, the hot path on the GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsing the N > 1 launcher, sharding, "
                         "broadcast and shard check on a one-GPU box; with --dist-backend gloo)")
    args = ap.parse_args(argv)
    if args.same_device and args.dist_backend != "gloo":
        # several RCCL ranks on one GPU fail at init or at the first collective
        ap.error("--same-device needs --dist-backend gloo")
    if args.warmup is None:
        args.warmup = 2 if args.device == "cpu" else 300
    return args


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(args, argv) -> int:
    """Start args.gpus ranks of this script (one process per GPU) under torch.distributed.run
    and return its exit status.  Called before anything touches the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------------------
# synthetic inputs
# ---------------------------------------------------------------------------------------
def pair_inputs(g, shapes, dtype):
    """Level inputs (x1, x2, flow) of global pair g, from a CPU generator seeded by g (any rank
    can regenerate any pair)."""
    gen = torch.Generator().manual_seed(PAIR_SEED + g)
    out = []
    for (C, h, w) in shapes:
        x1 = torch.randn(C, h, w, generator=gen)
        x2 = torch.randn(C, h, w, generator=gen)
        fl = torch.randn(2, h, w, generator=gen) * 2.0
        out.append((x1.to(dtype), x2.to(dtype), fl.to(dtype)))
    return out


def checked_set(pairs, shapes, dev, dtype):
    """Buffer set of the given global pairs (seeded inputs)."""
    per = [pair_inputs(g, shapes, dtype) for g in pairs]
    s = []
    for l, (C, h, w) in enumerate(shapes):
        s.append(dict(x1=torch.stack([p[l][0] for p in per]).to(dev),
                      x2=torch.stack([p[l][1] for p in per]).to(dev),
                      flow=torch.stack([p[l][2] for p in per]).to(dev),
                      corr=torch.empty(len(pairs), 81, h, w, device=dev, dtype=dtype)))
    return s


def random_set(shapes, B, dev, dtype, gen):
    s = []
    for (C, h, w) in shapes:
        s.append(dict(x1=torch.randn(B, C, h, w, device=dev, generator=gen).to(dtype),
                      x2=torch.randn(B, C, h, w, device=dev, generator=gen).to(dtype),
                      flow=(torch.randn(B, 2, h, w, device=dev, generator=gen) * 2.0).to(dtype),
                      corr=torch.empty(B, 81, h, w, device=dev, dtype=dtype)))
    return s


# ---------------------------------------------------------------------------------------
# the per-shard pass: HIP path (product) or the CPU rehearsal stand-in
# ---------------------------------------------------------------------------------------
class HipPass:
    """warp + Correlation(model.py:24) at l0..l4 through pwcnet_amd (C ABI); the l4
    correlation is a direct, pre-bound C-ABI call so it can carry the timing events."""

    P = (CORR_ARGS["pad_size"], CORR_ARGS["kernel_size"], CORR_ARGS["max_displacement"],
         CORR_ARGS["stride1"], CORR_ARGS["stride2"])

    def __init__(self, dev, dtype, fused, group=False, warp_group=False, corr_group=False,
                 group_desc=False):
        from pwcnet_amd import _lib
        from pwcnet_amd.ops import corr_forward, warp_forward
        self._lib = _lib
        self.lib = _lib.load()  # raises if the HIP library is missing: there is no fallback
        self.warp_forward, self.corr_forward = warp_forward, corr_forward
        self.dev, self.dtype, self.fused = dev, dtype, fused
        self.group = group
        self.warp_group = warp_group
        self.corr_group = corr_group
        self.group_desc = group_desc
        self.dcode = _lib.DTYPE_CODES[dtype]

    def bind(self, s):
        """Allocate every level's outputs (x2_warp, the volume) and split-channel workspace
        once, outside any capture, so the per-step graphs only hold kernel nodes."""
        L, P = self.lib, self.P
        for l, lv in enumerate(s):
            B, C, h, w = lv["x1"].shape
            OC, Ho, Wo = self._lib.corr_output_shape(h, w, *P)
            lv["x2w"] = torch.empty_like(lv["x2"])
            lv["corr"] = torch.empty((B, OC, Ho, Wo), dtype=self.dtype, device=self.dev)
            nws = (L.pwc_warp_corr_workspace_size(B, C, h, w, *P, self.dcode, 1)
                   if l in self.fused else L.pwc_corr_workspace_size(B, C, h, w, *P))
            lv["ws"] = torch.empty(max(int(nws), 1), dtype=torch.uint8, device=self.dev)
            lv["nws"] = int(nws)

    @property
    def sp(self):
        """The CURRENT stream (torch.cuda.graph captures on its own side stream)."""
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def prepare(self, s):
        """Pre-built (function, ctypes arguments) lists of pre() and of the l4 correlation on
        the current stream, so an eager step is a loop of foreign calls with nothing to convert
        (the Python side of a launch otherwise costs about as much as the kernel at l0-l2)."""
        L, P, p = self.lib, self.P, self._p
        sp = self.sp
        c_int = ctypes.c_int
        calls = []
        grouped = self.grouped_levels(s)
        wg = self.warp_levels(s)
        cg = self.corr_levels(s)
        for l, lv in enumerate(s):
            B, C, h, w = lv["x1"].shape
            dims = [c_int(B), c_int(C), c_int(h), c_int(w)]
            cp = [c_int(v) for v in P]
            if wg and l == min(wg):
                calls.append((L.pwc_warp_forward_group,
                              (self.warp_array(s, wg), c_int(len(wg)), c_int(self.dcode), sp),
                              f"warps {wg}"))
            if (l == len(s) - 1 or l not in self.fused) and l not in wg:
                calls.append((L.pwc_warp_forward, (p(lv["x2"]), p(lv["flow"]), p(lv["x2w"]),
                                                   *dims, c_int(self.dcode), sp), f"warp l{l}"))
            if l == len(s) - 1:
                continue
            if l in grouped:
                if l == grouped[0]:
                    arr = self.group_array(s, grouped)
                    calls.append((L.pwc_warp_corr_forward_group,
                                  (arr, c_int(len(grouped)), *cp, c_int(1), c_int(self.dcode),
                                   sp), f"levels {grouped}"))
            elif l in cg:
                if l == min(cg):
                    calls.append((L.pwc_corr_forward_group,
                                  (self.corr_array(s, cg), c_int(len(cg)), *cp, c_int(1),
                                   c_int(self.dcode), sp), f"corr levels {cg}"))
            elif l in self.fused:
                calls.append((L.pwc_warp_corr_forward,
                              (p(lv["x1"]), p(lv["x2"]), p(lv["flow"]), p(lv["x2w"]),
                               p(lv["corr"]), *dims, *cp, c_int(1), c_int(self.dcode),
                               p(lv["ws"]), ctypes.c_size_t(lv["nws"]), sp), f"level {l}"))
            else:
                calls.append((L.pwc_corr_forward_ws,
                              (p(lv["x1"]), p(lv["x2w"]), p(lv["corr"]), *dims, *cp, c_int(1),
                               c_int(self.dcode), p(lv["ws"]), ctypes.c_size_t(lv["nws"]), sp),
                              f"level {l}"))
        lv = s[-1]
        B, C, h, w = lv["x1"].shape
        corr = (L.pwc_corr_forward, (p(lv["x1"]), p(lv["x2w"]), p(lv["corr"]), c_int(B), c_int(C),
                                     c_int(h), c_int(w), *[c_int(v) for v in P], c_int(1),
                                     c_int(self.dcode), sp))
        return calls, corr

    def step_prepared(self, prep, events=None):
        """One eager step from prepare()'s lists; ``events`` arms the l4 correlation."""
        calls, (cfn, cargs) = prep
        for fn, args, what in calls:
            ret = fn(*args)
            if ret != 1:
                self._lib.check(ret, "bench " + what)
        if events is not None:
            self._lib.check(self.lib.pwc_time_next_corr(ctypes.c_void_p(events[0].cuda_event),
                                                        ctypes.c_void_p(events[1].cuda_event)),
                            "bench")
        ret = cfn(*cargs)
        if ret != 1:
            self._lib.check(ret, "bench corr_l4")

    def grouped_levels(self, s):
        """The fused levels issued as one pwc_warp_corr_forward_group call (>= 2 of them)."""
        lv = sorted(l for l in self.fused if l < len(s) - 1)
        # the paired kernel is the band kernel (fp32 or fp16 storage)
        ok = self.group and len(lv) >= 2
        return lv if ok else []

    def warp_levels(self, s):
        """The unfused levels whose warps run as one pwc_warp_forward_group call."""
        lv = [l for l in range(len(s)) if l == len(s) - 1 or l not in self.fused]
        ok = self.warp_group and len(lv) >= 2
        return (lv[::-1] if self.group_desc else lv) if ok else []

    def corr_levels(self, s):
        """The unfused levels below the last whose correlations run as one
        pwc_corr_forward_group call (after their warps: needs the warp group too)."""
        lv = [l for l in range(len(s) - 1) if l not in self.fused]
        ok = self.corr_group and self.warp_levels(s) and len(lv) >= 2
        return (lv[::-1] if self.group_desc else lv) if ok else []

    def corr_array(self, s, levels):
        key = ("corrs", tuple(levels))
        arr = s[0].get(key)
        if arr is None:
            T = self._lib.CorrProblem
            arr = (T * len(levels))()
            for i, l in enumerate(levels):
                lv = s[l]
                B, C, h, w = lv["x1"].shape
                arr[i] = T(lv["x1"].data_ptr(), lv["x2w"].data_ptr(), lv["corr"].data_ptr(),
                           B, C, h, w)
            s[0][key] = arr
        return arr

    def warp_array(self, s, levels):
        key = ("warps", tuple(levels))
        arr = s[0].get(key)
        if arr is None:
            T = self._lib.WarpProblem
            arr = (T * len(levels))()
            for i, l in enumerate(levels):
                lv = s[l]
                B, C, h, w = lv["x2"].shape
                arr[i] = T(lv["x2"].data_ptr(), lv["flow"].data_ptr(), lv["x2w"].data_ptr(),
                           B, C, h, w)
            s[0][key] = arr
        return arr

    def group_array(self, s, levels):
        """The problem list of one group call, kept alive on the buffer set."""
        key = ("group", tuple(levels))
        arr = s[0].get(key)
        if arr is None:
            T = self._lib.WarpCorrProblem
            arr = (T * len(levels))()
            for i, l in enumerate(levels):
                lv = s[l]
                B, C, h, w = lv["x1"].shape
                arr[i] = T(lv["x1"].data_ptr(), lv["x2"].data_ptr(), lv["flow"].data_ptr(),
                           lv["x2w"].data_ptr(), lv["corr"].data_ptr(), B, C, h, w)
            s[0][key] = arr
        return arr

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr())

    def pre(self, s):
        """l0..l3 (warp + corr; fused levels as one WarpCorrelation launch that also emits
        x2_warp) and the l4 warp, all direct C-ABI calls on the bound buffers."""
        L, P, p = self.lib, self.P, self._p
        grouped = self.grouped_levels(s)
        wg = self.warp_levels(s)
        cg = self.corr_levels(s)
        for l, lv in enumerate(s[:-1]):
            B, C, h, w = lv["x1"].shape
            if wg and l == min(wg):
                ret = L.pwc_warp_forward_group(self.warp_array(s, wg), len(wg), self.dcode,
                                               self.sp)
                if ret != 1:
                    self._lib.check(ret, f"bench warps {wg}")
            if l in cg:
                ret = 1
                if l == min(cg):
                    ret = L.pwc_corr_forward_group(self.corr_array(s, cg), len(cg), *P, 1,
                                                   self.dcode, self.sp)
            elif l in grouped:
                ret = 1
                if l == grouped[0]:
                    ret = L.pwc_warp_corr_forward_group(self.group_array(s, grouped),
                                                        len(grouped), *P, 1, self.dcode,
                                                        self.sp)
            elif l in self.fused:
                ret = L.pwc_warp_corr_forward(p(lv["x1"]), p(lv["x2"]), p(lv["flow"]),
                                              p(lv["x2w"]), p(lv["corr"]), B, C, h, w, *P, 1,
                                              self.dcode, p(lv["ws"]), lv["nws"], self.sp)
            else:
                ret = 1
                if l not in wg:
                    ret = L.pwc_warp_forward(p(lv["x2"]), p(lv["flow"]), p(lv["x2w"]), B, C, h,
                                             w, self.dcode, self.sp)
                if ret == 1:
                    ret = L.pwc_corr_forward_ws(p(lv["x1"]), p(lv["x2w"]), p(lv["corr"]), B, C,
                                                h, w, *P, 1, self.dcode, p(lv["ws"]), lv["nws"],
                                                self.sp)
            if ret != 1:
                self._lib.check(ret, f"bench level {l}")
        lv = s[-1]
        B, C, h, w = lv["x1"].shape
        if len(s) - 1 not in wg:
            ret = L.pwc_warp_forward(p(lv["x2"]), p(lv["flow"]), p(lv["x2w"]), B, C, h, w,
                                     self.dcode, self.sp)
            if ret != 1:
                self._lib.check(ret, "bench l4 warp")

    def corr_l4(self, s, events=None):
        """The l4 correlation; ``events`` (eager timing only) arms hipExtLaunchKernel's
        start/stop events for this one launch -- never during a capture."""
        lv = s[-1]
        B, C, h, w = lv["x1"].shape
        if events is not None:
            self._lib.check(self.lib.pwc_time_next_corr(ctypes.c_void_p(events[0].cuda_event),
                                                        ctypes.c_void_p(events[1].cuda_event)),
                            "bench")
        ret = self.lib.pwc_corr_forward(self._p(lv["x1"]), self._p(lv["x2w"]),
                                        self._p(lv["corr"]), B, C, h, w, *self.P, 1, self.dcode,
                                        self.sp)
        if ret != 1:
            self._lib.check(ret, "bench corr_l4")

    def full(self, s):
        if "ws" not in s[0]:
            self.bind(s)
        self.pre(s)
        self.corr_l4(s)

    def fresh(self, s):
        """Unfused eager recomputation of every level (the self-check's reference)."""
        out = []
        for lv in s:
            x2w = self.warp_forward(lv["x2"], lv["flow"])
            out.append(self.corr_forward(lv["x1"], x2w, **CORR_ARGS))
        return out


class CpuStandinPass:
    """--device cpu launcher rehearsal only: the same pass on the torch-CPU restatement."""

    def __init__(self):
        from oracle import torch_ref
        self.T = torch_ref

    def full(self, s):
        for lv in s:
            lv["x2w"] = self.T.warp(lv["x2"], lv["flow"])
            lv["corr"] = self.T.correlation(lv["x1"], lv["x2w"], **CORR_ARGS)

    def fresh(self, s):
        return [self.T.correlation(lv["x1"], self.T.warp(lv["x2"], lv["flow"]), **CORR_ARGS)
                for lv in s]


def _same(a, b):
    """Bit-identical, NaN == NaN (a 1-pixel level divides by W - 1 = 0, as the reference)."""
    return a.shape == b.shape and torch.allclose(a, b, rtol=0.0, atol=0.0, equal_nan=True)


def _diff(a, b):
    """max |a - b| / (1 + |b|) with NaN positions required to match (inf if they do not, or if
    the shapes differ).  The fused levels (one WarpCorrelation launch) may sum in a different
    order than the unfused recomputation; a skipped kernel leaves the NaN poison."""
    if a.shape != b.shape:
        return float("inf")
    na, nb = torch.isnan(a), torch.isnan(b)
    if not torch.equal(na, nb):
        return float("inf")
    if na.all():
        return 0.0
    d = ((a - b).abs() / (1 + b.abs()))[~na]
    return float(d.max()) if d.numel() else 0.0


def pair_checksums(s):
    """(pairs, levels, 2) float64: sum and sum of squares of each pair's volume per level."""
    cols = []
    for lv in s:
        c = lv["corr"].double().flatten(1)
        cols.append(torch.stack([c.sum(1), (c * c).sum(1)], 1))
    return torch.stack(cols, 1)


def shard_check(pass_, shapes, B, world, rank, dev, dtype, cdev=None):
    """Every rank computes its own pairs [rank*B, rank*B + B) of the checked set; rank 0
    gathers the per-pair checksums and compares them with its own computation of all
    world*B pairs (same batch composition -> bit-identical arithmetic)."""
    mine = list(range(rank * B, rank * B + B))
    s = checked_set(mine, shapes, dev, dtype)
    pass_.full(s)
    cs = pair_checksums(s)
    if world > 1:
        cs = cs.to(cdev or dev)
        parts = [torch.empty_like(cs) for _ in range(world)]
        dist.all_gather(parts, cs)
        parts = [p.to(dev) for p in parts]
    else:
        parts = [cs]
    if rank != 0:
        return None
    bad = []
    for r in range(world):
        ref = checked_set(list(range(r * B, r * B + B)), shapes, dev, dtype)
        pass_.full(ref)
        exp = pair_checksums(ref)
        if not _same(exp, parts[r]):
            bad.append(r)
    return {"pairs": world * B, "ranks": world, "ok": not bad, "bad_ranks": bad}


def broadcast_weights(dev):
    """one broadcast of the Net harness's weights from rank 0; every rank checks
    it holds rank 0's parameters afterwards (checksums all_gathered).  `dev` is where the
    collective runs: the GPU under RCCL, the CPU under the gloo rehearsal."""
    from pwcnet_amd.net import Net, NetArgs
    from pwcnet_amd.shard import broadcast_module
    torch.manual_seed(1000 + dist.get_rank())  # ranks start with different weights
    net = Net(NetArgs()).to(dev)
    nbytes = sum(p.numel() * p.element_size() for p in net.parameters())
    t0 = time.perf_counter()
    broadcast_module(net, src=0)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    cs = torch.stack([p.detach().double().sum() for p in net.parameters()]).to(dev)
    parts = [torch.empty_like(cs) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, cs)
    ok = all(torch.equal(p, parts[0]) for p in parts)
    return {"bytes": nbytes, "seconds": round(el, 4), "ok": ok}


# ---------------------------------------------------------------------------------------
# CPU baselines (rank 0, N = 1)
# ---------------------------------------------------------------------------------------
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_topology():
    """Host CPU facts for the baseline line: logical CPUs, this process's affinity, the cgroup
    CPU quota (the box's share; None if unlimited), physical cores and SMT from /proc/cpuinfo."""
    info = {"host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpus": None, "physical_cores": None, "smt": None, "cpu": cpu_model()}
    try:  # cgroup v2, then v1
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_cpus"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                info["cgroup_cpus"] = round(q / per, 2)
        except (OSError, ValueError):
            pass
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    try:
        cores = set()
        phys = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
            elif not line.strip() and core is not None:
                cores.add((phys, core))
                phys = core = None
        if core is not None:
            cores.add((phys, core))
        if cores:
            info["physical_cores"] = len(cores)
            info["smt"] = round(info["host_cpus"] / len(cores), 2)
    except OSError:
        pass
    return info


def progress(msg):
    """One line on stderr per bench phase (a long phase with no output looks hung)."""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def cpu_baseline_torch(shapes, batches=(8, 1), warmup=3, runs=5, max_seconds=12.0):
    """The reference's pure-PyTorch CPU path (WarpingLayer + CostVolumeLayer at l0..l4,
    oracle/torch_ref.py) as BASELINE.md's CPU-baseline plan times it: B = 8 and B = 1 synthetic
    pairs of the 384x448 pyramid shapes, 3 warm-up passes, then the median of >= 5 timed
    passes (more while the time budget lasts), at torch.set_num_threads(usable CPUs):
    os.cpu_count() unless an affinity mask or a cgroup CPU quota gives this process fewer
    (both are reported).  A line whose first pass alone overruns the budget is recorded as
    skipped."""
    from oracle import torch_ref as T
    topo = cpu_topology()
    usable = topo["affinity_cpus"]
    if topo["cgroup_cpus"]:
        usable = max(1, min(usable, int(topo["cgroup_cpus"])))
    # os.cpu_count() when this process may use every CPU; under an affinity mask or a cgroup
    # CPU quota (the GPU box: 16 of 256 host CPUs) the usable count -- more threads than the
    # quota only queue (one 256-thread pass under a 16-CPU quota took 60-120 s)
    counts = [usable]
    prev = torch.get_num_threads()
    lines, skipped = [], []
    per_budget = max_seconds / (len(counts) * len(batches))
    try:
        for thr in counts:
            torch.set_num_threads(thr)
            for B in batches:
                progress(f"cpu baseline: {thr} threads, B={B}")
                gen = torch.Generator().manual_seed(0)
                data = [(torch.randn(B, C, h, w, generator=gen),
                         torch.randn(B, C, h, w, generator=gen),
                         torch.randn(B, 2, h, w, generator=gen) * 2) for (C, h, w) in shapes]

                def one():
                    t0 = time.perf_counter()
                    with torch.no_grad():
                        for x1, x2, fl in data:
                            T.cost_volume(x1, T.warp(x2, fl), SEARCH_RANGE)
                    return time.perf_counter() - t0

                first = one()
                if first > 4 * per_budget:
                    skipped.append(dict(B=B, threads=thr, first_pass_s=round(first, 2)))
                    continue
                for _ in range(warmup - 1):
                    one()
                times = []
                t_end = time.perf_counter() + per_budget
                while len(times) < runs or (time.perf_counter() < t_end and len(times) < 200):
                    times.append(one())
                med = float(np.median(times))
                lines.append(dict(B=B, threads=thr, value=round(B / med, 2),
                                  median_ms=round(med * 1e3, 2), runs=len(times)))
    finally:
        torch.set_num_threads(prev)
    # the main batch's line; when its first pass overran the budget (skipped), the best line
    # timed at all, or no value -- the GPU line must not be lost to the CPU baseline
    main = [l for l in lines if l["B"] == max(batches)] or lines
    if not main:
        return dict(value=None, unit="image-pairs/s", cores=usable, kind="port",
                    usable_cpus=usable, lines=lines, skipped=skipped, **topo,
                    sample="every CPU-baseline line overran its time budget (see 'skipped')")
    b8 = max(main, key=lambda l: l["value"])
    return dict(value=b8["value"], unit="image-pairs/s", cores=b8["threads"], kind="port",
                usable_cpus=usable, lines=lines, skipped=skipped, **topo,
                sample=f"B={b8['B']} synthetic pairs, median of {b8['runs']} passes after "
                       f"{warmup} warm-ups at torch.set_num_threads({b8['threads']}) (the CPUs "
                       f"this process may use of the host's {os.cpu_count()}; B=1 in 'lines'): "
                       "the reference's pure-PyTorch CPU "
                       "path (WarpingLayer = grid_sample(align_corners=True) + "
                       "CostVolumeLayer(sr=4), modules.py:31-74) at l0-l4 of 384x448, fp32. "
                       "NOTE: the correlation timed here is CostVolumeLayer(sr=4) (the "
                       "reference's CPU correlation: 81 displacements -4..4 step 1, divided by "
                       "81), not the GPU path's Correlation(9,1,9,1,2) (81 displacements -8..8 "
                       "step 2, divided by C): both read the same C x H x W inputs, write the "
                       "same 81 x H x W volume and do the same 81*C multiply-adds per pixel")


def cpu_config1(seconds):
    """BASELINE config 1: the reference's whole predict forward on CPU -- model.py's Net with
    corr = CostVolumeLayer (pure PyTorch correlation + grid_sample), reference defaults, one
    centre-cropped example pair (example/1.png, 2.png -> 384x448, main.py:321-327; committed
    as tests/golden/example_crops_384x448.npz), random-init weights (no checkpoint)."""
    import warnings
    from oracle import torch_ref as T
    z = np.load(os.path.join(ROOT, "tests", "golden", "example_crops_384x448.npz"))
    x = torch.from_numpy(np.stack([z["img1"], z["img2"]])).float()  # 2 x H x W x 3
    x = x.permute(3, 0, 1, 2).unsqueeze(0).contiguous()            # 1 x 3 x 2 x H x W
    net = T.reference_cpu_net()
    times = []
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        net(x, fused=False)  # warm-up
        t_end = time.perf_counter() + seconds
        while True:
            t0 = time.perf_counter()
            net(x, fused=False)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() >= t_end or len(times) >= 20:
                break
    med = float(np.median(times))
    return dict(value=round(1.0 / med, 3), unit="image-pairs/s", ms_per_pair=round(med * 1e3, 1),
                cores=torch.get_num_threads(), kind="port",
                sample=f"median of {len(times)} full Net forwards (convs + CostVolumeLayer + "
                       "grid_sample) on the cropped example pair, B=1, fp32 CPU")


def cpu_baseline_port(shapes, B, seconds, threads):
    """fp32 C port of the GPU semantics (warp + Corr9, oracle/pwc_oracle.c, OpenMP)."""
    from oracle import oracle as O
    rng = np.random.default_rng(0)
    data = [(rng.standard_normal((B, C, h, w)).astype(np.float32),
             rng.standard_normal((B, C, h, w)).astype(np.float32),
             (rng.standard_normal((B, 2, h, w)) * 2).astype(np.float32)) for (C, h, w) in shapes]
    O.set_num_threads(threads, np.float32)
    used = O.num_threads(np.float32)

    def one():
        for x1, x2, fl in data:
            O.corr_forward(x1, O.warp_forward(x2, fl, dtype=np.float32), 9, 1, 9, 1, 2,
                           dtype=np.float32)

    one()
    reps, t0 = 0, time.perf_counter()
    while True:
        one()
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 2000:
            break
    return dict(value=round(reps * B / el, 2), unit="image-pairs/s", cores=used, kind="port",
                sample=f"{reps} reps x {B} pairs (warp + Corr9 at l0-l4, 384x448 shapes), fp32 "
                       f"C port oracle/pwc_oracle.c, {used} OpenMP threads, {el:.1f} s")


def corr4_roofline(dev, dtype, B, shape, launches=100, cargs=None, what=None):
    """Secondary roofline line (labelled, not the headline): the north star's literal "d=4",
    Correlation(pad 4, k 1, md 4, s1 1, s2 1) -- 81 displacements -4..4 step 1, the same bytes
    and multiply-adds as model.py:24's Corr9 -- at the l4 shape, B pairs, each launch timed
    with hipExtLaunchKernel start/stop events (pwc_time_next_corr) on buffer sets rotated past
    the Infinity Cache, launches back to back.  `cargs` / `what`: another correlation config
    and its label (config 4's synthetic 192x224x32 stress shape)."""
    from pwcnet_amd import _lib
    L = _lib.load()
    C, h, w = shape
    esz = 4 if dtype == torch.float32 else 2
    P = [(cargs or CORR4_ARGS)[k] for k in ("pad_size", "kernel_size", "max_displacement",
                                            "stride1", "stride2")]
    OC, Ho, Wo = _lib.corr_output_shape(h, w, *P)
    per = (2 * C * h * w + OC * Ho * Wo) * B * esz
    nsets = max(2, int(np.ceil(2 * 256 * 2 ** 20 / per)))
    gen = torch.Generator(device=dev).manual_seed(4)
    sets = [(torch.randn(B, C, h, w, device=dev, generator=gen).to(dtype),
             torch.randn(B, C, h, w, device=dev, generator=gen).to(dtype),
             torch.empty(B, OC, Ho, Wo, device=dev, dtype=dtype)) for _ in range(nsets)]
    dcode = _lib.DTYPE_CODES[dtype]
    sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def launch(i, ev=None):
        x1, x2, o = sets[i % nsets]
        if ev is not None:
            _lib.check(L.pwc_time_next_corr(ctypes.c_void_p(ev[0].cuda_event),
                                            ctypes.c_void_p(ev[1].cuda_event)), "corr4")
        _lib.check(L.pwc_corr_forward(ctypes.c_void_p(x1.data_ptr()),
                                      ctypes.c_void_p(x2.data_ptr()),
                                      ctypes.c_void_p(o.data_ptr()), B, C, h, w, *P, 1, dcode,
                                      sp), "corr4")

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(launches)]
    for a, b in evs:
        a.record()
        b.record()
    for i in range(20):
        launch(i)
    torch.cuda.synchronize(dev)
    for i in range(launches):
        launch(i, evs[i])
    torch.cuda.synchronize(dev)
    us = float(np.mean([a.elapsed_time(b) for a, b in evs])) * 1e3
    nbytes = corr_bytes_per_pair(C, h, w, esz) * B
    ach = nbytes / (us * 1e-6) / 1e9
    kind = what or "l4 Correlation(4, 1, 4, 1, 1)"
    why = "" if what else "the north star's literal d=4, "
    return {"kernel": f"{kind} ({C}x{h}x{w}, B={B}, "
                      f"{'fp32' if esz == 4 else 'fp16'}): {why}"
                      f"{launches} back-to-back launches, hipExtLaunchKernel start/stop events",
            "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": nbytes,
            "avg_launch_us": round(us, 3)}


def net_forward(dev, B, H, W, hot_ms, iters=5):
    """End-to-end forward of the whole network (model.py:48-115): pwcnet_amd.net.Net at the
    reference defaults, convs on MIOpen fp32 (out of this project's scope), the hot path on
    the HIP drop-ins (fused forms: UpsampleWarp, CorrelationCat), random-init weights
    (model.py:39-46 under manual_seed(0)), x ~ U[0,255) of B pairs; timed with events over
    `iters` forwards after two warm-up forwards (MIOpen's first calls)."""
    from pwcnet_amd.net import Net, NetArgs
    torch.manual_seed(0)
    net = Net(NetArgs()).to(dev).eval()
    gen = torch.Generator(device=dev).manual_seed(5)
    x = torch.rand(B, 3, 2, H, W, device=dev, generator=gen) * 255.0
    with torch.no_grad():
        for _ in range(2):
            net(x)
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            flows, _ = net(x)
        b.record()
        torch.cuda.synchronize(dev)
    ms = a.elapsed_time(b) / iters
    ok = bool(torch.isfinite(flows[-1]).all())
    del net, x, flows
    torch.cuda.empty_cache()
    return {"value": round(B / ms * 1e3, 2), "unit": "image-pairs/s", "ms_per_batch": round(ms, 3),
            "batch": B, "iters": iters, "finite": ok,
            "hot_path_ms_per_batch": round(hot_ms, 4),
            "hot_path_share": round(hot_ms / ms, 4),
            "what": "full Net forward (model.py:48-115) on 1 MI355X: feature pyramid, 5 "
                    "estimator levels and the full-resolution context network on MIOpen fp32 "
                    "(out of scope), warp + Correlation on the HIP drop-ins; hot_path_share = "
                    "the headline step's ms (warp + Correlation at l0-l4, same B) / this "
                    "forward's ms. Compare cpu_config1 (the same forward on the CPU path, B=1)"}


def load_pmc_traffic(path):
    """HBM bytes per launch of the l4 correlation from a committed rocprofv3 PMC summary."""
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        return None, None


def live_pmc_traffic(B, H, W, dtype, timeout=150, step=True):
    """HBM bytes per launch of the l4 correlation measured NOW: two rocprofv3 PMC passes (one
    counter each: FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md's HBM recipe), as child processes
    in their own process group (killed as a group on timeout).  step=True: over this bench's
    own dependency-order step (a short `bench.py --no-pmc` child at this run's shape: the l4
    correlation right after its warp, on the rotating buffer sets of the timed region; the l4
    dispatches picked by their C = 32 geometry); step=False: over tools/kbench.py's l4
    correlation alone.  FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads on
    gfx950 -> x2; both in KB.  Returns (bytes, note) or (None, reason)."""
    import csv
    import shutil
    import signal
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    kb = {}
    tmp = tempfile.mkdtemp(prefix="pwc_pmc_", dir="/tmp")
    shape = ["--batch", str(B), "--height", str(H), "--width", str(W), "--dtype", dtype]
    if step:
        child = [os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "20", "--no-pmc",
                 "--no-cpu-baseline", "--no-net-forward", "--no-corr4", "--grouped-mode",
                 "off"] + shape
        pick = L4_KERNEL_RE + r".*Geo<32,"
    else:
        child = [os.path.join(ROOT, "tools", "kbench.py"), "--levels", "4", "--ops", "corr",
                 "--iters", "20"] + shape
        pick = L4_KERNEL_RE
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        out = os.path.join(tmp, ctr)
        cmd = [prof, "--pmc", ctr, "--kernel-include-regex", L4_KERNEL_RE, "-d", out, "-o",
               "run", "--output-format", "csv", "--", sys.executable] + child
        env = dict(os.environ, TMPDIR="/tmp")
        p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                             stderr=subprocess.DEVNULL, start_new_session=True)
        try:
            p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return None, f"rocprofv3 --pmc {ctr} timed out"
        vals = []
        for root, _, files in os.walk(out):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    for r in csv.DictReader(open(os.path.join(root, f))):
                        if re.search(pick, r["Kernel_Name"]):
                            vals.append(float(r["Counter_Value"]))
        if p.returncode != 0 or not vals:
            return None, f"rocprofv3 --pmc {ctr} failed (rc {p.returncode}, {len(vals)} rows)"
        kb[ctr] = sum(vals) / len(vals)
        kb["n"] = len(vals)
    shutil.rmtree(tmp, ignore_errors=True)
    rd, wr = kb["FETCH_SIZE"] * 1024 * 2, kb["WRITE_SIZE"] * 1024
    where = (f"this bench's dependency-order step (a bench.py child at the same shape, the "
             f"{kb['n']} l4 correlation dispatches of 20 timed + 20 warm-up steps and its checks)"
             if step else "tools/kbench.py --levels 4")
    return int(rd + wr), (f"live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over {where} "
                          f"in this run (reads {int(rd)} B with the gfx950 x2 FETCH_SIZE "
                          f"correction, writes {int(wr)} B per launch)")


# ---------------------------------------------------------------------------------------
# main
# ---------------------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return spawn_ranks(args, argv)
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    cpu = args.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if not torch.cuda.is_available():
            print("bench.py: no HIP device (use --device cpu for the launcher rehearsal)",
                  file=sys.stderr)
            return 3
        dev = torch.device("cuda", 0 if args.same_device else local)
        torch.cuda.set_device(dev)
        if world > 1:
            if args.dist_backend == "gloo":
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=dev)
    # where the collectives run: the GPU under RCCL, CPU copies under gloo
    cdev = dev if (cpu or args.dist_backend == "nccl") else torch.device("cpu")
    from pwcnet_amd.shard import all_ranks, max_over_ranks

    dtype = torch.float32 if args.dtype == "fp32" else torch.float16
    esz = 4 if dtype == torch.float32 else 2
    B = args.batch
    shapes = level_shapes(args.height, args.width)
    fused = {int(v) for v in args.fused_levels.split(",") if v.strip()}
    bcast = broadcast_weights(cdev) if world > 1 else None

    gpass = None
    if cpu:
        pass_ = CpuStandinPass()
        sets = [checked_set(list(range(rank * B, rank * B + B)), shapes, dev, dtype)]
        nsets = 1
    else:
        # headline: dependency order -- level after level, each level's warp before its
        # correlation, nothing batched across levels (model.py:72-113 needs level l's flow
        # before level l+1's warp)
        pass_ = HipPass(dev, dtype, fused)
        if args.grouped_mode == "on":
            gpass = HipPass(dev, dtype, fused, group=args.group == "on",
                            warp_group=args.warp_group == "on",
                            corr_group=args.corr_group == "on",
                            group_desc=args.group_order == "desc")
            if not (gpass.grouped_levels(shapes) or gpass.warp_levels(shapes)):
                gpass = None
        per_set = sum((2 * C * h * w + 2 * h * w + 81 * h * w + C * h * w) * B * esz
                      for C, h, w in shapes)
        nsets = args.sets or max(2, int(np.ceil(2 * 256 * 2 ** 20 / per_set)))
        gen = torch.Generator(device=dev).manual_seed(1234 + rank)
        sets = [random_set(shapes, B, dev, dtype, gen) for _ in range(nsets)]

    graphs, preps, gpreps = [], [], []
    timing = "cpu" if cpu else ("eager" if args.no_graph else args.timing)
    if not cpu:
        for s in sets:
            pass_.bind(s)
        for s in sets:  # first calls (kernel attributes) outside any capture
            pass_.full(s)
            if gpass is not None:
                gpass.full(s)
        torch.cuda.synchronize(dev)

        def make_events():
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.steps)]
            for a, b in evs:  # materialise the hipEvent_t handles (torch creates them lazily)
                a.record()
                b.record()
            return evs

        evs = make_events()
        gevs = make_events() if gpass is not None else None
        torch.cuda.synchronize(dev)
        if timing == "graph-all":
            # comparison mode: one hipGraph per buffer set with the WHOLE step (l4 correlation
            # included); no per-kernel events (roofline timing is absent in this mode)
            pool = torch.cuda.graph_pool_handle()
            for s in sets:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    pass_.pre(s)
                    pass_.corr_l4(s)
                graphs.append(g)
        elif timing == "graph-eager":
            # one hipGraph per buffer set for l0..l3 and the l4 warp; the l4 correlation is an
            # eager launch after the replay with hipExtLaunchKernel start/stop events
            pool = torch.cuda.graph_pool_handle()
            for s in sets:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    pass_.pre(s)
                graphs.append(g)
        else:
            # eager: every launch a direct C-ABI call on pre-built ctypes arguments (on ROCm
            # this step runs faster as plain launches than as graph replays)
            preps = [pass_.prepare(s) for s in sets]
        if gpass is not None:
            gpreps = [gpass.prepare(s) for s in sets]
        torch.cuda.synchronize(dev)

    def step(i, ev=None):
        s = sets[i % nsets]
        if cpu:
            pass_.full(s)
            return
        if timing == "graph-all":
            graphs[i % nsets].replay()
            return
        if preps:
            pass_.step_prepared(preps[i % nsets], ev)
            return
        if graphs:
            graphs[i % nsets].replay()
        else:
            pass_.pre(s)
        pass_.corr_l4(s, ev)

    def gstep(i, ev=None):
        gpass.step_prepared(gpreps[i % nsets], ev)

    def sync():
        if not cpu:
            torch.cuda.synchronize(dev)

    def timed(stepf, events):
        """W untimed steps, then K timed ones between barrier + synchronize on both sides;
        returns (MAX over ranks of the elapsed time, this rank's issue time, every rank's
        elapsed time)."""
        for i in range(args.warmup):
            stepf(i)
        sync()
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for i in range(args.steps):
            stepf(i, None if events is None else events[i])
        issued = time.perf_counter() - t0  # host time to issue the steps (GPU-bound if << elapsed)
        sync()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        return max_over_ranks(el, device=cdev), issued, all_ranks(el, device=cdev)

    def self_check(stepf, p):
        """Poison one set's outputs, run one step, compare every level with a fresh eager
        computation (a skipped kernel leaves the NaN poison)."""
        k = (args.steps - 1) % nsets
        s = sets[k]
        for lv in s:
            lv["corr"].fill_(float("nan"))
        stepf(k)
        sync()
        ref = p.fresh(s)
        diff = [_diff(lv["corr"], r) for lv, r in zip(s, ref)]
        # fused / grouped levels sum in another order than the unfused recomputation: fp32
        # within 1e-5, fp16 storage within its output rounding
        tol = 1e-5 if dtype == torch.float32 else 2e-3
        ok = all(d <= tol for d in diff)
        if world > 1:
            flag = torch.tensor([int(ok)], device=cdev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(flag.item())
        return ok, diff

    progress(f"{args.warmup} warm-up + {args.steps} timed steps")
    elapsed, issued, per_rank = timed(step, None if cpu else evs)
    replay_ok, replay_diff = self_check(step, pass_)
    grouped = None
    if gpass is not None:
        progress("grouped mode")
        g_el, g_issued, g_per_rank = timed(gstep, gevs)
        g_ok, g_diff = self_check(gstep, gpass)
        g_kern = float(np.mean([a.elapsed_time(b) for a, b in gevs]))
        grouped = {
            "mode": "grouped (NOT the headline: independent levels batched into group launches, "
                    "which the network's level-to-level flow dependency does not allow)",
            "value": round(B * args.steps * world / g_el, 2),
            "ms_per_step": round(g_el / args.steps * 1e3, 5),
            "host_issue_ms_per_step": round(g_issued / args.steps * 1e3, 5),
            "per_rank_ms_per_step": [round(v / args.steps * 1e3, 5) for v in g_per_rank],
            "grouped_levels": gpass.grouped_levels(shapes),
            "warp_grouped_levels": gpass.warp_levels(shapes),
            "corr_grouped_levels": gpass.corr_levels(shapes),
            "l4_corr_us": round(g_kern * 1e3, 3),
            "replay": g_ok, "replay_max_rel_diff": g_diff,
        }
        replay_ok = replay_ok and g_ok
    shards = shard_check(pass_, shapes, B, world, rank, dev, dtype, cdev)

    C4, h4, w4 = shapes[-1]
    pairs = B * args.steps * world
    value = pairs / elapsed
    shape_cfg = (B, args.height, args.width, args.dtype)
    if shape_cfg == (8, 384, 448, "fp32"):
        workload = ("BASELINE config 2 (config 3 at N>1): B=8 pairs/GPU, 384x448 fp32, warp + "
                    "Correlation(pad 9, k 1, md 9, s1 1, s2 2) at levels l0-l4")
    elif shape_cfg == (16, 448, 1024, "fp16"):
        workload = ("BASELINE config 4: B=16 pairs/GPU, 448x1024 (Sintel shape) fp16 storage, "
                    "warp + Correlation(pad 9, k 1, md 9, s1 1, s2 2) at levels l0-l4")
    else:
        workload = (f"custom: B={B} pairs/GPU, {args.height}x{args.width} {args.dtype}, warp + "
                    "Correlation(pad 9, k 1, md 9, s1 1, s2 2) at levels l0-l4")
    result = {
        "metric": f"image-pairs/sec (forward, {args.height}x{args.width}) at {world} MI355X: "
                  "hot path = WarpingLayer + model.py:24's Correlation(pad 9, k 1, md 9, s1 1, "
                  "s2 2: 81 displacements -8..8 step 2) at all 5 pyramid levels; lvl2 corr HBM "
                  "GB/s vs peak",
        "value": round(value, 2),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "per_rank_ms_per_step": [round(v / args.steps * 1e3, 5) for v in per_rank],
        "host_issue_ms_per_step": round(issued / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (randn features / N(0,2^2) flows of the pyramid shapes; no weights on "
                "this path)",
        "config": {
            "workload": workload,
            "global_batch": B * world,
            "per_gpu_batch": B,
            "height": args.height,
            "width": args.width,
            "levels": [list(x) for x in shapes],
            "parallelism": (f"dp{world} (batch-sharded replicas, no data-path collective)"
                            if not args.same_device else
                            f"REHEARSAL: {world} ranks on one GPU over {args.dist_backend} "
                            "(launcher, sharding, broadcast and shard check; not a scaling run)"),
            "buffer_sets": nsets,
            "fused_levels": sorted(fused),
            "order": "dependency (level after level; warp before correlation within a level)",
            "graph": bool(graphs),
            "timing": timing,
            "device": "cpu (launcher rehearsal: torch-CPU stand-in, not the product path)"
                      if cpu else "cuda",
        },
        "checks": {"replay": replay_ok, "replay_max_rel_diff": replay_diff, "shards": shards,
                   "weights_broadcast": bcast},
    }
    if grouped is not None:
        result["grouped"] = grouped
    if not cpu and timing != "graph-all":
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        bytes_launch = corr_bytes_per_pair(C4, h4, w4, esz) * B
        achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = None, None
        if not args.no_pmc and rank == 0 and world == 1:
            progress("live PMC passes")
            traffic, tsrc = live_pmc_traffic(B, args.height, args.width, args.dtype)
            if traffic is None:  # the isolated kernel instead
                why = tsrc
                traffic, tsrc = live_pmc_traffic(B, args.height, args.width, args.dtype,
                                                 step=False)
                tsrc = f"{tsrc} (in-step passes not taken: {why})"
        if traffic is None and args.dtype == "fp32" and (B, args.height, args.width) == (
                8, 384, 448):
            why = tsrc
            traffic, tsrc = load_pmc_traffic(args.pmc)
            tsrc = f"{tsrc} (committed; live PMC not taken: {why})"
        result["roofline"] = {
            "kernel": f"l4 correlation ({C4}x{h4}x{w4}, B={B}, {args.dtype}), start/stop events "
                      f"per timed step ({'hipExtLaunchKernel start/stop events'})",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "algorithmic_bytes_per_launch": bytes_launch,
            "avg_launch_us": round(kern_ms * 1e3, 3),
        }
    if rank == 0 and world == 1 and not cpu and not args.no_corr4:
        progress("Corr4 line")
        result["roofline_corr4"] = corr4_roofline(dev, dtype, B, shapes[-1])
        if dtype == torch.float16:  # config 4's synthetic stress shape, labelled separately
            progress("192x224x32 stress line")
            result["stress_192x224x32"] = corr4_roofline(
                dev, dtype, B, (32, 192, 224), cargs=CORR_ARGS,
                what="synthetic stress shape (SURVEY.md §8: the north star's '192x224x32', no "
                     "correlated level of the model) Correlation(9, 1, 9, 1, 2)")
    if rank == 0 and world == 1 and not cpu and not args.no_net_forward:
        progress("Net forward")
        result["net_forward"] = net_forward(dev, B, args.height, args.width,
                                            elapsed / args.steps * 1e3)
    if rank == 0 and world == 1 and not cpu and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_torch(shapes, batches=(B, 1),
                                                    max_seconds=args.cpu_seconds)
        cpu_v = result["cpu_baseline"]["value"]
        result["cpu_baseline"]["speedup"] = round(value / cpu_v, 1) if cpu_v else None
        thr = result["cpu_baseline"]["cores"]
        progress(f"C port baseline ({thr} threads)")
        result["cpu_baseline_port"] = cpu_baseline_port(shapes, B, args.cpu_seconds / 2, thr)
        progress("config 1 (Net forward on the CPU)")
        prev = torch.get_num_threads()
        torch.set_num_threads(thr)
        try:
            result["cpu_config1"] = cpu_config1(args.cpu_seconds / 2)
        finally:
            torch.set_num_threads(prev)
    ok = replay_ok and (shards is None or shards["ok"]) and (bcast is None or bcast["ok"])
    if rank == 0:
        print(json.dumps(result), flush=True)
        if not ok:
            print("bench.py: self-check FAILED", file=sys.stderr)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
