"""Poison check of the correlation forward at config 2's l2-l4 under the dispatch knobs: the
output pre-filled with NaN, three calls through the C ABI; prints how many outputs the first
call left unwritten and the max difference between calls (must be 0 / 0 / 0)."""
import sys, os
sys.path.insert(0, "pwc-net_pytorch_amd"); sys.path.insert(0, ".")
import torch, bench
from pwcnet_amd import _lib
from pwcnet_amd.ops import corr_forward, _ptr, _stream, _workspace
lib = _lib.load()
dev = torch.device("cuda:0")
for lvl in (2, 3, 4):
    C, h, w = bench.level_shapes(384, 448)[lvl]
    B = 8
    g = torch.Generator(device=dev).manual_seed(7)
    x1 = torch.randn(B, C, h, w, device=dev, generator=g)
    x2 = torch.randn(B, C, h, w, device=dev, generator=g)
    for knob in ("", "strip_l3=0", "strip=0"):
        _lib.set_debug(knob)
        outs = []
        for it in range(3):
            out = torch.full((B, 81, h, w), float("nan"), device=dev)
            nws = lib.pwc_corr_workspace_size(B, C, h, w, 9, 1, 9, 1, 2)
            ws, wsp = _workspace(nws, dev)
            r = lib.pwc_corr_forward_ws(_ptr(x1), _ptr(x2), _ptr(out), B, C, h, w, 9, 1, 9, 1, 2, 1, 0, wsp, nws, _stream(dev))
            torch.cuda.synchronize()
            outs.append(out)
        nan = int(torch.isnan(outs[0]).sum())
        d01 = float((outs[0] - outs[1]).abs().nan_to_num(1e30).max())
        d12 = float((outs[1] - outs[2]).abs().nan_to_num(1e30).max())
        print(f"l{lvl} knob={knob!r:14} ret={r} nan_first={nan} d01={d01:.3g} d12={d12:.3g} ws={nws}", flush=True)
    _lib.set_debug("")
