"""Repeatability stress of the correlation forward in the bench's order (warp, then the
correlation of its output) at config 2's l3 and l4: each iteration warps a fresh random input,
runs the default dispatch and a reference path (the row-band / 56-px strip kernel through a
knob) on the same warped tensor, and counts the iterations whose volumes differ."""
import sys
sys.path.insert(0, "pwc-net_pytorch_amd")
sys.path.insert(0, ".")
import torch  # noqa: E402
import bench  # noqa: E402
from pwcnet_amd import _lib  # noqa: E402
from pwcnet_amd.ops import corr_forward, warp_forward  # noqa: E402

dev = torch.device("cuda:0")
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
for lvl, knob in ((2, "strip_l2=0"), (3, "strip_l3=0"), (4, "strip_geo=4")):
    C, h, w = bench.level_shapes(384, 448)[lvl]
    B = 8
    g = torch.Generator(device=dev).manual_seed(11)
    bad, worst = 0, 0.0
    for it in range(iters):
        x1 = torch.randn(B, C, h, w, device=dev, generator=g)
        x2 = torch.randn(B, C, h, w, device=dev, generator=g)
        fl = torch.randn(B, 2, h, w, device=dev, generator=g) * 2
        x2w = warp_forward(x2, fl)
        a = corr_forward(x1, x2w, 9, 1, 9, 1, 2)
        _lib.set_debug(knob)
        b = corr_forward(x1, x2w, 9, 1, 9, 1, 2)
        _lib.set_debug("")
        d = float((a - b).abs().max())
        if not d <= 1e-5:
            bad += 1
            worst = max(worst, d if d == d else 1e30)
            idx = torch.nonzero((a - b).abs() > 1e-5)
            if bad <= 3:
                print(f"l{lvl} it {it}: diff {d:.3g}, {idx.shape[0]} elements, first {idx[:4].tolist()}",
                      flush=True)
    torch.cuda.synchronize()
    print(f"l{lvl}: {bad} of {iters} iterations differ (worst {worst:.3g})", flush=True)
