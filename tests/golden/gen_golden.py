"""Generate the golden fixtures in tests/golden/ from the reference's own Python code.

Run in the build container (the only place /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

What is imported from the reference (read-only, /root/reference):
  * modules.CostVolumeLayer  (modules.py:45-74)   - pure-PyTorch cost volume
  * modules.WarpingLayer     (modules.py:25-42) + utils.get_grid (utils.py:3-8)
  * flow_utils.vis_flow      (flow_utils.py:114-149; cv2 stubbed, vis_flow does not use it)
  * model.Net                (model.py:11-115, CostVolumeLayer path; correlation_package
                              stubbed, that path never calls it)

The reference pins torch==0.4.0 (requirements.txt:62) whose F.grid_sample behaved as
align_corners=True; modern torch defaults to False (3.26 max error on an identity warp).
So ``modules.F`` is pointed at a namespace whose ``grid_sample`` passes
``align_corners=True`` explicitly.  Nothing else of the reference is altered.

The reference CUDA correlation package cannot be built or imported here (torch.utils.ffi,
THC, nvcc); its values are pinned through the CostVolumeLayer fixtures: for k=1, s1=1
Correlation(pad=md=r, s2=1) * C == CVL(sr=r)[perm] * (2r+1)^2 and
Correlation(pad=md=9, s2=2) * C == CVL(sr=8)[perm, even offsets] * 289.

Every fixture holds float32 inputs (the reference's dtype), the reference's outputs,
a seeded upstream gradient and the reference's autograd gradients.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _load_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import modules as ref_modules  # noqa: E402  (reference modules.py)

    ref_modules.F = types.SimpleNamespace(
        grid_sample=lambda x, g: F.grid_sample(
            x, g, mode="bilinear", padding_mode="zeros", align_corners=True))
    return ref_modules


def _cvl_case(M, name, seed, B, C, H, W, sr):
    g = torch.Generator().manual_seed(seed)
    src = torch.randn(B, C, H, W, generator=g)
    tgt = torch.randn(B, C, H, W, generator=g)
    args = types.SimpleNamespace(search_range=sr, device="cpu")
    s = src.clone().requires_grad_(True)
    t = tgt.clone().requires_grad_(True)
    out = M.CostVolumeLayer(args)(s, t)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), src=src.numpy(), tgt=tgt.numpy(),
                        out=out.detach().numpy(), gout=gout.numpy(), gsrc=s.grad.numpy(),
                        gtgt=t.grad.numpy(), sr=np.int32(sr))
    print(name, tuple(out.shape))


def _warp_case(M, name, seed, B, C, H, W, flow_std, zero_flow=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, H, W, generator=g)
    if zero_flow:
        flow = torch.zeros(B, 2, H, W)
    else:
        flow = torch.randn(B, 2, H, W, generator=g) * flow_std
    args = types.SimpleNamespace(device="cpu")
    xs = x.clone().requires_grad_(True)
    fs = flow.clone().requires_grad_(True)
    out = M.WarpingLayer(args)(xs, fs)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x.numpy(), flow=flow.numpy(),
                        out=out.detach().numpy(), gout=gout.numpy(), gx=xs.grad.numpy(),
                        gflow=fs.grad.numpy())
    print(name, tuple(out.shape))


def _upwarp_case(M, name, seed, B, C, h, w, flow_std):
    """model.py:78 (F.upsample(flow, scale_factor=2, mode='bilinear') * 2, called as the
    reference calls it: torch 0.4's default is align_corners=False, as is modern torch's) then
    model.py:80 (the reference WarpingLayer); gradients wrt x2 and the coarse flow for seeded
    upstream gradients of x2_warp and of the upsampled flow (model.py:89/91 concatenates it)."""
    g = torch.Generator().manual_seed(seed)
    x2 = torch.randn(B, C, 2 * h, 2 * w, generator=g)
    flow = torch.randn(B, 2, h, w, generator=g) * flow_std
    args = types.SimpleNamespace(device="cpu")
    xs = x2.clone().requires_grad_(True)
    fs = flow.clone().requires_grad_(True)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        fup = F.upsample(fs, scale_factor=2, mode="bilinear") * 2
    out = M.WarpingLayer(args)(xs, fup)
    gout = torch.randn(out.shape, generator=g)
    gfup = torch.randn(fup.shape, generator=g)
    torch.autograd.backward([out, fup], [gout, gfup])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x2=x2.numpy(), flow=flow.numpy(),
                        out=out.detach().numpy(), flow_up=fup.detach().numpy(),
                        gout=gout.numpy(), gflow_up=gfup.numpy(), gx2=xs.grad.numpy(),
                        gflow=fs.grad.numpy())
    print(name, tuple(out.shape))


def _vis_case(name, seed, H, W):
    """flow_utils.vis_flow (flow_utils.py:114-149) on a seeded flow with unknown (> 1e9)
    entries; flow_utils imports cv2 at the top but vis_flow never uses it, so a stub module
    stands in for it (cv2 is not installed here)."""
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    import flow_utils  # noqa: E402  (reference flow_utils.py)
    rng = np.random.default_rng(seed)
    flow = (rng.standard_normal((H, W, 2)) * 3).astype(np.float32)
    flow[0, 0, 0] = 2e9      # unknown flow (u > UNKNOWN_FLOW_THRESH)
    flow[1, 2, 1] = 5e9      # unknown flow (v)
    flow[3, 3] = 0.0         # zero motion
    img = flow_utils.vis_flow(flow.copy())
    np.savez_compressed(os.path.join(HERE, name + ".npz"), flow=flow, img=img)
    print(name, img.shape, img.dtype)


def _net_case(name, seed, H, W, corr="CostVolumeLayer"):
    """A reduced end-to-end run of the reference Net (model.py:11-115, CostVolumeLayer path,
    reference defaults otherwise) at H x W, weights from torch.manual_seed(seed) at
    construction (model.py:39-46 init).  correlation_package (CUDA/THC, unbuildable here) is a
    sys.modules stub: with args.corr == 'CostVolumeLayer' model.py never calls it.  Weights
    are not stored (20 MB): the fixture holds per-parameter sums so a harness seeded the same
    way can prove it built the same weights, the input, and every returned flow."""
    stub = types.ModuleType("correlation_package")
    sub = types.ModuleType("correlation_package.modules")
    leaf = types.ModuleType("correlation_package.modules.correlation")

    class Correlation(torch.nn.Module):  # never called on the CostVolumeLayer path
        def __init__(self, *a, **k):
            super().__init__()

    leaf.Correlation = Correlation
    sys.modules.update({"correlation_package": stub, "correlation_package.modules": sub,
                        "correlation_package.modules.correlation": leaf})
    import model as ref_model  # noqa: E402  (reference model.py)
    args = types.SimpleNamespace(search_range=4, num_levels=7, lv_chs=[16, 32, 64, 96, 128, 192],
                                 output_level=4, batch_norm=False, input_norm=False,
                                 rgb_max=255.0, residual=False, flow_norm=False, corr=corr,
                                 corr_activation=False, device="cpu")
    torch.manual_seed(seed)
    net = ref_model.Net(args)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.rand(1, 3, 2, H, W, generator=g) * 255.0
    import warnings
    with warnings.catch_warnings(), torch.no_grad():
        warnings.simplefilter("ignore")
        flows, summaries = net(x)
    names = [k for k, _ in net.named_parameters()]
    sums = np.array([float(p.double().sum()) for _, p in net.named_parameters()])
    out = dict(x=x.numpy(), param_names=np.array(names), param_sums=sums,
               n_flows=np.int32(len(flows)))
    for i, f in enumerate(flows):
        out[f"flow{i}"] = f.numpy()
    for i, w in enumerate(summaries["x2_warps"]):
        out[f"x2_warp{i}"] = w.numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, [tuple(f.shape) for f in flows])


def main():
    M = _load_reference()
    # CostVolumeLayer sr=4 ("Corr4" pin) and sr=8 ("Corr9" pin), SURVEY §8c shapes.
    _cvl_case(M, "cvl_sr4_b2c8_12x14", 1, 2, 8, 12, 14, 4)
    _cvl_case(M, "cvl_sr4_b2c32_24x28", 2, 2, 32, 24, 28, 4)
    _cvl_case(M, "cvl_sr8_b2c8_12x14", 3, 2, 8, 12, 14, 8)
    _cvl_case(M, "cvl_sr8_b1c32_12x14", 4, 1, 32, 12, 14, 8)
    # true pyramid shapes at 384x448, B=1 (l0 192x6x7, l1 128x12x14)
    _cvl_case(M, "cvl_sr4_l0_b1c192_6x7", 5, 1, 192, 6, 7, 4)
    _cvl_case(M, "cvl_sr8_l0_b1c192_6x7", 6, 1, 192, 6, 7, 8)
    _cvl_case(M, "cvl_sr4_l1_b1c128_12x14", 7, 1, 128, 12, 14, 4)
    # l2 true shape (96x24x28) and l1 with sr = 8 (the Corr9 pin at l1)
    _cvl_case(M, "cvl_sr4_l2_b1c96_24x28", 8, 1, 96, 24, 28, 4)
    _cvl_case(M, "cvl_sr8_l1_b1c128_12x14", 9, 1, 128, 12, 14, 8)
    # warp: flows ~ N(0, 2^2) incl. out-of-bounds samples; a large-flow case; zero flow.
    _warp_case(M, "warp_b2c8_12x14", 11, 2, 8, 12, 14, 2.0)
    _warp_case(M, "warp_b2c32_24x28", 12, 2, 32, 24, 28, 2.0)
    _warp_case(M, "warp_b1c16_9x31_far", 13, 1, 16, 9, 31, 12.0)
    _warp_case(M, "warp_b1c4_6x7_zero", 14, 1, 4, 6, 7, 0.0, zero_flow=True)
    # flow upsample x2 (model.py:78) then warp (model.py:80): l0 -> l1 shape and a ragged one
    _upwarp_case(M, "upwarp_b2c8_6x7", 21, 2, 8, 6, 7, 1.5)
    _upwarp_case(M, "upwarp_b1c4_5x9_far", 22, 1, 4, 5, 9, 6.0)
    # flow colour coding (flow_utils.py:114-149) and a reduced end-to-end Net (model.py)
    _vis_case("visflow_20x24", 31, 20, 24)
    _net_case("net_cvl_128x128", 0, 128, 128)
    example_crops()




def example_crops():
    """Config 1's inputs (BASELINE.json): example/1.png, 2.png (1024x436 RGB) centre-cropped
    to 384x448 as main.py's StaticCenterCrop does (main.py:321-327: rows 26:410, cols
    288:736), stored as uint8 HxWx3 (data files of the reference, not code)."""
    from PIL import Image
    crops = []
    for i in (1, 2):
        im = np.array(Image.open(os.path.join(REF, "example", f"{i}.png")).convert("RGB"))
        h, w = im.shape[:2]
        crops.append(im[(h - 384) // 2:(h + 384) // 2, (w - 448) // 2:(w + 448) // 2])
    np.savez_compressed(os.path.join(HERE, "example_crops_384x448.npz"), img1=crops[0],
                        img2=crops[1])


if __name__ == "__main__":
    main()
