#!/usr/bin/env python3
"""`pred` harness: an image pair -> PWC-Net flow on the MI355X drop-ins -> .flo + colour PNG.

The reference's `pred` subcommand (main.py:310-362) cannot run as written (it
calls model(x1, x2) on a one-argument forward, its parser lacks num_levels/lv_chs/corr/
crop_shape, and it needs cv2/imageio).  This harness does what it intends:

  1. read the two frames (PNG/JPEG via PIL, or the committed config-1 crops
     tests/golden/example_crops_384x448.npz = example/1.png, 2.png), centre-crop them to
     --crop-shape (StaticCenterCrop, main.py:321-327 / dataset.py:25-30);
  2. stack them as model.py's one input, B x 3 x 2 x H x W (model.py:48-56), and run
     pwcnet_amd.net.Net (model.py:11-115 with Correlation / WarpingLayer / CostVolumeLayer on
     the HIP library) on the GPU; weights from --load (a state_dict, loaded with
     weights_only=True) or the reference's init under --seed (model.py:39-46);
  3. write flows[-1] (the full-resolution flow, main.py:356) with save_flow (.flo,
     flow_utils.py:15-21) and its vis_flow colour image (flow_utils.py:114-149) as PNG.

    python tools/pred.py --output gpurun_out/pred/example.flo            # config-1 pair
    python tools/pred.py --input a.png b.png --output out.flo --load best.model

There is no CPU path (the product has none, like the reference's correlation.c stubs).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pwc-net_pytorch_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

EXAMPLE = os.path.join(ROOT, "tests", "golden", "example_crops_384x448.npz")


def center_crop(img, crop_shape):
    """StaticCenterCrop (main.py:318-327): rows (h-th)//2 : (h+th)//2, same for columns."""
    th, tw = crop_shape
    h, w = img.shape[:2]
    if th > h or tw > w:
        raise ValueError(f"crop {crop_shape} larger than the image {img.shape[:2]}")
    return img[(h - th) // 2:(h + th) // 2, (w - tw) // 2:(w + tw) // 2]


def read_pair(inputs, crop_shape):
    """Two H x W x 3 uint8 frames, centre-cropped."""
    if inputs is None:
        z = np.load(EXAMPLE)
        frames = [z["img1"], z["img2"]]
    else:
        from PIL import Image
        frames = [np.array(Image.open(p).convert("RGB")) for p in inputs]
    if frames[0].shape != frames[1].shape:
        raise ValueError(f"frame shapes differ: {frames[0].shape} vs {frames[1].shape}")
    return [center_crop(f, crop_shape) if crop_shape else f for f in frames]


def to_input(frames):
    """model.py:48-56's input: 1 x 3 x 2 x H x W float32 (frame index on dim 2)."""
    x = np.stack([f.transpose(2, 0, 1) for f in frames], axis=1).astype(np.float32)
    return x[np.newaxis]


def build_net(args, device):
    import torch
    from pwcnet_amd.net import Net, NetArgs
    torch.manual_seed(args.seed)
    net = Net(NetArgs(corr=args.corr, device=device))
    if args.load:
        net.load_state_dict(torch.load(args.load, map_location="cpu", weights_only=True))
    return net.to(device).eval()


def predict(net, x, device):
    """flows[-1] of Net.forward on x (numpy 1 x 3 x 2 x H x W) -> H x W x 2 numpy."""
    import torch
    from pwcnet_amd.flow_io import flow_to_hwc
    with torch.no_grad():
        flows, _ = net(torch.from_numpy(x).to(device))
    return flow_to_hwc(flows[-1])[0], flows


def write_outputs(flow, output):
    from PIL import Image
    from pwcnet_amd.flow_io import save_flow, vis_flow
    os.makedirs(os.path.dirname(os.path.abspath(output)), exist_ok=True)
    save_flow(output, flow)
    png = os.path.splitext(output)[0] + ".png"
    Image.fromarray(vis_flow(flow)).save(png)
    return png


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--input", nargs=2, default=None,
                    help="two frames (default: the config-1 example crops)")
    ap.add_argument("--output", default=os.path.join(ROOT, "gpurun_out", "pred", "example.flo"))
    ap.add_argument("--crop-shape", type=int, nargs=2, default=[384, 448])
    ap.add_argument("--corr", default="cost_volume",
                    help="'CostVolumeLayer' or anything else = Correlation(9,1,9,1,2) "
                         "(model.py:21-24; main.py:73's default 'cost_volume')")
    ap.add_argument("--load", default=None, help="state_dict (torch.save of Net.state_dict())")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args(argv)

    import torch
    if not args.device.startswith("cuda") or not torch.cuda.is_available():
        raise SystemExit("pred: the hot path runs on the HIP device only (no CPU path)")
    frames = read_pair(args.input, args.crop_shape)
    x = to_input(frames)
    net = build_net(args, args.device)
    predict(net, x, args.device)  # warm-up (MIOpen conv selection)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flow, _ = predict(net, x, args.device)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    png = write_outputs(flow, args.output)
    print(json.dumps({"flo": args.output, "png": png, "shape": list(flow.shape),
                      "forward_ms": round(ms, 3), "corr": args.corr,
                      "flow_abs_max": float(np.abs(flow).max())}))


if __name__ == "__main__":
    main()
