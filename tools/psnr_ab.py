"""A/B of the bf16 PSNR trajectory (bench.py psnr_check workload: 64^2 cameraman, 3x256, Adam
1e-4, 500 steps) under kernel options / loss implementations.

    python tools/psnr_ab.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from siren_mri_amd import _native, dataio, loss_functions, modules, training, utils  # noqa: E402


def run(prec="bf16", torch_loss=False, steps=(0, 50, 100, 200, 300, 400, 500)):
    dev = torch.device("cuda:0")
    img = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=64)[0][1]["img"][None].to(dev)
    coords = dataio.get_mgrid(64)[None].to(dev)
    torch.manual_seed(0)
    m = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=3, sidelength=(64, 64),
                             precision=prec).to(dev)
    opt = training.make_adam(m.parameters(), 1e-4)
    vals = []
    for s in range(max(steps) + 1):
        out = m({"coords": coords})
        if s in steps:
            vals.append(utils.psnr(dataio.lin2img(out["model_out"].detach()).cpu().numpy()[0],
                                   dataio.lin2img(img).cpu().numpy()[0]))
        if torch_loss:
            d = out["model_out"] - img
            loss = (d.abs() ** 2).sum() / (128 * 128)
        else:
            loss = loss_functions.image_mse(None, out, {"img": img}, high_freq=False)["img_loss"]
        loss.backward()
        opt.step()
        opt.zero_grad()
    return [round(v, 3) for v in vals]


_native.load_library()
if len(sys.argv) > 1 and sys.argv[1] == "magic":  # the register forward's epilogue forms
    fine = tuple(sorted(set(tuple(range(0, 801, 50)) + (480, 520, 540, 560, 580))))
    print("steps           ", list(fine), flush=True)
    for v in (1, 0):
        _native.set_option("freg_magic", v)
        print(f"bf16 freg_magic={v}", run(steps=fine), flush=True)
    _native.set_option("freg_magic", 1)
    sys.exit(0)
print("fp32            ", run("fp32"), flush=True)
print("bf16 default    ", run(), flush=True)
print("bf16 torch loss ", run(torch_loss=True), flush=True)
_native.set_option("pair_ring", 0)
print("bf16 pair_ring=0", run(), flush=True)
_native.set_option("pair_ring", 1)
_native.set_option("fused_forward", 0)
print("bf16 unfused fwd", run(), flush=True)
_native.set_option("fused_forward", 1)
_native.set_option("fused_backward", 0)
print("bf16 unfused bwd", run(), flush=True)
_native.set_option("fused_backward", 1)
