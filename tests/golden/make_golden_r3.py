"""Round-3 golden vectors from the REAL reference (run in the build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r3.py

  hypo256.npz  the configs-4/5 hypo-network at its real width, pinned to the reference itself:
               reference modules.SingleBVPNet(out 2, in 16, hidden 256, 3 hidden layers) run with
               per-slice (batched) parameters — the path HyperNetwork feeds (meta_modules.py:42-54,
               198-225, modules.py:16-27 with weights [B, out, in]) — on the reference's Fourier
               features (features.py:31-41) of a 64^2 grid, B = 2 slices. Stored: the FF matrix, the
               outputs, the loss-weighted gradients of the first and last layers, and every layer's
               gradient Frobenius norm. The parameters are NOT stored: they are the reference init
               under torch.manual_seed(4) (modules.py:86-90, 641-654; siren_mri_amd reproduces the RNG
               order bit for bit, tests/test_api_cpu.py) perturbed per slice by a seeded generator,
               which tests/test_gpu_modules.py regenerates with the same code (`batched_params`).
Only data leaves the reference: no source is copied.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference, quiet  # noqa: E402


def batched_params(named, B, seed):
    """Per-slice parameters from a SingleBVPNet's (name, tensor) pairs: W (1 + 0.1 g), b + 0.01 g."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, v in named:
        if k.endswith("weight"):
            out[k] = (v.detach().unsqueeze(0).repeat(B, 1, 1) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))).contiguous()
        else:
            out[k] = (v.detach().unsqueeze(0).repeat(B, 1) + 0.01 * torch.randn(B, v.shape[0], generator=g)).contiguous()
    return out


def main():
    R = import_reference()
    B, side = 2, 64
    torch.manual_seed(4)
    net = quiet(R.modules.SingleBVPNet, out_features=2, type="sine", in_features=16, hidden_features=256,
                num_hidden_layers=3, sidelength=(side, side))
    named = list(net.meta_named_parameters())
    params = batched_params(named, B, seed=11)
    for v in params.values():
        v.requires_grad_(True)
    torch.manual_seed(0)
    Bff = torch.randn(2, 8) * 21.0
    ff = R.features.GaussianFourierFeatureTransform(2, 8, 21, device="cpu")
    ff.set_B(Bff)
    coords = R.dataio.get_mgrid(side)[None].repeat(B, 1, 1)
    x = ff(coords)
    out = net({"coords": x}, params=params)
    y = out["model_out"]
    lw = torch.randn(y.shape, generator=torch.Generator().manual_seed(12))
    (y * lw).sum().backward()
    L = 5
    np.savez_compressed(
        os.path.join(OUT, "hypo256.npz"), B_ff=Bff.numpy(), y=y.detach().numpy(), lw=lw.numpy(),
        dW0=params["net.net.0.0.weight"].grad.numpy(), db0=params["net.net.0.0.bias"].grad.numpy(),
        dW4=params[f"net.net.{L - 1}.0.weight"].grad.numpy(), db4=params[f"net.net.{L - 1}.0.bias"].grad.numpy(),
        grad_norms=np.array([[params[f"net.net.{i}.0.weight"].grad.norm().item(),
                              params[f"net.net.{i}.0.bias"].grad.norm().item()] for i in range(L)]),
        seeds=np.array([4, 11, 0, 12]))
    print("wrote hypo256.npz", y.shape)


if __name__ == "__main__":
    main()
