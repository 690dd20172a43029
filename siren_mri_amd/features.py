"""Gaussian Fourier features (features.py:6-53 of jonbmartin/siren_mri).

forward: cat(sin(2 pi x B), cos(2 pi x B)) with B = randn(in, m) * scale (features.py:21-41).
On the GPU the transform is the native op siren_mri_amd::fourier_features (one launch).
B lives as a buffer on the module's device (the reference keeps it on the CPU and copies it to
the input's device on every call, features.py:28,36); save_B/load_B/get_B/set_B keep the
reference's file format (a bare tensor saved with torch.save).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _native
from .ops import _LIB

# siren_mri_amd::fourier_features(x, B) -> cat(sin(2 pi x B), cos(2 pi x B)) (one native launch);
# its gradient w.r.t. x (the reference differentiates through it when x requires grad) is the
# PyTorch expression's, recomputed on the backward (B is a constant buffer)
_LIB.define("fourier_features(Tensor x, Tensor B) -> Tensor")


def _ff_cuda(x, B):
    xc, Bc = x.contiguous(), B.contiguous()
    cin, m = Bc.shape
    out = torch.empty(xc.shape[:-1] + (2 * m,), dtype=torch.float32, device=x.device)
    rows = xc.numel() // cin
    _native.check(_native.lib().siren_fourier_features(xc.data_ptr(), Bc.data_ptr(), rows, cin, m, out.data_ptr(),
                                                       _native.stream_handle(x.device)), "siren_fourier_features")
    return out


class _FFAutograd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, B):
        with torch._C._AutoDispatchBelowAutograd():
            out = torch.ops.siren_mri_amd.fourier_features(x, B)
        ctx.save_for_backward(x, B)
        return out

    @staticmethod
    def backward(ctx, g):
        x, B = ctx.saved_tensors
        m = B.shape[1]
        z = 2 * np.pi * (x @ B)
        gs, gc = g[..., :m], g[..., m:]
        dz = gs * torch.cos(z) - gc * torch.sin(z)
        return (2 * np.pi) * (dz @ B.t()), None


_LIB.impl("fourier_features", _ff_cuda, "CUDA")
_LIB.impl("fourier_features", lambda x, B: _FFAutograd.apply(x, B), "Autograd")
torch.library.register_fake("siren_mri_amd::fourier_features",
                            lambda x, B: x.new_empty(x.shape[:-1] + (2 * B.shape[1],)), lib=_LIB)


# Fourier features formed in the SIREN's first layer (GaussianFourierFeatureTransform.model_input,
# ops.siren_mlp(ff_B=...)): ON by default since round 5 — the kernels form the features with the
# fourier_features op's own arithmetic (siren_common.h ff_feature = siren_kspace.hip fourier_kernel),
# so the fused and the materialised paths compute the same network bit for bit
# (tests/test_gpu_fourier_input.py). SIREN_MRI_AMD_FUSED_FOURIER=0 materialises the features with
# the fourier_features op (one launch), the reference's data flow.
FUSED_INPUT = os.environ.get("SIREN_MRI_AMD_FUSED_FOURIER", "1") == "1"


def fourier_features(x, B):
    """cat(sin(2 pi x B), cos(2 pi x B)) (features.py:21-41) for a given B."""
    B = B.to(x.device, x.dtype)
    if x.is_cuda and x.dtype == torch.float32:
        return torch.ops.siren_mri_amd.fourier_features(x, B)
    z = 2 * np.pi * (x @ B)
    return torch.cat([torch.sin(z), torch.cos(z)], dim=-1)


class GaussianFourierFeatureTransform(torch.nn.Module):
    def __init__(self, num_input_channels, mapping_size_spatial=256, scale=10, loaded_B=None, device=None):
        super().__init__()
        self._num_input_channels = num_input_channels
        self._mapping_size = mapping_size_spatial
        B = torch.randn((num_input_channels, mapping_size_spatial)) * scale if loaded_B is None else loaded_B
        self.register_buffer("_B_spatial", B.detach().clone(), persistent=False)
        self._fused_ok = _fused_range_ok(self._B_spatial)
        if device is not None:
            self.to(device)

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.float32:
            return torch.ops.siren_mri_amd.fourier_features(x, self._B_spatial.to(x.device, x.dtype))
        z = x @ self._B_spatial.to(x.device, x.dtype)
        z = 2 * np.pi * z
        return torch.cat([torch.sin(z), torch.cos(z)], dim=-1)

    def model_input(self, model, model_input):
        """Apply the transform to model_input["coords"] for `model` (training.py:61-64). A model that
        takes the Fourier-feature input in its SIREN's first layer (attribute fourier_input, e.g.
        the conv hypernetwork; the kernel forms the features) gets the raw
        coordinates and model_input["fourier_B"] when fusion is on and the coordinates need no
        gradient; every other model gets the materialised features, as in the reference."""
        from . import fusion
        x = model_input["coords"]
        inner = getattr(model, "module", model)  # (a DistributedDataParallel wrapper)
        if (FUSED_INPUT and self._fused_ok and getattr(inner, "fourier_input", False) and fusion.enabled()
                and x.is_cuda and x.dtype == torch.float32 and not x.requires_grad):
            model_input["fourier_B"] = self._B_spatial.to(x.device, x.dtype)
        else:
            model_input["coords"] = self(x)
        return model_input

    def save_B(self, filename):
        torch.save(self._B_spatial.detach().cpu(), filename)

    def load_B(self, filename):
        self.set_B(torch.load(filename, weights_only=True))

    def get_B(self):
        return self._B_spatial

    def set_B(self, B):
        self._B_spatial = B.detach().clone().to(self._B_spatial.device)
        self._fused_ok = _fused_range_ok(self._B_spatial)


# |2 pi x B| bound below which the kernels' Fourier-feature sin / cos (siren_common.h ff_feature,
# fourier_kernel: Cody-Waite + minimax) are accurate (kFFPolyRange): the in-kernel transform is
# used only when it holds for coordinates in [-1, 1] (get_mgrid's range); larger B entries take
# the materialised op, whose kernel calls the far-range sin / cos past it
FF_POLY_RANGE = 1.0e6


def _fused_range_ok(B):
    """Whether 2 pi max_k sum_c |B[c][k]| < FF_POLY_RANGE (computed once per B, on set)."""
    if B.numel() == 0:
        return True
    return float(2 * np.pi * B.detach().abs().sum(0).max()) < FF_POLY_RANGE
