"""k-space data consistency (data_consistency.py:8-48 of jonbmartin/siren_mri).

out = (1 - m) * pred + m * k0 (noiseless) or (1 - m) * pred + m * (pred + v k0) / (1 + v),
with k0/mask given as [B, 2, H, W] (NCHW planes) and pred as [B, H*W, 2].

On the GPU this is the native op siren_mri_amd::dc_forward (siren_kspace.hip: one launch that
reads k0 and the mask where they lie instead of permuting copies of them; bit-identical to the
reference's elementwise chain) with dc_backward as its autograd formula. The output remembers its
inputs (attribute `_siren_dc`), so loss_functions.image_mse of a DC output runs the fused
DC + masked-SSE op, whose backward writes dL/dpred in one launch.
Inputs on the CPU (or other dtypes) take the reference's PyTorch expression.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.nn as nn
from torch import Tensor

from . import _native, fusion
from .ops import _LIB

_LIB.define("dc_forward(Tensor pred, Tensor k0, Tensor mask, float noise) -> Tensor")
_LIB.define("dc_backward(Tensor g, Tensor mask, float noise) -> Tensor")


def _planes(pred, k0):
    b, n, c = pred.shape
    if k0.shape[0] != b or k0.shape[1] != c or k0[0, 0].numel() != n:
        raise RuntimeError(f"siren_mri_amd.dc: k-space planes {tuple(k0.shape)} do not match the prediction "
                           f"{tuple(pred.shape)}")
    return b, n, c


def _dc_forward_cuda(pred: Tensor, k0: Tensor, mask: Tensor, noise: float) -> Tensor:
    b, n, c = _planes(pred, k0)
    pc, kc, mc = pred.contiguous(), k0.contiguous(), mask.contiguous()
    out = torch.empty_like(pc)
    _native.check(_native.lib().siren_dc_forward(pc.data_ptr(), kc.data_ptr(), mc.data_ptr(), b, n, c, float(noise),
                                                 out.data_ptr(), _native.stream_handle(pred.device)), "siren_dc_forward")
    return out


def _dc_backward_cuda(g: Tensor, mask: Tensor, noise: float) -> Tensor:
    b, n, c = g.shape
    gc, mc = g.contiguous(), mask.contiguous()
    out = torch.empty_like(gc)
    _native.check(_native.lib().siren_dc_backward(gc.data_ptr(), mc.data_ptr(), b, n, c, float(noise), out.data_ptr(),
                                                  _native.stream_handle(g.device)), "siren_dc_backward")
    return out


class _DCAutograd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, k0, mask, noise):
        with torch._C._AutoDispatchBelowAutograd():
            out = torch.ops.siren_mri_amd.dc_forward(pred, k0, mask, noise)
        ctx.save_for_backward(mask)
        ctx.noise = noise
        return out

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return torch.ops.siren_mri_amd.dc_backward(g, mask, ctx.noise), None, None, None


_LIB.impl("dc_forward", _dc_forward_cuda, "CUDA")
_LIB.impl("dc_backward", _dc_backward_cuda, "CUDA")
_LIB.impl("dc_forward", lambda pred, k0, mask, noise: _DCAutograd.apply(pred, k0, mask, noise), "Autograd")
torch.library.register_fake("siren_mri_amd::dc_forward", lambda pred, k0, mask, noise: torch.empty_like(pred), lib=_LIB)
torch.library.register_fake("siren_mri_amd::dc_backward", lambda g, mask, noise: torch.empty_like(g), lib=_LIB)


def data_consistency(pred, k0, mask, noise_lvl=None):
    """data_consistency.py:8-20 on tensors of one layout (the reference's expression)."""
    v = noise_lvl
    if v:
        return (1 - mask) * pred + mask * (pred + v * k0) / (1 + v)
    return (1 - mask) * pred + mask * k0


def _native_ok(pred, k0, mask):
    return (pred.is_cuda and pred.dtype == torch.float32 and k0.dtype == torch.float32 and mask.dtype == torch.float32
            and pred.dim() == 3 and k0.dim() == 4 and k0.shape == mask.shape and pred.shape[-1] <= 8
            and k0.device == pred.device and mask.device == pred.device and not k0.requires_grad
            and not mask.requires_grad)


class DataConsistencyInKspace(nn.Module):
    def __init__(self, noise_lvl=None):
        super().__init__()
        self.noise_lvl = noise_lvl

    def forward(self, prediction, k0, mask):
        if _native_ok(prediction, k0, mask):
            noise = float(self.noise_lvl) if self.noise_lvl else 0.0
            st = fusion.staged(prediction.device)
            if st is not None and st.result is not None and st.result[0] is prediction and st.result[1] is not None:
                sk0, smask, snoise = st.result[4]
                if sk0 is k0 and smask is mask and snoise == noise:
                    # computed by the forward's fused output epilogue (fusion.py)
                    out = st.result[1]
                    out._siren_dc = (prediction, k0, mask, noise)
                    return out
            out = torch.ops.siren_mri_amd.dc_forward(prediction, k0, mask, noise)
            out._siren_dc = (prediction, k0, mask, noise)
            return out
        b = k0.shape[0]
        k0 = k0.permute(0, 2, 3, 1).reshape(b, -1, 2)
        mask = mask.permute(0, 2, 3, 1).reshape(b, -1, 2)
        return data_consistency(prediction, k0, mask, self.noise_lvl)


def dc_source(t: Tensor) -> Optional[tuple]:
    """(pred, k0, mask, noise) if t is the output of DataConsistencyInKspace's native path."""
    return getattr(t, "_siren_dc", None)
