"""Autograd wrappers of the native SIREN layer stack.

``siren_mlp(x, weights, biases, w0=..., precision=..., outermost_linear=...)`` is the fused
replacement of ``FCBlock.forward`` with nonlinearity='sine' (modules.py:92-97): the whole
[BatchLinear -> Sine] x L stack (modules.py:16-27, 35-38) runs as one native forward call and
one native backward call. Weights may be shared ([out, in]) or batched per sample
([B, out, in], the hypernetwork case of meta_modules.py:42-54, 198-225).

No CPU or eager-PyTorch fallback exists: a CPU tensor, a float64 tensor or an unsupported
shape raises.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch
from torch.autograd.function import once_differentiable

from . import _native

_DEFAULT_PRECISION = "fp32"


def set_default_precision(precision: str) -> None:
    """Process-wide default arithmetic for SIREN layers ('fp32' or 'bf16')."""
    global _DEFAULT_PRECISION
    _native.precision_code(precision)
    _DEFAULT_PRECISION = precision


def get_default_precision() -> str:
    return _DEFAULT_PRECISION


def _require_device(x: torch.Tensor):
    if x.device.type != "cuda":
        raise RuntimeError(
            "siren_mri_amd: the SIREN layer stack runs only on an MI355X (HIP) device; got a "
            f"{x.device.type} tensor. There is no CPU fallback by design.")
    if x.dtype != torch.float32:
        raise RuntimeError(f"siren_mri_amd: SIREN kernels take float32 inputs, got {x.dtype}")


class _Geometry:
    """Row/batch geometry of one call. Shared weights collapse all rows into one weight set;
    batched weights ([B, out, in]) need x of shape [B, N, in]."""
    __slots__ = ("dims", "batch", "rows", "batched", "lead_shape", "squeeze_w")

    def __init__(self, x: torch.Tensor, weights: Sequence[torch.Tensor]):
        w_first = weights[0]
        if w_first.dim() not in (2, 3):
            raise RuntimeError(f"siren_mri_amd: weight of shape {tuple(w_first.shape)} unsupported")
        batched = w_first.dim() == 3
        squeeze_w = False
        if batched and w_first.shape[0] == 1 and not (x.dim() == 3 and x.shape[0] == 1):
            batched, squeeze_w = False, True
        if batched:
            if x.dim() != 3 or w_first.shape[0] != x.shape[0]:
                raise RuntimeError(
                    f"siren_mri_amd: batched weights {tuple(w_first.shape)} need x of shape "
                    f"[{w_first.shape[0]}, N, in]; got {tuple(x.shape)}")
            B, N = x.shape[0], x.shape[1]
        else:
            B, N = 1, x.numel() // max(1, x.shape[-1])
        dims = [int(x.shape[-1])] + [int(w.shape[-2]) for w in weights]
        for l, w in enumerate(weights):
            if int(w.shape[-1]) != dims[l]:
                raise RuntimeError(f"siren_mri_amd: layer {l} weight {tuple(w.shape)} does not "
                                   f"take {dims[l]} inputs")
            if w.dim() != w_first.dim():
                raise RuntimeError("siren_mri_amd: mixed batched and shared weights")
        if N == 0:
            raise RuntimeError("siren_mri_amd: empty coordinate tensor")
        self.dims = dims
        self.batch = B
        self.rows = N
        self.batched = batched
        self.lead_shape = tuple(x.shape[:-1])
        self.squeeze_w = squeeze_w


def _flat_params(weights, biases, geo: _Geometry):
    ws, bs = [], []
    for w, b in zip(weights, biases):
        if geo.squeeze_w:
            w, b = w[0], b[0]
        ws.append(w.contiguous())
        bs.append(b.contiguous())
    return ws, bs


_SIZES = {}


def _sizes(L, desc, geo: _Geometry, prec: int, outermost_linear: bool, need_saved: bool):
    """(saved, workspace) bytes of a geometry after siren_mlp_check. They depend only on the
    geometry and options (not on the pointers), so they are asked once per geometry."""
    key = (tuple(geo.dims), geo.batch, geo.rows, geo.batched, prec, outermost_linear,
           _native.options_epoch())
    hit = _SIZES.get(key)
    if hit is None:
        _native.check(L.siren_mlp_check(ctypes.byref(desc)), "siren_mlp_check")
        hit = (L.siren_mlp_saved_bytes(ctypes.byref(desc)), L.siren_mlp_workspace_bytes(ctypes.byref(desc)))
        if len(_SIZES) > 256:
            _SIZES.clear()
        _SIZES[key] = hit
    return (hit[0] if need_saved else 0), hit[1]


class _SirenMLPFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, x, *params):
        w0, prec, outermost_linear, n_layers, grad_on = cfg
        weights = list(params[:n_layers])
        biases = list(params[n_layers:])
        _require_device(x)
        geo = _Geometry(x, weights)
        ws, bs = _flat_params(weights, biases, geo)
        xc = x.contiguous()
        dev = x.device
        desc = _native.make_desc(geo.dims, ws, bs, w0=w0, prec=prec,
                                 outermost_linear=outermost_linear, weights_batched=geo.batched,
                                 batch=geo.batch, rows_per_batch=geo.rows)
        L = _native.lib()
        need_saved = grad_on and any(ctx.needs_input_grad)
        saved_bytes, ws_bytes = _sizes(L, desc, geo, prec, outermost_linear, need_saved)
        saved = torch.empty(max(saved_bytes, 1), dtype=torch.uint8, device=dev) if need_saved else None
        work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        y = torch.empty(geo.lead_shape + (geo.dims[-1],), dtype=torch.float32, device=dev)
        rc = L.siren_mlp_forward(ctypes.byref(desc), xc.data_ptr(), y.data_ptr(),
                                 saved.data_ptr() if saved is not None else None, saved_bytes,
                                 work.data_ptr(), ws_bytes, _native.stream_handle(dev))
        _native.check(rc, "siren_mlp_forward")
        ctx.cfg = cfg
        ctx.geo = geo
        ctx.desc = desc  # its pointers are the tensors saved below
        ctx.saved_buf = saved
        ctx.saved_bytes = saved_bytes
        ctx.save_for_backward(xc, *ws, *bs)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        w0, prec, outermost_linear, n_layers, _ = ctx.cfg
        if ctx.saved_buf is None and ctx.saved_bytes:
            # the saved activations are released at the end of the first backward (they are the
            # largest allocation of a step); the reference's autograd graph could be re-entered
            raise RuntimeError(
                "siren_mri_amd: the native SIREN backward runs once per forward; backward through "
                "the same graph a second time (retain_graph=True) is not supported")
        geo = ctx.geo
        tensors = ctx.saved_tensors
        xc = tensors[0]
        ws = list(tensors[1:1 + n_layers])
        bs = list(tensors[1 + n_layers:])
        dev = xc.device
        dyc = dy.contiguous().to(torch.float32)
        desc = ctx.desc
        L = _native.lib()
        ws_bytes = _sizes(L, desc, geo, prec, outermost_linear, False)[1]
        work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        dW = [torch.empty_like(w) for w in ws]
        db = [torch.empty_like(b) for b in bs]
        need_dx = ctx.needs_input_grad[1]
        dx = torch.empty_like(xc) if need_dx else None
        VP = ctypes.c_void_p * n_layers
        dW_ptrs = VP(*[t.data_ptr() for t in dW])
        db_ptrs = VP(*[t.data_ptr() for t in db])
        rc = L.siren_mlp_backward(ctypes.byref(desc), xc.data_ptr(), dyc.data_ptr(),
                                  ctx.saved_buf.data_ptr(), ctx.saved_bytes, work.data_ptr(),
                                  ws_bytes, dW_ptrs, db_ptrs,
                                  dx.data_ptr() if dx is not None else None,
                                  _native.stream_handle(dev))
        _native.check(rc, "siren_mlp_backward")
        ctx.saved_buf = None
        ctx.desc = None
        if geo.squeeze_w:
            dW = [g.unsqueeze(0) for g in dW]
            db = [g.unsqueeze(0) for g in db]
        return (None, dx, *dW, *db)


def siren_mlp(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor], *,
              w0: float = 30.0, precision: str | None = None,
              outermost_linear: bool = True) -> torch.Tensor:
    """Fused SIREN stack: y = Linear_L(sin(w0 Linear_{L-1}(... sin(w0 Linear_0(x)))))."""
    prec = _native.precision_code(precision or _DEFAULT_PRECISION)
    n = len(weights)
    if len(biases) != n:
        raise ValueError("siren_mlp: weights and biases differ in length")
    cfg = (float(w0), prec, bool(outermost_linear), n, torch.is_grad_enabled())
    return _SirenMLPFunction.apply(cfg, x, *weights, *biases)
