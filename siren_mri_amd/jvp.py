"""Analytic SIREN derivatives as autograd Functions (native tangent-stream kernels).

siren_gradient(x, fcblock, params) == diff_operators.gradient(y, x) for y = fcblock(x)
    (diff_operators.py:39-43): sum over output channels of dy/dx, shape of x. Differentiable:
    its backward is siren_jvp_backward, the hand-derived adjoint of the tangent streams (what
    loss_functions.gradients_mse's double backward computes through autograd in the reference).
siren_laplace(x, fcblock, params) == diff_operators.laplace(y, x) (diff_operators.py:27-36):
    sum over outputs and input dims of d2y/dx2. Differentiable: its backward adds the Laplacian
    adjoint stream (what laplace_mse's triple backward computes through autograd).
"""
from __future__ import annotations

import ctypes

import torch
from torch.autograd.function import once_differentiable

from . import _native
from .ops import _Geometry, _flat_params, _require_device, get_default_precision


def _desc(geo, ws, bs, fcblock, prec):
    return _native.make_desc(geo.dims, ws, bs, w0=fcblock.w0, prec=prec, outermost_linear=True,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows)


class _SirenJVP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, x, *params):
        fcblock, prec, order, n_layers, grad_on = cfg
        weights, biases = list(params[:n_layers]), list(params[n_layers:])
        _require_device(x)
        geo = _Geometry(x, weights)
        ws, bs = _flat_params(weights, biases, geo)
        xc = x.contiguous()
        dev = x.device
        desc = _desc(geo, ws, bs, fcblock, prec)
        L = _native.lib()
        keep = grad_on and any(ctx.needs_input_grad)
        saved_bytes = L.siren_jvp_saved_bytes(ctypes.byref(desc), order)
        if saved_bytes < 0:
            raise _native.NativeError(f"siren_jvp: {_native.last_error()}")
        ws_bytes = L.siren_jvp_workspace_bytes(ctypes.byref(desc), order)
        saved = torch.empty(saved_bytes, dtype=torch.uint8, device=dev) if keep else None
        work = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        grad = torch.empty(xc.shape, dtype=torch.float32, device=dev)
        lap = torch.empty(xc.shape[:-1] + (1,), dtype=torch.float32, device=dev) if order == 2 else None
        rc = L.siren_jvp_forward(ctypes.byref(desc), order, xc.data_ptr(), grad.data_ptr(),
                                 lap.data_ptr() if lap is not None else None,
                                 saved.data_ptr() if saved is not None else None, saved_bytes if keep else 0,
                                 work.data_ptr(), ws_bytes, _native.stream_handle(dev))
        _native.check(rc, "siren_jvp_forward")
        ctx.cfg, ctx.geo, ctx.saved_buf, ctx.saved_bytes = cfg, geo, saved, saved_bytes
        ctx.save_for_backward(xc, *ws, *bs)
        return grad if order == 1 else lap

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        fcblock, prec, order, n_layers, _ = ctx.cfg
        if ctx.saved_buf is None:
            raise RuntimeError(
                "siren_mri_amd: the native tangent-stream backward runs once per forward; backward "
                "through the same graph a second time (retain_graph=True) is not supported")
        geo = ctx.geo
        t = ctx.saved_tensors
        xc, ws, bs = t[0], list(t[1:1 + n_layers]), list(t[1 + n_layers:])
        dev = xc.device
        desc = _desc(geo, ws, bs, fcblock, prec)
        L = _native.lib()
        ws_bytes = L.siren_jvp_workspace_bytes(ctypes.byref(desc), order)
        work = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        dW = [torch.empty_like(w) for w in ws]
        db = [torch.empty_like(b) for b in bs]
        dx = torch.empty_like(xc) if ctx.needs_input_grad[1] else None
        VP = ctypes.c_void_p * n_layers
        rc = L.siren_jvp_backward(ctypes.byref(desc), order, xc.data_ptr(), dout.contiguous().float().data_ptr(),
                                  ctx.saved_buf.data_ptr(), ctx.saved_bytes, work.data_ptr(), ws_bytes,
                                  VP(*[g.data_ptr() for g in dW]), VP(*[g.data_ptr() for g in db]),
                                  dx.data_ptr() if dx is not None else None, _native.stream_handle(dev))
        _native.check(rc, "siren_jvp_backward")
        ctx.saved_buf = None
        if geo.squeeze_w:
            dW = [g.unsqueeze(0) for g in dW]
            db = [g.unsqueeze(0) for g in db]
        # the output bias does not reach dy/dx or the Laplacian: autograd leaves its .grad as None in the reference
        db[-1] = None
        return (None, dx, *dW, *db)


def _apply(x, fcblock, params, order):
    from .meta import get_subdict
    ws, bs = fcblock.layer_params(get_subdict(params, "net") if params is not None else None)
    prec = _native.precision_code(fcblock.precision or get_default_precision())
    cfg = (fcblock, prec, order, len(ws), torch.is_grad_enabled())
    return _SirenJVP.apply(cfg, x, *ws, *bs)


def siren_gradient(x, fcblock, params=None):
    return _apply(x, fcblock, params, 1)


def siren_laplace(x, fcblock, params=None):
    return _apply(x, fcblock, params, 2)
