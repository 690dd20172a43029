"""Analytic SIREN derivatives as PyTorch custom ops (native tangent-stream kernels).

siren_gradient(x, fcblock, params) == diff_operators.gradient(y, x) for y = fcblock(x)
    (diff_operators.py:39-43): sum over output channels of dy/dx, shape of x. Differentiable:
    its backward is siren_jvp_backward, the hand-derived adjoint of the tangent streams (what
    loss_functions.gradients_mse's double backward computes through autograd in the reference).
siren_laplace(x, fcblock, params) == diff_operators.laplace(y, x) (diff_operators.py:27-36):
    sum over outputs and input dims of d2y/dx2. Differentiable: its backward adds the Laplacian
    adjoint stream (what laplace_mse's triple backward computes through autograd).
siren_jacobian(x, fcblock, params) == diff_operators.jacobian(y, x)[0] (diff_operators.py:46-59):
    dy_c/dx_k per output channel. Differentiable (the same adjoint with a per-channel cotangent);
    it also carries gradient(y, x, grad_outputs=g) for any g, and the double backward of the
    SIREN forward through autograd (ops._SineMLPAutograd under create_graph=True).

Custom ops (torch.library.Library "siren_mri_amd", with fake kernels and an Autograd-key
formula), over the C ABI siren_jvp_forward/backward:
  siren_mri_amd::sine_mlp_jvp(x, W[], b[], w0, prec, batched, order, keep) -> (out, saved)
  siren_mri_amd::sine_mlp_jvp_bwd(dout, x, W[], b[], saved, w0, prec, batched, order, need_dx)
        -> (dx, dW[], db[])
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

import torch
from torch import Tensor

from . import _native
from .ops import _LIB, _Geometry, _geo_of, _require_device, get_default_precision


def _desc(geo, ws, bs, w0, prec):
    return _native.make_desc(geo.dims, ws, bs, w0=w0, prec=prec, outermost_linear=True,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows)


def _jvp_sizes(geo, prec, order):
    L = _native.lib()
    d = _native.describe_only(geo.dims, prec=prec, weights_batched=geo.batched, batch=geo.batch,
                              rows_per_batch=geo.rows)
    saved = L.siren_jvp_saved_bytes(ctypes.byref(d), order)
    if saved < 0:
        raise _native.NativeError(f"siren_jvp: {_native.last_error()}")
    return saved, L.siren_jvp_workspace_bytes(ctypes.byref(d), order)


GRADIENT, LAPLACE, JACOBIAN = 1, 2, 3  # SIREN_JVP_* of include/siren_mri_amd.h

_LIB.define("sine_mlp_jvp(Tensor x, Tensor[] weights, Tensor[] biases, float w0, int prec, bool batched, int order, "
            "bool keep, Tensor? primal=None) -> (Tensor, Tensor)")
_LIB.define("sine_mlp_jvp_bwd(Tensor dout, Tensor x, Tensor[] weights, Tensor[] biases, Tensor saved, float w0, "
            "int prec, bool batched, int order, bool need_dx, Tensor? primal=None) -> (Tensor, Tensor[], Tensor[])")


def sine_mlp_jvp(x: Tensor, weights: List[Tensor], biases: List[Tensor], w0: float, prec: int, batched: bool,
                 order: int, keep: bool, primal: Tensor | None = None) -> Tuple[Tensor, Tensor]:
    """siren_jvp_forward_ex: order 1 -> sum_c dy_c/dx (shape of x); order 2 -> the Laplacian [.., 1];
    order 3 -> the per-channel Jacobian dy_c/dx_k [.., out, in]. primal: the saved buffer of the
    plain forward of this stack on this x (fp32): its phases are the primal stream."""
    _require_device(x)
    geo = _geo_of(x, weights, batched)
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    desc = _desc(geo, ws, bs, w0, prec)
    saved_bytes, ws_bytes = _jvp_sizes(geo, prec, order)
    saved = torch.empty(saved_bytes if keep else 0, dtype=torch.uint8, device=dev)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    gshape = xc.shape[:-1] + (geo.dims[-1], xc.shape[-1]) if order == JACOBIAN else xc.shape
    grad = torch.empty(gshape, dtype=torch.float32, device=dev)
    lap = torch.empty(xc.shape[:-1] + (1,), dtype=torch.float32, device=dev) if order == LAPLACE else None
    rc = _native.lib().siren_jvp_forward_ex(ctypes.byref(desc), order, xc.data_ptr(), grad.data_ptr(),
                                            lap.data_ptr() if lap is not None else None,
                                            saved.data_ptr() if keep else None, saved_bytes if keep else 0,
                                            work.data_ptr(), ws_bytes,
                                            primal.data_ptr() if primal is not None else None,
                                            primal.numel() if primal is not None else 0, _native.stream_handle(dev))
    _native.check(rc, "siren_jvp_forward_ex")
    return (lap if order == LAPLACE else grad), saved


def _sine_mlp_jvp_fake(x, weights, biases, w0, prec, batched, order, keep, primal=None):
    geo = _geo_of(x, weights, batched)
    saved_bytes, _ = _jvp_sizes(geo, prec, order)
    if order == JACOBIAN:
        out = x.new_empty(x.shape[:-1] + (geo.dims[-1], x.shape[-1]))
    else:
        out = x.new_empty(x.shape) if order == GRADIENT else x.new_empty(x.shape[:-1] + (1,))
    return out, x.new_empty((saved_bytes if keep else 0,), dtype=torch.uint8)


def sine_mlp_jvp_bwd(dout: Tensor, x: Tensor, weights: List[Tensor], biases: List[Tensor], saved: Tensor, w0: float,
                     prec: int, batched: bool, order: int, need_dx: bool,
                     primal: Tensor | None = None) -> Tuple[Tensor, List[Tensor], List[Tensor]]:
    """siren_jvp_backward: the adjoint of the tangent streams -> (dx or empty, dW, db)."""
    if saved.numel() == 0:
        raise RuntimeError("siren_mri_amd: sine_mlp_jvp_bwd needs the saved buffer of a forward with keep=True")
    geo = _geo_of(x, weights, batched)
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    desc = _desc(geo, ws, bs, w0, prec)
    saved_bytes, ws_bytes = _jvp_sizes(geo, prec, order)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    dW = [torch.empty_like(w) for w in ws]
    db = [torch.empty_like(b) for b in bs]
    dx = torch.empty_like(xc) if need_dx else xc.new_empty((0,))
    VP = ctypes.c_void_p * len(ws)
    rc = _native.lib().siren_jvp_backward_ex(ctypes.byref(desc), order, xc.data_ptr(),
                                             dout.contiguous().float().data_ptr(), saved.data_ptr(), saved_bytes,
                                             work.data_ptr(), ws_bytes, VP(*[g.data_ptr() for g in dW]),
                                             VP(*[g.data_ptr() for g in db]), dx.data_ptr() if need_dx else None,
                                             primal.data_ptr() if primal is not None else None,
                                             primal.numel() if primal is not None else 0, _native.stream_handle(dev))
    _native.check(rc, "siren_jvp_backward_ex")
    return dx, dW, db


def _sine_mlp_jvp_bwd_fake(dout, x, weights, biases, saved, w0, prec, batched, order, need_dx, primal=None):
    return (torch.empty_like(x) if need_dx else x.new_empty((0,)),
            [torch.empty_like(w) for w in weights], [torch.empty_like(b) for b in biases])


class _SineMLPJVPAutograd(torch.autograd.Function):
    """Autograd formula of sine_mlp_jvp: its backward is sine_mlp_jvp_bwd (lists passed flattened)."""

    @staticmethod
    def forward(ctx, meta, x, primal, *params):
        w0, prec, batched, order, n, keep = meta
        with torch._C._AutoDispatchBelowAutograd():
            out, saved = torch.ops.siren_mri_amd.sine_mlp_jvp(x, list(params[:n]), list(params[n:]), w0, prec,
                                                              batched, order, keep, primal)
        ctx.meta = meta
        # the primal buffer is read again by the backward: kept alive here
        ctx.primal = primal
        ctx.save_for_backward(x, saved, *params)
        ctx.mark_non_differentiable(saved)
        ctx.set_materialize_grads(False)
        return out, saved

    @staticmethod
    def backward(ctx, dout, _dsaved):
        w0, prec, batched, order, n, keep = ctx.meta
        if dout is None:
            return (None,) * (3 + 2 * n)
        if not keep:
            raise RuntimeError("siren_mri_amd: the tangent-stream forward ran without keeping its streams "
                               "(grad mode was off); it cannot be differentiated")
        t = ctx.saved_tensors
        x, saved, ws, bs = t[0], t[1], list(t[2:2 + n]), list(t[2 + n:])
        need_dx = ctx.needs_input_grad[1]
        with torch.no_grad():
            dx, dW, db = torch.ops.siren_mri_amd.sine_mlp_jvp_bwd(dout, x, ws, bs, saved, w0, prec, batched, order,
                                                                  need_dx, ctx.primal)
        db = list(db)
        # the output bias does not reach dy/dx or the Laplacian: autograd leaves its .grad None in the reference
        db[-1] = None
        outs = [dx if need_dx else None, *dW, *db]
        if torch.is_grad_enabled():
            # create_graph=True over a derivative op: one more order is not provided; the gradients
            # are exact, differentiating them again raises (instead of silently giving zeros)
            outs = guard_higher_order(outs, [x, *ws, *bs],
                                      "siren_mri_amd: derivatives of the tangent-stream backward (a third "
                                      "derivative of the SIREN) are not provided")
        return (None, outs[0], None, *outs[1:])


def _sine_mlp_jvp_autograd(x, weights, biases, w0, prec, batched, order, keep, primal=None):
    return _SineMLPJVPAutograd.apply((w0, prec, batched, order, len(weights), keep), x, primal, *weights, *biases)


_LIB.impl("sine_mlp_jvp", sine_mlp_jvp, "CUDA")
_LIB.impl("sine_mlp_jvp_bwd", sine_mlp_jvp_bwd, "CUDA")
_LIB.impl("sine_mlp_jvp", _sine_mlp_jvp_autograd, "Autograd")
torch.library.register_fake("siren_mri_amd::sine_mlp_jvp", _sine_mlp_jvp_fake, lib=_LIB)
torch.library.register_fake("siren_mri_amd::sine_mlp_jvp_bwd", _sine_mlp_jvp_bwd_fake, lib=_LIB)


def _apply(x, fcblock, params, order, primal=None):
    from .meta import get_subdict
    ws, bs = fcblock.layer_params(get_subdict(params, "net") if params is not None else None)
    prec = _native.precision_code(fcblock.precision or get_default_precision())
    _require_device(x)
    geo = _Geometry(x, ws)
    if geo.squeeze_w:
        ws, bs = [w[0] for w in ws], [b[0] for b in bs]
    keep = torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in list(ws) + list(bs)))
    if primal is not None and (prec != _native.PREC_F32 or not fcblock.outermost_linear):
        primal = None
    out, _ = torch.ops.siren_mri_amd.sine_mlp_jvp(x, list(ws), list(bs), float(fcblock.w0), prec, geo.batched,
                                                  order, keep, primal)
    return out


def siren_gradient(x, fcblock, params=None, primal=None):
    return _apply(x, fcblock, params, GRADIENT, primal)


def siren_laplace(x, fcblock, params=None, primal=None):
    return _apply(x, fcblock, params, LAPLACE, primal)


def siren_jacobian(x, fcblock, params=None, primal=None):
    """dy_c/dx_k per output channel, [..., out_features, in_features] (diff_operators.jacobian)."""
    return _apply(x, fcblock, params, JACOBIAN, primal)


def jacobian_of(x, weights, biases, w0, prec, batched):
    """The per-channel Jacobian of the SIREN stack with these (autograd-tracked) tensors, on the
    tangent-stream op: differentiable w.r.t. the weights, the biases and x."""
    keep = torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in list(weights) + list(biases)))
    out, _ = torch.ops.siren_mri_amd.sine_mlp_jvp(x, list(weights), list(biases), float(w0), prec, batched,
                                                  JACOBIAN, keep)
    return out


class _HigherOrderGuard(torch.autograd.Function):
    """Passes tensors through; differentiating them raises `msg`. The anchors (the op's inputs)
    make the outputs part of the graph whenever those inputs are, so a derivative that is not
    provided is an error, never a silent zero."""

    @staticmethod
    def forward(ctx, msg, n, *args):
        ctx.msg = msg
        return tuple(t.view_as(t) for t in args[:n])

    @staticmethod
    def backward(ctx, *grads):
        raise RuntimeError(ctx.msg)


def guard_higher_order(outs, anchors, msg):
    idx = [i for i, t in enumerate(outs) if t is not None]
    if not idx or not any(a.requires_grad for a in anchors):
        return outs
    res = _HigherOrderGuard.apply(msg, len(idx), *[outs[i] for i in idx], *anchors)
    outs = list(outs)
    for i, t in zip(idx, res):
        outs[i] = t
    return outs
