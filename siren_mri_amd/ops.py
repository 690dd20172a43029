"""The native SIREN layer stack as PyTorch custom ops (torch.library, namespace siren_mri_amd).

``siren_mlp(x, weights, biases, w0=..., precision=..., outermost_linear=...)`` is the fused
replacement of ``FCBlock.forward`` with nonlinearity='sine' (modules.py:92-97): the whole
[BatchLinear -> Sine] x L stack (modules.py:16-27, 35-38) runs as one native forward call and
one native backward call. Weights may be shared ([out, in]) or batched per sample
([B, out, in], the hypernetwork case of meta_modules.py:42-54, 198-225).

Custom ops (SURVEY.md §8(b) 'Custom-op layer'), each a thin wrapper of the C ABI in
include/siren_mri_amd.h, registered with the dispatcher together with fake (meta) kernels, so
FakeTensor tracing / torch.compile see shapes without running anything:
  siren_mri_amd::sine_mlp_fwd(x, W[], b[], w0, prec, outermost_linear, batched, keep)
        -> (y, saved)                         siren_mlp_forward
  siren_mri_amd::sine_mlp_bwd(dy, x, W[], b[], saved, w0, prec, outermost_linear, batched, need_dx)
        -> (dx, dW[], db[])                   siren_mlp_backward
`saved` is the uint8 buffer of prepared weights and stored phases the backward reads (never
writes), so a graph may be back-propagated more than once (retain_graph=True). The autograd
formula of sine_mlp_fwd (its Autograd dispatch key) is sine_mlp_bwd; under create_graph=True
(double backward through an autograd graph) the input gradient is formed instead from the
per-channel Jacobian of the tangent-stream op (jvp.py), which is itself differentiable, and the
weight gradients are exact but raise if differentiated again.

float64 inputs and parameters (the reference's double_precision=True with the model cast by
.double(), training.py:56-58) take the fp64 stack (siren_mlp64_*, csrc/siren_f64.hip) through
  siren_mri_amd::sine_mlp64_fwd / sine_mlp64_bwd
whatever `precision` says (first-order gradients; no Fourier-feature input, no fused loss).

No CPU or eager-PyTorch fallback exists: a CPU tensor, a mixed-dtype call or an unsupported
shape raises.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import torch
from torch import Tensor

from . import _native, fusion

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

    def __init__(self, x: torch.Tensor, weights: Sequence[torch.Tensor], in_features: int | None = None):
        # in_features: layer 0's inputs when x holds something else per row (the raw coordinates
        # of a Fourier-feature input, siren_mlp_desc.ff_B)
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
        dims = [int(in_features or x.shape[-1])] + [int(w.shape[-2]) for w in weights]
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


def _sizes(geo: _Geometry, prec: int, outermost_linear: bool, ff_in: int = 0):
    """(saved, workspace) bytes of a geometry after siren_mlp_check. They depend only on the
    geometry and options (not on the pointers), so they are asked once per geometry, with a
    pointer-free descriptor (also what the fake kernels use)."""
    key = (tuple(geo.dims), geo.batch, geo.rows, geo.batched, prec, outermost_linear, ff_in,
           _native.options_epoch())
    hit = _SIZES.get(key)
    if hit is None:
        L = _native.lib()
        desc = _native.describe_only(geo.dims, prec=prec, outermost_linear=outermost_linear,
                                     weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows,
                                     ff_in=ff_in)
        _native.check(L.siren_mlp_check(ctypes.byref(desc)), "siren_mlp_check")
        hit = (L.siren_mlp_saved_bytes(ctypes.byref(desc)), L.siren_mlp_workspace_bytes(ctypes.byref(desc)))
        if len(_SIZES) > 256:
            _SIZES.clear()
        _SIZES[key] = hit
    return hit


def _geo_of(x, weights, batched, ff_B=None):
    geo = _Geometry(x, weights, 2 * int(ff_B.shape[1]) if ff_B is not None else None)
    if geo.batched != batched:
        raise RuntimeError("siren_mri_amd: weight batching does not match the op's `batched` flag")
    return geo


# --------------------------------------------------------------------------- custom ops
# Registered with the low-level torch.library.Library API (schema + CUDA kernel + fake kernel +
# an Autograd-key formula): the dispatcher round trip costs ~15 us per call on the host, against
# ~100 us for the torch.library.custom_op wrapper, which would make small fits host-bound.
_LIB = torch.library.Library("siren_mri_amd", "DEF")
_LIB.define("sine_mlp_fwd(Tensor x, Tensor[] weights, Tensor[] biases, float w0, int prec, bool outermost_linear, "
            "bool batched, bool keep) -> (Tensor, Tensor)")
_LIB.define("sine_mlp_bwd(Tensor dy, Tensor x, Tensor[] weights, Tensor[] biases, Tensor saved, float w0, int prec, "
            "bool outermost_linear, bool batched, bool need_dx, Tensor? dy_scale=None, Tensor? ff_B=None) "
            "-> (Tensor, Tensor[], Tensor[])")
_LIB.define("sine_mlp_fwd_loss(Tensor x, Tensor[] weights, Tensor[] biases, float w0, int prec, bool batched, "
            "Tensor tgt, Tensor? k0, Tensor? mask, Tensor? hf, float noise, float weight, Tensor? ff_B=None) "
            "-> (Tensor, Tensor, Tensor, Tensor, Tensor)")


def sine_mlp_fwd(x: Tensor, weights: List[Tensor], biases: List[Tensor], w0: float, prec: int,
                 outermost_linear: bool, batched: bool, keep: bool) -> Tuple[Tensor, Tensor]:
    """siren_mlp_forward: y = the SIREN stack on x; saved = the backward's buffer (empty unless keep)."""
    _require_device(x)
    geo = _geo_of(x, weights, batched)
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    desc = _native.make_desc(geo.dims, ws, bs, w0=w0, prec=prec, outermost_linear=outermost_linear,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows)
    saved_bytes, ws_bytes = _sizes(geo, prec, outermost_linear)
    saved = torch.empty(saved_bytes if keep else 0, dtype=torch.uint8, device=dev)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    y = torch.empty(geo.lead_shape + (geo.dims[-1],), dtype=torch.float32, device=dev)
    rc = _native.lib().siren_mlp_forward(ctypes.byref(desc), xc.data_ptr(), y.data_ptr(),
                                         saved.data_ptr() if keep else None, saved_bytes if keep else 0,
                                         work.data_ptr(), ws_bytes, _native.stream_handle(dev))
    _native.check(rc, "siren_mlp_forward")
    return y, saved


def _sine_mlp_fwd_fake(x, weights, biases, w0, prec, outermost_linear, batched, keep):
    geo = _geo_of(x, weights, batched)
    saved_bytes, _ = _sizes(geo, prec, outermost_linear)
    return (x.new_empty(geo.lead_shape + (geo.dims[-1],), dtype=torch.float32),
            x.new_empty((saved_bytes if keep else 0,), dtype=torch.uint8))


def sine_mlp_bwd(dy: Tensor, x: Tensor, weights: List[Tensor], biases: List[Tensor], saved: Tensor, w0: float,
                 prec: int, outermost_linear: bool, batched: bool,
                 need_dx: bool, dy_scale: Tensor | None = None,
                 ff_B: Tensor | None = None) -> Tuple[Tensor, List[Tensor], List[Tensor]]:
    """siren_mlp_backward_ex: (dx or an empty tensor, dW per layer, db per layer); dL/dy = dy times
    the device scalar dy_scale when given (a fused loss's upstream gradient). ff_B: x holds the raw
    coordinates of a Fourier-feature input (no input gradient)."""
    if saved.numel() == 0:
        raise RuntimeError("siren_mri_amd: sine_mlp_bwd needs the saved buffer of a forward run with keep=True")
    if ff_B is not None and need_dx:
        raise RuntimeError("siren_mri_amd: no input gradient through a fused Fourier-feature input")
    geo = _geo_of(x, weights, batched, ff_B)
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    dyc = dy.contiguous().to(torch.float32)
    desc = _native.make_desc(geo.dims, ws, bs, w0=w0, prec=prec, outermost_linear=outermost_linear,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows, ff_B=ff_B)
    saved_bytes, ws_bytes = _sizes(geo, prec, outermost_linear, int(ff_B.shape[0]) if ff_B is not None else 0)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    dW = [torch.empty_like(w) for w in ws]
    db = [torch.empty_like(b) for b in bs]
    dx = torch.empty_like(xc) if need_dx else xc.new_empty((0,))
    n = len(ws)
    VP = ctypes.c_void_p * n
    sc = None
    if dy_scale is not None:
        sc = dy_scale.detach().reshape(()).to(device=dev, dtype=torch.float32).contiguous()
    rc = _native.lib().siren_mlp_backward_ex(ctypes.byref(desc), xc.data_ptr(), dyc.data_ptr(),
                                             sc.data_ptr() if sc is not None else None, saved.data_ptr(),
                                             saved_bytes, work.data_ptr(), ws_bytes,
                                             VP(*[t.data_ptr() for t in dW]), VP(*[t.data_ptr() for t in db]),
                                             dx.data_ptr() if need_dx else None, _native.stream_handle(dev))
    _native.check(rc, "siren_mlp_backward_ex")
    return dx, dW, db


def _sine_mlp_bwd_fake(dy, x, weights, biases, saved, w0, prec, outermost_linear, batched, need_dx, dy_scale=None,
                       ff_B=None):
    return (torch.empty_like(x) if need_dx else x.new_empty((0,)),
            [torch.empty_like(w) for w in weights], [torch.empty_like(b) for b in biases])


class _SineMLPAutograd(torch.autograd.Function):
    """Autograd formula of sine_mlp_fwd (the Autograd dispatch key): its backward is sine_mlp_bwd.
    The weight and bias lists are passed flattened so autograd tracks every tensor."""

    @staticmethod
    def forward(ctx, meta, x, *params):
        w0, prec, outermost_linear, batched, n, keep = meta
        weights, biases = list(params[:n]), list(params[n:])
        with torch._C._AutoDispatchBelowAutograd():
            y, saved = torch.ops.siren_mri_amd.sine_mlp_fwd(x, weights, biases, w0, prec, outermost_linear,
                                                            batched, keep)
        ctx.meta = meta
        ctx.save_for_backward(x, saved, *params)
        ctx.mark_non_differentiable(saved)
        # no zero-filled gradient for the uint8 saved buffer (a full-size fill kernel per step)
        ctx.set_materialize_grads(False)
        return y, saved

    @staticmethod
    def backward(ctx, dy, _dsaved):
        w0, prec, outermost_linear, batched, n, keep = ctx.meta
        if dy is None:
            return (None,) * (2 + 2 * n)
        if not keep:
            raise RuntimeError("siren_mri_amd: the SIREN forward ran without keeping activations "
                               "(grad mode was off); it cannot be differentiated")
        t = ctx.saved_tensors
        x, saved, ws, bs = t[0], t[1], list(t[2:2 + n]), list(t[2 + n:])
        need_dx = ctx.needs_input_grad[1]
        if torch.is_grad_enabled():
            return (None, *_differentiable_backward(ctx, dy, x, saved, ws, bs, need_dx))
        dx, dW, db = torch.ops.siren_mri_amd.sine_mlp_bwd(dy, x, ws, bs, saved, w0, prec, outermost_linear,
                                                          batched, need_dx)
        return (None, dx if need_dx else None, *dW, *db)


def _differentiable_backward(ctx, dy, x, saved, ws, bs, need_dx):
    """The SIREN backward under create_graph=True (diff_operators.gradient through autograd,
    diff_operators.py:39-43, for any y derived from the SIREN output and any grad_outputs): the input
    gradient as dx_k = sum_c dy_c J[c, k] with J the per-channel Jacobian of the tangent-stream op,
    which is differentiable w.r.t. dy, the weights, the biases and x (its backward is the native
    adjoint). The weight gradients are exact but not differentiable again (differentiating them
    raises)."""
    from .jvp import guard_higher_order, jacobian_of
    w0, prec, outermost_linear, batched, n, keep = ctx.meta
    dx = None
    need_w = any(ctx.needs_input_grad[2:])
    dW, db = [None] * n, [None] * n
    if need_dx:
        if not outermost_linear or x.shape[-1] > 4:
            # no tangent-stream form for this stack: the native first-order input gradient, which
            # raises only if it is differentiated again; the same launch's dW / db are
            # kept when the weights need gradients (one native backward, not two)
            with torch.no_grad():
                dx, dW, db = torch.ops.siren_mri_amd.sine_mlp_bwd(dy, x, ws, bs, saved, w0, prec, outermost_linear,
                                                                  batched, True)
            dW, db = list(dW), list(db)
            dx = guard_higher_order([dx], [dy, x, *ws, *bs],
                                    "siren_mri_amd: a differentiable SIREN input gradient (create_graph=True) "
                                    "needs outermost_linear=True and in_features <= 4 (the tangent-stream "
                                    "kernels)")[0]
        else:
            J = jacobian_of(x, ws, bs, w0, prec, batched)
            dx = (J * dy.unsqueeze(-1)).sum(-2)
    if need_w:
        if dW[0] is None:
            with torch.no_grad():
                _, dW, db = torch.ops.siren_mri_amd.sine_mlp_bwd(dy, x, ws, bs, saved, w0, prec, outermost_linear,
                                                                 batched, False)
        wb = guard_higher_order([*dW, *db], [dy, x, *ws, *bs],
                                "siren_mri_amd: second derivatives of the SIREN's weight gradients are not "
                                "provided (derivatives of its input gradient are)")
        dW, db = wb[:n], wb[n:]
    return (dx, *dW, *db)


def _sine_mlp_fwd_autograd(x, weights, biases, w0, prec, outermost_linear, batched, keep):
    meta = (w0, prec, outermost_linear, batched, len(weights), keep)
    return _SineMLPAutograd.apply(meta, x, *weights, *biases)


_LIB.impl("sine_mlp_fwd", sine_mlp_fwd, "CUDA")
_LIB.impl("sine_mlp_bwd", sine_mlp_bwd, "CUDA")
_LIB.impl("sine_mlp_fwd", _sine_mlp_fwd_autograd, "Autograd")
torch.library.register_fake("siren_mri_amd::sine_mlp_fwd", _sine_mlp_fwd_fake, lib=_LIB)
torch.library.register_fake("siren_mri_amd::sine_mlp_bwd", _sine_mlp_bwd_fake, lib=_LIB)


# ---------------------------------------------------------------- fp64 stack (double_precision=True)
_LIB.define("sine_mlp64_fwd(Tensor x, Tensor[] weights, Tensor[] biases, float w0, bool outermost_linear, "
            "bool batched, bool keep) -> (Tensor, Tensor)")
_LIB.define("sine_mlp64_bwd(Tensor dy, Tensor x, Tensor[] weights, Tensor[] biases, Tensor saved, float w0, "
            "bool outermost_linear, bool batched, bool need_dx) -> (Tensor, Tensor[], Tensor[])")

_SIZES64 = {}


def _sizes64(geo: _Geometry, outermost_linear: bool):
    key = (tuple(geo.dims), geo.batch, geo.rows, geo.batched, outermost_linear)
    hit = _SIZES64.get(key)
    if hit is None:
        L = _native.lib()
        desc = _native.describe_only(geo.dims, prec=_native.PREC_F64, outermost_linear=outermost_linear,
                                     weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows)
        saved = L.siren_mlp64_saved_bytes(ctypes.byref(desc))
        if saved < 0:
            _native.check(-1, "siren_mlp64_saved_bytes")
        hit = (saved, L.siren_mlp64_workspace_bytes(ctypes.byref(desc)))
        if len(_SIZES64) > 256:
            _SIZES64.clear()
        _SIZES64[key] = hit
    return hit


def _require_f64(x, weights, biases):
    if x.device.type != "cuda":
        raise RuntimeError("siren_mri_amd: the SIREN layer stack runs only on an MI355X (HIP) device; got a "
                           f"{x.device.type} tensor. There is no CPU fallback by design.")
    for t in list(weights) + list(biases):
        if t.dtype != torch.float64 or t.device != x.device:
            raise RuntimeError("siren_mri_amd: a float64 input needs float64 weights and biases on its device "
                               f"(model.double(), as the reference's double_precision=True); got {t.dtype}")


def sine_mlp64_fwd(x: Tensor, weights: List[Tensor], biases: List[Tensor], w0: float, outermost_linear: bool,
                   batched: bool, keep: bool) -> Tuple[Tensor, Tensor]:
    """siren_mlp64_forward: y (float64); saved = the pre-activations of the sine layers (empty unless keep)."""
    _require_f64(x, weights, biases)
    geo = _geo_of(x, weights, batched)
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    desc = _native.make_desc(geo.dims, ws, bs, w0=w0, prec=_native.PREC_F64, outermost_linear=outermost_linear,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows)
    saved_bytes, ws_bytes = _sizes64(geo, outermost_linear)
    saved = torch.empty(saved_bytes if keep else 0, dtype=torch.uint8, device=dev)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    y = torch.empty(geo.lead_shape + (geo.dims[-1],), dtype=torch.float64, device=dev)
    rc = _native.lib().siren_mlp64_forward(ctypes.byref(desc), xc.data_ptr(), y.data_ptr(),
                                           saved.data_ptr() if keep else None, saved_bytes if keep else 0,
                                           work.data_ptr(), ws_bytes, _native.stream_handle(dev))
    _native.check(rc, "siren_mlp64_forward")
    return y, saved


def _sine_mlp64_fwd_fake(x, weights, biases, w0, outermost_linear, batched, keep):
    geo = _geo_of(x, weights, batched)
    saved_bytes, _ = _sizes64(geo, outermost_linear)
    return (x.new_empty(geo.lead_shape + (geo.dims[-1],), dtype=torch.float64),
            x.new_empty((saved_bytes if keep else 0,), dtype=torch.uint8))


def sine_mlp64_bwd(dy: Tensor, x: Tensor, weights: List[Tensor], biases: List[Tensor], saved: Tensor, w0: float,
                   outermost_linear: bool, batched: bool, need_dx: bool) -> Tuple[Tensor, List[Tensor], List[Tensor]]:
    """siren_mlp64_backward: (dx or an empty tensor, dW per layer, db per layer), all float64."""
    if saved.numel() == 0:
        raise RuntimeError("siren_mri_amd: sine_mlp64_bwd needs the saved buffer of a forward run with keep=True")
    geo = _geo_of(x, weights, batched)
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    dyc = dy.contiguous().to(torch.float64)
    desc = _native.make_desc(geo.dims, ws, bs, w0=w0, prec=_native.PREC_F64, outermost_linear=outermost_linear,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows)
    saved_bytes, ws_bytes = _sizes64(geo, outermost_linear)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    dW = [torch.empty_like(w) for w in ws]
    db = [torch.empty_like(b) for b in bs]
    dx = torch.empty_like(xc) if need_dx else xc.new_empty((0,))
    n = len(ws)
    VP = ctypes.c_void_p * n
    rc = _native.lib().siren_mlp64_backward(ctypes.byref(desc), xc.data_ptr(), dyc.data_ptr(), saved.data_ptr(),
                                            saved_bytes, work.data_ptr(), ws_bytes,
                                            VP(*[t.data_ptr() for t in dW]), VP(*[t.data_ptr() for t in db]),
                                            dx.data_ptr() if need_dx else None, _native.stream_handle(dev))
    _native.check(rc, "siren_mlp64_backward")
    return dx, dW, db


def _sine_mlp64_bwd_fake(dy, x, weights, biases, saved, w0, outermost_linear, batched, need_dx):
    return (torch.empty_like(x) if need_dx else x.new_empty((0,)),
            [torch.empty_like(w) for w in weights], [torch.empty_like(b) for b in biases])


class _SineMLP64Autograd(torch.autograd.Function):
    """Autograd formula of sine_mlp64_fwd: its backward is sine_mlp64_bwd (first order)."""

    @staticmethod
    def forward(ctx, meta, x, *params):
        w0, outermost_linear, batched, n, keep = meta
        with torch._C._AutoDispatchBelowAutograd():
            y, saved = torch.ops.siren_mri_amd.sine_mlp64_fwd(x, list(params[:n]), list(params[n:]), w0,
                                                              outermost_linear, batched, keep)
        ctx.meta = meta
        ctx.save_for_backward(x, saved, *params)
        ctx.mark_non_differentiable(saved)
        ctx.set_materialize_grads(False)
        return y, saved

    @staticmethod
    def backward(ctx, dy, _dsaved):
        w0, outermost_linear, batched, n, keep = ctx.meta
        if dy is None:
            return (None,) * (2 + 2 * n)
        if not keep:
            raise RuntimeError("siren_mri_amd: the SIREN forward ran without keeping activations "
                               "(grad mode was off); it cannot be differentiated")
        if torch.is_grad_enabled():
            raise RuntimeError("siren_mri_amd: second derivatives of the fp64 SIREN stack are not provided "
                               "(create_graph=True); the fp32 / bf16 stacks provide them")
        t = ctx.saved_tensors
        x, saved, ws, bs = t[0], t[1], list(t[2:2 + n]), list(t[2 + n:])
        need_dx = ctx.needs_input_grad[1]
        dx, dW, db = torch.ops.siren_mri_amd.sine_mlp64_bwd(dy, x, ws, bs, saved, w0, outermost_linear, batched,
                                                            need_dx)
        return (None, dx if need_dx else None, *dW, *db)


def _sine_mlp64_fwd_autograd(x, weights, biases, w0, outermost_linear, batched, keep):
    meta = (w0, outermost_linear, batched, len(weights), keep)
    return _SineMLP64Autograd.apply(meta, x, *weights, *biases)


_LIB.impl("sine_mlp64_fwd", sine_mlp64_fwd, "CUDA")
_LIB.impl("sine_mlp64_bwd", sine_mlp64_bwd, "CUDA")
_LIB.impl("sine_mlp64_fwd", _sine_mlp64_fwd_autograd, "Autograd")
torch.library.register_fake("siren_mri_amd::sine_mlp64_fwd", _sine_mlp64_fwd_fake, lib=_LIB)
torch.library.register_fake("siren_mri_amd::sine_mlp64_bwd", _sine_mlp64_bwd_fake, lib=_LIB)


def _siren_mlp64(x, weights, biases, w0, outermost_linear, return_saved, ff_B):
    if ff_B is not None:
        raise RuntimeError("siren_mri_amd: no Fourier-feature input in the fp64 stack (the reference's "
                           "double_precision=True cannot combine them either: its B is float32)")
    _require_f64(x, weights, biases)
    geo = _Geometry(x, weights)
    ws, bs = list(weights), list(biases)
    if geo.squeeze_w:
        ws, bs = [w[0] for w in ws], [b[0] for b in bs]
    keep = torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in ws + bs))
    y, saved = torch.ops.siren_mri_amd.sine_mlp64_fwd(x, ws, bs, float(w0), bool(outermost_linear), geo.batched, keep)
    return (y, saved) if return_saved else y


# ---------------------------------------------------------------- forward with the fused image loss
def _loss_desc(tgt, k0, mask, hf, noise, weight, y_dc, dy, loss, lws):
    ld = _native.SirenLossDesc()
    ld.target = tgt.data_ptr()
    ld.k0 = k0.data_ptr() if k0 is not None else None
    ld.mask = mask.data_ptr() if mask is not None else None
    ld.hf = hf.data_ptr() if hf is not None else None
    ld.hf_len = hf.numel() if hf is not None else 0
    ld.noise = float(noise)
    ld.weight = float(weight)
    ld.y_dc = y_dc.data_ptr() if (k0 is not None and y_dc is not None) else None
    ld.dy = dy.data_ptr()
    ld.loss = loss.data_ptr()
    ld.loss_workspace = lws.data_ptr()
    ld.loss_workspace_bytes = lws.numel()
    return ld


_LOSS_OK = {}


def fused_loss_supported(geo: _Geometry, prec: int, has_dc: bool, hf_len: int, ff_in: int = 0) -> bool:
    """siren_mlp_loss_check for a geometry (cached; pointer-free descriptors)."""
    key = (tuple(geo.dims), geo.batch, geo.rows, geo.batched, prec, has_dc, hf_len, ff_in, _native.options_epoch())
    hit = _LOSS_OK.get(key)
    if hit is None:
        d = _native.describe_only(geo.dims, prec=prec, weights_batched=geo.batched, batch=geo.batch,
                                  rows_per_batch=geo.rows, ff_in=ff_in)
        ld = _native.SirenLossDesc()
        ld.target = ld.dy = ld.loss = ld.loss_workspace = 256
        if has_dc:
            ld.k0 = ld.mask = ld.y_dc = 256
        if hf_len:
            ld.hf, ld.hf_len = 256, hf_len
        ld.loss_workspace_bytes = int(_native.lib().siren_sse_workspace_bytes())
        hit = _native.lib().siren_mlp_loss_check(ctypes.byref(d), ctypes.byref(ld)) == 0
        if len(_LOSS_OK) > 256:
            _LOSS_OK.clear()
        _LOSS_OK[key] = hit
    return hit


def sine_mlp_fwd_loss(x: Tensor, weights: List[Tensor], biases: List[Tensor], w0: float, prec: int, batched: bool,
                      tgt: Tensor, k0: Tensor | None, mask: Tensor | None, hf: Tensor | None, noise: float,
                      weight: float, ff_B: Tensor | None = None):
    """siren_mlp_forward_loss: (y, DC(y) or an empty tensor, loss, dL/dy for a unit upstream
    gradient, saved). ff_B: x holds raw coordinates, layer 0's inputs are their Fourier features
    cat(sin(2 pi x B), cos(2 pi x B)) formed in the kernel (features.py:21-41)."""
    _require_device(x)
    geo = _geo_of(x, weights, batched, ff_B)
    ff_in = int(ff_B.shape[0]) if ff_B is not None else 0
    ws = [w.contiguous() for w in weights]
    bs = [b.contiguous() for b in biases]
    xc = x.contiguous()
    dev = x.device
    desc = _native.make_desc(geo.dims, ws, bs, w0=w0, prec=prec, outermost_linear=True,
                             weights_batched=geo.batched, batch=geo.batch, rows_per_batch=geo.rows, ff_B=ff_B)
    saved_bytes, ws_bytes = _sizes(geo, prec, True, ff_in)
    saved = torch.empty(saved_bytes, dtype=torch.uint8, device=dev)
    work = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    shape = geo.lead_shape + (geo.dims[-1],)
    y = torch.empty(shape, dtype=torch.float32, device=dev)
    y_dc = torch.empty(shape, dtype=torch.float32, device=dev) if k0 is not None else y.new_empty((0,))
    dy = torch.empty(shape, dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    tc = tgt.contiguous()
    kc = k0.contiguous() if k0 is not None else None
    mc = mask.contiguous() if mask is not None else None
    hc = hf.contiguous() if hf is not None else None
    ld = _loss_desc(tc, kc, mc, hc, noise, weight, y_dc, dy, loss, _native.sse_workspace(dev))
    rc = _native.lib().siren_mlp_forward_loss(ctypes.byref(desc), ctypes.byref(ld), xc.data_ptr(), y.data_ptr(),
                                              saved.data_ptr(), saved_bytes, work.data_ptr(), ws_bytes,
                                              _native.stream_handle(dev))
    _native.check(rc, "siren_mlp_forward_loss")
    return y, y_dc, loss, dy, saved


def _sine_mlp_fwd_loss_fake(x, weights, biases, w0, prec, batched, tgt, k0, mask, hf, noise, weight, ff_B=None):
    geo = _geo_of(x, weights, batched, ff_B)
    saved_bytes, _ = _sizes(geo, prec, True, int(ff_B.shape[0]) if ff_B is not None else 0)
    shape = geo.lead_shape + (geo.dims[-1],)
    y = x.new_empty(shape, dtype=torch.float32)
    return (y, x.new_empty(shape if k0 is not None else (0,), dtype=torch.float32), x.new_empty((), dtype=torch.float32),
            x.new_empty(shape, dtype=torch.float32), x.new_empty((saved_bytes,), dtype=torch.uint8))


class _SineMLPLossAutograd(torch.autograd.Function):
    """One autograd node for the forward with the fused image loss: outputs (y, DC(y), loss). Its
    backward forms dL/dy = dL/dloss * dy_unit (+ the gradients arriving at y and DC(y), if any) and
    runs the native backward; with only the loss's gradient, dL/dloss goes to the output-layer
    kernels as a device scalar (no dL/dy tensor, no extra launch)."""

    @staticmethod
    def forward(ctx, meta, x, tgt, k0, mask, hf, ff_B, *params):
        w0, prec, batched, n, noise, weight = meta
        with torch._C._AutoDispatchBelowAutograd():
            y, y_dc, loss, dyu, saved = torch.ops.siren_mri_amd.sine_mlp_fwd_loss(
                x, list(params[:n]), list(params[n:]), w0, prec, batched, tgt, k0, mask, hf, noise, weight, ff_B)
        ctx.meta = meta
        ctx.has_dc = k0 is not None
        ctx.ff_B = ff_B
        ctx.save_for_backward(x, saved, dyu, mask, *params)
        ctx.set_materialize_grads(False)
        return y, y_dc, loss

    @staticmethod
    def backward(ctx, gy, gdc, gloss):
        w0, prec, batched, n, noise, weight = ctx.meta
        t = ctx.saved_tensors
        x, saved, dyu, mask, ws, bs = t[0], t[1], t[2], t[3], list(t[4:4 + n]), list(t[4 + n:])
        if torch.is_grad_enabled():
            raise RuntimeError("siren_mri_amd: double backward through a fused SIREN loss is not provided; "
                               "run it unfused (siren_mri_amd.fusion.set_enabled(False))")
        parts = []
        if gy is not None:
            parts.append(gy)
        if gdc is not None and ctx.has_dc:
            parts.append(torch.ops.siren_mri_amd.dc_backward(gdc, mask, noise))
        scale = None
        if gloss is not None and not parts:
            dy, scale = dyu, gloss
        elif parts:
            dy = parts[0] if len(parts) == 1 else sum(parts)
            if gloss is not None:
                dy = dy + dyu * gloss
        else:
            return (None,) * (7 + 2 * n)
        need_dx = ctx.needs_input_grad[1]
        dx, dW, db = torch.ops.siren_mri_amd.sine_mlp_bwd(dy, x, ws, bs, saved, w0, prec, True, batched, need_dx,
                                                          scale, ctx.ff_B)
        return (None, dx if need_dx else None, None, None, None, None, None, *dW, *db)


def _fused_loss_forward(st, x, ws, bs, w0, prec, geo, ff_B=None):
    """The staged image loss (fusion.py) on this SIREN forward, or None when it does not apply.
    ff_B: x holds raw coordinates of a Fourier-feature input (formed in the kernel)."""
    from . import loss_functions
    O = geo.dims[-1]
    shape = geo.lead_shape + (O,)
    tgt = st.tgt
    if tuple(tgt.shape) != tuple(shape) or tgt.device != x.device:
        return None
    side = int(round(geo.rows ** 0.5))
    hf = loss_functions.high_freq_flat(x.device) if (st.high_freq and side * side == geo.rows and side == 128) else None
    k0 = mask = None
    noise = 0.0
    if st.dc is not None:
        k0, mask, noise = st.dc
        if not (isinstance(k0, Tensor) and isinstance(mask, Tensor) and k0.is_cuda and k0.dtype == torch.float32
                and mask.dtype == torch.float32 and k0.dim() == 4 and k0.shape == mask.shape
                and k0.shape[0] == geo.batch and k0.shape[1] == O and k0[0, 0].numel() == geo.rows
                and not k0.requires_grad and not mask.requires_grad):
            k0 = mask = None
    if not fused_loss_supported(geo, prec, k0 is not None, hf.numel() if hf is not None else 0,
                                int(ff_B.shape[0]) if ff_B is not None else 0):
        return None
    meta = (float(w0), prec, geo.batched, len(ws), float(noise), float(st.weight))
    y, y_dc, loss = _SineMLPLossAutograd.apply(meta, x, tgt, k0, mask, hf, ff_B, *ws, *bs)
    st.result = (y, y_dc if k0 is not None else None, loss, hf is not None, (k0, mask, noise) if k0 is not None else None)
    return y


_LIB.impl("sine_mlp_fwd_loss", sine_mlp_fwd_loss, "CUDA")
torch.library.register_fake("siren_mri_amd::sine_mlp_fwd_loss", _sine_mlp_fwd_loss_fake, lib=_LIB)


def _fourier_input_forward(x, weights, biases, w0, prec, outermost_linear, return_saved, ff_B):
    """siren_mlp with a Fourier-feature input formed in the kernel, or None
    when that path does not apply (then the caller materialises the features)."""
    from . import features
    st = fusion.pending(x.device)
    if (not features.FUSED_INPUT or st is None or prec != _native.PREC_BF16 or not outermost_linear or return_saved
            or x.requires_grad
            or not torch.is_grad_enabled() or not x.is_cuda or x.dtype != torch.float32
            or not ff_B.is_cuda or ff_B.dtype != torch.float32 or ff_B.dim() != 2
            or not 1 <= ff_B.shape[0] <= 4 or x.shape[-1] != ff_B.shape[0]
            or 2 * ff_B.shape[1] != weights[0].shape[-1]):
        return None
    geo = _Geometry(x, weights, 2 * int(ff_B.shape[1]))
    ws, bs = list(weights), list(biases)
    if geo.squeeze_w:
        ws, bs = [w[0] for w in ws], [b[0] for b in bs]
    if not any(t.requires_grad for t in ws + bs):
        return None
    return _fused_loss_forward(st, x, ws, bs, w0, prec, geo, ff_B.contiguous())


def siren_mlp(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor], *,
              w0: float = 30.0, precision: str | None = None, outermost_linear: bool = True,
              return_saved: bool = False, ff_B: torch.Tensor | None = None):
    """Fused SIREN stack: y = Linear_L(sin(w0 Linear_{L-1}(... sin(w0 Linear_0(x))))).
    return_saved=True also returns the op's saved buffer (diagnostics). ff_B: x holds raw
    coordinates and the stack's input is their Gaussian Fourier features (features.py:21-41):
    formed inside the forward's first layer with a staged image loss (bf16 wide form, no input
    gradient), else materialised by the fourier_features op first."""
    n = len(weights)
    if len(biases) != n:
        raise ValueError("siren_mlp: weights and biases differ in length")
    if x.device.type == "cpu":
        # a CPU tensor: the stack as plain PyTorch ops on the host (config 1 "on CPU", cpu_stack.py);
        # CUDA tensors never come here — they take the native kernels or raise
        if return_saved:
            raise RuntimeError("siren_mri_amd: return_saved needs the native (GPU) stack")
        from . import cpu_stack
        if ff_B is not None:
            from .features import fourier_features
            x = fourier_features(x, ff_B)
        return cpu_stack.sine_stack(x, weights, biases, float(w0), outermost_linear)
    if x.dtype == torch.float64:
        return _siren_mlp64(x, weights, biases, w0, outermost_linear, return_saved, ff_B)
    prec = _native.precision_code(precision or _DEFAULT_PRECISION)
    _require_device(x)
    if ff_B is not None:
        y = _fourier_input_forward(x, weights, biases, w0, prec, outermost_linear, return_saved, ff_B)
        if y is not None:
            return y
        from . import features  # noqa: F401  (registers the fourier_features op)
        x = torch.ops.siren_mri_amd.fourier_features(x, ff_B.to(x.device, x.dtype))
    geo = _Geometry(x, weights)
    ws, bs = list(weights), list(biases)
    if geo.squeeze_w:
        ws, bs = [w[0] for w in ws], [b[0] for b in bs]
    keep = torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in ws + bs))
    st = fusion.pending(x.device)
    if st is not None and keep and outermost_linear and not return_saved:
        # the staged image loss in the forward's output epilogue: the bf16 register forward, or the
        # per-layer path's output kernel (fp32 mode; siren_mlp_loss_check decides)
        y = _fused_loss_forward(st, x, ws, bs, w0, prec, geo)
        if y is not None:
            return y
    y, saved = torch.ops.siren_mri_amd.sine_mlp_fwd(x, ws, bs, float(w0), prec, bool(outermost_linear),
                                                    geo.batched, keep)
    if return_saved:
        return y, saved
    if keep and outermost_linear and prec == _native.PREC_F32:
        # diff_operators hands this to the tangent-stream op on (y, x): its primal stream is these phases
        y._siren_primal = saved
    return y
