"""Differential operators (drop-in for diff_operators.py of jonbmartin/siren_mri).

gradient(y, x)  diff_operators.py:39-43   sum_c dy_c/dx, differentiable (create_graph=True)
laplace(y, x)   diff_operators.py:27-29   sum_k d2y/dx_k2
divergence      diff_operators.py:32-36
jacobian        diff_operators.py:46-59
hessian         diff_operators.py:5-24

For y produced by a SIREN (SingleBVPNet / FCBlock with nonlinearity='sine') w.r.t. its own
`model_in`, gradient() and laplace() do not build an autograd graph: they call the native
forward-mode (tangent-stream) kernels, which carry dh/dx (and d2h/dx2) analytically through
every layer next to the primal activations, and whose backward is the hand-derived second-order
adjoint. Any other (y, x) pair goes through torch.autograd exactly as the reference does.
"""
from __future__ import annotations

import weakref

import torch
from torch.autograd import grad

# id(y) -> (weakref(y), weakref(x), fcblock, params). Entries die with y.
_SIREN_OUTPUTS: dict = {}


def register_siren_output(y: torch.Tensor, x: torch.Tensor, fcblock, params) -> None:
    """Called by SingleBVPNet.forward: remember that `y` is the SIREN output of leaf `x`."""
    key = id(y)

    def _drop(_ref, key=key):
        _SIREN_OUTPUTS.pop(key, None)

    _SIREN_OUTPUTS[key] = (weakref.ref(y, _drop), weakref.ref(x), fcblock, params)


def _lookup(y, x):
    ent = _SIREN_OUTPUTS.get(id(y))
    if ent is None:
        return None
    yref, xref, fcblock, params = ent
    if yref() is not y or xref() is not x:
        return None
    return fcblock, params


def siren_source(y, x):
    """(fcblock, params) if y is the registered SIREN output of x, else None."""
    return _lookup(y, x)


def _primal(y):
    """The saved buffer of the forward that produced y (ops.siren_mlp, fp32 mode), or None: the
    tangent-stream op then takes its primal phases from it instead of recomputing the forward."""
    return getattr(y, "_siren_primal", None)


_ANALYTIC = True


def set_analytic(enabled: bool) -> None:
    """Enable/disable the native tangent-stream path for SIREN outputs (for A/B tests)."""
    global _ANALYTIC
    _ANALYTIC = bool(enabled)


def gradient(y, x, grad_outputs=None):
    """sum_c g_c dy_c/dx (g = grad_outputs, ones by default), differentiable. For a SIREN output
    the analytic path: g = ones -> the summed tangent streams; one output channel -> g times that;
    any other g -> the per-channel Jacobian contracted with g (no host synchronisation in any
    case). Other (y, x) pairs go through autograd, whose SIREN backward is itself differentiable
    (ops._differentiable_backward)."""
    if _ANALYTIC:
        src = _lookup(y, x)
        if src is not None:
            from .jvp import siren_gradient, siren_jacobian
            if grad_outputs is None:
                return siren_gradient(x, *src, primal=_primal(y))
            g = grad_outputs
            if g.shape == y.shape:
                if y.shape[-1] == 1:
                    return siren_gradient(x, *src, primal=_primal(y)) * g
                return (siren_jacobian(x, *src, primal=_primal(y)) * g.unsqueeze(-1)).sum(-2)
    if grad_outputs is None:
        grad_outputs = torch.ones_like(y)
    return torch.autograd.grad(y, [x], grad_outputs=grad_outputs, create_graph=True)[0]


def divergence(y, x):
    div = 0.0
    for i in range(y.shape[-1]):
        div += grad(y[..., i], x, torch.ones_like(y[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


def laplace(y, x):
    if _ANALYTIC:
        src = _lookup(y, x)
        if src is not None:
            from .jvp import siren_laplace
            return siren_laplace(x, *src, primal=_primal(y))
    return divergence(gradient(y, x), x)


def jacobian(y, x):
    """Per-output-channel jacobian [B, N, C_out, C_in] and a NaN status flag (for a SIREN output:
    the tangent-stream op, one native forward)."""
    if _ANALYTIC and y.dim() == 3:
        src = _lookup(y, x)
        if src is not None:
            from .jvp import siren_jacobian
            jac = siren_jacobian(x, *src, primal=_primal(y))
            return jac, (-1 if torch.any(torch.isnan(jac)) else 0)
    b, n = y.shape[:2]
    jac = torch.zeros(b, n, y.shape[-1], x.shape[-1], device=y.device)
    for i in range(y.shape[-1]):
        y_flat = y[..., i].view(-1, 1)
        jac[:, :, i, :] = grad(y_flat, x, torch.ones_like(y_flat), create_graph=True)[0]
    status = -1 if torch.any(torch.isnan(jac)) else 0
    return jac, status


def hessian(y, x):
    """Hessian [B, N, C_out, C_in, C_in] and a NaN status flag."""
    b, n = y.shape[:2]
    grad_y = torch.ones_like(y[..., 0])
    h = torch.zeros(b, n, y.shape[-1], x.shape[-1], x.shape[-1], device=y.device)
    for i in range(y.shape[-1]):
        dydx = grad(y[..., i], x, grad_y, create_graph=True)[0]
        for j in range(x.shape[-1]):
            h[..., i, j, :] = grad(dydx[..., j], x, grad_y, create_graph=True)[0][..., :]
    status = -1 if torch.any(torch.isnan(h)) else 0
    return h, status
