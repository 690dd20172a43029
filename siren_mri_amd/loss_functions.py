"""Losses on the SIREN hot path (drop-in for loss_functions.py of jonbmartin/siren_mri).

  image_mse                loss_functions.py:66-101
  latent_loss              loss_functions.py:275-276
  hypo_weight_loss         loss_functions.py:279-287
  image_hypernetwork_loss  loss_functions.py:290-293
  function_mse             loss_functions.py:326-327
  gradients_mse            loss_functions.py:330-335
  laplace_mse              loss_functions.py:350-355

image_mse runs on the native k-space op (siren_kspace.hip), with the data consistency of a native
DataConsistencyInKspace output folded in.

Deliberate deviation (bug 0.2): the reference builds its high-frequency mask
on a fixed 128x128 grid, so image_mse(high_freq=True) raises for any other image size; here the
mask applies when the image is 128x128 and the loss is the plain SSE otherwise.
"""
from __future__ import annotations

import torch

from . import _native, diff_operators, fusion
from .data_consistency import dc_source
from .dataio import lin2img
from .utils import create_circular_mask_torch

_KSPACE_WEIGHT = 1.0 / (128 * 128)
KSPACE_WEIGHT = _KSPACE_WEIGHT  # image_mse's normalisation (loss_functions.py:101)
_MASKS: dict = {}


def _high_freq_mask(device):
    m = _MASKS.get(device)
    if m is None:
        # float32 (the reference's mask is int64; 1 - mask promotes the product with pred to float
        # either way), so the native weighted-SSE kernel takes it
        m = (1 - create_circular_mask_torch(129, 129, center=None, radius=20)).to(torch.float32)
        m = m.to(device)
        _MASKS[device] = m
    return m


def _sse_workspace(device):
    # one workspace per (device, stream): its block sums and ticket must not be shared by two
    # launches that may run concurrently
    return _native.sse_workspace(device)


class _WeightedSSE(torch.autograd.Function):
    """sum((m * (pred - tgt))^2) * w for real pred and a constant target on the native kernels
    (siren_sse_forward / siren_sse_backward, siren_loss.hip): forward = one launch (d = m (pred -
    tgt) and the deterministic weighted sum), backward = one launch, 2 w m^2 (pred - tgt) g — the
    values of the autograd chain of (diff.abs() ** 2).sum() * w in 2 launches instead of ~6."""

    @staticmethod
    def forward(ctx, pred, tgt, mask, weight):
        predc, tgtc = pred.contiguous(), tgt.contiguous()
        maskc = mask.contiguous() if mask is not None else None
        n = predc.numel()
        d = torch.empty_like(predc)
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        ws = _sse_workspace(pred.device)
        rc = _native.lib().siren_sse_forward(
            predc.data_ptr(), tgtc.data_ptr(), maskc.data_ptr() if maskc is not None else None, n,
            maskc.numel() if maskc is not None else 0, float(weight), d.data_ptr(), loss.data_ptr(),
            ws.data_ptr(), ws.numel(), _native.stream_handle(pred.device))
        _native.check(rc, "siren_sse_forward")
        ctx.save_for_backward(d, maskc)
        ctx.weight = weight
        ctx.shape = pred.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        d, mask = ctx.saved_tensors
        gc = g.contiguous().to(torch.float32)
        out = torch.empty_like(d)
        rc = _native.lib().siren_sse_backward(
            d.data_ptr(), mask.data_ptr() if mask is not None else None, d.numel(),
            mask.numel() if mask is not None else 0, gc.data_ptr(), float(2.0 * ctx.weight), out.data_ptr(),
            _native.stream_handle(d.device))
        _native.check(rc, "siren_sse_backward")
        return out.view(ctx.shape), None, None, None


# image_mse on the SIREN output layout [B, N, C], optionally with data consistency folded in
# (siren_kspace.hip): siren_mri_amd::kspace_sse(pred, k0?, mask?, tgt, hf?, noise, weight) -> (loss, d)
from .ops import _LIB  # noqa: E402

_LIB.define("kspace_sse(Tensor pred, Tensor? k0, Tensor? mask, Tensor tgt, Tensor? hf, float noise, float weight) "
            "-> (Tensor, Tensor)")
_LIB.define("kspace_sse_bwd(Tensor d, Tensor? mask, Tensor? hf, Tensor g, float noise, float scale) -> Tensor")


def _kspace_sse_cuda(pred, k0, mask, tgt, hf, noise, weight):
    b, n, c = pred.shape
    pc, tc = pred.contiguous(), tgt.contiguous()
    kc = k0.contiguous() if k0 is not None else None
    mc = mask.contiguous() if mask is not None else None
    hc = hf.contiguous() if hf is not None else None
    d = torch.empty_like(pc)
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    ws = _sse_workspace(pred.device)
    rc = _native.lib().siren_kspace_sse_forward(
        pc.data_ptr(), kc.data_ptr() if kc is not None else None, mc.data_ptr() if mc is not None else None,
        tc.data_ptr(), hc.data_ptr() if hc is not None else None, b, n, c, float(noise), float(weight), d.data_ptr(),
        loss.data_ptr(), ws.data_ptr(), ws.numel(), _native.stream_handle(pred.device))
    _native.check(rc, "siren_kspace_sse_forward")
    return loss, d


def _kspace_sse_bwd_cuda(d, mask, hf, g, noise, scale):
    b, n, c = d.shape
    out = torch.empty_like(d)
    mc = mask.contiguous() if mask is not None else None
    hc = hf.contiguous() if hf is not None else None
    gc = g.contiguous().to(torch.float32)
    rc = _native.lib().siren_kspace_sse_backward(d.data_ptr(), mc.data_ptr() if mc is not None else None,
                                                 hc.data_ptr() if hc is not None else None, b, n, c, float(noise),
                                                 gc.data_ptr(), float(scale), out.data_ptr(),
                                                 _native.stream_handle(d.device))
    _native.check(rc, "siren_kspace_sse_backward")
    return out


class _KspaceSSEAutograd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, k0, mask, tgt, hf, noise, weight):
        with torch._C._AutoDispatchBelowAutograd():
            loss, d = torch.ops.siren_mri_amd.kspace_sse(pred, k0, mask, tgt, hf, noise, weight)
        ctx.save_for_backward(d, mask, hf)
        ctx.noise, ctx.weight = noise, weight
        ctx.mark_non_differentiable(d)
        ctx.set_materialize_grads(False)
        return loss, d

    @staticmethod
    def backward(ctx, g, _gd):
        if g is None:
            return (None,) * 7
        d, mask, hf = ctx.saved_tensors
        dpred = torch.ops.siren_mri_amd.kspace_sse_bwd(d, mask, hf, g, ctx.noise, 2.0 * ctx.weight)
        return dpred, None, None, None, None, None, None


_LIB.impl("kspace_sse", _kspace_sse_cuda, "CUDA")
_LIB.impl("kspace_sse_bwd", _kspace_sse_bwd_cuda, "CUDA")
_LIB.impl("kspace_sse", lambda pred, k0, mask, tgt, hf, noise, weight:
          _KspaceSSEAutograd.apply(pred, k0, mask, tgt, hf, noise, weight), "Autograd")
torch.library.register_fake("siren_mri_amd::kspace_sse", lambda pred, k0, mask, tgt, hf, noise, weight:
                            (pred.new_empty(()), torch.empty_like(pred)), lib=_LIB)
torch.library.register_fake("siren_mri_amd::kspace_sse_bwd", lambda d, mask, hf, g, noise, scale: torch.empty_like(d),
                            lib=_LIB)

_FUSE_DC = True


def set_kspace_fusion(enabled: bool) -> None:
    """Fold a native DataConsistencyInKspace output's DC into image_mse's loss op (default on)."""
    global _FUSE_DC
    _FUSE_DC = bool(enabled)


def high_freq_flat(device):
    """image_mse's 128x128 high-frequency mask, flattened to the SIREN's [N] row order."""
    return _hf_flat(device)


def _staged_loss(out, tgt, hf_applied, weight):
    """The forward's fused loss (fusion.py) when `out` is its output (DC(y) with data consistency),
    `tgt` the staged target and the reduction the same; None otherwise."""
    st = fusion.staged(out.device)
    if st is None or st.result is None:
        return None
    y, y_dc, loss, st_hf, _dc = st.result
    if out is not (y_dc if y_dc is not None else y) or tgt is not st.tgt:
        return None
    if bool(hf_applied) != bool(st_hf) or float(weight) != st.weight:
        return None
    return loss


def _hf_flat(device):
    key = ("flat", device)
    m = _MASKS.get(key)
    if m is None:
        m = _high_freq_mask(device).reshape(-1).contiguous()
        _MASKS[key] = m
    return m


def _kspace_image_mse(out, tgt, high_freq):
    """image_mse on [B, N, C] (N a square): the native k-space op, or None when not applicable."""
    if not (out.is_cuda and out.dtype == torch.float32 and out.dim() == 3 and tgt.shape == out.shape
            and tgt.dtype == torch.float32 and tgt.device == out.device and not tgt.requires_grad
            and out.shape[-1] <= 8):
        return None
    n = out.shape[1]
    side = int(round(n ** 0.5))
    if side * side != n:
        return None
    hf = _hf_flat(out.device) if (high_freq and side == 128) else None
    src = dc_source(out) if _FUSE_DC else None
    if src is not None and src[0].shape == out.shape:
        pred, k0, mask, noise = src
        return torch.ops.siren_mri_amd.kspace_sse(pred, k0, mask, tgt, hf, noise, _KSPACE_WEIGHT)[0]
    return torch.ops.siren_mri_amd.kspace_sse(out, None, None, tgt, hf, 0.0, _KSPACE_WEIGHT)[0]


def weighted_sse(pred, tgt, weight=_KSPACE_WEIGHT, mask=None):
    """sum |m (pred - tgt)|^2 * weight over any shape (image_mse's reduction without the
    lin2img reshape): the loss of a coordinate shard of an image in a sharded fit, whose partial
    sums over the ranks' shards add up to image_mse of the whole image."""
    if mask is None:
        staged = _staged_loss(pred, tgt, False, weight)
        if staged is not None:
            return staged
    if pred.is_cuda and pred.dtype == torch.float32 and tgt.dtype == torch.float32 and not tgt.requires_grad:
        return _WeightedSSE.apply(pred, tgt.to(pred.device), mask, weight)
    diff = pred - tgt
    if mask is not None:
        diff = mask * diff
    return (diff.abs() ** 2).sum() * weight


def image_mse(mask, model_output, gt, high_freq=True):
    """Weighted k-space SSE: sum |m * (pred - gt)|^2 / 128^2 (a sum over the batch). On the GPU
    the native k-space op reads model_out / gt in their [B, N, C] layout (no lin2img copies); a
    model_out produced by the native DataConsistencyInKspace has the DC folded into the op."""
    out, tgt = model_output["model_out"], gt["img"]
    if out.dim() == 3:
        side = int(round(out.shape[1] ** 0.5))
        staged = _staged_loss(out, tgt, high_freq and side * side == out.shape[1] and side == 128, _KSPACE_WEIGHT)
        if staged is not None:
            return {"img_loss": staged}
    fused = _kspace_image_mse(model_output["model_out"], gt["img"], high_freq)
    if fused is not None:
        return {"img_loss": fused}
    pred = lin2img(model_output["model_out"])
    tgt = lin2img(gt["img"])
    hf = _high_freq_mask(pred.device) if (high_freq and pred.shape[-2:] == (128, 128)) else None
    if (pred.is_cuda and pred.dtype == torch.float32 and tgt.dtype == torch.float32 and not tgt.requires_grad
            and pred.shape == tgt.shape and tgt.device == pred.device
            and (hf is None or (hf.dtype == torch.float32 and pred.shape[-hf.dim():] == hf.shape))):
        return {"img_loss": _WeightedSSE.apply(pred, tgt, hf, _KSPACE_WEIGHT)}
    diff = pred - tgt
    if hf is not None:
        diff = hf * diff
    loss = (diff.abs() ** 2).sum() * _KSPACE_WEIGHT
    return {"img_loss": loss}


def latent_loss(model_output):
    return torch.mean(model_output["latent_vec"] ** 2)


_SUMSQ_WS = {}


def _sumsq_workspace(device, total):
    """Per-(device, stream) zeroed workspace of siren_sumsq_forward (left zeroed by every launch)."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    need = int(_native.lib().siren_sumsq_workspace_bytes(total))
    ws = _SUMSQ_WS.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.zeros(need, dtype=torch.uint8, device=device)
        _SUMSQ_WS[key] = ws
    return ws


class _SumSquares(torch.autograd.Function):
    """sum over tensors of torch.sum(w ** 2) in one native launch (siren_sumsq_forward), its
    gradient 2 g w in one more (siren_sumsq_backward)."""

    @staticmethod
    def forward(ctx, *ws):
        import ctypes
        ts = [w.detach().contiguous() for w in ws]
        n = len(ts)
        numel = (ctypes.c_int64 * n)(*[t.numel() for t in ts])
        out = torch.empty((), dtype=torch.float32, device=ts[0].device)
        work = _sumsq_workspace(ts[0].device, sum(t.numel() for t in ts))
        _native.check(_native.lib().siren_sumsq_forward(n, (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]), numel,
                                                        out.data_ptr(), work.data_ptr(), work.numel(),
                                                        _native.stream_handle(ts[0].device)), "siren_sumsq_forward")
        ctx.save_for_backward(*ws)  # the inputs: a create_graph backward differentiates through them
        return out

    @staticmethod
    def backward(ctx, g):
        import ctypes
        if torch.is_grad_enabled():
            # create_graph=True: the exact gradient 2 g w in differentiable PyTorch
            return tuple(2 * g * w if need else None for w, need in zip(ctx.saved_tensors, ctx.needs_input_grad))
        ts = [w.detach().contiguous() for w in ctx.saved_tensors]
        n = len(ts)
        gc = g.detach().reshape(()).to(torch.float32).contiguous()
        outs = [torch.empty_like(t) for t in ts]
        _native.check(_native.lib().siren_sumsq_backward(n, (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]),
                                                         (ctypes.c_int64 * n)(*[t.numel() for t in ts]), gc.data_ptr(),
                                                         (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs]),
                                                         _native.stream_handle(ts[0].device)), "siren_sumsq_backward")
        return tuple(o if need else None for o, need in zip(outs, ctx.needs_input_grad))


def hypo_weight_loss(model_output):
    """loss_functions.py:279-287: the mean of the squared hypo-parameters; on CUDA fp32 the sum of
    squares is one native launch (and its gradient one more)."""
    ws = list(model_output["hypo_params"].values())
    total = sum(w.numel() for w in ws)
    if ws and 0 < len(ws) <= 32 and all(w.is_cuda and w.dtype == torch.float32 and w.device == ws[0].device
                                        for w in ws):
        return _SumSquares.apply(*ws) * (1 / total)
    weight_sum = 0
    for w in ws:
        weight_sum = weight_sum + torch.sum(w ** 2)
    return weight_sum * (1 / total)


def image_hypernetwork_loss(mask, kl, fw, model_output, gt):
    return {"img_loss": image_mse(mask, model_output, gt)["img_loss"],
            "latent_loss": kl * latent_loss(model_output),
            "hypo_weight_loss": fw * hypo_weight_loss(model_output)}


def function_mse(model_output, gt):
    return {"func_loss": ((model_output["model_out"] - gt["func"]) ** 2).mean()}


def gradients_mse(model_output, gt):
    """mean_n sum_k (dy/dx_k - gt_k)^2 with the analytic SIREN gradient (config 3)."""
    g = diff_operators.gradient(model_output["model_out"], model_output["model_in"])
    return {"gradients_loss": torch.mean((g - gt["gradients"]).pow(2).sum(-1))}


def laplace_mse(model_output, gt):
    lap = diff_operators.laplace(model_output["model_out"], model_output["model_in"])
    return {"laplace_loss": torch.mean((lap - gt["laplace"]) ** 2)}
