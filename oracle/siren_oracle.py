"""ORACLE — CPU restatement of the jonbmartin/siren_mri SIREN hot path (TEST INFRASTRUCTURE).

This module is the checker, never the product: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it. The product path (siren_mri_amd) must not, and it
fails loudly instead of falling back to anything here.

It restates, with plain PyTorch CPU ops (fp32 by default, fp64 optional), the reference
algorithm at:
  dataio.py:28-48      get_mgrid             dataio.py:51-63     lin2img
  modules.py:11-27     BatchLinear           modules.py:30-38    Sine
  modules.py:45-97     FCBlock               modules.py:122-164  SingleBVPNet
  modules.py:641-654   sine_init / first_layer_sine_init (+ nn.Linear default init)
  diff_operators.py:27-43  gradient / laplace / divergence (autograd, create_graph=True)
  loss_functions.py:66-101 image_mse         loss_functions.py:275-293 hypernet losses
  loss_functions.py:330-335 gradients_mse    loss_functions.py:350-355 laplace_mse
  utils.py:25-40       create_circular_mask_torch
  utils.py:593-616     write_psnr (skimage compare_psnr, data_range=1)
  features.py:31-41    GaussianFourierFeatureTransform.forward
  data_consistency.py:8-48 DataConsistencyInKspace
  training.py:19-146   train (Adam, clip, accumulation) — as `train_steps`

Parity pinning: tests/golden/*.npz were produced by tests/golden/make_golden.py, which imports
the real reference in the survey container (PyTorch 2.10 CPU) and records its outputs; the
tests in tests/test_oracle_golden.py check this restatement against them.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
from torch import nn


# --------------------------------------------------------------------------- data layout
def get_mgrid(sidelen, dim: int = 2) -> torch.Tensor:
    """dataio.py:28-48 — flattened row-major grid in [-1, 1]: x_k = 2*i_k/(S_k-1) - 1."""
    if isinstance(sidelen, int):
        sidelen = dim * (sidelen,)
    if dim == 2:
        pc = np.stack(np.mgrid[:sidelen[0], :sidelen[1]], axis=-1)[None, ...].astype(np.float32)
        pc[0, :, :, 0] = pc[0, :, :, 0] / (sidelen[0] - 1)
        pc[0, :, :, 1] = pc[0, :, :, 1] / (sidelen[1] - 1)
    elif dim == 3:
        pc = np.stack(np.mgrid[:sidelen[0], :sidelen[1], :sidelen[2]], axis=-1)[None, ...].astype(np.float32)
        pc[..., 0] = pc[..., 0] / max(sidelen[0] - 1, 1)
        pc[..., 1] = pc[..., 1] / (sidelen[1] - 1)
        pc[..., 2] = pc[..., 2] / (sidelen[2] - 1)
    else:
        raise NotImplementedError(dim)
    pc -= 0.5
    pc *= 2.0
    return torch.from_numpy(pc).view(-1, dim)


def lin2img(t: torch.Tensor, image_resolution=None) -> torch.Tensor:
    """dataio.py:51-63 — [B, N, C] -> [B, C, H, W] (square unless a resolution is given)."""
    b, n, c = t.shape
    if image_resolution is None:
        h = w = int(np.sqrt(n))
    else:
        h, w = image_resolution
    return t.permute(0, 2, 1).reshape(b, c, h, w)


# --------------------------------------------------------------------------- SIREN model
def siren_dims(in_features: int, hidden_features: int, num_hidden_layers: int, out_features: int):
    """FCBlock layer widths (modules.py:68-85): in -> hidden x (1 + nh) -> out."""
    return [in_features] + [hidden_features] * (num_hidden_layers + 1) + [out_features]


def siren_init(dims, seed: int | None = None, generator_state=None):
    """Parameters in the reference's RNG order (modules.py:68-90, 641-654):
    1) every BatchLinear (nn.Linear subclass) is constructed in order -> kaiming_uniform_(W,
       a=sqrt(5)) then U(+-1/sqrt(fan_in)) for b (nn.Linear.reset_parameters);
    2) net.apply(sine_init): W_l ~ U(+-sqrt(6/in)/30), layers in order;
    3) net[0].apply(first_layer_sine_init): W_0 ~ U(+-1/in)."""
    if seed is not None:
        torch.manual_seed(seed)
    lins = [nn.Linear(dims[l], dims[l + 1]) for l in range(len(dims) - 1)]
    with torch.no_grad():
        for lin in lins:
            n = lin.weight.size(-1)
            lin.weight.uniform_(-np.sqrt(6 / n) / 30, np.sqrt(6 / n) / 30)
        n0 = lins[0].weight.size(-1)
        lins[0].weight.uniform_(-1 / n0, 1 / n0)
    return [(l.weight.detach().clone(), l.bias.detach().clone()) for l in lins]


def siren_forward(x: torch.Tensor, params, w0: float = 30.0, outermost_linear: bool = True):
    """FCBlock.forward with nonlinearity='sine' (modules.py:16-38, 92-97).
    params: list of (W, b); W is [out, in] or batched [B, out, in]."""
    h = x
    L = len(params)
    for l, (W, b) in enumerate(params):
        perm = list(range(W.dim() - 2)) + [-1, -2]
        h = h.matmul(W.permute(*perm))
        h = h + b.unsqueeze(-2)
        if l < L - 1 or not outermost_linear:
            h = torch.sin(w0 * h)
    return h


def param_dict(params) -> OrderedDict:
    """state_dict key names of SingleBVPNet (net.net.{i}.0.weight/bias)."""
    d = OrderedDict()
    for i, (W, b) in enumerate(params):
        d[f"net.net.{i}.0.weight"] = W
        d[f"net.net.{i}.0.bias"] = b
    return d


class OracleSiren(nn.Module):
    """CPU SingleBVPNet restatement (modules.py:122-164) — the reference CPU path used by the
    CPU baseline and the CPU multi-process tests. Same param names as the reference."""

    def __init__(self, out_features=1, in_features=2, hidden_features=256, num_hidden_layers=3,
                 w0=30.0, seed=None):
        super().__init__()
        dims = siren_dims(in_features, hidden_features, num_hidden_layers, out_features)
        params = siren_init(dims, seed)
        self.w0 = w0
        self.weights = nn.ParameterList([nn.Parameter(W) for W, _ in params])
        self.biases = nn.ParameterList([nn.Parameter(b) for _, b in params])

    def forward(self, model_input, params=None):
        coords_org = model_input["coords"].clone().detach().requires_grad_(True)
        p = list(zip(self.weights, self.biases))
        return {"model_in": coords_org, "model_out": siren_forward(coords_org, p, self.w0)}


# --------------------------------------------------------------------------- derivatives
def gradient(y, x, grad_outputs=None):
    """diff_operators.py:39-43."""
    if grad_outputs is None:
        grad_outputs = torch.ones_like(y)
    return torch.autograd.grad(y, [x], grad_outputs=grad_outputs, create_graph=True)[0]


def divergence(y, x):
    """diff_operators.py:32-36."""
    div = 0.0
    for i in range(y.shape[-1]):
        div += torch.autograd.grad(y[..., i], x, torch.ones_like(y[..., i]), create_graph=True)[0][..., i:i + 1]
    return div


def laplace(y, x):
    """diff_operators.py:27-29."""
    return divergence(gradient(y, x), x)


# --------------------------------------------------------------------------- losses
def create_circular_mask(h, w, center=None, radius=None):
    """utils.py:25-40 — note arange(1, h) gives h-1 points (129 -> 128x128)."""
    if center is None:
        center = (int(w / 2), int(h / 2))
    if radius is None:
        radius = min(center[0], center[1], w - center[0], h - center[1])
    y = torch.arange(1, h)
    x = torch.arange(1, w)
    Y, X = torch.meshgrid(y, x, indexing="ij")
    dist = torch.sqrt((X - center[0]) ** 2 + (Y - center[1]) ** 2)
    return (dist <= radius).long()


def image_mse(mask, model_output, gt, high_freq=True):
    """loss_functions.py:66-101 — k-space SSE / 128^2 (a SUM over the batch), optionally with the
    high-frequency mask 1 - circle(r=20) on a 128x128 grid."""
    pred = lin2img(model_output["model_out"])
    tgt = lin2img(gt["img"])
    if high_freq:
        m = (1 - create_circular_mask(129, 129, center=None, radius=20)).to(pred.device)
        loss = (torch.abs(m * (pred - tgt)) ** 2).sum()
    else:
        loss = (torch.abs(pred - tgt) ** 2).sum()
    return {"img_loss": loss * (1 / (128 * 128))}


def latent_loss(model_output):
    """loss_functions.py:275-276."""
    return torch.mean(model_output["latent_vec"] ** 2)


def hypo_weight_loss(model_output):
    """loss_functions.py:279-287."""
    s, n = 0, 0
    for w in model_output["hypo_params"].values():
        s = s + torch.sum(w ** 2)
        n += w.numel()
    return s * (1 / n)


def image_hypernetwork_loss(mask, kl, fw, model_output, gt):
    """loss_functions.py:290-293."""
    return {"img_loss": image_mse(mask, model_output, gt)["img_loss"],
            "latent_loss": kl * latent_loss(model_output),
            "hypo_weight_loss": fw * hypo_weight_loss(model_output)}


def gradients_mse(model_output, gt):
    """loss_functions.py:330-335."""
    g = gradient(model_output["model_out"], model_output["model_in"])
    return {"gradients_loss": torch.mean((g - gt["gradients"]).pow(2).sum(-1))}


def laplace_mse(model_output, gt):
    """loss_functions.py:350-355."""
    lap = laplace(model_output["model_out"], model_output["model_in"])
    return {"laplace_loss": torch.mean((lap - gt["laplace"]) ** 2)}


def function_mse(model_output, gt):
    """loss_functions.py:326-327."""
    return {"func_loss": ((model_output["model_out"] - gt["func"]) ** 2).mean()}


def psnr(pred_img: np.ndarray, gt_img: np.ndarray) -> float:
    """utils.py:604-610 + skimage compare_psnr(data_range=1): p = clip(p/2+.5, 0, 1),
    t = t/2+.5 (unclipped), PSNR = 10 log10(1 / mean((p - t)^2))."""
    p = np.clip(pred_img / 2.0 + 0.5, 0.0, 1.0).astype(np.float64)
    t = (gt_img / 2.0 + 0.5).astype(np.float64)
    mse = np.mean((p - t) ** 2)
    return float(10 * np.log10(1.0 / mse))


# --------------------------------------------------------------------------- MRI helpers
def fourier_features(x: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """features.py:31-41: cat(sin(2 pi x B), cos(2 pi x B))."""
    z = 2 * np.pi * (x @ B.to(x.device))
    return torch.cat([torch.sin(z), torch.cos(z)], dim=2)


def data_consistency(pred, k0, mask):
    """data_consistency.py:8-20, 32-48 (noiseless): (1 - m) pred + m k0 on [B, N, 2]."""
    b = k0.shape[0]
    k0 = torch.permute(k0, (0, 2, 3, 1)).reshape(b, -1, 2)
    mask = torch.permute(mask, (0, 2, 3, 1)).reshape(b, -1, 2)
    return (1 - mask) * pred + mask * k0


# --------------------------------------------------------------------------- training
def train_steps(params, coords, gt, loss_fn, steps: int, lr: float = 1e-4, w0: float = 30.0,
                clip_grad=False, record_params_every: int = 0):
    """training.py:19-146 restated for a single full-batch image: per step forward, loss sum of
    `.mean()`s, backward, optional clip_grad_norm_(1.0), Adam(lr) step + zero_grad.
    Returns (losses, final params, [param snapshots])."""
    ps = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in params]
    flat = [t for wb in ps for t in wb]
    opt = torch.optim.Adam(lr=lr, params=flat)
    losses, snaps = [], []
    for step in range(steps):
        x = coords.clone().detach().requires_grad_(True)
        out = {"model_in": x, "model_out": siren_forward(x, ps, w0)}
        parts = loss_fn(out, gt)
        total = 0.0
        for v in parts.values():
            total = total + v.mean()
        losses.append(float(total.item()))
        total.backward()
        if clip_grad:
            torch.nn.utils.clip_grad_norm_(flat, max_norm=1.0 if isinstance(clip_grad, bool) else clip_grad)
        opt.step()
        opt.zero_grad()
        if record_params_every and (step + 1) % record_params_every == 0:
            snaps.append([t.detach().clone() for t in flat])
    return losses, [(W.detach(), b.detach()) for W, b in ps], snaps


def norm_rel(a, b) -> float:
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    den = torch.linalg.vector_norm(b).item()
    return torch.linalg.vector_norm(a - b).item() / (den if den > 0 else 1.0)
