"""Mask and metric helpers on the hot path (utils.py of jonbmartin/siren_mri).

  cond_mkdir                 utils.py:15-17
  create_circular_mask_torch utils.py:25-40 (arange(1, h): a 129 request yields 128 points)
  psnr / write_psnr          utils.py:593-616 with skimage compare_psnr(data_range=1):
                             p = clip(p/2 + 0.5, 0, 1), t = t/2 + 0.5, 10 log10(1/MSE)
The tensorboard image/gradient summaries (visualisation) are out of scope.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def cond_mkdir(path):
    if not os.path.exists(path):
        os.makedirs(path, exist_ok=True)


def create_circular_mask_torch(h, w, center=None, radius=None):
    if center is None:
        center = (int(w / 2), int(h / 2))
    if radius is None:
        radius = min(center[0], center[1], w - center[0], h - center[1])
    y = torch.arange(1, h)
    x = torch.arange(1, w)
    Y, X = torch.meshgrid(y, x, indexing="ij")
    dist = torch.sqrt((X - center[0]) ** 2 + (Y - center[1]) ** 2)
    return (dist <= radius).long()


def _host(a) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().double().numpy()
    return np.asarray(a, dtype=np.float64)


def psnr(pred_img, gt_img) -> float:
    """PSNR of one image pair in the reference's [-1, 1] convention (utils.py:604-610);
    numpy arrays or tensors on any device."""
    p = _host(pred_img) / 2.0 + 0.5
    p = np.clip(p, 0.0, 1.0)
    t = _host(gt_img) / 2.0 + 0.5
    mse = float(np.mean((p - t) ** 2))
    return float("inf") if mse == 0 else float(10.0 * np.log10(1.0 / mse))


def batch_psnr(pred_img: torch.Tensor, gt_img: torch.Tensor) -> list:
    """Per-image PSNR of [B, C, H, W] tensors (the loop of write_psnr, utils.py:593-611)."""
    p = pred_img.detach().float().cpu().numpy()
    t = gt_img.detach().float().cpu().numpy()
    return [psnr(p[i], t[i]) for i in range(p.shape[0])]


def write_psnr(pred_img, gt_img, writer, iter, prefix):
    vals = batch_psnr(pred_img, gt_img)
    if writer is not None:
        writer.add_scalar(prefix + "psnr", float(np.mean(vals)), iter)
    return vals
