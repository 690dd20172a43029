"""k-space data consistency (data_consistency.py:8-48 of jonbmartin/siren_mri).

out = (1 - m) * pred + m * k0 (noiseless) or (1 - m) * pred + m * (pred + v k0) / (1 + v),
with k0/mask given as [B, 2, H, W] and pred as [B, H*W, 2].
"""
from __future__ import annotations

import torch
import torch.nn as nn


def data_consistency(pred, k0, mask, noise_lvl=None):
    v = noise_lvl
    if v:
        return (1 - mask) * pred + mask * (pred + v * k0) / (1 + v)
    return (1 - mask) * pred + mask * k0


class DataConsistencyInKspace(nn.Module):
    def __init__(self, noise_lvl=None):
        super().__init__()
        self.noise_lvl = noise_lvl

    def forward(self, prediction, k0, mask):
        b = k0.shape[0]
        k0 = k0.permute(0, 2, 3, 1).reshape(b, -1, 2)
        mask = mask.permute(0, 2, 3, 1).reshape(b, -1, 2)
        return data_consistency(prediction, k0, mask, self.noise_lvl)
