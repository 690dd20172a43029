"""Gaussian Fourier features (features.py:6-53 of jonbmartin/siren_mri).

forward: cat(sin(2 pi x B), cos(2 pi x B)) with B = randn(in, m) * scale (features.py:21-41).
B lives as a buffer on the module's device (the reference keeps it on the CPU and copies it to
the input's device on every call, features.py:28,36); save_B/load_B/get_B/set_B keep the
reference's file format (a bare tensor saved with torch.save).
"""
from __future__ import annotations

import numpy as np
import torch


class GaussianFourierFeatureTransform(torch.nn.Module):
    def __init__(self, num_input_channels, mapping_size_spatial=256, scale=10, loaded_B=None, device=None):
        super().__init__()
        self._num_input_channels = num_input_channels
        self._mapping_size = mapping_size_spatial
        B = torch.randn((num_input_channels, mapping_size_spatial)) * scale if loaded_B is None else loaded_B
        self.register_buffer("_B_spatial", B.detach().clone(), persistent=False)
        if device is not None:
            self.to(device)

    def forward(self, x):
        z = x @ self._B_spatial.to(x.device, x.dtype)
        z = 2 * np.pi * z
        return torch.cat([torch.sin(z), torch.cos(z)], dim=-1)

    def save_B(self, filename):
        torch.save(self._B_spatial.detach().cpu(), filename)

    def load_B(self, filename):
        self.set_B(torch.load(filename, weights_only=True))

    def get_B(self):
        return self._B_spatial

    def set_B(self, B):
        self._B_spatial = B.detach().clone().to(self._B_spatial.device)
