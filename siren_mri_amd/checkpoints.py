"""Checkpoint and Fourier-matrix file compatibility with jonbmartin/siren_mri (SURVEY.md §8(f)
row 4), so the reference's evaluation scripts and this package read each other's files.

* Model files are plain `state_dict`s saved with `torch.save`; parameter names follow the
  reference's module tree (`net.net.{i}.0.weight` / `.bias` for SingleBVPNet, modules.py:68-85).
* The reference's data-parallel loop saves `model_current.pth` / `model_final.pth` from the DDP
  wrapper, so their keys carry a `module.` prefix (training_ddp.py:89,146), while
  `model_epoch_*.pth` come from `model.module` without it (training_ddp.py:53). Its test scripts
  call `model.load_state_dict(torch.load(path))` on a plain model (e.g.
  test_mri_conv_neural_process_kspace_fourierfeat.py:222), which only works for the unprefixed
  files. `load_state_dict_compat` accepts both forms. This package's loops never wrap the model
  (one flattened gradient all-reduce, training_ddp.py here), so every file they write is
  unprefixed — loadable by the reference's test scripts as they stand.
* The Fourier matrix B of each rank goes to `<model_dir>/current_B_DDP_mp<rank>.pt`, a bare
  tensor (train_mri_neural_process_ddp.py:254-256, features.py:43-47), where the reference's
  test script looks for it (test_mri_conv_neural_process_kspace_fourierfeat.py:214-215).

Files are read with `torch.load(..., weights_only=True)`: tensors and containers only.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

DDP_PREFIX = "module."


def strip_ddp_prefix(state_dict):
    """The state_dict without the DDP wrapper's `module.` prefix when every key carries it
    (the reference's model_current/model_final files); otherwise unchanged."""
    keys = list(state_dict.keys())
    if keys and all(k.startswith(DDP_PREFIX) for k in keys):
        return OrderedDict((k[len(DDP_PREFIX):], v) for k, v in state_dict.items())
    return state_dict


def load_state_dict_file(path, map_location="cpu"):
    """A model file written by either code base, as an unprefixed state_dict."""
    sd = torch.load(path, map_location=map_location, weights_only=True)
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: expected a state_dict, found {type(sd).__name__}")
    return strip_ddp_prefix(sd)


def load_state_dict_compat(model, path_or_state_dict, strict=True):
    """model.load_state_dict for a reference or siren_mri_amd checkpoint (file path or dict),
    with or without the DDP `module.` prefix. Returns load_state_dict's result."""
    sd = (load_state_dict_file(path_or_state_dict) if isinstance(path_or_state_dict, (str, os.PathLike))
          else strip_ddp_prefix(path_or_state_dict))
    return model.load_state_dict(sd, strict=strict)


def ddp_state_dict(model):
    """The model's state_dict with the `module.` prefix the reference's DDP wrapper gives its
    model_current/model_final files (training_ddp.py:89,146), for tools that expect that form."""
    return OrderedDict((DDP_PREFIX + k, v) for k, v in model.state_dict().items())


def b_matrix_path(model_dir, rank):
    """`<model_dir>/current_B_DDP_mp<rank>.pt` (train_mri_neural_process_ddp.py:254)."""
    return os.path.join(model_dir, f"current_B_DDP_mp{int(rank)}.pt")


def save_b_matrix(transform, model_dir, rank):
    """Save a GaussianFourierFeatureTransform's B where the reference's scripts expect it."""
    os.makedirs(model_dir, exist_ok=True)
    path = b_matrix_path(model_dir, rank)
    transform.save_B(path)
    return path


def load_b_matrix(transform, model_dir, rank):
    path = b_matrix_path(model_dir, rank)
    transform.load_B(path)
    return path
