"""Staged image loss for the forward's fused output epilogue.

The reference computes the loss after the model (training.py:67-78):

    model_output = model(model_input)              # SingleBVPNet / hypernetwork (+ DC)
    losses = loss_fn(model_output, gt)             # image_mse: (masked) k-space SSE / 128^2

so the SIREN forward cannot know the target. The fitting loops (training.train, bench.py) stage
it first — ``stage_image_loss(gt["img"])`` — and the first SIREN forward of the step whose output
matches the target's shape then runs the native forward-with-loss (one launch: the SIREN, the data
consistency of DataConsistencyInKspace when ``stage_dc`` supplied its planes, the loss, dL/dy),
as one autograd node with outputs (y, DC(y), loss). The modules and losses downstream recognise
its outputs by identity:

  * DataConsistencyInKspace(y, k0, mask) returns the already computed DC(y) when y, k0, mask and
    the noise level are the staged ones;
  * image_mse(mask, out, gt) / weighted_sse(pred, tgt) return the fused loss when their input is
    that output, their target the staged tensor and their parameters (high-frequency mask, weight)
    the staged ones;

anything else computes as usual (a staged loss nobody asks for costs its epilogue and nothing
else). The backward of the node takes dL/dloss as a device scalar into the native backward's
output-layer kernels (no dL/dy tensor is formed), so the two SSE launches of the unfused step
disappear. ``clear()`` ends the step.
"""
from __future__ import annotations

import torch

_ENABLED = True


def set_enabled(enabled: bool) -> None:
    """Process-wide switch (tests A/B the fused and the unfused paths)."""
    global _ENABLED
    _ENABLED = bool(enabled)
    if not enabled:
        clear()


def enabled() -> bool:
    return _ENABLED


class Staged:
    __slots__ = ("tgt", "high_freq", "weight", "dc", "result")

    def __init__(self, tgt, high_freq, weight):
        self.tgt = tgt
        self.high_freq = high_freq
        self.weight = float(weight)
        self.dc = None        # (k0, mask, noise)
        self.result = None    # (y, y_dc or None, loss)


_STAGED = [None]


def stage_image_loss(tgt: torch.Tensor, high_freq: bool = True, weight: float = 1.0 / (128 * 128)):
    """Stage image_mse's target for the next SIREN forward (see the module docstring)."""
    if not _ENABLED or not isinstance(tgt, torch.Tensor) or not tgt.is_cuda or tgt.dtype != torch.float32 \
            or tgt.requires_grad:
        _STAGED[0] = None
        return None
    st = Staged(tgt, bool(high_freq), weight)
    _STAGED[0] = st
    return st


def stage_dc(k0, mask, noise: float) -> None:
    """The k-space planes of the DataConsistencyInKspace that will follow the staged SIREN."""
    st = _STAGED[0]
    if st is not None and st.result is None:
        st.dc = (k0, mask, float(noise))


def pending():
    """The staged record whose forward has not run yet, or None."""
    st = _STAGED[0]
    return st if (st is not None and st.result is None) else None


def staged():
    return _STAGED[0]


def clear() -> None:
    _STAGED[0] = None
