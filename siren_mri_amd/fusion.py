"""Staged image loss for the forward's fused output epilogue.

The reference computes the loss after the model (training.py:67-78):

    model_output = model(model_input)              # SingleBVPNet / hypernetwork (+ DC)
    losses = loss_fn(model_output, gt)             # image_mse: (masked) k-space SSE / 128^2

so the SIREN forward cannot know the target. The fitting loops (training.train, bench.py) stage
it first — ``stage_image_loss(gt["img"])`` — and the first SIREN forward of the step whose output
matches the target's shape then runs the native forward-with-loss (one launch: the SIREN, the data
consistency of DataConsistencyInKspace when ``stage_dc`` supplied its planes, the loss, dL/dy),
as one autograd node with outputs (y, DC(y), loss). A record belongs to the thread that staged it
and to the stream current on the target's device at that time. The modules and losses downstream recognise
its outputs by identity:

  * DataConsistencyInKspace(y, k0, mask) returns the already computed DC(y) when y, k0, mask and
    the noise level are the staged ones;
  * image_mse(mask, out, gt) / weighted_sse(pred, tgt) return the fused loss when their input is
    that output, their target the staged tensor and their parameters (high-frequency mask, weight)
    the staged ones;

anything else computes as usual (a staged loss nobody asks for costs its epilogue and nothing
else). The backward of the node takes dL/dloss as a device scalar into the native backward's
output-layer kernels (no dL/dy tensor is formed), so the two SSE launches of the unfused step
disappear. ``clear(record)`` ends the step (or the ``image_loss`` context manager).
"""
from __future__ import annotations

import threading

import torch

_ENABLED = True


def set_enabled(enabled: bool) -> None:
    """Switch fusion on or off for this process (the tests use it to A/B the fused and unfused
    paths). Switching it off also clears the calling thread's staged records."""
    global _ENABLED
    _ENABLED = bool(enabled)
    if not enabled:
        clear()


def enabled() -> bool:
    return _ENABLED


class Staged:
    __slots__ = ("tgt", "high_freq", "weight", "dc", "result", "key")

    def __init__(self, tgt, high_freq, weight, key=None):
        self.tgt = tgt
        self.high_freq = high_freq
        self.weight = float(weight)
        self.dc = None        # (k0, mask, noise)
        self.result = None    # (y, y_dc or None, loss, hf applied, dc planes)
        self.key = key


# Staged records live per thread, keyed by (device, stream): a forward picks up only the record
# staged on its own thread for the stream it is launched on. So two models fitted in one process
# on two streams, or on two threads, never see each other's target.
_LOCAL = threading.local()


def _slots() -> dict:
    d = getattr(_LOCAL, "slots", None)
    if d is None:
        d = _LOCAL.slots = {}
    return d


def stream_key(device) -> tuple:
    """(device type, index, stream handle) of `device` (a torch.device or a tensor's device)."""
    if isinstance(device, torch.Tensor):
        device = device.device
    device = torch.device(device)
    if device.type != "cuda":
        return (device.type, device.index, 0)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return ("cuda", idx, torch.cuda.current_stream(idx).cuda_stream)


def stage_image_loss(tgt: torch.Tensor, high_freq: bool = True, weight: float = 1.0 / (128 * 128)):
    """Stage image_mse's target for the next SIREN forward on the current thread and the current
    stream of tgt's device (see the module docstring). Returns the record, or None when the
    target cannot be fused (then the forward runs unfused)."""
    if not isinstance(tgt, torch.Tensor):
        return None
    key = stream_key(tgt.device)
    if not _ENABLED or not tgt.is_cuda or tgt.dtype != torch.float32 or tgt.requires_grad:
        _slots().pop(key, None)
        return None
    st = Staged(tgt, bool(high_freq), weight, key)
    _slots()[key] = st
    return st


def stage_dc(k0, mask, noise: float, device=None) -> None:
    """The k-space planes of the DataConsistencyInKspace that will follow the staged SIREN
    (device: that of k0 unless given)."""
    st = _slots().get(stream_key(k0 if device is None else device))
    if st is not None and st.result is None:
        st.dc = (k0, mask, float(noise))


def pending(device):
    """The record staged for `device`'s current stream on this thread whose forward has not run
    yet, or None."""
    st = _slots().get(stream_key(device))
    return st if (st is not None and st.result is None) else None


def staged(device):
    """The record staged for `device`'s current stream on this thread (run or not), or None."""
    return _slots().get(stream_key(device))


_ALL = object()


def clear(record=_ALL) -> None:
    """End a step: drop `record` (as stage_image_loss returned it; None: nothing), or every record
    of this thread when called without an argument."""
    if record is _ALL:
        _slots().clear()
    elif record is not None:
        d = _slots()
        if d.get(record.key) is record:
            del d[record.key]


class image_loss:
    """Context manager: ``with fusion.image_loss(gt["img"]): out = model(...); loss = loss_fn(...)``
    stages the target for the block and clears exactly that record afterwards."""

    def __init__(self, tgt, high_freq: bool = True, weight: float = 1.0 / (128 * 128)):
        self.args = (tgt, high_freq, weight)
        self.record = None

    def __enter__(self):
        self.record = stage_image_loss(*self.args)
        return self.record

    def __exit__(self, *exc):
        clear(self.record)
        return False
