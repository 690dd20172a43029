"""Data-parallel fitting (drop-in for training_ddp.py:23-164 of jonbmartin/siren_mri).

One process per GPU over torch.distributed ('nccl' = RCCL on ROCm, over xGMI; 'gloo' on CPU).
The reference wraps the model in DDP (train_mri_neural_process_ddp.py:238) and lets its
backward hooks all-reduce ~25 MB buckets. Here the exchange is explicit and minimal:

  * GradAllReducer flattens every parameter gradient into ONE contiguous buffer after backward
    and issues ONE all-reduce (averaged, DDP semantics, or summed, for coordinate-sharded fits
    whose loss is a sum over coordinates) — for the 5x256 SIREN that is a single 793.6 KB
    message per step; for the config-5 hypernetwork model (31.3 M params) a few large buckets.
  * parameters are broadcast from rank 0 once at construction (the DDP constructor's broadcast).
  * shard_rows / DistributedSampler split the coordinate grid or the slice list across ranks.

Deliberate deviations: MASTER_ADDR/PORT come from the environment or 127.0.0.1:12355 instead of
a hard-coded host (bug 0.6); checkpoints, loss files and summaries are written by rank 0 only
(the reference lets every rank write the same files).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist

from . import training


def ddp_setup(rank: int, world_size: int, backend: str | None = None):
    """training_ddp.py:155-164 with the address taken from the environment."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(rank % torch.cuda.device_count())
    dist.init_process_group(backend=backend, rank=rank, world_size=world_size)


def shard_rows(n_rows: int, rank: int, world_size: int):
    """Contiguous row block of the flattened grid owned by `rank`."""
    base, rem = divmod(n_rows, world_size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


class GradAllReducer:
    """Single flattened all-reduce of all parameter gradients (see module docstring)."""

    def __init__(self, params, op: str = "mean", group=None, bucket_bytes: int = 256 << 20,
                 broadcast: bool = True):
        self.params = [p for p in params if p.requires_grad]
        if op not in ("mean", "sum"):
            raise ValueError("op must be 'mean' or 'sum'")
        self.op = op
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # group parameters into buckets of <= bucket_bytes (one for small models)
        self.buckets = []
        cur, size = [], 0
        for p in self.params:
            nbytes = p.numel() * p.element_size()
            if cur and size + nbytes > bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._flat = [None] * len(self.buckets)
        self._base = None  # snapshot of the accumulated gradient (micro-step deltas)
        if broadcast and self.world > 1:
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, src=0, group=group)

    @torch.no_grad()
    def snapshot(self):
        """Remember the current (already exchanged) gradient; the next call with delta=True
        exchanges only what was added since."""
        if self.world == 1:
            return
        self._base = [[None if p.grad is None else p.grad.detach().clone() for p in b] for b in self.buckets]

    @torch.no_grad()
    def __call__(self, delta: bool = False):
        if self.world == 1:
            return
        base = self._base if delta else None
        self._base = None
        for i, bucket in enumerate(self.buckets):
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            if base is not None:
                grads = [g if b is None else g - b for g, b in zip(grads, base[i])]
            numel = sum(g.numel() for g in grads)
            flat = self._flat[i]
            if flat is None or flat.numel() != numel or flat.device != grads[0].device:
                flat = torch.empty(numel, dtype=grads[0].dtype, device=grads[0].device)
                self._flat[i] = flat
            off = 0
            views = []
            for g in grads:
                n = g.numel()
                flat[off:off + n].copy_(g.reshape(-1))
                views.append((off, n))
                off += n
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            if self.op == "mean":
                flat.mul_(1.0 / self.world)
            for j, (p, (o, n)) in enumerate(zip(bucket, views)):
                red = flat[o:o + n].view_as(p)
                if base is not None and base[i][j] is not None:
                    red = red + base[i][j]
                if p.grad is None:
                    p.grad = red.clone()
                else:
                    p.grad.copy_(red)


def train_ddp(model, train_dataloader, epochs, lr, steps_til_summary, epochs_til_checkpoint, model_dir, loss_fn,
              summary_fn, val_dataloader=None, double_precision=False, clip_grad=False, use_lbfgs=False,
              loss_schedules=None, fourier_feat_transformer=None, device=0, ddp_run=False, accumulation_steps=1,
              grad_op: str = "mean"):
    """training_ddp.py:23-152: the train loop with a per-step gradient all-reduce, the sampler's
    epoch set for shuffling, and rank-0-only I/O. `model` may be a plain module (preferred) or a
    torch DDP wrapper (then DDP performs the exchange and no extra all-reduce is issued)."""
    is_ddp_wrapper = isinstance(model, torch.nn.parallel.DistributedDataParallel)
    module = model.module if is_ddp_wrapper else model
    rank = dist.get_rank() if dist.is_initialized() else 0
    reducer = None if is_ddp_wrapper else GradAllReducer(module.parameters(), op=grad_op)

    sampler = getattr(train_dataloader, "sampler", None)

    class _EpochLoader:
        def __init__(self, dl):
            self.dl = dl
            self.epoch = 0

        def __len__(self):
            return len(self.dl)

        def __iter__(self):
            if sampler is not None and hasattr(sampler, "set_epoch"):
                sampler.set_epoch(self.epoch)
            self.epoch += 1
            return iter(self.dl)

    out = training.train(model, _EpochLoader(train_dataloader), epochs, lr, steps_til_summary,
                         epochs_til_checkpoint, model_dir, loss_fn,
                         summary_fn if rank == 0 else (lambda *a, **k: None),
                         val_dataloader=val_dataloader if rank == 0 else None,
                         double_precision=double_precision, clip_grad=clip_grad, loss_schedules=loss_schedules,
                         fourier_feat_transformer=fourier_feat_transformer,
                         # rank 0 replaces model_dir unconditionally, as training_ddp.py:29-33 does
                         hyperopt_run=True,
                         accumulation_steps=accumulation_steps, grad_reducer=reducer,
                         write_outputs=(rank == 0))
    return out
