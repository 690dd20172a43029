"""Generic fitting loop (drop-in for training.py:19-146 of jonbmartin/siren_mri).

Same signature and step semantics: optional Fourier-feature transform of the coordinates
(:61-64), forward, loss dict summed from per-term `.mean()`s with optional schedules (:67-78),
loss / accumulation_steps, backward, optional clip_grad_norm_ every micro-step (:93-97), Adam
step + zero_grad every `accumulation_steps` micro-steps or at the last batch (:101-103),
checkpoints (`model_epoch_%04d.pth`, `model_current.pth`, `model_final.pth`) and loss text files
with the reference's names.

Deliberate deviations:
  * batches are moved to the model's device (bug 0.1, training.py:53-66);
  * the function returns the mean validation loss, or the last training loss when there is no
    validation loader (bug 0.3, training.py:145);
  * the per-step loss is kept on the device and read back only at summary steps and at the end
    (the reference calls .item() every step, a host sync per step);
  * an existing model_dir is never deleted without consent: interactively the reference's prompt
    asks (training.py:25-33); in a non-interactive run (nohup, a batch scheduler, a pipe) the
    reference's input() raises EOFError and nothing is lost — here a FileExistsError says so,
    unless overwrite=True (or hyperopt_run=True, as in the reference) was passed;
  * with accumulation_steps > 1 and a data-parallel grad_reducer, each micro-step's exchange
    carries only the gradient added since the previous exchange (see the note above validate).
"""
from __future__ import annotations

import os
import shutil
import sys
import time

import numpy as np
import torch

from . import fusion, utils


class _NullWriter:
    def __getattr__(self, name):
        return lambda *a, **k: None


def make_writer(path):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(path)
    except Exception:  # tensorboard is optional
        return _NullWriter()


def to_device(d, device):
    return {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in d.items()}


def model_device(model):
    for p in model.parameters():
        return p.device
    return torch.device("cpu")


def prepare_model_dir(model_dir, hyperopt_run=False, overwrite=False):
    """training.py:25-37. Deletes an existing model_dir only on consent: hyperopt_run or overwrite,
    or a 'y' at the interactive prompt. A non-interactive run raises instead of deleting."""
    if os.path.exists(model_dir):
        if hyperopt_run or overwrite:
            val = "y"
        elif sys.stdin is not None and sys.stdin.isatty():
            val = input("The model directory %s exists. Overwrite? (y/n)" % model_dir)
        else:
            raise FileExistsError(
                f"model directory {model_dir} exists and stdin is not interactive; pass "
                "overwrite=True (scripts: --overwrite) to replace it, or choose another experiment name")
        if val == "y":
            shutil.rmtree(model_dir)
    os.makedirs(model_dir, exist_ok=True)
    summaries_dir = os.path.join(model_dir, "summaries")
    checkpoints_dir = os.path.join(model_dir, "checkpoints")
    utils.cond_mkdir(summaries_dir)
    utils.cond_mkdir(checkpoints_dir)
    return summaries_dir, checkpoints_dir


def compute_loss(losses, loss_schedules, total_steps, writer):
    train_loss = 0.0
    for name, loss in losses.items():
        single = loss.mean()
        if loss_schedules is not None and name in loss_schedules:
            w = loss_schedules[name](total_steps)
            writer.add_scalar(name + "_weight", w, total_steps)
            single = single * w
        train_loss = train_loss + single
    return train_loss


def make_adam(params, lr):
    """The optimizer of training.py:29 (torch.optim.Adam(lr=lr, params=...)): siren_mri_amd.optim.Adam,
    torch's Adam with the update of all fp32 CUDA parameters in one native launch."""
    from .optim import Adam
    return Adam(params, lr=lr)


def train(model, train_dataloader, epochs, lr, steps_til_summary, epochs_til_checkpoint, model_dir, loss_fn,
          summary_fn, val_dataloader=None, double_precision=False, clip_grad=False, use_lbfgs=False,
          loss_schedules=None, fourier_feat_transformer=None, device=None, hyperopt_run=False,
          accumulation_steps=1, grad_reducer=None, write_outputs=True, overwrite=False, model_dir_hook=None):
    """Fit `model` (training.py:19-146). `grad_reducer`, if given, is the data-parallel gradient
    exchange of training_ddp (see the note above validate for when it runs). With write_outputs=False
    (non-zero data-parallel ranks) nothing is written to disk. model_dir_hook(model_dir) runs once the
    model directory has been prepared (writing ranks only)."""
    optim = make_adam(model.parameters(), lr)
    dev = model_device(model) if device is None else torch.device(device)
    if write_outputs:
        summaries_dir, checkpoints_dir = prepare_model_dir(model_dir, hyperopt_run, overwrite)
        writer = make_writer(summaries_dir)
        if model_dir_hook is not None:
            model_dir_hook(model_dir)
    else:
        checkpoints_dir, writer = None, _NullWriter()

    def save(obj_fn, name):
        if checkpoints_dir is not None:
            obj_fn(os.path.join(checkpoints_dir, name))

    total_steps = 0
    train_losses_dev = []
    mean_val_loss = None
    last_loss = None
    n_batches = len(train_dataloader)
    for epoch in range(epochs):
        if not epoch % epochs_til_checkpoint and epoch:
            save(lambda p: torch.save(model.state_dict(), p), "model_epoch_%04d.pth" % epoch)
            hist = torch.stack(train_losses_dev).cpu().numpy() if train_losses_dev else np.array([])
            save(lambda p: np.savetxt(p, hist), "train_losses_epoch_%04d.txt" % epoch)
        for step, (model_input, gt) in enumerate(train_dataloader):
            start_time = time.time()
            model_input = to_device(model_input, dev)
            gt = to_device(gt, dev)
            if double_precision:
                model_input = {k: v.double() for k, v in model_input.items()}
                gt = {k: v.double() for k, v in gt.items()}
            if fourier_feat_transformer is not None:
                model_input = _fourier_input(model, model_input, fourier_feat_transformer)

            # image_mse's target, staged for the SIREN forward's fused loss epilogue (fusion.py:
            # one launch for forward + data consistency + loss; the losses pick its result up)
            staged = fusion.stage_image_loss(gt["img"]) if "img" in gt else None
            try:
                model_output = model(model_input)
                losses = loss_fn(model_output, gt)
            finally:
                fusion.clear(staged)
            train_loss = compute_loss(losses, loss_schedules, total_steps, writer)
            train_losses_dev.append(train_loss.detach().reshape(()))
            summary_step = not total_steps % steps_til_summary
            if summary_step:
                writer.add_scalar("total_train_loss", float(train_loss.detach()), total_steps)
                save(lambda p: torch.save(model.state_dict(), p), "model_current.pth")
                summary_fn(model, model_input, gt, model_output, writer, total_steps)
            del model_output, losses

            train_loss = train_loss / accumulation_steps
            last_micro = (step + 1) % accumulation_steps == 0 or (step + 1 == n_batches)
            window_start = step % accumulation_steps == 0
            exchange = grad_reducer is not None and (clip_grad or last_micro)
            if exchange:
                grad_reducer.begin(delta=clip_grad and not window_start)
            train_loss.backward()
            if exchange:
                grad_reducer()
            if clip_grad:
                max_norm = 1.0 if isinstance(clip_grad, bool) else clip_grad
                torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
            if last_micro:
                optim.step()
                optim.zero_grad()

            if summary_step:
                print("Epoch %d, Total loss %0.6f, iteration time %0.6f"
                      % (epoch, float(train_loss.detach()), time.time() - start_time))
                if val_dataloader is not None:
                    mean_val_loss = validate(model, val_dataloader, loss_fn, fourier_feat_transformer, dev)
                    writer.add_scalar("val_loss", mean_val_loss, total_steps)
                    print(f"val loss (img_loss_only): {mean_val_loss}")
            last_loss = train_loss
            total_steps += 1

    save(lambda p: torch.save(model.state_dict(), p), "model_final.pth")
    losses_host = torch.stack(train_losses_dev).cpu().numpy() if train_losses_dev else np.array([])
    save(lambda p: np.savetxt(p, losses_host), "train_losses_final.txt")
    if mean_val_loss is not None:
        return mean_val_loss
    return None if last_loss is None else float(last_loss.detach()) * accumulation_steps


# When the data-parallel exchange runs inside an accumulation window (training.py:90-103): the
# reference's DDP all-reduces (averages) the accumulated .grad after every backward
# (training_ddp.py:96-109, no no_sync) and clips every micro-step. Exchanging the whole accumulated
# gradient each micro-step is right only for an average and only because the earlier part is
# already identical on every rank; with a sum it would add the earlier micro-steps W times over. So:
#   * without clipping, only the micro-step followed by optim.step() exchanges (DDP no_sync
#     semantics: one collective per optimizer step, identical result for 'mean' and 'sum');
#   * with clipping (which needs the exchanged gradient every micro-step, as in the reference), each
#     exchange after the window's first carries only what its backward added (GradAllReducer.begin
#     with delta=True), so 'sum' and 'mean' both give sum/average over ranks of every micro-step.


def _fourier_input(model, model_input, transform):
    """training.py:61-64: coords -> Fourier features, under the caller's grad mode (the reference
    transforms with autograd on in training and under no_grad in validation); a
    GaussianFourierFeatureTransform may hand the raw coordinates and B to a model that forms the
    features in its first layer (features.py)."""
    if hasattr(transform, "model_input"):
        return transform.model_input(model, model_input)
    model_input["coords"] = transform(model_input["coords"])
    return model_input


@torch.no_grad()
def validate(model, val_dataloader, loss_fn, fourier_feat_transformer, dev):
    """training.py:111-136: mean of the 'img_loss' term over the validation loader, under
    torch.no_grad() as in the reference (training.py:114)."""
    model.eval()
    vals = []
    for model_input, gt in val_dataloader:
        model_input = to_device(model_input, dev)
        gt = to_device(gt, dev)
        if fourier_feat_transformer is not None:
            model_input = _fourier_input(model, model_input, fourier_feat_transformer)
        out = model(model_input)
        vals.append(loss_fn(out, gt)["img_loss"])
    model.train()
    return float(torch.mean(torch.stack(vals)))
