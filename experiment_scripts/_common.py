"""Shared helpers for the experiment-script counterparts (argparse instead of configargparse,
which is not installed; a printing summary instead of tensorboard image summaries)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def base_parser(batch_size=1, lr=1e-4, num_epochs=10000, epochs_til_ckpt=25, steps_til_summary=1000):
    p = argparse.ArgumentParser()
    p.add_argument("--logging_root", type=str, default="./logs")
    p.add_argument("--experiment_name", type=str, required=True)
    p.add_argument("--batch_size", type=int, default=batch_size)
    p.add_argument("--lr", type=float, default=lr)
    p.add_argument("--num_epochs", type=int, default=num_epochs)
    p.add_argument("--epochs_til_ckpt", type=int, default=epochs_til_ckpt)
    p.add_argument("--steps_til_summary", type=int, default=steps_til_summary)
    p.add_argument("--model_type", type=str, default="sine")
    p.add_argument("--precision", type=str, default="fp32", choices=["fp32", "bf16"],
                   help="arithmetic of the native SIREN stack (fp32 = reference numerics)")
    p.add_argument("--checkpoint_path", default=None)
    p.add_argument("--overwrite", action="store_true",
                   help="replace an existing logging_root/experiment_name without asking")
    return p


def psnr_summary(key="img"):
    """summary_fn(model, model_input, gt, model_output, writer, total_steps): logs PSNR."""
    from siren_mri_amd import utils

    def fn(model, model_input, gt, model_output, writer, total_steps):
        out = model_output["model_out"].detach()
        ref = gt[key].to(out.device)
        p = utils.psnr(out, ref)
        writer.add_scalar("psnr", p, total_steps)
        print(f"step {total_steps}: psnr {p:.3f} dB", flush=True)
    return fn
