"""GPU: the experiment-script counterparts run end to end for a few epochs (train_img.py,
train_poisson_grad_img.py, train_mri_neural_process.py) and leave the reference's output layout
(checkpoints/model_final.pth, train_losses_final.txt)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(script, tmp_path, *args):
    cmd = [sys.executable, os.path.join(ROOT, "experiment_scripts", script), "--logging_root", str(tmp_path),
           "--experiment_name", "run", *args]
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    ck = tmp_path / "run" / "checkpoints"
    assert (ck / "model_final.pth").exists()
    return np.atleast_1d(np.loadtxt(ck / "train_losses_final.txt"))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_train_img_script(tmp_path, precision):
    losses = run("train_img.py", tmp_path, "--num_epochs", "30", "--steps_til_summary", "10",
                 "--precision", precision)
    assert losses.shape == (30,) and losses[-1] < losses[0]


def test_train_poisson_grad_img_script(tmp_path):
    losses = run("train_poisson_grad_img.py", tmp_path, "--num_epochs", "20", "--steps_til_summary", "10")
    assert losses.shape == (20,) and losses[-1] < losses[0]


def test_train_mri_neural_process_script(tmp_path):
    losses = run("train_mri_neural_process.py", tmp_path, "--num_epochs", "2", "--batch_size", "4",
                 "--n_slices", "16", "--steps_til_summary", "2")
    assert np.all(np.isfinite(losses))
