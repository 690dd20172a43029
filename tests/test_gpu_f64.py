"""GPU: the fp64 SIREN stack (siren_mlp64_*, csrc/siren_f64.hip) — the reference's
double_precision=True training (training.py:56-58) with the model cast to float64 — against the
fp64 oracle (oracle/siren_oracle.py: FCBlock.forward restated, autograd for the gradients).

Both sides compute in IEEE double with different summation orders, so forward, every dW / db and
dx agree to ~1e-15 norm-relative (measured 1e-16 - 1.7e-15; bound 1e-13); the 3-step Adam fit
through training.train with double_precision=True reproduces the oracle's training loop losses
to 1e-11.
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _params(dims, B=None, seed=0):
    g = torch.Generator().manual_seed(seed)
    ps = []
    for i in range(len(dims) - 1):
        shape = (dims[i + 1], dims[i]) if B is None else (B, dims[i + 1], dims[i])
        bound = (np.sqrt(6 / dims[i]) / 30) if i else 1 / dims[i]
        W = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * bound
        b = (torch.rand(shape[:-1], generator=g, dtype=torch.float64) * 2 - 1) * 0.5
        ps.append((W, b))
    return ps


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("outermost_linear", [True, False])
def test_f64_forward_and_every_gradient(batched, outermost_linear):
    from siren_mri_amd.ops import siren_mlp
    dims = (3, 40, 72, 72, 2)  # widths off the 64-tiles, a ragged row count
    B, rows = (3, 333) if batched else (None, 1000)
    ps = _params(dims, B)
    g = torch.Generator().manual_seed(7)
    lead = (B, rows) if batched else (1, rows)
    x = torch.rand(lead + (dims[0],), generator=g, dtype=torch.float64) * 2 - 1
    lw = torch.randn(lead + (dims[-1],), generator=g, dtype=torch.float64)
    # oracle
    rp = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in ps]
    rx = x.clone().requires_grad_(True)
    ry = orc.siren_forward(rx, rp, outermost_linear=outermost_linear)
    (ry * lw).sum().backward()
    # native fp64
    ws = [W.to(DEV).requires_grad_(True) for W, _ in ps]
    bs = [b.to(DEV).requires_grad_(True) for _, b in ps]
    xd = x.to(DEV).requires_grad_(True)
    y = siren_mlp(xd, ws, bs, outermost_linear=outermost_linear)
    assert y.dtype == torch.float64
    (y * lw.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    errs = {"y": orc.norm_rel(y.detach().cpu(), ry.detach()), "dx": orc.norm_rel(xd.grad.cpu(), rx.grad)}
    for l, ((rW, rb), w, b) in enumerate(zip(rp, ws, bs)):
        errs[f"dW{l}"] = orc.norm_rel(w.grad.cpu(), rW.grad)
        errs[f"db{l}"] = orc.norm_rel(b.grad.cpu(), rb.grad)
    print(f"\n[fp64 batched={batched} linear={outermost_linear}] " + " ".join(f"{k} {v:.1e}" for k, v in errs.items()))
    assert max(errs.values()) < 1e-13, errs


def test_f64_is_deterministic_and_rejects_mixed_dtypes():
    from siren_mri_amd.ops import siren_mlp
    dims = (2, 64, 64, 1)
    ps = _params(dims)
    x = (torch.rand(1, 4099, 2, dtype=torch.float64) * 2 - 1).to(DEV)
    ws = [W.to(DEV).requires_grad_(True) for W, _ in ps]
    bs = [b.to(DEV).requires_grad_(True) for _, b in ps]
    outs = []
    for _ in range(2):
        for t in ws + bs:
            t.grad = None
        y = siren_mlp(x, ws, bs)
        y.square().sum().backward()
        outs.append([y.detach().clone()] + [t.grad.clone() for t in ws + bs])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    with pytest.raises(RuntimeError, match="float64"):
        siren_mlp(x, [w.float() for w in ws], [b.float() for b in bs])
    with pytest.raises(RuntimeError, match="second derivatives"):
        xg = x.clone().requires_grad_(True)
        y = siren_mlp(xg, ws, bs)
        torch.autograd.grad(y.sum(), xg, create_graph=True)[0].sum().backward()


def test_train_double_precision_matches_oracle_loop(tmp_path):
    """training.train(double_precision=True) on model.double() (training.py:56-58): 3 Adam steps of
    a 2-64-64-64-1 SIREN on a 64^2 image, per-step losses vs the oracle's loop in fp64."""
    from siren_mri_amd import loss_functions, modules, training
    torch.manual_seed(0)
    model = modules.SingleBVPNet(type="sine", in_features=2, out_features=1, hidden_features=64,
                                 num_hidden_layers=2).to(DEV).double()
    init = [(model.net.net[i][0].weight.detach().cpu().clone(), model.net.net[i][0].bias.detach().cpu().clone())
            for i in range(4)]
    coords = orc.get_mgrid(64)[None]
    img = torch.sin(3 * coords[..., :1]) * torch.cos(2 * coords[..., 1:])
    losses = []

    def loss_fn(out, gt):
        parts = loss_functions.image_mse(None, out, gt, high_freq=False)
        losses.append(float(parts["img_loss"].detach()))
        return parts

    training.train(model, [({"coords": coords}, {"img": img})], epochs=3, lr=1e-4, steps_til_summary=1000,
                   epochs_til_checkpoint=1000, model_dir=str(tmp_path / "m"), loss_fn=loss_fn,
                   summary_fn=lambda *a, **k: None, double_precision=True, write_outputs=False)
    ref, _, _ = orc.train_steps([(W.double(), b.double()) for W, b in init], coords.double(), {"img": img.double()},
                                lambda o, gt: orc.image_mse(None, o, gt, high_freq=False), steps=3)
    print(f"\n[fp64 train] {losses} vs oracle {ref}")
    np.testing.assert_allclose(losses, ref, rtol=1e-11)
