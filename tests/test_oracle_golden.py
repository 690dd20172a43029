"""Pin the CPU oracle (oracle/siren_oracle.py) to the REFERENCE's own outputs.

tests/golden/*.npz were produced by tests/golden/make_golden.py, which imports the real
jonbmartin/siren_mri code in the build container and records what it computes. The reference
ships no known-answer tests of its own for this path, so these fixtures
are the parity anchor. Tolerances: bit-exact for init/grids (same RNG/ops); 1e-6 norm-relative
for fp32 forward/derivative outputs computed by identical torch ops; 1e-5 for 10-step training
trajectories.
"""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def params_from(d, prefix, n_layers):
    return [(torch.from_numpy(d[f"{prefix}net.net.{i}.0.weight"]), torch.from_numpy(d[f"{prefix}net.net.{i}.0.bias"]))
            for i in range(n_layers)]


def test_mgrid_and_lin2img():
    d = load("mgrid.npz")
    assert np.array_equal(orc.get_mgrid(5).numpy(), d["mgrid5"])
    assert np.array_equal(orc.get_mgrid((4, 6)).numpy(), d["mgrid4x6"])
    assert np.array_equal(orc.lin2img(torch.from_numpy(d["lin2img_in"])).numpy(), d["lin2img_out"])


@pytest.mark.parametrize("seed,hid,nh", [(0, 64, 1), (1, 64, 1), (0, 256, 3)])
def test_init_rng_order_bit_exact(seed, hid, nh):
    d = load("init.npz")
    params = orc.siren_init(orc.siren_dims(2, hid, nh, 1), seed=seed)
    for i, (W, b) in enumerate(params):
        key = f"s{seed}_h{hid}_n{nh}/net.net.{i}.0."
        assert np.array_equal(W.numpy(), d[key + "weight"])
        assert np.array_equal(b.numpy(), d[key + "bias"])


def test_forward_gradient_laplace():
    d = load("forward.npz")
    params = params_from(d, "param/", 4)
    x = torch.from_numpy(d["coords"]).clone().requires_grad_(True)
    y = orc.siren_forward(x, params)
    assert orc.norm_rel(y.detach(), torch.from_numpy(d["model_out"])) < 1e-6
    g = orc.gradient(y, x)
    assert orc.norm_rel(g.detach(), torch.from_numpy(d["gradient"])) < 1e-6
    lap = orc.laplace(y, x)
    assert orc.norm_rel(lap.detach(), torch.from_numpy(d["laplace"])) < 1e-6
    # batched (hypernetwork) weights
    pb = [(torch.stack([W, W * 1.05]), torch.stack([b, b * 1.05])) for W, b in params]
    yb = orc.siren_forward(torch.from_numpy(d["coords"]).repeat(2, 1, 1), pb)
    assert orc.norm_rel(yb.detach(), torch.from_numpy(d["batched_out"])) < 1e-6


def test_losses_and_mask():
    d = load("losses.npz")
    pred, tgt = torch.from_numpy(d["pred"]), torch.from_numpy(d["tgt"])
    assert np.array_equal(orc.create_circular_mask(129, 129, radius=20).numpy(), d["circ_mask"])
    hf = orc.image_mse(None, {"model_out": pred}, {"img": tgt})["img_loss"].item()
    plain = orc.image_mse(None, {"model_out": pred}, {"img": tgt}, high_freq=False)["img_loss"].item()
    assert hf == pytest.approx(float(d["image_mse_hf"]), rel=1e-6)
    assert plain == pytest.approx(float(d["image_mse_plain"]), rel=1e-6)
    out = {"model_out": pred, "latent_vec": torch.from_numpy(d["latent"]),
           "hypo_params": {"a": torch.from_numpy(d["hp_a"]), "b": torch.from_numpy(d["hp_b"])}}
    hl = orc.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, out, {"img": tgt})
    assert hl["img_loss"].item() == pytest.approx(float(d["hyper_img"]), rel=1e-6)
    assert hl["latent_loss"].item() == pytest.approx(float(d["hyper_latent"]), rel=1e-6)
    assert hl["hypo_weight_loss"].item() == pytest.approx(float(d["hyper_weight"]), rel=1e-6)


def test_gradients_and_laplace_mse():
    d = load("forward.npz")
    L = load("losses.npz")
    params = params_from(d, "param/", 4)
    x = torch.from_numpy(d["coords"]).clone().requires_grad_(True)
    out = {"model_in": x, "model_out": orc.siren_forward(x, params)}
    gm = orc.gradients_mse(out, {"gradients": torch.ones(1, 256, 2) * 0.3})["gradients_loss"].item()
    assert gm == pytest.approx(float(L["gradients_mse"]), rel=1e-5)
    lm = orc.laplace_mse(out, {"laplace": torch.ones(1, 256, 1) * 0.1})["laplace_loss"].item()
    assert lm == pytest.approx(float(L["laplace_mse"]), rel=1e-5)


def test_train_c1_trajectory():
    """training.train, 10 Adam steps, 64^2 cameraman, 3x256 — oracle loop vs reference loop."""
    d = load("train_c1.npz")
    params = params_from(d, "init/", 3)
    coords = orc.get_mgrid(64)[None]
    gt = {"img": torch.from_numpy(d["img"])}
    loss_fn = lambda o, g: orc.image_mse(None, o, g, high_freq=False)  # noqa: E731
    losses, final, _ = orc.train_steps(params, coords, gt, loss_fn, steps=10, lr=1e-4)
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-5)
    for i, (W, b) in enumerate(final):
        assert orc.norm_rel(W, torch.from_numpy(d[f"final/net.net.{i}.0.weight"])) < 1e-5
        assert orc.norm_rel(b, torch.from_numpy(d[f"final/net.net.{i}.0.bias"])) < 1e-5


def test_train_c3_gradient_loss_trajectory():
    d = load("train_c3.npz")
    params = params_from(d, "init/", 4)
    coords = orc.get_mgrid(32)[None]
    losses, final, _ = orc.train_steps(params, coords, {"gradients": torch.from_numpy(d["gradients"])},
                                       orc.gradients_mse, steps=10, lr=1e-4)
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4)
    for i, (W, b) in enumerate(final):
        assert orc.norm_rel(W, torch.from_numpy(d[f"final/net.net.{i}.0.weight"])) < 1e-4


def test_psnr_trajectory_first_steps():
    """Oracle reproduces the reference PSNR trajectory (steps 0/50/100) of SURVEY.md §6."""
    d = load("psnr_c1.npz")
    from PIL import Image
    from siren_mri_amd.dataio import camera_image
    u8 = camera_image()
    img = np.asarray(Image.fromarray(u8).resize((64, 64), Image.BILINEAR), dtype=np.float32) / 255.0
    img = torch.from_numpy((img - 0.5) / 0.5)
    gt = {"img": img.reshape(1, -1, 1)}
    params = orc.siren_init(orc.siren_dims(2, 256, 3, 1), seed=0)
    coords = orc.get_mgrid(64)[None]
    ps = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in params]
    opt = torch.optim.Adam(lr=1e-4, params=[t for wb in ps for t in wb])
    got = []
    for step in range(101):
        y = orc.siren_forward(coords, ps)
        if step in (0, 50, 100):
            got.append(orc.psnr(orc.lin2img(y.detach()).numpy()[0], img.numpy()[None]))
        loss = orc.image_mse(None, {"model_out": y}, gt, high_freq=False)["img_loss"]
        loss.backward()
        opt.step()
        opt.zero_grad()
    np.testing.assert_allclose(got, d["nh3_psnr"][:3], atol=1e-3)


def test_fourier_features_and_dc():
    d = load("features.npz")
    ff = orc.fourier_features(torch.from_numpy(d["x"]), torch.from_numpy(d["B"]))
    assert orc.norm_rel(ff, torch.from_numpy(d["ff"])) < 1e-6
    dc = orc.data_consistency(torch.from_numpy(d["pred"]), torch.from_numpy(d["k0"]), torch.from_numpy(d["mask"]))
    assert np.array_equal(dc.numpy(), d["dc"])


def hypo256_params(B=2):
    """The per-slice parameters of hypo256.npz (tests/golden/make_golden_r3.py `batched_params`):
    the reference init under seed 4, weights x (1 + 0.1 g), biases + 0.01 g, generator seed 11."""
    base = orc.siren_init([16, 256, 256, 256, 256, 2], seed=4)
    g = torch.Generator().manual_seed(11)
    out = []
    for W, b in base:
        Wb = (W.unsqueeze(0).repeat(B, 1, 1) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))).contiguous()
        bb = (b.unsqueeze(0).repeat(B, 1) + 0.01 * torch.randn(B, b.shape[0], generator=g)).contiguous()
        out.append((Wb, bb))
    return out


def test_hypo256_batched_siren_matches_reference():
    """The 256-wide hypo-network with per-slice weights (configs 4/5) against the reference itself."""
    d = load("hypo256.npz")
    ps = [(W.clone().requires_grad_(True), b.clone().requires_grad_(True)) for W, b in hypo256_params()]
    x = orc.fourier_features(orc.get_mgrid(64)[None].repeat(2, 1, 1), torch.from_numpy(d["B_ff"]))
    y = orc.siren_forward(x, ps)
    (y * torch.from_numpy(d["lw"])).sum().backward()
    assert orc.norm_rel(y.detach(), torch.from_numpy(d["y"])) < 1e-6
    assert orc.norm_rel(ps[0][0].grad, torch.from_numpy(d["dW0"])) < 1e-5
    assert orc.norm_rel(ps[-1][0].grad, torch.from_numpy(d["dW4"])) < 1e-5
    norms = np.array([[W.grad.norm().item(), b.grad.norm().item()] for W, b in ps])
    np.testing.assert_allclose(norms, d["grad_norms"], rtol=1e-5)
