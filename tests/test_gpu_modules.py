"""GPU: the drop-in modules and loop against the REFERENCE's recorded outputs (tests/golden).

  * SingleBVPNet forward (shared and hypernetwork-batched params) vs forward.npz
  * training.train, 10 Adam steps on the 64^2 cameraman, fp32 path vs the reference loop's own
    losses and final parameters (train_c1.npz)
  * the config-4 hypernetwork model (reduced sizes) with the reference's state_dict vs the
    reference's model_out and losses (hypernet.npz)
fp32 tolerances: 1e-5 norm-relative (north_star); bf16 path: 3e-2.
"""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-5), ("bf16", 3e-2)])
def test_singlebvpnet_forward_matches_reference(precision, tol):
    from siren_mri_amd import modules
    d = load("forward.npz")
    m = modules.SingleBVPNet(type="sine", hidden_features=64, num_hidden_layers=2, precision=precision)
    m.load_state_dict({k[len("param/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("param/")})
    m = m.to(DEV)
    out = m({"coords": torch.from_numpy(d["coords"]).to(DEV)})
    assert orc.norm_rel(out["model_out"].detach().cpu(), torch.from_numpy(d["model_out"])) < tol
    params = {k: torch.stack([v, v * 1.05]) for k, v in m.state_dict().items()}
    outb = m({"coords": torch.from_numpy(d["coords"]).to(DEV).repeat(2, 1, 1)}, params=params)
    assert orc.norm_rel(outb["model_out"].detach().cpu(), torch.from_numpy(d["batched_out"])) < tol


def test_training_train_matches_reference_loop(tmp_path):
    from siren_mri_amd import dataio, loss_functions, modules, training
    d = load("train_c1.npz")
    m = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=1, precision="fp32")
    m.load_state_dict({k[len("init/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("init/")})
    m = m.to(DEV)
    loader = [({"coords": dataio.get_mgrid(64)[None]}, {"img": torch.from_numpy(d["img"])})]
    loss_fn = lambda o, g: loss_functions.image_mse(None, o, g, high_freq=False)  # noqa: E731
    training.train(m, loader, epochs=10, lr=1e-4, steps_til_summary=1000, epochs_til_checkpoint=1000,
                   model_dir=str(tmp_path / "run"), loss_fn=loss_fn, summary_fn=lambda *a, **k: None)
    losses = np.loadtxt(tmp_path / "run" / "checkpoints" / "train_losses_final.txt")
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-5)
    sd = m.state_dict()
    for k in sd:
        assert orc.norm_rel(sd[k].cpu(), torch.from_numpy(d["final/" + k])) < 1e-4, k


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-5), ("bf16", 5e-2)])
def test_hypernetwork_forward_matches_reference(precision, tol):
    from siren_mri_amd import dataio, features, loss_functions, meta_modules
    d = load("hypernet.npz")
    model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=16, out_features=2, image_resolution=(128, 128), fourier_features_size=16, latent_dim=16,
        hidden_features=32, num_hidden_layers=1, hyper_hidden_features=16, hyper_hidden_layers=1,
        conv_kernel_size=3, num_conv_res_blocks=1, w0=30, precision=precision)
    model.load_state_dict({k[len("state/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("state/")})
    model = model.to(DEV)
    ff = features.GaussianFourierFeatureTransform(2, 8, 21, loaded_B=torch.from_numpy(d["B"]), device=DEV)
    kspace = torch.from_numpy(d["kspace"]).to(DEV)
    mask = torch.from_numpy(d["mask"].astype(np.float32)).to(DEV)
    coords = dataio.get_mgrid(128)[None].repeat(2, 1, 1).to(DEV)
    torch.backends.cudnn.allow_tf32 = False
    with torch.no_grad():
        out = model({"coords": ff(coords), "img_sparse": mask * kspace, "dc_mask": mask})
    assert orc.norm_rel(out["latent_vec"].cpu(), torch.from_numpy(d["latent"])) < 1e-4
    assert orc.norm_rel(out["model_out"].cpu(), torch.from_numpy(d["model_out"])) < tol
    gt = {"img": kspace.permute(0, 2, 3, 1).reshape(2, -1, 2)}
    hl = loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, out, gt)
    assert hl["img_loss"].item() == pytest.approx(float(d["img_loss"]), rel=max(tol, 1e-5))


def test_hypernetwork_backward_reaches_hypernet_params():
    from siren_mri_amd import dataio, features, loss_functions, meta_modules
    d = load("hypernet.npz")
    model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=16, out_features=2, image_resolution=(128, 128), fourier_features_size=16, latent_dim=16,
        hidden_features=32, num_hidden_layers=1, hyper_hidden_features=16, hyper_hidden_layers=1,
        conv_kernel_size=3, num_conv_res_blocks=1, w0=30, precision="fp32")
    model.load_state_dict({k[len("state/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("state/")})
    model = model.to(DEV)
    ff = features.GaussianFourierFeatureTransform(2, 8, 21, loaded_B=torch.from_numpy(d["B"]), device=DEV)
    kspace = torch.from_numpy(d["kspace"]).to(DEV)
    mask = torch.from_numpy(d["mask"].astype(np.float32)).to(DEV)
    coords = dataio.get_mgrid(128)[None].repeat(2, 1, 1).to(DEV)
    torch.backends.cudnn.allow_tf32 = False
    out = model({"coords": ff(coords), "img_sparse": mask * kspace, "dc_mask": mask})
    gt = {"img": kspace.permute(0, 2, 3, 1).reshape(2, -1, 2)}
    hl = loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, out, gt)
    (hl["img_loss"].mean() + hl["latent_loss"].mean() + hl["hypo_weight_loss"].mean()).backward()
    checked = 0
    for n, p in model.named_parameters():
        key = "gradnorm/" + n
        if key in d.files and p.grad is not None and n.startswith("hyper_net"):
            assert p.grad.norm().item() == pytest.approx(float(d[key]), rel=1e-3), n
            checked += 1
    assert checked > 0


@pytest.mark.parametrize("precision,tol", [("fp32", (1e-5, 1e-4)), ("bf16", (2e-3, 2e-2))])
def test_hypo256_batched_against_reference_fixture(precision, tol):
    """The configs-4/5 hypo-network at its real width (16-256-256-256-256-2, per-slice weights, the
    path HyperNetwork feeds) on the native stack against the REFERENCE's own outputs and gradients
    (hypo256.npz, tests/golden/make_golden_r3.py); bf16 runs the wide-first-layer register forward."""
    from test_oracle_golden import hypo256_params
    from siren_mri_amd import dataio, features, modules
    d = np.load(os.path.join(G, "hypo256.npz"), allow_pickle=False)
    torch.manual_seed(4)
    net = modules.SingleBVPNet(out_features=2, type="sine", in_features=16, hidden_features=256,
                               num_hidden_layers=3, precision=precision).to(DEV)
    params = {}
    for i, (W, b) in enumerate(hypo256_params()):
        params[f"net.net.{i}.0.weight"] = W.to(DEV).requires_grad_(True)
        params[f"net.net.{i}.0.bias"] = b.to(DEV).requires_grad_(True)
    ff = features.GaussianFourierFeatureTransform(2, 8, loaded_B=torch.from_numpy(d["B_ff"]), device=DEV)
    x = ff(dataio.get_mgrid(64)[None].repeat(2, 1, 1).to(DEV))
    y = net({"coords": x}, params=params)["model_out"]
    (y * torch.from_numpy(d["lw"]).to(DEV)).sum().backward()
    ty, tg = tol
    assert orc.norm_rel(y.detach().cpu(), torch.from_numpy(d["y"])) < ty
    assert orc.norm_rel(params["net.net.0.0.weight"].grad.cpu(), torch.from_numpy(d["dW0"])) < tg
    assert orc.norm_rel(params["net.net.4.0.weight"].grad.cpu(), torch.from_numpy(d["dW4"])) < tg
    norms = np.array([[params[f"net.net.{i}.0.weight"].grad.norm().item(),
                       params[f"net.net.{i}.0.bias"].grad.norm().item()] for i in range(5)])
    np.testing.assert_allclose(norms, d["grad_norms"], rtol=tg)


def test_wide_output_linear_matches_matmul_chain():
    """BatchLinear's wide-output form (the HyperNetwork heads emitting a 256x256 hypo-weight):
    forward and all three gradients equal the matmul + add chain to fp32 rounding."""
    from siren_mri_amd import modules
    torch.manual_seed(0)
    lin = modules.BatchLinear(128, 65536).to(DEV)
    x = torch.randn(32, 128, device=DEV, requires_grad=True)
    g = torch.randn(32, 65536, device=DEV)
    y = lin(x)
    y.backward(g)
    gx, gw, gb = x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()
    x2 = x.detach().clone().requires_grad_(True)
    w2 = lin.weight.detach().clone().requires_grad_(True)
    b2 = lin.bias.detach().clone().requires_grad_(True)
    y2 = x2.matmul(w2.t()) + b2.unsqueeze(-2)
    y2.backward(g)
    torch.backends.cuda.matmul.allow_tf32 = False
    assert orc.norm_rel(y.detach().cpu(), y2.detach().cpu()) < 1e-6
    assert orc.norm_rel(gx.cpu(), x2.grad.cpu()) < 1e-5
    assert orc.norm_rel(gw.cpu(), w2.grad.cpu()) < 1e-6
    assert orc.norm_rel(gb.cpu(), b2.grad.cpu()) < 1e-6
