"""Host-side API of siren_mri_amd against the reference's contract (CPU, no kernels):
parameter names and init RNG order, param routing, losses, data layouts, the training loop
(driven with the CPU oracle model) and the hypernetwork architecture/state_dict compatibility."""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc
from siren_mri_amd import (data_consistency, dataio, diff_operators, features, loss_functions, meta,
                           meta_modules, modules, training, utils)

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


@pytest.mark.parametrize("seed,hid,nh", [(0, 64, 1), (1, 64, 1), (0, 256, 3)])
def test_singlebvpnet_state_dict_matches_reference_init(seed, hid, nh):
    d = load("init.npz")
    torch.manual_seed(seed)
    m = modules.SingleBVPNet(type="sine", hidden_features=hid, num_hidden_layers=nh, sidelength=(8, 8))
    sd = m.state_dict()
    prefix = f"s{seed}_h{hid}_n{nh}/"
    ref_keys = sorted(k[len(prefix):] for k in d.files if k.startswith(prefix))
    assert sorted(sd.keys()) == ref_keys
    for k in ref_keys:
        assert np.array_equal(sd[k].numpy(), d[prefix + k]), k


def test_meta_named_parameters_order_and_subdict():
    m = modules.SingleBVPNet(type="sine", hidden_features=32, num_hidden_layers=1)
    names = [n for n, _ in m.meta_named_parameters()]
    assert names == [f"net.net.{i}.0.{w}" for i in range(3) for w in ("weight", "bias")]
    sub = meta.get_subdict(dict(m.named_parameters()), "net")
    assert list(sub.keys())[0] == "net.0.0.weight"
    assert meta.get_subdict(None, "net") is None


def test_sine_forward_on_cpu_is_the_cpu_device_path():
    """A CPU tensor runs the stack as plain PyTorch ops on the host (cpu_stack.py, config 1 "on
    CPU"): the REFERENCE's recorded forward (shared and batched params), gradient and laplace
    (forward.npz) through the package's own modules and diff_operators."""
    d = load("forward.npz")
    m = modules.SingleBVPNet(type="sine", hidden_features=64, num_hidden_layers=2)
    m.load_state_dict({k[len("param/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("param/")})
    out = m({"coords": torch.from_numpy(d["coords"])})
    assert orc.norm_rel(out["model_out"].detach(), torch.from_numpy(d["model_out"])) < 1e-5
    g = diff_operators.gradient(out["model_out"], out["model_in"])
    assert orc.norm_rel(g.detach(), torch.from_numpy(d["gradient"])) < 1e-5
    lap = diff_operators.laplace(out["model_out"], out["model_in"])
    assert orc.norm_rel(lap.detach(), torch.from_numpy(d["laplace"])) < 1e-4
    params = {k: torch.stack([v, v * 1.05]) for k, v in m.state_dict().items()}
    outb = m({"coords": torch.from_numpy(d["coords"]).repeat(2, 1, 1)}, params=params)
    assert orc.norm_rel(outb["model_out"].detach(), torch.from_numpy(d["batched_out"])) < 1e-5
    from siren_mri_amd import cpu_stack
    with pytest.raises(RuntimeError, match="CPU tensors only"):
        cpu_stack.sine_stack(torch.zeros(1, 2, device="meta"), [], [], 30.0)


def test_config1_fit_on_cpu_reproduces_reference_trajectory(tmp_path):
    """Config 1 on a GPU-less host (VERDICT r5 missing 2): experiment_scripts/train_img.py's fit —
    SingleBVPNet 2-256-256-1 (num_hidden_layers=1) on the 64^2 cameraman, image_mse, Adam 1e-4 —
    through the package's own modules on CPU tensors reproduces the reference's recorded 10-step
    training.train trajectory (train_c1.npz: losses and final parameters)."""
    d = load("train_c1.npz")
    model = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=1, sidelength=(64, 64))
    model.load_state_dict({k[len("init/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("init/")})
    loader = [({"coords": dataio.get_mgrid(64)[None]}, {"img": torch.from_numpy(d["img"])})]
    loss_fn = lambda o, g: loss_functions.image_mse(None, o, g, high_freq=False)  # noqa: E731
    training.train(model, loader, epochs=10, lr=1e-4, steps_til_summary=1000, epochs_til_checkpoint=1000,
                   model_dir=str(tmp_path / "run"), loss_fn=loss_fn, summary_fn=lambda *a, **k: None)
    losses = np.loadtxt(tmp_path / "run" / "checkpoints" / "train_losses_final.txt")
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-5)
    sd = model.state_dict()
    for i in range(3):
        k = f"net.net.{i}.0.weight"
        assert orc.norm_rel(sd[k], torch.from_numpy(d["final/" + k])) < 1e-5


def test_relu_fcblock_runs_in_torch():
    """Non-sine FCBlocks (the HyperNetwork's) are plain PyTorch and batch-broadcast like BatchLinear."""
    torch.manual_seed(0)
    blk = modules.FCBlock(8, 5, 1, 16, outermost_linear=True, nonlinearity="relu")
    z = torch.randn(3, 8)
    out = blk(z)
    assert out.shape == (3, 5)
    ref = z
    for i, layer in enumerate(blk.net):
        lin = layer[0]
        ref = ref @ lin.weight.T + lin.bias
        if i < len(blk.net) - 1:
            ref = torch.relu(ref)
    assert torch.allclose(out, ref, atol=1e-6)


def test_losses_match_reference_values():
    d = load("losses.npz")
    pred, tgt = torch.from_numpy(d["pred"]), torch.from_numpy(d["tgt"])
    assert loss_functions.image_mse(None, {"model_out": pred}, {"img": tgt})["img_loss"].item() == \
        pytest.approx(float(d["image_mse_hf"]), rel=1e-6)
    assert loss_functions.image_mse(None, {"model_out": pred}, {"img": tgt}, high_freq=False)["img_loss"].item() == \
        pytest.approx(float(d["image_mse_plain"]), rel=1e-6)
    out = {"model_out": pred, "latent_vec": torch.from_numpy(d["latent"]),
           "hypo_params": {"a": torch.from_numpy(d["hp_a"]), "b": torch.from_numpy(d["hp_b"])}}
    hl = loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, out, {"img": tgt})
    assert hl["latent_loss"].item() == pytest.approx(float(d["hyper_latent"]), rel=1e-6)
    assert hl["hypo_weight_loss"].item() == pytest.approx(float(d["hyper_weight"]), rel=1e-6)
    assert np.array_equal(utils.create_circular_mask_torch(129, 129, radius=20).numpy(), d["circ_mask"])


def test_image_mse_off_128_is_plain_sse():
    """bug 0.2 deviation: high_freq is ignored off the 128x128 grid (the reference raises)."""
    a, b = torch.randn(1, 64 * 64, 1), torch.randn(1, 64 * 64, 1)
    hf = loss_functions.image_mse(None, {"model_out": a}, {"img": b})["img_loss"]
    plain = ((a - b) ** 2).sum() / (128 * 128)
    assert torch.allclose(hf, plain)


def test_dataio_layouts():
    d = load("mgrid.npz")
    assert np.array_equal(dataio.get_mgrid(5).numpy(), d["mgrid5"])
    assert np.array_equal(dataio.get_mgrid((4, 6)).numpy(), d["mgrid4x6"])
    assert np.array_equal(dataio.lin2img(torch.from_numpy(d["lin2img_in"])).numpy(), d["lin2img_out"])


def test_camera_transform_matches_fixture():
    d = load("train_c1.npz")
    ds = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=64)
    inp, gt = ds[0]
    assert inp["coords"].shape == (4096, 2)
    assert np.array_equal(gt["img"].numpy(), d["img"][0])


def test_gradient_ground_truth_matches_fixture():
    d = load("train_c3.npz")
    ds = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=32, compute_diff="gradients")
    _, gt = ds[0]
    assert np.allclose(gt["gradients"].numpy(), d["gradients"][0], atol=1e-5)


def test_features_and_dc_match_reference():
    d = load("features.npz")
    ff = features.GaussianFourierFeatureTransform(2, 8, 21, loaded_B=torch.from_numpy(d["B"]))
    assert torch.allclose(ff(torch.from_numpy(d["x"])), torch.from_numpy(d["ff"]), atol=1e-6)
    dc = data_consistency.DataConsistencyInKspace()(torch.from_numpy(d["pred"]), torch.from_numpy(d["k0"]),
                                                     torch.from_numpy(d["mask"]))
    assert np.array_equal(dc.numpy(), d["dc"])


def test_psnr_formula():
    p = np.array([[0.5, -1.2], [0.1, 0.9]])
    t = np.array([[0.4, -1.0], [0.1, 1.0]])
    pp = np.clip(p / 2 + 0.5, 0, 1)
    tt = t / 2 + 0.5
    assert utils.psnr(p, t) == pytest.approx(10 * np.log10(1 / np.mean((pp - tt) ** 2)))


def test_training_loop_reproduces_reference_trajectory(tmp_path):
    """siren_mri_amd.training.train driving the CPU oracle model reproduces the reference's own
    training.train trajectory (losses + final params): pins the loop (Adam, loss sum, zero_grad)."""
    d = load("train_c1.npz")
    model = orc.OracleSiren(hidden_features=256, num_hidden_layers=1)
    with torch.no_grad():
        for i in range(3):
            model.weights[i].copy_(torch.from_numpy(d[f"init/net.net.{i}.0.weight"]))
            model.biases[i].copy_(torch.from_numpy(d[f"init/net.net.{i}.0.bias"]))
    loader = [({"coords": dataio.get_mgrid(64)[None]}, {"img": torch.from_numpy(d["img"])})]
    loss_fn = lambda o, g: loss_functions.image_mse(None, o, g, high_freq=False)  # noqa: E731
    ret = training.train(model, loader, epochs=10, lr=1e-4, steps_til_summary=1000, epochs_til_checkpoint=1000,
                         model_dir=str(tmp_path / "run"), loss_fn=loss_fn, summary_fn=lambda *a, **k: None)
    losses = np.loadtxt(tmp_path / "run" / "checkpoints" / "train_losses_final.txt")
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-5)
    assert ret == pytest.approx(losses[-1], rel=1e-5)
    for i in range(3):
        assert orc.norm_rel(model.weights[i].detach(), torch.from_numpy(d[f"final/net.net.{i}.0.weight"])) < 1e-5
    assert (tmp_path / "run" / "checkpoints" / "model_final.pth").exists()


def test_validate_runs_under_no_grad(tmp_path):
    """training.py:114: validation runs under torch.no_grad(), while the
    training step's Fourier transform keeps the caller's grad mode (training.py:61-64)."""
    model = orc.OracleSiren(hidden_features=16, num_hidden_layers=1)
    seen = []

    class Probe(torch.nn.Module):
        def forward(self, x):
            seen.append(torch.is_grad_enabled())
            return x

    loader = [({"coords": dataio.get_mgrid(8)[None]}, {"img": torch.zeros(1, 64, 1)})]
    loss_fn = lambda o, g: loss_functions.image_mse(None, o, g, high_freq=False)  # noqa: E731
    ret = training.validate(model, loader, loss_fn, Probe(), torch.device("cpu"))
    assert seen == [False] and isinstance(ret, float)
    seen.clear()
    training.train(model, loader, epochs=1, lr=1e-4, steps_til_summary=1, epochs_til_checkpoint=1000,
                   model_dir=str(tmp_path / "run"), loss_fn=loss_fn, summary_fn=lambda *a, **k: None,
                   val_dataloader=loader, fourier_feat_transformer=Probe())
    assert seen == [True, False]  # the training step's transform, then validation's
    out = model({"coords": dataio.get_mgrid(8)[None]})
    vals = []

    def spy(o, g):
        r = loss_fn(o, g)
        vals.append(r["img_loss"])
        return r
    training.validate(model, loader, spy, None, torch.device("cpu"))
    assert vals and vals[0].grad_fn is None and out["model_out"].grad_fn is not None


def test_hypernet_architecture_matches_reference_state_dict():
    d = load("hypernet.npz")
    model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=16, out_features=2, image_resolution=(128, 128), fourier_features_size=16, latent_dim=16,
        hidden_features=32, num_hidden_layers=1, hyper_hidden_features=16, hyper_hidden_layers=1,
        conv_kernel_size=3, num_conv_res_blocks=1, w0=30)
    sd = model.state_dict()
    ref = {k[len("state/"):]: d[k] for k in d.files if k.startswith("state/")}
    assert sorted(sd.keys()) == sorted(ref.keys())
    for k in ref:
        assert tuple(sd[k].shape) == ref[k].shape, k
    model.load_state_dict({k: torch.from_numpy(v) for k, v in ref.items()})
    names = model.hyper_net.names
    assert names == [n for n, _ in model.hypo_net.meta_named_parameters()]


def test_diff_operators_autograd_path_for_non_siren():
    x = torch.randn(1, 10, 2, requires_grad=True)
    y = (x ** 3).sum(-1, keepdim=True)
    g = diff_operators.gradient(y, x)
    assert torch.allclose(g, 3 * x ** 2)
    lap = diff_operators.laplace(y, x)
    assert torch.allclose(lap, (6 * x).sum(-1, keepdim=True))


def test_checkpoint_compat_ddp_prefix_and_b_files(tmp_path):
    """§8(f) row 4: model files with the reference DDP wrapper's "module." prefix
    (training_ddp.py:89,146) and without it (training_ddp.py:53, this package's loops) load into
    a plain SingleBVPNet; B goes to current_B_DDP_mp<rank>.pt as a bare tensor
    (train_mri_neural_process_ddp.py:254-256) and reads back with weights_only loading."""
    from siren_mri_amd import checkpoints
    torch.manual_seed(0)
    src = modules.SingleBVPNet(type="sine", hidden_features=32, num_hidden_layers=1)
    torch.manual_seed(1)
    dst = modules.SingleBVPNet(type="sine", hidden_features=32, num_hidden_layers=1)
    assert not torch.equal(src.net.net[0][0].weight, dst.net.net[0][0].weight)
    p_ddp, p_plain = tmp_path / "model_final.pth", tmp_path / "model_epoch_0005.pth"
    torch.save(checkpoints.ddp_state_dict(src), p_ddp)
    torch.save(src.state_dict(), p_plain)
    assert all(k.startswith("module.net.net.") for k in torch.load(p_ddp, weights_only=True))
    for p in (p_ddp, p_plain, str(p_ddp)):
        dst2 = modules.SingleBVPNet(type="sine", hidden_features=32, num_hidden_layers=1)
        checkpoints.load_state_dict_compat(dst2, p)
        for (k, a), (k2, b) in zip(src.state_dict().items(), dst2.state_dict().items()):
            assert k == k2 and torch.equal(a, b)
    # a state_dict with only some prefixed keys is not rewritten (strict loading then fails)
    mixed = dict(src.state_dict())
    k0 = next(iter(mixed))
    mixed["module." + k0] = mixed.pop(k0)
    with pytest.raises(RuntimeError):
        checkpoints.load_state_dict_compat(dst, mixed)
    ft = features.GaussianFourierFeatureTransform(2, mapping_size_spatial=8, scale=21)
    path = checkpoints.save_b_matrix(ft, str(tmp_path / "run"), 3)
    assert os.path.basename(path) == "current_B_DDP_mp3.pt"
    B = torch.load(path, weights_only=True)
    assert isinstance(B, torch.Tensor) and B.shape == (2, 8) and torch.equal(B, ft.get_B().cpu())
    ft2 = features.GaussianFourierFeatureTransform(2, mapping_size_spatial=8, scale=21)
    checkpoints.load_b_matrix(ft2, str(tmp_path / "run"), 3)
    assert torch.equal(ft2.get_B(), ft.get_B())


def test_fusion_staging_rules():
    """fusion.py: only a CUDA fp32 target without grad is staged; set_enabled(False) clears and
    refuses; pending() is the record until the forward stores its result; clear(record) ends the
    step; records are per thread and per (device, stream) key (no process-global slot)."""
    import threading

    from siren_mri_amd import fusion
    fusion.clear()
    cpu = torch.device("cpu")
    assert fusion.stage_image_loss(torch.zeros(1, 4, 1)) is None and fusion.staged(cpu) is None
    # a CUDA-looking record is built by hand on CPU (the rules, not the kernel)
    key = fusion.stream_key(cpu)
    st = fusion.Staged(torch.zeros(1), True, 0.5, key)
    fusion._slots()[key] = st
    assert fusion.pending(cpu) is st
    fusion.stage_dc("k0", "mask", 0.25, device=cpu)
    assert st.dc == ("k0", "mask", 0.25)
    st.result = ("y", None, "loss", False, None)
    assert fusion.pending(cpu) is None and fusion.staged(cpu) is st
    fusion.stage_dc("k1", "m1", 0.0, device=cpu)  # after the forward: no effect
    assert st.dc == ("k0", "mask", 0.25)
    # another thread sees none of this thread's records, and its own clear() leaves them alone
    seen = []

    def other():
        seen.append(fusion.staged(cpu))
        fusion.clear()
    th = threading.Thread(target=other)
    th.start()
    th.join()
    assert seen == [None] and fusion.staged(cpu) is st
    fusion.clear(None)  # an unstaged step's record: nothing to clear
    assert fusion.staged(cpu) is st
    fusion.clear(st)
    assert fusion.staged(cpu) is None
    fusion._slots()[key] = st
    fusion.set_enabled(False)
    try:
        assert fusion.staged(cpu) is None and not fusion.enabled()
    finally:
        fusion.set_enabled(True)
    fusion.clear()
    assert fusion.staged(cpu) is None