"""GPU: the forward's fused image-loss epilogue (siren_mri_amd/fusion.py)
against the unfused chain (SIREN forward -> [DataConsistencyInKspace] -> image_mse / weighted_sse on
the native k-space SSE op) on the same inputs and weights:

  * loss within 1e-5 relative (the same fp32 terms, summed in a different order);
  * y and DC(y) bit-identical (the same register forward; the DC formula of siren_kspace.hip);
  * every parameter gradient within 5e-3 norm-relative (dL/dy differs only in fp32 rounding, the
    bf16 backward then rounds the same way or one ulp apart);
  * the fused node really ran (the staged record holds its outputs) and the step launches fewer
    kernels than the unfused one.
"""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _run(step, fused):
    from siren_mri_amd import fusion
    fusion.set_enabled(fused)
    try:
        return step()
    finally:
        fusion.set_enabled(True)


def _net(hidden_layers=2, seed=0):
    from siren_mri_amd import modules
    torch.manual_seed(seed)
    return modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=hidden_layers,
                                precision="bf16").to(DEV)


def _grads(model):
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("side,high_freq", [(128, True), (128, False), (64, False), (96, True)])
def test_image_mse_fused_matches_unfused(side, high_freq):
    from siren_mri_amd import dataio, fusion, loss_functions
    model = _net()
    coords = dataio.get_mgrid(side)[None].to(DEV)
    g = torch.Generator().manual_seed(side)
    tgt = torch.randn(1, side * side, 1, generator=g).to(DEV)
    ran = []

    def step():
        model.zero_grad(set_to_none=True)
        fusion.stage_image_loss(tgt, high_freq=high_freq)
        out = model({"coords": coords})
        st = fusion.staged(DEV)
        ran.append(st is not None and st.result is not None)
        loss = loss_functions.image_mse(None, out, {"img": tgt}, high_freq=high_freq)["img_loss"]
        fusion.clear()
        (2.5 * loss).backward()
        return out["model_out"].detach().clone(), loss.detach().clone(), _grads(model)

    yf, lf, gf = _run(step, True)
    yu, lu, gu = _run(step, False)
    assert ran == [True, False]
    assert torch.equal(yf, yu)
    assert float(lf) == pytest.approx(float(lu), rel=1e-5)
    assert gf.keys() == gu.keys() and len(gf) == 8
    for k in gf:
        assert orc.norm_rel(gf[k].cpu(), gu[k].cpu()) < 5e-3, k


def test_weighted_sse_fused_matches_unfused():
    """bench.py's M step: weighted_sse(model_out, tgt) with image_mse's 1/128^2 weight."""
    from siren_mri_amd import dataio, fusion, loss_functions
    model = _net(hidden_layers=3, seed=1)
    side = 160
    coords = dataio.get_mgrid(side)[None].to(DEV)
    tgt = torch.from_numpy(dataio.smooth_random_image(side, seed=3)).float().reshape(1, -1, 1).to(DEV)
    ran = []

    def step():
        model.zero_grad(set_to_none=True)
        fusion.stage_image_loss(tgt, weight=loss_functions.KSPACE_WEIGHT)
        out = model({"coords": coords})
        loss = loss_functions.weighted_sse(out["model_out"], tgt)
        st = fusion.staged(DEV)
        ran.append(st is not None and st.result is not None and st.result[2] is loss)
        fusion.clear()
        loss.backward()
        return loss.detach().clone(), _grads(model)

    lf, gf = _run(step, True)
    lu, gu = _run(step, False)
    assert ran == [True, False]
    assert float(lf) == pytest.approx(float(lu), rel=1e-5)
    for k in gf:
        assert orc.norm_rel(gf[k].cpu(), gu[k].cpu()) < 5e-3, k


def test_fused_loss_with_other_uses_of_y():
    """A gradient arriving at y besides the loss's (here 0.1 * sum y^2) joins dL/dy: the node's
    backward forms the sum and runs the same backward."""
    from siren_mri_amd import dataio, fusion, loss_functions
    model = _net(seed=2)
    coords = dataio.get_mgrid(64)[None].to(DEV)
    tgt = torch.randn(1, 64 * 64, 1, generator=torch.Generator().manual_seed(5)).to(DEV)

    def step():
        model.zero_grad(set_to_none=True)
        fusion.stage_image_loss(tgt, high_freq=False)
        out = model({"coords": coords})
        loss = loss_functions.image_mse(None, out, {"img": tgt}, high_freq=False)["img_loss"]
        fusion.clear()
        (loss + 0.1 * (out["model_out"] ** 2).sum()).backward()
        return _grads(model)

    gf = _run(step, True)
    gu = _run(step, False)
    for k in gf:
        assert orc.norm_rel(gf[k].cpu(), gu[k].cpu()) < 5e-3, k


def test_unmatched_consumers_compute_their_own_loss():
    """A staged target the loss does not use (another target tensor, another weight) leaves the
    loss to the unfused op: same values as with fusion off."""
    from siren_mri_amd import dataio, fusion, loss_functions
    model = _net(seed=3)
    coords = dataio.get_mgrid(64)[None].to(DEV)
    tgt = torch.randn(1, 64 * 64, 1, generator=torch.Generator().manual_seed(6)).to(DEV)
    fusion.stage_image_loss(tgt, high_freq=False)
    out = model({"coords": coords})
    assert fusion.staged(DEV).result is not None
    other = tgt.clone()
    l_other = loss_functions.image_mse(None, out, {"img": other}, high_freq=False)["img_loss"]
    l_w = loss_functions.weighted_sse(out["model_out"], tgt, weight=0.5)
    fusion.clear()
    with torch.no_grad():
        y = out["model_out"]
        ref = ((y - tgt) ** 2).sum()
    assert float(l_other) == pytest.approx(float(ref) * loss_functions.KSPACE_WEIGHT, rel=1e-5)
    assert float(l_w) == pytest.approx(float(ref) * 0.5, rel=1e-5)


def _hypernet(seed=0):
    from siren_mri_amd import meta_modules
    torch.manual_seed(seed)
    return meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=16, out_features=2, image_resolution=(128, 128), fourier_features_size=16, latent_dim=16,
        hidden_features=256, num_hidden_layers=3, hyper_hidden_features=32, hyper_hidden_layers=1,
        conv_kernel_size=3, num_conv_res_blocks=1, w0=30, precision="bf16").to(DEV)


@pytest.mark.parametrize("noise", [None, 0.25])
def test_hypernetwork_dc_loss_fused_matches_unfused(noise):
    """Configs 4/5: hypernetwork -> per-slice SIREN -> DataConsistencyInKspace -> image_mse (high
    frequency mask) with the DC and the loss in the SIREN forward's epilogue."""
    from siren_mri_amd import dataio, features, fusion, loss_functions
    model = _hypernet()
    model.dc.noise_lvl = noise
    B = 3
    g = torch.Generator().manual_seed(11)
    kspace = torch.randn(B, 2, 128, 128, generator=g).to(DEV)
    mask = (torch.rand(B, 2, 128, 128, generator=g) < 0.3).float().to(DEV)
    torch.manual_seed(0)
    ff = features.GaussianFourierFeatureTransform(2, 8, 21, device=DEV)
    coords = ff(dataio.get_mgrid(128)[None].repeat(B, 1, 1).to(DEV))
    mi = {"coords": coords, "img_sparse": mask * kspace, "dc_mask": mask}
    gt = {"img": kspace.permute(0, 2, 3, 1).reshape(B, -1, 2).contiguous()}
    ran = []

    def step():
        model.zero_grad(set_to_none=True)
        fusion.stage_image_loss(gt["img"])
        out = model(mi)
        st = fusion.staged(DEV)
        ran.append(st is not None and st.result is not None and st.result[1] is out["model_out"])
        hl = loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, out, gt)
        fusion.clear()
        sum(v.mean() for v in hl.values()).backward()
        return out["model_out"].detach().clone(), hl["img_loss"].detach().clone(), _grads(model)

    yf, lf, gf = _run(step, True)
    yu, lu, gu = _run(step, False)
    assert ran == [True, False]
    assert torch.equal(yf, yu)
    assert float(lf) == pytest.approx(float(lu), rel=1e-5)
    checked = 0
    for k in gf:
        if k.startswith("hyper_net"):
            assert orc.norm_rel(gf[k].cpu(), gu[k].cpu()) < 5e-3, k
            checked += 1
    assert checked >= 4


def _launches(fn):
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return sum(1 for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA)


def test_fused_step_launches_fewer_kernels():
    from siren_mri_amd import dataio, fusion, loss_functions
    model = _net(seed=4)
    coords = dataio.get_mgrid(128)[None].to(DEV)
    tgt = torch.randn(1, 128 * 128, 1, generator=torch.Generator().manual_seed(8)).to(DEV)
    one = torch.ones((), device=DEV)

    def step():
        fusion.stage_image_loss(tgt)
        out = model({"coords": coords})
        loss = loss_functions.image_mse(None, out, {"img": tgt})["img_loss"]
        fusion.clear()
        loss.backward(one)
        model.zero_grad(set_to_none=True)

    _run(step, True)
    n_fused = _run(lambda: _launches(step), True)
    n_chain = _run(lambda: _launches(step), False)
    print(f"\n[fused loss] kernel launches per step: fused {n_fused}, unfused {n_chain}")
    assert n_fused <= n_chain - 2


def test_fused_loss_rejects_double_backward():
    from siren_mri_amd import dataio, fusion, loss_functions
    model = _net(seed=5)
    coords = dataio.get_mgrid(64)[None].to(DEV)
    tgt = torch.randn(1, 64 * 64, 1, generator=torch.Generator().manual_seed(9)).to(DEV)
    fusion.stage_image_loss(tgt, high_freq=False)
    out = model({"coords": coords})
    loss = loss_functions.image_mse(None, out, {"img": tgt}, high_freq=False)["img_loss"]
    fusion.clear()
    with pytest.raises(RuntimeError, match="double backward"):
        torch.autograd.grad(loss, list(model.parameters()), create_graph=True)


def test_two_models_staged_on_two_streams_each_get_their_own_loss():
    """Staged records are per thread and per (device, stream): two models
    fitted in one process, each staged and run on its own stream, each get their own fused loss
    (equal to the unfused loss of their own target); a forward on a stream nothing was staged for
    runs unfused."""
    from siren_mri_amd import dataio, fusion, loss_functions
    ma, mb = _net(seed=6), _net(seed=7)
    coords = dataio.get_mgrid(64)[None].to(DEV)
    g = torch.Generator().manual_seed(12)
    ta = torch.randn(1, 64 * 64, 1, generator=g).to(DEV)
    tb = 3.0 * torch.randn(1, 64 * 64, 1, generator=g).to(DEV)
    with torch.no_grad():
        ref = {}
        fusion.set_enabled(False)
        try:
            for name, m, t in (("a", ma, ta), ("b", mb, tb)):
                out = m({"coords": coords})
                ref[name] = float(loss_functions.image_mse(None, out, {"img": t}, high_freq=False)["img_loss"])
        finally:
            fusion.set_enabled(True)
    sa, sb = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        rec_a = fusion.stage_image_loss(ta, high_freq=False)
    with torch.cuda.stream(sb):
        rec_b = fusion.stage_image_loss(tb, high_freq=False)
    assert rec_a is not rec_b and fusion.staged(DEV) is None  # nothing on the default stream
    losses = {}
    for name, m, t, s, rec in (("b", mb, tb, sb, rec_b), ("a", ma, ta, sa, rec_a)):
        with torch.cuda.stream(s):
            out = m({"coords": coords})
            loss = loss_functions.image_mse(None, out, {"img": t}, high_freq=False)["img_loss"]
            assert rec.result is not None and rec.result[2] is loss  # this stream's record ran fused
            loss.backward()
            losses[name] = float(loss)
    fusion.clear(rec_a)
    assert fusion.staged(DEV) is None
    with torch.cuda.stream(sb):
        assert fusion.staged(DEV) is rec_b
    fusion.clear(rec_b)
    torch.cuda.synchronize()
    for name in ("a", "b"):
        assert losses[name] == pytest.approx(ref[name], rel=1e-5), (name, losses, ref)
    # staged on sa, run on the default stream: not picked up
    with torch.cuda.stream(sa):
        rec = fusion.stage_image_loss(ta, high_freq=False)
    out = ma({"coords": coords})
    assert rec.result is None
    fusion.clear(rec)


@pytest.mark.parametrize("side,high_freq,hidden", [(128, True, 256), (128, False, 256), (96, True, 128)])
def test_fp32_image_mse_fused_matches_unfused(side, high_freq, hidden):
    """fp32 mode (the reference's arithmetic, precision's default): the staged image loss runs in the
    per-layer path's output kernel (last_fwd_kernel's LOSS form) — y bit-identical to the unfused
    forward, the loss and every gradient at the fp32 level of a reordered sum."""
    from siren_mri_amd import dataio, fusion, loss_functions, modules
    torch.manual_seed(side + hidden)
    model = modules.SingleBVPNet(type="sine", hidden_features=hidden, num_hidden_layers=2, precision="fp32").to(DEV)
    coords = dataio.get_mgrid(side)[None].to(DEV)
    tgt = torch.randn(1, side * side, 1, generator=torch.Generator().manual_seed(side)).to(DEV)
    ran = []

    def step():
        model.zero_grad(set_to_none=True)
        st = fusion.stage_image_loss(tgt, high_freq=high_freq)
        out = model({"coords": coords})
        loss = loss_functions.image_mse(None, out, {"img": tgt}, high_freq=high_freq)["img_loss"]
        ran.append(st is not None and st.result is not None and st.result[2] is loss)
        fusion.clear(st)
        (1.5 * loss).backward()
        return out["model_out"].detach().clone(), loss.detach().clone(), _grads(model)

    yf, lf, gf = _run(step, True)
    yu, lu, gu = _run(step, False)
    assert ran == [True, False]
    assert torch.equal(yf, yu)
    assert float(lf) == pytest.approx(float(lu), rel=1e-6)
    assert gf.keys() == gu.keys() and len(gf) == 8
    for k in gf:
        assert orc.norm_rel(gf[k].cpu(), gu[k].cpu()) < 1e-6, k


def test_fp32_hypernetwork_dc_loss_fused_matches_unfused():
    """Configs 4/5's chain (DC + high-frequency-masked k-space loss) with an fp32 hypo-net: the
    DC and the loss in last_fwd_kernel's epilogue."""
    from siren_mri_amd import dataio, features, fusion, loss_functions, meta_modules
    torch.manual_seed(1)
    model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=16, out_features=2, image_resolution=(128, 128), fourier_features_size=16, latent_dim=16,
        hidden_features=128, num_hidden_layers=2, hyper_hidden_features=32, hyper_hidden_layers=1,
        conv_kernel_size=3, num_conv_res_blocks=1, w0=30, precision="fp32").to(DEV)
    model.dc.noise_lvl = 0.25
    B = 2
    g = torch.Generator().manual_seed(13)
    kspace = torch.randn(B, 2, 128, 128, generator=g).to(DEV)
    mask = (torch.rand(B, 2, 128, 128, generator=g) < 0.3).float().to(DEV)
    torch.manual_seed(0)
    ff = features.GaussianFourierFeatureTransform(2, 8, 21, device=DEV)
    coords = ff(dataio.get_mgrid(128)[None].repeat(B, 1, 1).to(DEV))
    mi = {"coords": coords, "img_sparse": mask * kspace, "dc_mask": mask}
    gt = {"img": kspace.permute(0, 2, 3, 1).reshape(B, -1, 2).contiguous()}
    ran = []

    def step():
        model.zero_grad(set_to_none=True)
        st = fusion.stage_image_loss(gt["img"])
        out = model(mi)
        ran.append(st is not None and st.result is not None and st.result[1] is out["model_out"])
        hl = loss_functions.image_hypernetwork_loss(None, 2.78e-8, 6.4e-6, out, gt)
        fusion.clear(st)
        sum(v.mean() for v in hl.values()).backward()
        return out["model_out"].detach().clone(), hl["img_loss"].detach().clone(), _grads(model)

    yf, lf, gf = _run(step, True)
    yu, lu, gu = _run(step, False)
    assert ran == [True, False]
    assert torch.equal(yf, yu)
    assert float(lf) == pytest.approx(float(lu), rel=1e-6)
    checked = 0
    for k in gf:
        if k.startswith("hyper_net"):
            assert orc.norm_rel(gf[k].cpu(), gu[k].cpu()) < 1e-5, k
            checked += 1
    assert checked >= 4
