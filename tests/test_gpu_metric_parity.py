"""GPU parity at the configurations BASELINE.json names, against the fp64 oracle.

  M   512^2 grid, SingleBVPNet 2-256-256-256-256-1 (modules.py:122-164): forward y AND every
      dW_l / db_l / dx, in fp32 and in bf16 mode, through the default kernels (register-resident
      forward, paired ring backward with the split-K tail reductions of pair_tail_reduce).
  C3  512^2 grid + gradients_mse (loss_functions.py:330-335, diff_operators.py:39-43), fp32:
      the analytic gradient field and the double-backward parameter gradients of one step.
  C2  256^2 IRData slice (dataio.py:507-525; / max, x2 - 1, bilinear 256^2), 5x256: 3 fp32 Adam
      steps against the oracle's training loop (training.py:19-146 restated), and a 400-step bf16
      fit whose PSNR (utils.py:593-616) stays within 0.1 dB of the fp32 path's at equal steps.

Tolerances (norm-relative ||a-b|| / ||b||, SURVEY.md §7 'Parity tolerances'):
  fp32 : forward <= 1e-5 (north_star), gradients <= 1e-4.
  bf16 : forward <= 2e-3 (fp16-operand forward, measured ~5e-4), gradients <= 2e-2 (bf16
         operands, fp32 accumulation over 2^18 rows).
The measured errors are printed (pytest -s) so a run records them.
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

TOL = {"fp32": (1e-5, 1e-4), "bf16": (2e-3, 2e-2)}


@pytest.fixture(scope="module")
def metric_reference():
    """fp64 oracle forward + backward of the metric shape (seed 0, random loss weights)."""
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    dims = orc.siren_dims(2, 256, 3, 1)
    params = orc.siren_init(dims, seed=0)
    x = orc.get_mgrid(512).unsqueeze(0)
    lw = torch.randn(1, 512 * 512, 1, generator=torch.Generator().manual_seed(5))
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    xx = x.double().requires_grad_(True)
    y = orc.siren_forward(xx, ps)
    (y * lw.double()).sum().backward()
    ref = (y.detach(), [(W.grad, b.grad) for W, b in ps], xx.grad)
    return params, x, lw, ref


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_metric_size_forward_and_every_gradient(metric_reference, precision):
    from siren_mri_amd import _native
    from siren_mri_amd.ops import siren_mlp
    params, x, lw, (y_ref, g_ref, dx_ref) = metric_reference
    assert _native.get_option("pair_tail_reduce") == 1  # the default split-K tail path is the one checked
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    xd = x.to(DEV).requires_grad_(True)
    y = siren_mlp(xd, ws, bs, precision=precision)
    (y * lw.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    ty, tg = TOL[precision]
    errs = {"y": orc.norm_rel(y.detach().cpu(), y_ref)}
    for l, ((rW, rb), w, b) in enumerate(zip(g_ref, ws, bs)):
        errs[f"dW{l}"] = orc.norm_rel(w.grad.cpu(), rW)
        errs[f"db{l}"] = orc.norm_rel(b.grad.cpu(), rb)
    errs["dx"] = orc.norm_rel(xd.grad.cpu(), dx_ref)
    print(f"\n[metric 512^2 5x256 {precision}] " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
    assert errs["y"] <= ty, errs
    for k, v in errs.items():
        if k != "y":
            assert v <= tg, (k, errs)


def test_c3_metric_size_gradients_mse_fp32():
    """Config C3 at its size: 512^2, 5x256, gradients_mse, fp32 — one step against the oracle."""
    from siren_mri_amd import dataio, diff_operators, loss_functions, modules
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    side = 512
    torch.manual_seed(0)
    m = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=3, precision="fp32").to(DEV)
    _, gt = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=side, compute_diff="gradients")[0]
    coords = dataio.get_mgrid(side)[None]
    gtg = gt["gradients"][None]
    o = m({"coords": coords.to(DEV)})
    g = diff_operators.gradient(o["model_out"], o["model_in"])
    loss = loss_functions.gradients_mse(o, {"gradients": gtg.to(DEV)})["gradients_loss"]
    loss.backward()
    torch.cuda.synchronize()

    sd = m.state_dict()
    ps = [(sd[f"net.net.{i}.0.weight"].double().cpu().clone().requires_grad_(True),
           sd[f"net.net.{i}.0.bias"].double().cpu().clone().requires_grad_(True)) for i in range(5)]
    x = coords.double().clone().requires_grad_(True)
    out = {"model_in": x, "model_out": orc.siren_forward(x, ps)}
    g_ref = orc.gradient(out["model_out"], x)
    ref = orc.gradients_mse(out, {"gradients": gtg.double()})["gradients_loss"]
    ref.backward()
    errs = {"grad": orc.norm_rel(g.detach().cpu(), g_ref.detach()),
            "loss": abs(loss.item() - ref.item()) / abs(ref.item())}
    for i, (W, b) in enumerate(ps):
        lw = m.net.net[i][0]
        errs[f"dW{i}"] = orc.norm_rel(lw.weight.grad.cpu(), W.grad)
        if b.grad is not None:
            errs[f"db{i}"] = orc.norm_rel(lw.bias.grad.cpu(), b.grad)
        else:
            assert lw.bias.grad is None
    print("\n[C3 512^2 gradients_mse fp32] " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
    assert errs["grad"] <= 1e-5 and errs["loss"] <= 1e-5, errs
    for k, v in errs.items():
        assert v <= 1e-4, (k, errs)


def _c2_fit(precision, steps, record):
    from siren_mri_amd import dataio, loss_functions, modules, training, utils
    img = dataio.irdata_image(0, 256)[None].to(DEV)
    coords = dataio.get_mgrid(256)[None].to(DEV)
    torch.manual_seed(0)
    m = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=3, precision=precision).to(DEV)
    init = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    opt = training.make_adam(m.parameters(), 1e-4)
    psnr, losses = {}, []
    for s in range(steps + 1):
        out = m({"coords": coords})
        if s in record:
            psnr[s] = utils.psnr(dataio.lin2img(out["model_out"].detach()).cpu().numpy()[0],
                                 dataio.lin2img(img).cpu().numpy()[0])
        if s == steps:
            break
        loss = loss_functions.image_mse(None, out, {"img": img}, high_freq=False)["img_loss"]
        losses.append(loss.detach())
        loss.backward()
        opt.step()
        opt.zero_grad()
    return init, [float(v) for v in torch.stack(losses).cpu()], psnr


def test_c2_irdata_fit_fp32_matches_oracle_loop():
    """C2 input path: 3 fp32 Adam steps on the 256^2 IRData slice vs the oracle's training loop."""
    from siren_mri_amd import dataio
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    init, losses, _ = _c2_fit("fp32", 3, ())
    ps = [(init[f"net.net.{i}.0.weight"], init[f"net.net.{i}.0.bias"]) for i in range(5)]
    img = dataio.irdata_image(0, 256)[None]
    ref_losses, _, _ = orc.train_steps(ps, orc.get_mgrid(256)[None], {"img": img},
                                       lambda o, gt: orc.image_mse(None, o, gt, high_freq=False), steps=3)
    print(f"\n[C2 fp32 losses] {losses} vs oracle {ref_losses}")
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)


def test_c2_irdata_bf16_psnr_tracks_fp32():
    """C2 (256^2 IRData slice, 5x256, bf16): PSNR within 0.1 dB of the fp32 path at equal steps."""
    rec = (0, 100, 200, 400)
    _, _, p32 = _c2_fit("fp32", 400, rec)
    _, _, p16 = _c2_fit("bf16", 400, rec)
    print(f"\n[C2 PSNR dB] fp32 {p32} bf16 {p16}")
    assert p32[400] > p32[0] + 10  # the fit makes progress
    for s in rec:
        assert abs(p16[s] - p32[s]) <= 0.1, (s, p16, p32)


@pytest.mark.parametrize("rows", [100_000, 65536 * 2 + 513])
def test_fwdreg_one_hidden_layer_several_rounds(rows):
    """[2, 256, 256, 1] (one hidden MFMA layer: the weight ring is never refilled) with more rows
    than one round of 256 workgroups x 256 rows: every round's x tile is read after its LDS-DMA
    landed. Oracle-checked and run-to-run bit-identical (y and the stored phase codes)."""
    from siren_mri_amd.ops import siren_mlp
    dims = [2, 256, 256, 1]
    params = orc.siren_init(dims, seed=rows % 97)
    x = torch.rand(1, rows, 2, generator=torch.Generator().manual_seed(rows)) * 2 - 1
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    outs = []
    for rep in range(2):
        junk = torch.full((64 << 20,), rep + 7, dtype=torch.uint8, device=DEV)  # dirty the pool
        del junk
        y, saved = siren_mlp(x.to(DEV), ws, bs, precision="bf16", return_saved=True)
        torch.cuda.synchronize()
        outs.append((y.detach().cpu(), saved.clone().cpu()))
    with torch.no_grad():
        y_ref = orc.siren_forward(x.double(), [(W.double(), b.double()) for W, b in params])
    assert orc.norm_rel(outs[0][0], y_ref) <= 2e-3
    assert torch.equal(outs[0][0], outs[1][0])
    # the saved buffer: prepared weights, then the phase codes of sine layer 1 (P_0 is rebuilt)
    assert torch.equal(outs[0][1][-rows * 512:], outs[1][1][-rows * 512:])


def test_metric_size_fused_loss_step_vs_oracle():
    """The bench's M step exactly as it runs (bench.py step): the staged weighted_sse (image_mse's
    1/128^2 weight) fused into the register forward's output epilogue — at 512^2 that is 1,024
    row tiles over 256 persistent workgroups, 4 rounds of per-lane partial sums and the
    workgroup ticket hand-off — then the native backward with dL/dloss as a device scalar.
    Against the fp64 oracle: the loss, y, and every dW_l / db_l at the bf16 tolerances."""
    from siren_mri_amd import dataio, fusion, loss_functions
    from siren_mri_amd.ops import siren_mlp
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    dims = orc.siren_dims(2, 256, 3, 1)
    params = orc.siren_init(dims, seed=11)
    x = orc.get_mgrid(512).unsqueeze(0)
    tgt = torch.from_numpy(dataio.smooth_random_image(512, seed=1)).float().reshape(1, -1, 1)
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    y_ref = orc.siren_forward(x.double(), ps)
    l_ref = ((y_ref - tgt.double()) ** 2).sum() * loss_functions.KSPACE_WEIGHT
    l_ref.backward()

    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    td = tgt.to(DEV)
    st = fusion.stage_image_loss(td, weight=loss_functions.KSPACE_WEIGHT)
    try:
        y = siren_mlp(x.to(DEV), ws, bs, precision="bf16")
        loss = loss_functions.weighted_sse(y, td)
        assert st is not None and st.result is not None and st.result[2] is loss  # the fused node ran
    finally:
        fusion.clear(st)
    loss.backward()
    torch.cuda.synchronize()
    errs = {"loss": abs(float(loss) - float(l_ref)) / abs(float(l_ref)),
            "y": orc.norm_rel(y.detach().cpu(), y_ref.detach())}
    for l, ((rW, rb), w, b) in enumerate(zip(ps, ws, bs)):
        errs[f"dW{l}"] = orc.norm_rel(w.grad.cpu(), rW.grad)
        errs[f"db{l}"] = orc.norm_rel(b.grad.cpu(), rb.grad)
    print("\n[M fused loss step 512^2 bf16] " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
    ty, tg = TOL["bf16"]
    assert errs["loss"] <= ty and errs["y"] <= ty, errs
    for k, v in errs.items():
        assert v <= tg, (k, errs)


def test_c4_size_fused_dc_loss_forward_vs_oracle():
    """Configs 4/5's hypo-net forward with the data consistency and the high-frequency-masked
    k-space loss in its epilogue, at C4's size (32 slices x 128^2 rows, per-slice weights,
    16 Fourier-feature inputs): y, DC(y) and the loss against the fp64 oracle
    (data_consistency.py:32-48, loss_functions.py:66-101)."""
    from siren_mri_amd import _native, loss_functions
    import siren_mri_amd.ops  # noqa: F401
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    B, N = 32, 16384
    g = torch.Generator().manual_seed(21)
    dims = [16, 256, 256, 256, 256, 2]
    ws, bs = [], []
    for l in range(len(dims) - 1):
        W, b = orc.siren_init(dims, seed=30 + l)[l]
        ws.append((W.unsqueeze(0) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))).contiguous())
        bs.append((b.unsqueeze(0) + 0.01 * torch.randn(B, dims[l + 1], generator=g)).contiguous())
    x = torch.sin(torch.rand(B, N, 16, generator=g) * 6.28)
    kspace = torch.randn(B, 2, 128, 128, generator=g) * 0.05
    mask = (torch.rand(B, 2, 128, 128, generator=g) < 0.3).float()
    k0 = mask * kspace
    tgt = kspace.permute(0, 2, 3, 1).reshape(B, N, 2).contiguous()
    with torch.no_grad():
        y_ref = orc.siren_forward(x.double(), list(zip([w.double() for w in ws], [b.double() for b in bs])))
        dc_ref = orc.data_consistency(y_ref, k0.double(), mask.double())
        l_ref = orc.image_mse(None, {"model_out": dc_ref}, {"img": tgt.double()}, high_freq=True)["img_loss"]
    hf = loss_functions.high_freq_flat(DEV)
    y, y_dc, loss, _, _ = torch.ops.siren_mri_amd.sine_mlp_fwd_loss(
        x.to(DEV), [w.to(DEV) for w in ws], [b.to(DEV) for b in bs], 30.0, _native.PREC_BF16, True, tgt.to(DEV),
        k0.to(DEV), mask.to(DEV), hf, 0.0, loss_functions.KSPACE_WEIGHT)
    torch.cuda.synchronize()
    errs = {"y": orc.norm_rel(y.cpu(), y_ref), "dc": orc.norm_rel(y_dc.cpu(), dc_ref),
            "loss": abs(float(loss) - float(l_ref)) / abs(float(l_ref))}
    print("\n[C4 fused DC + hf loss forward, 32 x 128^2, bf16] " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
    for k, v in errs.items():
        assert v <= TOL["bf16"][0], (k, errs)


def test_metric_size_fp32_fused_loss_step_vs_oracle():
    """The metric fit in fp32 (the reference's arithmetic) with the staged loss fused into the
    per-layer path's output kernel: loss, y and every gradient vs the fp64 oracle at the fp32
    tolerances."""
    from siren_mri_amd import dataio, fusion, loss_functions
    from siren_mri_amd.ops import siren_mlp
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    dims = orc.siren_dims(2, 256, 3, 1)
    params = orc.siren_init(dims, seed=12)
    x = orc.get_mgrid(512).unsqueeze(0)
    tgt = torch.from_numpy(dataio.smooth_random_image(512, seed=2)).float().reshape(1, -1, 1)
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    y_ref = orc.siren_forward(x.double(), ps)
    l_ref = ((y_ref - tgt.double()) ** 2).sum() * loss_functions.KSPACE_WEIGHT
    l_ref.backward()
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    td = tgt.to(DEV)
    st = fusion.stage_image_loss(td, weight=loss_functions.KSPACE_WEIGHT)
    try:
        y = siren_mlp(x.to(DEV), ws, bs, precision="fp32")
        loss = loss_functions.weighted_sse(y, td)
        assert st is not None and st.result is not None and st.result[2] is loss
    finally:
        fusion.clear(st)
    loss.backward()
    torch.cuda.synchronize()
    errs = {"loss": abs(float(loss) - float(l_ref)) / abs(float(l_ref)),
            "y": orc.norm_rel(y.detach().cpu(), y_ref.detach())}
    for l, ((rW, rb), w, b) in enumerate(zip(ps, ws, bs)):
        errs[f"dW{l}"] = orc.norm_rel(w.grad.cpu(), rW.grad)
        errs[f"db{l}"] = orc.norm_rel(b.grad.cpu(), rb.grad)
    print("\n[M fused loss step 512^2 fp32] " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
    ty, tg = TOL["fp32"]
    assert errs["loss"] <= ty and errs["y"] <= ty, errs
    for k, v in errs.items():
        assert v <= tg, (k, errs)
