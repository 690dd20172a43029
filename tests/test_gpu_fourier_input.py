"""GPU: the Fourier-feature input formed in the SIREN's first layer (SURVEY.md §8(f) row 1:
features.py:21-41 applied by training.py:61-64, fused into the wide register forward's layer-0
prologue and the first-layer weight-gradient kernel) against the materialised features.

The kernels form the features with the same fp32 arithmetic as the fourier_features op (the fma
chain x.B, the argument 2 pi z, siren_common.h sincos_poly), so the fused path computes the SAME
network: y, the loss and every gradient equal the materialised path's (tolerances 1e-6, the
level of a reordered fp32 sum; the forward is checked for bit equality row by row, for SIREN-init
weights (the magic-form kernel) and N(0, 1/in) weights (phases past its bound: the fract form)).
"""
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _c4_run(fused, monkeypatch, steps=2):
    import bench
    from siren_mri_amd import features
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-psnr", "--no-cpu-baseline", "--no-other-configs"])
    monkeypatch.setattr(features, "FUSED_INPUT", fused)
    args = bench.parse()
    wl = bench.build("c4", args, DEV, 0, 1)
    losses = [float(wl.step()) for _ in range(steps)]
    params = [p.detach().clone() for g in wl.extra["optimizer"].param_groups for p in g["params"]]
    return losses, params


def test_c4_fused_fourier_input_matches_materialised(monkeypatch):
    from oracle import siren_oracle as orc
    l1, p1 = _c4_run(True, monkeypatch)
    l0, p0 = _c4_run(False, monkeypatch)
    print(f"\n[C4 fused vs materialised Fourier input] losses {l1} vs {l0}")
    assert l1[0] == pytest.approx(l0[0], rel=1e-6)
    assert l1[1] == pytest.approx(l0[1], rel=1e-5)
    for a, b in zip(p1, p0):
        assert orc.norm_rel(a.cpu(), b.cpu()) < 1e-5


def _hyper_case(seed=0, B=2, N=4096):
    g = torch.Generator().manual_seed(seed)
    Bm = torch.randn(2, 8, generator=g) * 3
    x = torch.rand(B, N, 2, generator=g) * 2 - 1
    shapes = [(256, 16), (256, 256), (256, 256), (2, 256)]
    ws = [torch.randn(B, o, i, generator=g) / i ** 0.5 for o, i in shapes]
    bs = [torch.randn(B, o, generator=g) * 0.1 for o, _ in shapes]
    tgt = torch.randn(B, N, 2, generator=g) * 0.1
    return Bm.to(DEV), x.to(DEV), [w.to(DEV) for w in ws], [b.to(DEV) for b in bs], tgt.to(DEV)


@pytest.mark.parametrize("init", ["siren", "randn"])
@pytest.mark.parametrize("B,N,scale", [(2, 4096, 3.0), (2, 4096, 21.0), (32, 16384, 3.0), (32, 16384, 21.0)])
def test_fused_input_forward_rows_match_materialised(B, N, scale, init):
    """y alone (no loss gradient, no backward): the forward with the features formed in layer 0's
    prologue against the forward on the materialised features, row by row. A row that differs is
    reported with its position in the 256-row workgroup tile, its 32-row wave tile and its lane
    half (the round-4 fault: the tile's last row read its coordinates as (0, 0))."""
    from siren_mri_amd import _native, features
    import siren_mri_amd.ops  # noqa: F401
    g = torch.Generator().manual_seed(7)
    Bm = (torch.randn(2, 8, generator=g) * scale).to(DEV)
    x = (torch.rand(B, N, 2, generator=g) * 2 - 1).to(DEV)
    shapes = [(256, 16), (256, 256), (256, 256), (256, 256), (2, 256)]
    if init == "siren":
        # SIREN init ranges (modules.py:641-654): first layer U(-1/in, 1/in), then U(-sqrt(6/in)/w0, ..)
        # (hidden phases within the register forward's magic-form bound)
        ws = [((torch.rand(B, o, i, generator=g) * 2 - 1) * (1 / i if k == 0 else (6 / i) ** 0.5 / 30)).to(DEV)
              for k, (o, i) in enumerate(shapes)]
    else:  # N(0, 1/in) weights: phases past the bound, the fract-form kernel
        ws = [(torch.randn(B, o, i, generator=g) / i ** 0.5).to(DEV) for o, i in shapes]
    bs = [(torch.randn(B, o, generator=g) * 0.1).to(DEV) for o, _ in shapes]
    tgt = torch.zeros(B, N, 2, device=DEV)
    bf = _native.PREC_BF16
    y1 = torch.ops.siren_mri_amd.sine_mlp_fwd_loss(x, ws, bs, 30.0, bf, True, tgt, None, None, None, 0.0, 1.0, Bm)[0]
    feats = features.fourier_features(x, Bm)
    y0, _ = torch.ops.siren_mri_amd.sine_mlp_fwd(feats, ws, bs, 30.0, bf, True, True, False)
    torch.cuda.synchronize()
    assert torch.equal(feats, torch.ops.siren_mri_amd.fourier_features(x, Bm))  # (deterministic)
    err = (y1 - y0).abs().amax(-1).reshape(-1).cpu()
    bad = torch.nonzero(err > 0).flatten()
    if bad.numel():
        r = bad % N
        report = {"rows": bad.numel(), "of": B * N, "first": bad[:8].tolist(), "max": float(err.max()),
                  "row%256==255": int((r % 256 == 255).sum()), "row%32": torch.bincount(r % 32, minlength=32).tolist()}
        pytest.fail(f"fused-input forward differs on {report}")


def _fit_grads(fused, monkeypatch):
    from siren_mri_amd import features, fusion, loss_functions
    monkeypatch.setattr(features, "FUSED_INPUT", True)
    from siren_mri_amd.ops import siren_mlp
    Bm, x, ws, bs, tgt = _hyper_case()
    ws = [w.requires_grad_(True) for w in ws]
    bs = [b.requires_grad_(True) for b in bs]
    fusion.stage_image_loss(tgt)
    try:
        if fused:
            y = siren_mlp(x, ws, bs, precision="bf16", ff_B=Bm)
        else:
            y = siren_mlp(features.fourier_features(x, Bm), ws, bs, precision="bf16")
        loss = loss_functions.image_mse(None, {"model_out": y}, {"img": tgt})["img_loss"]
    finally:
        fusion.clear()
    loss.backward()
    return y, float(loss), [w.grad for w in ws] + [b.grad for b in bs]


def test_fused_node_and_gradients(monkeypatch):
    """The fused forward + image loss node carries B (no feature tensor, no fourier_features launch)
    and its loss / gradients match the materialised features'."""
    from oracle import siren_oracle as orc
    y1, l1, g1 = _fit_grads(True, monkeypatch)
    y0, l0, g0 = _fit_grads(False, monkeypatch)
    assert getattr(y1.grad_fn, "ff_B", None) is not None
    assert getattr(y0.grad_fn, "ff_B", 0) is None
    assert torch.equal(y1, y0)
    assert l1 == pytest.approx(l0, rel=1e-6)
    for a, b in zip(g1, g0):
        if b is None:
            assert a is None
        else:
            assert orc.norm_rel(a.cpu(), b.cpu()) < 1e-6


def test_siren_mlp_ff_input_with_coordinate_gradient():  # (the default path: materialised features)
    """Raw coordinates that require grad take the materialised path: the input gradient exists
    (w.r.t. the raw coordinates, through the fourier_features op's backward)."""
    from siren_mri_amd import fusion
    from siren_mri_amd.ops import siren_mlp
    Bm, x, ws, bs, tgt = _hyper_case(seed=1, N=256)
    x.requires_grad_(True)
    fusion.stage_image_loss(tgt)
    try:
        y = siren_mlp(x, [w.requires_grad_(True) for w in ws], [b.requires_grad_(True) for b in bs],
                      precision="bf16", ff_B=Bm)
    finally:
        fusion.clear()
    y.sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()


@pytest.mark.parametrize("scale", [21.0, 3.0e3, 4.0e4])
def test_fourier_features_op_against_fp64_over_the_argument_range(scale):
    """the materialised op (and so the fused path, bit-identical to it) forms sin / cos
    with the Cody-Waite + minimax sincos_poly below kFFPolyRange (1e6 rad). Checked against fp64
    sin / cos of the SAME fp32 argument (fma chain x.B from 0, then fl(2 pi) z, emulated here in
    fp64 with one rounding per step) over grid coordinates in [-1, 1] and B scales from the configs'
    21 up to arguments of ~1e6: abs error <= 2e-7. The host's fused-path gate
    (features._fused_range_ok) admits the scales whose arguments stay inside the range."""
    import numpy as np
    from siren_mri_amd import dataio, features
    g = torch.Generator().manual_seed(3)
    B = torch.randn(2, 8, generator=g) * scale
    x = dataio.get_mgrid(128)[None]
    out = features.fourier_features(x.to(DEV), B.to(DEV)).cpu().double().numpy()[0]
    f32 = np.float32
    xn, Bn = x[0].numpy(), B.numpy()
    z = f32(np.float64(xn[:, :1]) * np.float64(Bn[0][None]))  # fma(x0, B0, 0): one rounding
    z = f32(np.float64(xn[:, 1:2]) * np.float64(Bn[1][None]) + np.float64(z))
    arg = np.float64(f32(np.float64(f32(2 * np.pi)) * np.float64(z)))
    err_s = np.abs(out[:, :8] - np.sin(arg)).max()
    err_c = np.abs(out[:, 8:] - np.cos(arg)).max()
    print(f"\n[fourier_features vs fp64] scale {scale}: max |arg| {np.abs(arg).max():.3g}, "
          f"sin err {err_s:.2e}, cos err {err_c:.2e}")
    assert err_s <= 2e-7 and err_c <= 2e-7
    inside = 2 * np.pi * np.abs(Bn).sum(0).max() < features.FF_POLY_RANGE
    assert features._fused_range_ok(B) == inside
    assert features.GaussianFourierFeatureTransform(2, 8, loaded_B=B)._fused_ok == inside


def test_fused_fourier_gate_rejects_out_of_range_B():
    """A B whose arguments could leave the in-kernel range on [-1, 1] coordinates is handed to the
    model materialised (the op's kernel takes the far-range sin / cos past 1e6), never fused."""
    from siren_mri_amd import features
    ff = features.GaussianFourierFeatureTransform(2, 8, loaded_B=torch.full((2, 8), 1.0e5), device=DEV)

    class M(torch.nn.Module):
        fourier_input = True
    mi = ff.model_input(M(), {"coords": torch.zeros(1, 4, 2, device=DEV)})
    assert "fourier_B" not in mi and mi["coords"].shape == (1, 4, 16)
