"""GPU: the register-resident forward with a wide first layer (5..16 inputs: the Fourier-feature
coordinates of configs 4/5, features.py:31-41 -> modules.py:16-27), against the fp64 oracle.

Layer 0 runs as one f16 MFMA K step split into hi + lo halves (siren_fwdreg.hip, C = 16 form),
the hidden layers as in the narrow form; P_0 is kept and the backward runs layer 1 on the paired
ring kernels and layer 0 on the per-layer kernels. Tolerances as tests/test_gpu_metric_parity.py
(bf16 mode: forward 2e-3, gradients 2e-2, norm-relative)."""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _params(dims, B, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for l in range(len(dims) - 1):
        W, b = orc.siren_init(dims, seed=seed + l)[l]
        if B is not None:
            W = (W.unsqueeze(0).repeat(B, 1, 1) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))).contiguous()
            b = (b.unsqueeze(0).repeat(B, 1) + 0.01 * torch.randn(B, dims[l + 1], generator=g)).contiguous()
        out.append((W, b))
    return out


def _check(dims, B, N, seed, tol=(2e-3, 2e-2), need_dx=False):
    from siren_mri_amd import _native
    from siren_mri_amd.ops import siren_mlp
    assert _native.get_option("fused_forward_reg") == 1
    params = _params(dims, B, seed)
    g = torch.Generator().manual_seed(seed + 100)
    lead = (B if B is not None else 1, N)
    x = torch.sin(torch.rand(*lead, dims[0], generator=g) * 6.28)  # Fourier-feature-like inputs
    lw = torch.randn(*lead, dims[-1], generator=g)
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    xx = x.double().requires_grad_(need_dx)
    y_ref = orc.siren_forward(xx, ps)
    (y_ref * lw.double()).sum().backward()
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    xd = x.to(DEV).requires_grad_(need_dx)
    y = siren_mlp(xd, ws, bs, precision="bf16")
    (y * lw.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    errs = {"y": orc.norm_rel(y.detach().cpu(), y_ref.detach())}
    # the last rows of every weight set: their inputs come through 16-byte loads that cross the end
    # of x (bounded per dword by the buffer resource); a dropped input would show as an O(1) row
    # error that the norm over ~10^5 rows hides
    yl, rl = y.detach().cpu()[..., -3:, :], y_ref.detach()[..., -3:, :]
    scale = float(y_ref.detach().pow(2).mean().sqrt())
    assert float((yl - rl).abs().max()) <= 0.05 * scale, (yl, rl)
    for l, (w, b, (rW, rb)) in enumerate(zip(ws, bs, ps)):
        errs[f"dW{l}"] = orc.norm_rel(w.grad.cpu(), rW.grad)
        errs[f"db{l}"] = orc.norm_rel(b.grad.cpu(), rb.grad)
    if need_dx:
        errs["dx"] = orc.norm_rel(xd.grad.cpu(), xx.grad)
    print(f"\n[wide {dims} B={B} N={N}] " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()))
    assert errs["y"] <= tol[0], errs
    for k, v in errs.items():
        assert v <= tol[1] or k == "y", (k, errs)
    return y.detach()


@pytest.mark.parametrize("need_dx", [False, True])
def test_config4_siren_batched_32x16384(need_dx):
    # the hypo-net of configs 4/5 (reference config hyperoptIV_homebrew): 8 Fourier features -> 16
    # inputs, 3 hidden x 256, 2 outputs, 32 slices of 128^2 coordinates with per-slice weights.
    # need_dx: SingleBVPNet's coordinate leaf requires grad, so the models ask for dx (the
    # first_dx_wide MFMA launch beside first_bwd_wide)
    _check([16, 256, 256, 256, 256, 2], 32, 16384, seed=3, need_dx=need_dx)


def test_config4_small_siren_in120_32x16384():
    # hyperoptIV_homebrew_small (train_mri_neural_process_ddp.py:114-128): 60 Fourier features ->
    # 120 inputs, past the register forward's 16; runs on the per-layer bf16 kernels (MFMA first layer
    # on bf16 x and W_0, no hi/lo split: y ~5e-3 norm-relative, the bf16-operand forward's level)
    _check([120, 256, 256, 256, 256, 2], 32, 16384, seed=4, tol=(1e-2, 2e-2))


@pytest.mark.parametrize("C", [5, 7, 12, 16])
def test_wide_inputs_shared_ragged(C):
    _check([C, 256, 256, 256, 1], None, 70000 + C, seed=C, need_dx=True)


def test_wide_weight_gradient_kernel_generic_inputs():
    # first_bwd_wide_kernel's runtime-C form (C != 16, no input gradient), ragged rows, per-set weights
    _check([12, 256, 256, 256, 1], None, 70001, seed=5)
    _check([7, 256, 256, 256, 2], 3, 5003, seed=6)


def test_wide_one_hidden_layer_and_six():
    _check([16, 256, 256, 2], None, 3001, seed=1)
    _check([9, 256, 256, 256, 256, 256, 256, 256, 1], None, 1000, seed=2)


def test_wide_forward_deterministic():
    from siren_mri_amd.ops import siren_mlp
    dims = [16, 256, 256, 256, 256, 2]
    params = _params(dims, 4, 9)
    x = torch.sin(torch.rand(4, 5000, 16, generator=torch.Generator().manual_seed(1)) * 6.28).to(DEV)
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    outs = []
    for rep in range(3):
        junk = torch.full((64 << 20,), rep + 7, dtype=torch.uint8, device=DEV)
        del junk
        y, saved = siren_mlp(x, ws, bs, precision="bf16", return_saved=True)
        torch.cuda.synchronize()
        outs.append((y.cpu(), saved.cpu()))
    rows = 4 * 5000
    for y, sv in outs[1:]:
        assert torch.equal(y, outs[0][0])
        # P_0 .. P_3 (the last 4 phase regions): identical codes
        assert torch.equal(sv[-4 * rows * 512:], outs[0][1][-4 * rows * 512:])


def test_fourier_features_native_vs_reference():
    """siren_mri_amd::fourier_features (one launch) against the reference's recorded output
    (features.npz, features.py:31-41) and, for its x-gradient, the oracle's autograd."""
    import os

    import numpy as np
    from siren_mri_amd.features import GaussianFourierFeatureTransform
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "features.npz"), allow_pickle=False)
    ff = GaussianFourierFeatureTransform(2, 8, loaded_B=torch.from_numpy(d["B"]), device=DEV)
    x = torch.from_numpy(d["x"]).to(DEV).requires_grad_(True)
    out = ff(x)
    assert orc.norm_rel(out.detach().cpu(), torch.from_numpy(d["ff"])) < 2e-5
    g = torch.randn(out.shape, generator=torch.Generator().manual_seed(2))
    (out * g.to(DEV)).sum().backward()
    xr = torch.from_numpy(d["x"]).double().requires_grad_(True)
    (orc.fourier_features(xr, torch.from_numpy(d["B"]).double()) * g.double()).sum().backward()
    assert orc.norm_rel(x.grad.cpu(), xr.grad) < 1e-4
