"""GPU: analytic SIREN derivatives (tangent-stream kernels) vs the oracle's autograd in float64.

  gradient  == diff_operators.gradient (diff_operators.py:39-43)
  laplace   == diff_operators.laplace  (diff_operators.py:27-36)
  backward of gradients_mse == the reference's double backward (loss_functions.py:330-335)
  backward of laplace_mse   == the reference's triple backward (loss_functions.py:350-355)
Tolerance (fp32 path): 1e-5 norm-relative for values, 1e-4 for parameter gradients of the
gradient loss (second-order adjoints through 2^10..2^12 rows). bf16 path: 5e-2.
Also: 10 Adam steps of gradients_mse with the reference's own trajectory (train_c3.npz), and 10
Adam steps of laplace_mse against the oracle's loop (training.py:19-146 restated, float64) —
the Laplacian training trajectory has no reference fixture: parity pinned through the oracle's
autograd, whose forward laplace/laplace_mse values are pinned by forward.npz / losses.npz.
"""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _model(hidden, nh, seed, precision, out=1, inp=2):
    from siren_mri_amd import modules
    torch.manual_seed(seed)
    return modules.SingleBVPNet(out_features=out, in_features=inp, type="sine", hidden_features=hidden,
                                num_hidden_layers=nh, precision=precision).to(DEV)


def _oracle_params(m):
    sd = m.state_dict()
    L = len(m.net.net)
    return [(sd[f"net.net.{i}.0.weight"].double().cpu().clone().requires_grad_(True),
             sd[f"net.net.{i}.0.bias"].double().cpu().clone().requires_grad_(True)) for i in range(L)]


TOL = {"fp32": (1e-5, 1e-4), "bf16": (5e-2, 8e-2)}


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("side,hidden,nh,out", [(16, 64, 2, 1), (32, 256, 3, 1), (20, 128, 1, 2)])
def test_gradient_and_laplace_forward(precision, side, hidden, nh, out):
    from siren_mri_amd import diff_operators
    m = _model(hidden, nh, side, precision, out=out)
    coords = orc.get_mgrid(side)[None]
    o = m({"coords": coords.to(DEV)})
    g = diff_operators.gradient(o["model_out"], o["model_in"])
    lap = diff_operators.laplace(o["model_out"], o["model_in"])
    ps = _oracle_params(m)
    x = coords.double().clone().requires_grad_(True)
    y = orc.siren_forward(x, ps)
    g_ref = orc.gradient(y, x)
    lap_ref = orc.laplace(y, x)
    tv, _ = TOL[precision]
    assert g.shape == x.shape and lap.shape == y.shape[:-1] + (1,)
    assert orc.norm_rel(g.detach().cpu(), g_ref.detach()) < tv
    assert orc.norm_rel(lap.detach().cpu(), lap_ref.detach()) < max(tv, 1e-5) * 4


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_gradients_mse_double_backward(precision):
    from siren_mri_amd import loss_functions
    side, hidden, nh = 24, 64, 2
    m = _model(hidden, nh, 3, precision)
    coords = orc.get_mgrid(side)[None]
    gt = torch.randn(1, side * side, 2, generator=torch.Generator().manual_seed(2))
    o = m({"coords": coords.to(DEV)})
    loss = loss_functions.gradients_mse(o, {"gradients": gt.to(DEV)})["gradients_loss"]
    loss.backward()
    ps = _oracle_params(m)
    x = coords.double().clone().requires_grad_(True)
    out = {"model_in": x, "model_out": orc.siren_forward(x, ps)}
    ref = orc.gradients_mse(out, {"gradients": gt.double()})["gradients_loss"]
    ref.backward()
    tv, tg = TOL[precision]
    assert loss.item() == pytest.approx(ref.item(), rel=tv)
    for i, (W, b) in enumerate(ps):
        lw = m.net.net[i][0]
        assert orc.norm_rel(lw.weight.grad.cpu(), W.grad) < tg, f"layer {i} dW"
        if b.grad is None:  # output bias: no path to the gradient
            assert lw.bias.grad is None
        else:
            assert orc.norm_rel(lw.bias.grad.cpu(), b.grad) < tg, f"layer {i} db"


def test_batched_weights_gradient():
    """Hypernetwork-style per-sample weights through the analytic gradient."""
    from siren_mri_amd import diff_operators
    m = _model(64, 1, 5, "fp32")
    B = 3
    params = {k: torch.stack([v * (1 + 0.05 * i) for i in range(B)]) for k, v in m.state_dict().items()}
    coords = orc.get_mgrid(12)[None].repeat(B, 1, 1)
    o = m({"coords": coords.to(DEV)}, params=params)
    g = diff_operators.gradient(o["model_out"], o["model_in"])
    for bi in range(B):
        ps = [(params[f"net.net.{i}.0.weight"][bi].double().cpu(), params[f"net.net.{i}.0.bias"][bi].double().cpu())
              for i in range(3)]
        x = coords[bi:bi + 1].double().clone().requires_grad_(True)
        ref = orc.gradient(orc.siren_forward(x, ps), x)
        assert orc.norm_rel(g[bi:bi + 1].detach().cpu(), ref.detach()) < 1e-5


def test_gradient_loss_training_matches_reference(tmp_path):
    """training.train + gradients_mse (config 3 analogue, 32^2) vs the reference loop's losses."""
    from siren_mri_amd import dataio, loss_functions, modules, training
    d = np.load(os.path.join(G, "train_c3.npz"), allow_pickle=False)
    m = modules.SingleBVPNet(type="sine", hidden_features=64, num_hidden_layers=2, precision="fp32")
    m.load_state_dict({k[len("init/"):]: torch.from_numpy(d[k]) for k in d.files if k.startswith("init/")})
    m = m.to(DEV)
    loader = [({"coords": dataio.get_mgrid(32)[None]}, {"gradients": torch.from_numpy(d["gradients"])})]
    training.train(m, loader, epochs=10, lr=1e-4, steps_til_summary=1000, epochs_til_checkpoint=1000,
                   model_dir=str(tmp_path / "run"), loss_fn=loss_functions.gradients_mse,
                   summary_fn=lambda *a, **k: None)
    losses = np.loadtxt(tmp_path / "run" / "checkpoints" / "train_losses_final.txt")
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4)
    sd = m.state_dict()
    for k in sd:
        assert orc.norm_rel(sd[k].cpu(), torch.from_numpy(d["final/" + k])) < 1e-4, k


def _oracle_check_grads(m, ps, tg):
    for i, (W, b) in enumerate(ps):
        lw = m.net.net[i][0]
        assert orc.norm_rel(lw.weight.grad.cpu(), W.grad) < tg, f"layer {i} dW"
        if b.grad is None:  # output bias: no path to the derivative
            assert lw.bias.grad is None
        else:
            assert orc.norm_rel(lw.bias.grad.cpu(), b.grad) < tg, f"layer {i} db"


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("side,hidden,nh,out", [(24, 64, 2, 1), (16, 256, 3, 1), (20, 128, 1, 2)])
def test_laplace_mse_backward(precision, side, hidden, nh, out):
    from siren_mri_amd import loss_functions
    m = _model(hidden, nh, 7, precision, out=out)
    coords = orc.get_mgrid(side)[None]
    gt = torch.randn(1, side * side, 1, generator=torch.Generator().manual_seed(3)) * 100.0
    o = m({"coords": coords.to(DEV)})
    loss = loss_functions.laplace_mse(o, {"laplace": gt.to(DEV)})["laplace_loss"]
    loss.backward()
    ps = _oracle_params(m)
    x = coords.double().clone().requires_grad_(True)
    outd = {"model_in": x, "model_out": orc.siren_forward(x, ps)}
    ref = orc.laplace_mse(outd, {"laplace": gt.double()})["laplace_loss"]
    ref.backward()
    tv, tg = TOL[precision]
    assert loss.item() == pytest.approx(ref.item(), rel=max(tv, 1e-5) * 4)
    _oracle_check_grads(m, ps, tg)


def test_laplace_backward_input_grad_and_batched_weights():
    """dL/dx through the analytic Laplacian and per-sample (hypernetwork) weights."""
    from siren_mri_amd import diff_operators, modules
    torch.manual_seed(11)
    m = modules.SingleBVPNet(type="sine", hidden_features=64, num_hidden_layers=1, precision="fp32").to(DEV)
    B = 2
    params = {k: torch.stack([v * (1 + 0.03 * i) for i in range(B)]).requires_grad_(True)
              for k, v in m.state_dict().items()}
    coords = orc.get_mgrid(10)[None].repeat(B, 1, 1)
    o = m({"coords": coords.to(DEV)}, params=params)
    xin = o["model_in"]  # SingleBVPNet's detached leaf copy of the coordinates (modules.py:151)
    lap = diff_operators.laplace(o["model_out"], o["model_in"])
    wts = torch.randn(lap.shape, generator=torch.Generator().manual_seed(4))
    (lap * wts.to(DEV)).sum().backward()
    for bi in range(B):
        ps = [(params[f"net.net.{i}.0.weight"][bi].detach().double().cpu().requires_grad_(True),
               params[f"net.net.{i}.0.bias"][bi].detach().double().cpu().requires_grad_(True)) for i in range(3)]
        x = coords[bi:bi + 1].double().clone().requires_grad_(True)
        ref = orc.laplace(orc.siren_forward(x, ps), x)
        (ref * wts[bi:bi + 1].double()).sum().backward()
        for i, (W, b) in enumerate(ps):
            gW = params[f"net.net.{i}.0.weight"].grad[bi].cpu()
            assert orc.norm_rel(gW, W.grad) < 1e-4, f"sample {bi} layer {i} dW"
            if i < 2:
                assert orc.norm_rel(params[f"net.net.{i}.0.bias"].grad[bi].cpu(), b.grad) < 1e-4
        assert orc.norm_rel(xin.grad[bi:bi + 1].cpu(), x.grad) < 1e-4, f"sample {bi} dx"


def test_laplace_loss_training_matches_oracle(tmp_path):
    """training.train + laplace_mse (Poisson-style fit, 32^2, 2x64): 10 Adam steps vs the oracle."""
    from siren_mri_amd import dataio, loss_functions, modules, training
    torch.manual_seed(5)
    m = modules.SingleBVPNet(type="sine", hidden_features=64, num_hidden_layers=2, precision="fp32")
    init = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    coords = dataio.get_mgrid(32)[None]
    gt = torch.sin(3 * coords[..., :1]) * torch.cos(2 * coords[..., 1:]) * 50.0
    loader = [({"coords": coords}, {"laplace": gt})]
    training.train(m, loader, epochs=10, lr=1e-4, steps_til_summary=1000, epochs_til_checkpoint=1000,
                   model_dir=str(tmp_path / "run"), loss_fn=loss_functions.laplace_mse,
                   summary_fn=lambda *a, **k: None)
    losses = np.loadtxt(tmp_path / "run" / "checkpoints" / "train_losses_final.txt")
    ps = [(init[f"net.net.{i}.0.weight"].double(), init[f"net.net.{i}.0.bias"].double()) for i in range(4)]
    ref_losses, ref_ps, _ = orc.train_steps(ps, coords.double(), {"laplace": gt.double()}, orc.laplace_mse,
                                            steps=10, lr=1e-4)
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    for i, (W, b) in enumerate(ref_ps):
        assert orc.norm_rel(m.net.net[i][0].weight.detach().cpu(), W) < 1e-4, f"layer {i} W"


# ------------------------------------------------------------------ per-channel Jacobian, double backward
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_jacobian_and_channel_weighted_gradient(precision):
    """diff_operators.jacobian (diff_operators.py:46-59) and gradient(y, x, grad_outputs=g) with g
    varying across output channels, on the SIREN_JVP_JACOBIAN tangent-stream op; both
    differentiable (the parameter gradients of a loss on them vs the oracle's double backward)."""
    from siren_mri_amd import diff_operators
    side, out = 20, 3
    m = _model(64, 2, 13, precision, out=out)
    coords = orc.get_mgrid(side)[None]
    g = torch.randn(1, side * side, out, generator=torch.Generator().manual_seed(6))
    o = m({"coords": coords.to(DEV)})
    jac, status = diff_operators.jacobian(o["model_out"], o["model_in"])
    gr = diff_operators.gradient(o["model_out"], o["model_in"], grad_outputs=g.to(DEV))
    (gr.square().sum() + 0.5 * jac.square().sum()).backward()
    ps = _oracle_params(m)
    x = coords.double().clone().requires_grad_(True)
    y = orc.siren_forward(x, ps)
    jac_ref = torch.stack([torch.autograd.grad(y[..., c].sum(), x, create_graph=True)[0] for c in range(out)], dim=-2)
    gr_ref = torch.autograd.grad(y, x, grad_outputs=g.double(), create_graph=True)[0]
    (gr_ref.square().sum() + 0.5 * jac_ref.square().sum()).backward()
    tv, tg = TOL[precision]
    assert status == 0 and jac.shape == (1, side * side, out, 2)
    assert orc.norm_rel(jac.detach().cpu(), jac_ref.detach()) < tv
    assert orc.norm_rel(gr.detach().cpu(), gr_ref.detach()) < tv
    _oracle_check_grads(m, ps, tg)


@pytest.mark.parametrize("batched", [False, True])
def test_autograd_double_backward_through_further_ops(batched):
    """A derivative of a function OF the SIREN output (here a data-consistency-like mix with a
    channel-varying mask, data_consistency.py:32-48) w.r.t. the coordinates, through
    torch.autograd.grad(create_graph=True) — the reference's generic path (diff_operators.py:39-43)
    — then a loss on it, backward: every parameter gradient and dL/dx vs the oracle (fp32)."""
    from siren_mri_amd import modules
    torch.manual_seed(21)
    side, out = 16, 2
    m = modules.SingleBVPNet(out_features=out, type="sine", hidden_features=64, num_hidden_layers=1,
                             precision="fp32").to(DEV)
    B = 2 if batched else 1
    params = None
    if batched:
        params = {k: torch.stack([v * (1 + 0.04 * i) for i in range(B)]).requires_grad_(True)
                  for k, v in m.state_dict().items()}
    coords = orc.get_mgrid(side)[None].repeat(B, 1, 1)
    gen = torch.Generator().manual_seed(8)
    mask = (torch.rand(B, side * side, out, generator=gen) > 0.5).float()
    k0 = torch.randn(B, side * side, out, generator=gen)
    o = m({"coords": coords.to(DEV)}, params=params)
    x = o["model_in"]
    z = (1 - mask.to(DEV)) * o["model_out"] ** 2 + mask.to(DEV) * k0.to(DEV)
    dz = torch.autograd.grad(z, [x], grad_outputs=torch.ones_like(z), create_graph=True)[0]
    loss = (dz * torch.linspace(0.5, 1.5, 2, device=DEV)).square().sum()
    loss.backward()
    sd = m.state_dict() if params is None else None
    for bi in range(B):
        if batched:
            ps = [(params[f"net.net.{i}.0.weight"][bi].detach().double().cpu().requires_grad_(True),
                   params[f"net.net.{i}.0.bias"][bi].detach().double().cpu().requires_grad_(True)) for i in range(3)]
        else:
            ps = [(sd[f"net.net.{i}.0.weight"].double().cpu().clone().requires_grad_(True),
                   sd[f"net.net.{i}.0.bias"].double().cpu().clone().requires_grad_(True)) for i in range(3)]
        xr = coords[bi:bi + 1].double().clone().requires_grad_(True)
        y = orc.siren_forward(xr, ps)
        zr = (1 - mask[bi:bi + 1].double()) * y ** 2 + mask[bi:bi + 1].double() * k0[bi:bi + 1].double()
        dzr = torch.autograd.grad(zr, [xr], grad_outputs=torch.ones_like(zr), create_graph=True)[0]
        ref = (dzr * torch.linspace(0.5, 1.5, 2, dtype=torch.float64)).square().sum()
        ref.backward()
        assert orc.norm_rel(dz[bi:bi + 1].detach().cpu(), dzr.detach()) < 1e-5
        for i, (W, b) in enumerate(ps):
            gW = (params[f"net.net.{i}.0.weight"].grad[bi] if batched else m.net.net[i][0].weight.grad).cpu()
            gb = (params[f"net.net.{i}.0.bias"].grad[bi] if batched else m.net.net[i][0].bias.grad).cpu()
            assert orc.norm_rel(gW, W.grad) < 1e-4, f"sample {bi} layer {i} dW"
            assert orc.norm_rel(gb, b.grad) < 1e-4, f"sample {bi} layer {i} db"
        assert orc.norm_rel(x.grad[bi:bi + 1].cpu(), xr.grad) < 1e-4, f"sample {bi} dx"


def test_unprovided_higher_orders_raise():
    """Differentiating the SIREN's weight gradients (create_graph=True), or a derivative of the
    tangent-stream backward, raises instead of giving silent zeros."""
    from siren_mri_amd import diff_operators, modules
    torch.manual_seed(2)
    m = modules.SingleBVPNet(type="sine", hidden_features=32, num_hidden_layers=1, precision="fp32").to(DEV)
    o = m({"coords": orc.get_mgrid(8)[None].to(DEV)})
    gw = torch.autograd.grad(o["model_out"].square().sum(), list(m.parameters()), create_graph=True)
    with pytest.raises(RuntimeError, match="not provided"):
        gw[0].square().sum().backward()
    o = m({"coords": orc.get_mgrid(8)[None].to(DEV)})
    g = diff_operators.gradient(o["model_out"], o["model_in"])
    gw = torch.autograd.grad(g.square().sum(), list(m.parameters())[:2], create_graph=True)
    with pytest.raises(RuntimeError, match="not provided"):
        gw[0].sum().backward()


@pytest.mark.parametrize("order", ["gradient", "laplace", "jacobian"])
@pytest.mark.parametrize("batched", [False, True])
def test_primal_reuse_matches_recomputed_primal(order, batched):
    """The fp32 forward's saved phases as the tangent op's primal stream (y._siren_primal) give the
    same values and parameter / input gradients as the op recomputing its own primal stream."""
    from siren_mri_amd import jvp
    from siren_mri_amd.meta import get_subdict
    out = 2 if order == "jacobian" else 1
    m = _model(128, 2, 21, "fp32", out=out)
    B = 2 if batched else 1
    coords = orc.get_mgrid(20)[None].repeat(B, 1, 1).to(DEV)
    params = None
    if batched:
        params = {k: torch.stack([v * (1 + 0.03 * i) for i in range(B)]).requires_grad_(True)
                  for k, v in m.state_dict().items()}
    fn = {"gradient": jvp.siren_gradient, "laplace": jvp.siren_laplace, "jacobian": jvp.siren_jacobian}[order]
    res = []
    for use_primal in (True, False):
        m.zero_grad(set_to_none=True)
        if params is not None:
            for p in params.values():
                p.grad = None
        x = coords.clone().requires_grad_(True)
        o = m({"coords": x}, params=params)
        y = o["model_out"]
        primal = getattr(y, "_siren_primal", None)
        assert primal is not None
        sub = get_subdict(params, "net") if params is not None else None
        val = fn(o["model_in"], m.net, sub, primal=primal if use_primal else None)
        torch.manual_seed(5)
        w = torch.randn_like(val)
        (val * w).sum().backward()
        grads = [p.grad.clone() for p in (params.values() if params is not None else m.parameters())
                 if p.grad is not None]
        res.append((val.detach(), grads, o["model_in"].grad))
    (v1, g1, dx1), (v0, g0, dx0) = res
    assert orc.norm_rel(v1.cpu(), v0.cpu()) < 1e-6
    assert len(g1) == len(g0)
    for a, b in zip(g1, g0):
        assert orc.norm_rel(a.cpu(), b.cpu()) < 1e-5
    if dx0 is not None:
        assert orc.norm_rel(dx1.cpu(), dx0.cpu()) < 1e-5


@pytest.mark.parametrize("order", ["gradient", "laplace", "jacobian"])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("batched", [False, True])
def test_fused_adjoint_combine_matches_two_launches(order, precision, batched):
    """jvp_adj_kernel (the hidden layers' adjoint GEMM with the adjoint combine in its epilogue,
    option jvp_adj, default on) against the two-launch path (jvp_nt adjoint GEMM, then
    jvp_combine): the same formula on the same fp32 accumulators. Ragged rows (41^2, not a
    multiple of the 64-row tile)."""
    from siren_mri_amd import _native, jvp
    from siren_mri_amd.meta import get_subdict
    out = 2 if order == "jacobian" else 1
    m = _model(256, 3, 33, precision, out=out)
    B = 2 if batched else 1
    coords = orc.get_mgrid(41)[None].repeat(B, 1, 1).to(DEV)
    params = None
    if batched:
        params = {k: torch.stack([v * (1 + 0.03 * i) for i in range(B)]).requires_grad_(True)
                  for k, v in m.state_dict().items()}
    fn = {"gradient": jvp.siren_gradient, "laplace": jvp.siren_laplace, "jacobian": jvp.siren_jacobian}[order]
    res = []
    assert _native.get_option("jvp_adj") == 1 and _native.get_option("jvp_tn2") == 1
    for fused, tn2 in ((1, 1), (0, 1), (1, 0)):
        _native.set_option("jvp_adj", fused)
        _native.set_option("jvp_tn2", tn2)
        try:
            m.zero_grad(set_to_none=True)
            if params is not None:
                for p in params.values():
                    p.grad = None
            x = coords.clone().requires_grad_(True)
            o = m({"coords": x}, params=params)
            sub = get_subdict(params, "net") if params is not None else None
            val = fn(o["model_in"], m.net, sub)
            torch.manual_seed(5)
            w = torch.randn_like(val)
            (val * w).sum().backward()
            torch.cuda.synchronize()
            grads = [p.grad.clone() for p in (params.values() if params is not None else m.parameters())
                     if p.grad is not None]
            res.append((grads, o["model_in"].grad.clone()))
        finally:
            _native.set_option("jvp_adj", 1)
            _native.set_option("jvp_tn2", 1)
    (g1, dx1), (g0, dx0), (gt, dxt) = res
    assert len(g1) == len(g0) > 0
    # the combine's fp32 arithmetic is the two-launch path's formula; the compiler contracts its
    # products into FMAs differently in the two kernels (1-ulp differences), which the bf16 path's
    # stored adjoints can round either way
    tol = 1e-6 if precision == "fp32" else 5e-3
    for a, b in zip(g1, g0):
        assert orc.norm_rel(a.cpu(), b.cpu()) < tol
    assert orc.norm_rel(dx1.cpu(), dx0.cpu()) < tol
    # jvp_tn2 (fp32 weight gradients, all 256 rows per workgroup) vs the 128x128-tile kernel: the
    # same products, split-K sums over other row ranges (fp32 rounding)
    for a, b in zip(g1, gt):
        assert orc.norm_rel(a.cpu(), b.cpu()) < 1e-6
    assert torch.equal(dx1, dxt)


def test_create_graph_first_order_dx_without_tangent_form():
    """create_graph=True on a stack the tangent-stream kernels do not take (a sine output layer):
    the input gradient is the native first-order one (equal to create_graph=False), and only
    differentiating it again raises."""
    from siren_mri_amd.ops import siren_mlp
    g = torch.Generator().manual_seed(3)
    ws = [(torch.randn(64, 2, generator=g) * 0.5).to(DEV).requires_grad_(True),
          (torch.randn(1, 64, generator=g) * 0.1).to(DEV).requires_grad_(True)]
    bs = [torch.zeros(64, device=DEV).requires_grad_(True), torch.zeros(1, device=DEV).requires_grad_(True)]
    x = (torch.rand(1, 500, 2, generator=g) * 2 - 1).to(DEV).requires_grad_(True)
    y = siren_mlp(x, ws, bs, outermost_linear=False)
    d1 = torch.autograd.grad(y.sum(), x, create_graph=True)[0]
    y2 = siren_mlp(x, ws, bs, outermost_linear=False)
    d0 = torch.autograd.grad(y2.sum(), x)[0]
    assert torch.equal(d1.detach(), d0)
    with pytest.raises(RuntimeError, match="tangent-stream"):
        d1.square().sum().backward()


@pytest.mark.parametrize("order,inp", [("gradient", 2), ("gradient", 1), ("gradient", 3), ("jacobian", 2)])
@pytest.mark.parametrize("batched", [False, True])
def test_row_stacked_tangents_match_stream_stacked(order, inp, batched):
    """jvp_tan_kernel (the hidden layers' tangent streams stacked by ROW: one phase load and one
    cosine per operand element for the C streams; option jvp_tan, default on, fp32 with the
    forward's primal) against jvp_nt_kernel's stream-stacked rows: the same operand products and
    the same K order, so the values and every gradient are bit-identical. Ragged rows (41^2, not
    a multiple of the 64-row tile); 1..3 input dimensions."""
    from siren_mri_amd import _native, jvp
    from siren_mri_amd.meta import get_subdict
    out = 2 if order == "jacobian" else 1
    m = _model(256, 3, 35, "fp32", out=out, inp=inp)
    B = 2 if batched else 1
    g = torch.Generator().manual_seed(7)
    coords = (torch.rand(B, 41 * 41, inp, generator=g) * 2 - 1).to(DEV)
    params = None
    if batched:
        params = {k: torch.stack([v * (1 + 0.03 * i) for i in range(B)]).requires_grad_(True)
                  for k, v in m.state_dict().items()}
    fn = {"gradient": jvp.siren_gradient, "jacobian": jvp.siren_jacobian}[order]
    res = []
    assert _native.get_option("jvp_tan") == 1
    for tan in (1, 0):
        _native.set_option("jvp_tan", tan)
        try:
            m.zero_grad(set_to_none=True)
            if params is not None:
                for p in params.values():
                    p.grad = None
            x = coords.clone().requires_grad_(True)
            o = m({"coords": x}, params=params)
            primal = getattr(o["model_out"], "_siren_primal", None)
            assert primal is not None
            sub = get_subdict(params, "net") if params is not None else None
            val = fn(o["model_in"], m.net, sub, primal=primal)
            torch.manual_seed(5)
            w = torch.randn_like(val)
            (val * w).sum().backward()
            torch.cuda.synchronize()
            grads = [p.grad.clone() for p in (params.values() if params is not None else m.parameters())
                     if p.grad is not None]
            res.append((val.detach().clone(), grads, o["model_in"].grad.clone()))
        finally:
            _native.set_option("jvp_tan", 1)
    (v1, g1, dx1), (v0, g0, dx0) = res
    assert torch.equal(v1, v0)
    assert len(g1) == len(g0) > 0
    for a, b in zip(g1, g0):
        assert torch.equal(a, b)
    assert torch.equal(dx1, dx0)
