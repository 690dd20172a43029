"""GPU parity of the native SIREN layer stack (siren_mlp, C ABI siren_mlp_forward/backward)
against the CPU oracle (oracle/siren_oracle.py, a restatement of modules.py:11-97).

Tolerances (norm-relative, ||a-b||/||b||, per SURVEY.md §7 'Parity tolerances'):
  fp32 mode : forward <= 1e-5 (north_star), gradients <= 1e-4 (fp32 reduction order over up
              to 2^18 rows differs from the CPU's)
  bf16 mode : forward <= 3e-2, gradients <= 5e-2 (bf16 operands, fp32 accumulation)
The reference is the oracle evaluated in float64 on the same fp32 parameters.
"""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _ref(x, params, w0=30.0, outermost_linear=True, loss_w=None):
    ps = [(W.double().clone().requires_grad_(True), b.double().clone().requires_grad_(True))
          for W, b in params]
    xx = x.double().clone().requires_grad_(True)
    y = orc.siren_forward(xx, ps, w0, outermost_linear)
    lw = loss_w.double() if loss_w is not None else torch.ones_like(y)
    (y * lw).sum().backward()
    return y.detach(), [(W.grad, b.grad) for W, b in ps], xx.grad


def _run(x, params, precision, w0=30.0, outermost_linear=True, loss_w=None):
    from siren_mri_amd.ops import siren_mlp
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    xd = x.to(DEV).requires_grad_(True)
    y = siren_mlp(xd, ws, bs, w0=w0, precision=precision, outermost_linear=outermost_linear)
    lw = loss_w.to(DEV) if loss_w is not None else torch.ones_like(y)
    (y * lw).sum().backward()
    torch.cuda.synchronize()
    return y.detach().cpu(), [(w.grad.cpu(), b.grad.cpu()) for w, b in zip(ws, bs)], xd.grad.cpu()


TOL = {"fp32": (1e-5, 1e-4), "bf16": (3e-2, 5e-2)}


def _check(x, params, precision, **kw):
    torch.manual_seed(123)
    y_ref, g_ref, dx_ref = _ref(x, params, **kw)
    y, g, dx = _run(x, params, precision, **kw)
    ty, tg = TOL[precision]
    ey = orc.norm_rel(y, y_ref)
    assert ey <= ty, f"forward norm-rel {ey:.3e} > {ty}"
    for l, ((dW, db), (rW, rb)) in enumerate(zip(g, g_ref)):
        eW, eb = orc.norm_rel(dW, rW), orc.norm_rel(db, rb)
        assert eW <= tg, f"layer {l} dW norm-rel {eW:.3e} > {tg}"
        assert eb <= tg, f"layer {l} db norm-rel {eb:.3e} > {tg}"
    edx = orc.norm_rel(dx, dx_ref)
    assert edx <= tg, f"dx norm-rel {edx:.3e} > {tg}"
    return ey


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("side,hidden,nh", [(32, 256, 3), (33, 64, 1), (20, 128, 2), (64, 256, 1)])
def test_plain_siren(precision, side, hidden, nh):
    dims = orc.siren_dims(2, hidden, nh, 1)
    params = orc.siren_init(dims, seed=side)
    x = orc.get_mgrid(side).unsqueeze(0)
    lw = torch.randn(1, side * side, 1, generator=torch.Generator().manual_seed(5))
    _check(x, params, precision, loss_w=lw)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_batched_weights_hypernet_shape(precision):
    # configs 4/5 shape at reduced size: B weight sets, Fourier-feature input (2m = 16), out 2
    B, N = 3, 300
    dims = [16, 256, 256, 256, 256, 2]
    g = torch.Generator().manual_seed(7)
    params = []
    for l in range(len(dims) - 1):
        base = orc.siren_init(dims, seed=l)[l]
        W = base[0].unsqueeze(0).repeat(B, 1, 1) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))
        b = base[1].unsqueeze(0).repeat(B, 1) + 0.01 * torch.randn(B, dims[l + 1], generator=g)
        params.append((W.contiguous(), b.contiguous()))
    x = torch.rand(B, N, 16, generator=g) * 2 - 1
    lw = torch.randn(B, N, 2, generator=g)
    _check(x, params, precision, loss_w=lw)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("dims", [[2, 96, 96, 1], [2, 160, 224, 96, 1], [3, 32, 480, 2]])
def test_irregular_hidden_widths(precision, dims):
    # widths that are multiples of 32 but not powers of two (LDS swizzle must stay inside a row);
    # fp32 widths above 256 run the two-chunk K = 512 form of the fp32 GEMM
    params = orc.siren_init(dims, seed=sum(dims))
    x = torch.rand(1, 517, dims[0], generator=torch.Generator().manual_seed(2)) * 2 - 1
    _check(x, params, precision)


def _wide_params(dims, B, seed):
    g = torch.Generator().manual_seed(seed)
    params = []
    for l in range(len(dims) - 1):
        base = orc.siren_init(dims, seed=seed + l)[l]
        if B is None:
            params.append(base)
            continue
        W = base[0].unsqueeze(0).repeat(B, 1, 1) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))
        b = base[1].unsqueeze(0).repeat(B, 1) + 0.01 * torch.randn(B, dims[l + 1], generator=g)
        params.append((W.contiguous(), b.contiguous()))
    return params


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("C", [20, 120, 122])
def test_wide_input_first_layer(precision, C):
    # in_features > 16 (Fourier-feature coordinates, configs 4/5: 2*60 = 120) run layer 0 on the
    # MFMA GEMM path; C = 122 exercises the unaligned-row load path
    dims = [C, 256, 256, 2]
    params = _wide_params(dims, None, C)
    g = torch.Generator().manual_seed(C)
    x = torch.sin(torch.rand(1, 700, C, generator=g) * 6.28)
    lw = torch.randn(1, 700, 2, generator=g)
    _check(x, params, precision, loss_w=lw)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_wide_input_batched_config4_shape(precision):
    # config 4's SIREN (in 120, 3 hidden x 256, out 2) with per-slice hypernetwork weights
    B, N = 3, 333
    dims = [120, 256, 256, 256, 256, 2]
    params = _wide_params(dims, B, 11)
    g = torch.Generator().manual_seed(4)
    x = torch.sin(torch.rand(B, N, 120, generator=g) * 6.28)
    lw = torch.randn(B, N, 2, generator=g)
    _check(x, params, precision, loss_w=lw)


def test_wide_input_config5_shape_bf16():
    # config 5's SIREN widths (in 2*228 = 456, hidden 512, out 2), reduced depth and rows
    B, N = 2, 130
    dims = [456, 512, 512, 2]
    params = _wide_params(dims, B, 5)
    g = torch.Generator().manual_seed(5)
    x = torch.sin(torch.rand(B, N, 456, generator=g) * 6.28)
    _check(x, params, "bf16")


def test_wide_input_fp32_456():
    """Config 5's Fourier-feature width (2 x 228 = 456 inputs) in fp32: layer 0 on the two-chunk
    K = 512 fp32 GEMM (it was rejected before round 4)."""
    dims = [456, 256, 1]
    params = orc.siren_init(dims, seed=1)
    x = torch.rand(1, 300, 456, generator=torch.Generator().manual_seed(6)) * 2 - 1
    _check(x, params, "fp32")


def test_wide_input_bound():
    from siren_mri_amd.ops import siren_mlp
    from siren_mri_amd._native import NativeError
    dims = [600, 256, 1]
    params = orc.siren_init(dims, seed=1)
    for prec in ("fp32", "bf16"):
        with pytest.raises(NativeError, match="in_features"):
            siren_mlp(torch.zeros(1, 4, 600, device=DEV), [W.to(DEV) for W, _ in params],
                      [b.to(DEV) for _, b in params], precision=prec)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_sine_output_layer(precision):
    dims = [3, 64, 64, 4]
    params = orc.siren_init(dims, seed=3)
    x = torch.rand(1, 129, 3, generator=torch.Generator().manual_seed(1)) * 2 - 1
    _check(x, params, precision, outermost_linear=False)


def test_wide_hidden_bf16():
    # 512-wide hidden layers use the K=512 bf16 kernel variant (32-row tiles)
    dims = orc.siren_dims(2, 512, 1, 1)
    params = orc.siren_init(dims, seed=9)
    x = orc.get_mgrid(23).unsqueeze(0)
    _check(x, params, "bf16")


def test_hidden_width_bound():
    """Hidden widths above 512 are rejected in both arithmetics (fp32 supports up to 512 since
    round 4: test_fp32_hidden_512)."""
    from siren_mri_amd.ops import siren_mlp
    from siren_mri_amd._native import NativeError
    dims = orc.siren_dims(2, 544, 1, 1)
    params = orc.siren_init(dims, seed=9)
    for prec in ("fp32", "bf16"):
        with pytest.raises(NativeError, match="hidden width"):
            siren_mlp(torch.zeros(1, 4, 2, device=DEV), [W.to(DEV) for W, _ in params],
                      [b.to(DEV) for _, b in params], precision=prec)


def test_metric_size_fp32_forward():
    # the metric configuration (512^2, 5x256) forward in fp32 against the fp64 oracle
    from siren_mri_amd.ops import siren_mlp
    dims = orc.siren_dims(2, 256, 3, 1)
    params = orc.siren_init(dims, seed=0)
    x = orc.get_mgrid(512).unsqueeze(0)
    with torch.no_grad():
        y_ref = orc.siren_forward(x.double(), [(W.double(), b.double()) for W, b in params])
        y = siren_mlp(x.to(DEV), [W.to(DEV) for W, _ in params], [b.to(DEV) for _, b in params],
                      precision="fp32")
    assert orc.norm_rel(y.cpu(), y_ref) <= 1e-5


def test_device_selects_the_path(monkeypatch):
    """A CPU tensor takes the host path (cpu_stack.py, config 1 on a GPU-less host); a CUDA tensor
    takes the native kernels and never reaches the host path (the GPU-side result is checked
    against the oracle elsewhere; here the host path is made to raise while the CUDA call runs)."""
    from siren_mri_amd import cpu_stack
    from siren_mri_amd.ops import siren_mlp
    dims = orc.siren_dims(2, 64, 1, 1)
    params = orc.siren_init(dims, seed=0)
    x = orc.get_mgrid(6)[None]
    y_cpu = siren_mlp(x, [W for W, _ in params], [b for _, b in params])
    assert y_cpu.device.type == "cpu"
    assert orc.norm_rel(y_cpu, orc.siren_forward(x, params)) < 1e-6

    def refuse(*a, **k):
        raise AssertionError("a CUDA tensor reached the host path")
    monkeypatch.setattr(cpu_stack, "sine_stack", refuse)
    y = siren_mlp(x.to(DEV), [W.to(DEV) for W, _ in params], [b.to(DEV) for _, b in params], precision="fp32")
    assert y.is_cuda and orc.norm_rel(y.cpu(), y_cpu) < 1e-5


@pytest.mark.parametrize("hidden,nh,B", [(256, 3, 1), (128, 2, 2), (512, 1, 1), (64, 2, 3)])
def test_fp32_row_stacked_layers_equal_nt_f32(hidden, nh, B):
    """The fp32 hidden layers' forward and input gradient on the row-stacked tile (jvp_tan_kernel
    JT_FWD / JT_DX, option f32_rows, default on) against nt_f32_kernel: the same products, K order
    and epilogues, so y and dx are bit-identical; the 256-wide layers' weight gradients (jvp_tn2
    over the primal stream, under the same option) split the row sum differently from tn_dw_kernel:
    fp32 rounding level (1e-6). Ragged rows (37^2), shared and batched weights, hidden 64 .. 512."""
    from siren_mri_amd import _native
    from siren_mri_amd.ops import siren_mlp
    dims = orc.siren_dims(2, hidden, nh, 1)
    params = orc.siren_init(dims, seed=hidden + nh)
    g = torch.Generator().manual_seed(9)
    x = (torch.rand(B, 37 * 37, 2, generator=g) * 2 - 1).to(DEV)
    lw = torch.randn(B, 37 * 37, 1, generator=g).to(DEV)
    ws0 = [(W if B == 1 else torch.stack([W * (1 + 0.02 * i) for i in range(B)])).to(DEV) for W, _ in params]
    bs0 = [(b if B == 1 else torch.stack([b * (1 + 0.02 * i) for i in range(B)])).to(DEV) for _, b in params]
    res = []
    assert _native.get_option("f32_rows") == 1
    for rows in (1, 0):
        _native.set_option("f32_rows", rows)
        try:
            ws = [w.clone().requires_grad_(True) for w in ws0]
            bs = [b.clone().requires_grad_(True) for b in bs0]
            xd = x.clone().requires_grad_(True)
            y = siren_mlp(xd, ws, bs, precision="fp32")
            (y * lw).sum().backward()
            torch.cuda.synchronize()
            res.append((y.detach(), xd.grad, [w.grad for w in ws], [b.grad for b in bs]))
        finally:
            _native.set_option("f32_rows", 1)
    (y1, dx1, dw1, db1), (y0, dx0, dw0, db0) = res
    assert torch.equal(y1, y0) and torch.equal(dx1, dx0)
    for a_, b_ in zip(dw1 + db1, dw0 + db0):
        assert orc.norm_rel(a_.cpu(), b_.cpu()) < 1e-6


@pytest.mark.parametrize("nh", [1, 3])
def test_fp32_hidden_512(nh):
    """SingleBVPNet(hidden_features=512) in the default (fp32) arithmetic — modules.py:125-126 allows
    any width: forward, every gradient and dx against the fp64 oracle at the fp32 tolerances."""
    dims = orc.siren_dims(2, 512, nh, 1)
    params = orc.siren_init(dims, seed=512 + nh)
    x = orc.get_mgrid(40).unsqueeze(0)
    lw = torch.randn(1, 40 * 40, 1, generator=torch.Generator().manual_seed(3))
    _check(x, params, "fp32", loss_w=lw)


def test_fp32_hidden_512_module_and_gradient():
    """The module path (SingleBVPNet, default precision) at hidden 512 and its analytic gradient."""
    from siren_mri_amd import diff_operators, modules
    torch.manual_seed(4)
    m = modules.SingleBVPNet(type="sine", hidden_features=512, num_hidden_layers=2).to(DEV)
    coords = orc.get_mgrid(24)[None]
    o = m({"coords": coords.to(DEV)})
    g = diff_operators.gradient(o["model_out"], o["model_in"])
    sd = m.state_dict()
    ps = [(sd[f"net.net.{i}.0.weight"].double().cpu(), sd[f"net.net.{i}.0.bias"].double().cpu()) for i in range(4)]
    x = coords.double().clone().requires_grad_(True)
    y = orc.siren_forward(x, ps)
    assert orc.norm_rel(o["model_out"].detach().cpu(), y.detach()) < 1e-5
    assert orc.norm_rel(g.detach().cpu(), orc.gradient(y, x).detach()) < 1e-5
