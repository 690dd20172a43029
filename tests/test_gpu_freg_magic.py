"""GPU: the register-resident forward's two epilogue forms (siren_fwdreg.hip epi_part, option
"freg_magic").

The magic form starts every hidden-layer accumulator at fract(b k1) + 192 revolutions, so the
accumulator's low 16 mantissa bits are the phase code and v_sin takes it unreduced; it holds while
k1 sum_k |W_fk| < 62 for every hidden row (prep_reg_kernel's bound), and each weight set whose
weights break that runs the fract form instead (both forms are launched; the one that does not
apply exits). Checked here: the magic form against the fp64 oracle and the fract form at the
shapes it takes; bit-equality run to run; weights past the bound take the fract form bit for bit;
a batch mixing sets on both sides of the bound."""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _params(dims, B, seed, hidden_scale=1.0, big_sets=()):
    g = torch.Generator().manual_seed(seed)
    out = []
    for l in range(len(dims) - 1):
        W, b = orc.siren_init(dims, seed=seed + l)[l]
        if 0 < l < len(dims) - 2:
            W = W * hidden_scale
        if B is not None:
            W = (W.unsqueeze(0).repeat(B, 1, 1) * (1 + 0.1 * torch.randn(B, 1, 1, generator=g))).contiguous()
            b = (b.unsqueeze(0).repeat(B, 1) + 0.01 * torch.randn(B, dims[l + 1], generator=g)).contiguous()
            if 0 < l < len(dims) - 2:
                for s in big_sets:
                    W[s] *= 40.0
        out.append((W, b))
    return out


def _run(x, params, magic):
    from siren_mri_amd import _native
    from siren_mri_amd.ops import siren_mlp
    _native.set_option("freg_magic", 1 if magic else 0)
    try:
        ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
        bs = [b.to(DEV).requires_grad_(True) for _, b in params]
        y = siren_mlp(x.to(DEV), ws, bs, precision="bf16", outermost_linear=True)
        (y.square().sum() * (1.0 / y.numel())).backward()
        torch.cuda.synchronize()
        return y.detach().cpu(), [(w.grad.cpu(), b.grad.cpu()) for w, b in zip(ws, bs)]
    finally:
        _native.set_option("freg_magic", 0)


def _oracle(x, params):
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    y = orc.siren_forward(x.double(), ps)
    (y.square().sum() * (1.0 / y.numel())).backward()
    return y.detach(), [(W.grad, b.grad) for W, b in ps]


def _max_grad_err(g, g_ref):
    return max(max(orc.norm_rel(dW, rW), orc.norm_rel(db, rb)) for (dW, db), (rW, rb) in zip(g, g_ref))


CASES = [
    ([2, 256, 256, 256, 256, 1], None, 4096),
    ([2, 256, 256, 256, 256, 1], None, 65536 + 77),
    ([2, 256, 256, 1], None, 1000),
    ([3, 256, 256, 256, 8], None, 255),
    ([2, 256, 256, 256, 2], 3, 500),
    ([16, 256, 256, 256, 256, 2], 4, 2048),  # wide first layer (configs 4/5's hypo-net)
]


@pytest.mark.parametrize("dims,B,n", CASES)
def test_magic_form_matches_oracle_and_fract_form(dims, B, n):
    params = _params(dims, B, seed=7 * len(dims) + n)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(B or 1, n, dims[0], generator=g) * 2 - 1
    y_m, g_m = _run(x, params, magic=True)
    y_f, g_f = _run(x, params, magic=False)
    y_ref, g_ref = _oracle(x, params)
    e_m, e_f = orc.norm_rel(y_m, y_ref), orc.norm_rel(y_f, y_ref)
    assert torch.isfinite(y_m).all()
    # bf16-mode tolerances: forward 2e-3, gradients 2e-2; and the magic form's
    # forward within 1.5x (+ 5e-5) of the fract form's error
    assert e_m < 2e-3 and e_m <= 1.5 * e_f + 5e-5, (e_m, e_f)
    gm, gf = _max_grad_err(g_m, g_ref), _max_grad_err(g_f, g_ref)
    assert gm < 2e-2 and gm <= 1.5 * gf + 1e-3, (gm, gf)


def test_magic_form_deterministic():
    dims = [2, 256, 256, 256, 256, 1]
    params = _params(dims, None, seed=3)
    x = torch.rand(1, 65536 + 300, 2, generator=torch.Generator().manual_seed(1)) * 2 - 1
    y1, g1 = _run(x, params, magic=True)
    y2, g2 = _run(x, params, magic=True)
    assert torch.equal(y1, y2)
    for (a, b), (c, d) in zip(g1, g2):
        assert torch.equal(a, c) and torch.equal(b, d)


def test_weights_past_the_bound_take_the_fract_form():
    """Hidden weights 40x the SIREN init (k1 sum |W| ~ 100-200 revolutions > 62): the magic launch
    exits and the fract form does the work, so the result is bit-equal to freg_magic = 0."""
    dims = [2, 256, 256, 256, 256, 1]
    params = _params(dims, None, seed=11, hidden_scale=40.0)
    x = torch.rand(1, 8192 + 5, 2, generator=torch.Generator().manual_seed(2)) * 2 - 1
    y_m, g_m = _run(x, params, magic=True)
    y_f, g_f = _run(x, params, magic=False)
    assert torch.equal(y_m, y_f)
    for (a, b), (c, d) in zip(g_m, g_f):
        assert torch.equal(a, c) and torch.equal(b, d)
    # (no oracle comparison: at phases of ~100 revolutions the f16 weights' 2^-11 rounding moves a
    # phase by ~0.05 revolution, in either form — the claim here is the fallback, bit for bit)


def test_mixed_weight_sets():
    """Per-set weights with sets 1 and 3 past the bound: the other sets match the oracle, and the
    sets past the bound are bit-equal to the fract form's."""
    dims = [2, 256, 256, 256, 2]
    B, n = 4, 3000
    params = _params(dims, B, seed=5, big_sets=(1, 3))
    x = torch.rand(B, n, 2, generator=torch.Generator().manual_seed(3)) * 2 - 1
    y_m, _ = _run(x, params, magic=True)
    y_f, _ = _run(x, params, magic=False)
    with torch.no_grad():
        y_ref = orc.siren_forward(x.double(), [(W.double(), b.double()) for W, b in params])
    for s in (0, 2):
        assert orc.norm_rel(y_m[s], y_ref[s]) < 2e-3, s
    assert torch.equal(y_m[1], y_f[1]) and torch.equal(y_m[3], y_f[3])
