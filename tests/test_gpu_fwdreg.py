"""GPU: the register-resident forward (siren_fwdreg.hip, option "fused_forward_reg") against the
fp64 oracle and against the LDS-staged fused forward it replaces, over the shapes it takes
(hidden width 256, 1..4 inputs, 1..8 outputs, 1..4+ hidden MFMA layers, shared and per-set
weights, ragged row counts, several persistent rounds per workgroup, sine output layer).

Both forwards multiply the hidden layers with fp16 operands and fp32 accumulation; the reg
kernel runs layer 0 on the exact-fp32 MFMA and takes sin of the unrounded phase, but its output
layer also multiplies f16 operands (the staged kernel's is fp32 VALU), so its y error stays at
the 1e-4 level, within 2x of the staged kernel's.
The phase codes it stores for the backward feed the same bf16 backward, so the parameter
gradients agree with the staged path to bf16 accuracy."""
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


def _run(x, params, reg, grad, outermost_linear=True):
    from siren_mri_amd import _native
    from siren_mri_amd.ops import siren_mlp
    _native.set_option("fused_forward_reg", 1 if reg else 0)
    try:
        ws = [W.to(DEV).requires_grad_(grad) for W, _ in params]
        bs = [b.to(DEV).requires_grad_(grad) for _, b in params]
        with torch.set_grad_enabled(grad):
            y = siren_mlp(x.to(DEV), ws, bs, precision="bf16", outermost_linear=outermost_linear)
            if grad:
                (y.square().sum() * (1.0 / y.numel())).backward()
        torch.cuda.synchronize()
        grads = [(w.grad.cpu(), b.grad.cpu()) for w, b in zip(ws, bs)] if grad else None
        return y.detach().cpu(), grads
    finally:
        _native.set_option("fused_forward_reg", 1)


CASES = [
    # dims, weight sets, rows per set
    ([2, 256, 256, 256, 256, 1], None, 4096),      # metric architecture
    ([2, 256, 256, 256, 256, 1], None, 65536 + 77),  # several rounds per workgroup, ragged
    ([2, 256, 256, 1], None, 1000),                # one hidden layer (ring never refilled), ragged
    ([2, 256, 256, 256, 2], None, 300),            # two hidden layers, O = 2
    ([1, 256, 256, 256, 256, 256, 3], None, 513),  # C = 1, four hidden layers, O = 3
    ([3, 256, 256, 256, 8], None, 255),            # C = 3 (two K pairs), O = 8, under one round
    ([4, 256, 256, 256, 256, 256, 256, 1], None, 2048),  # C = 4, five hidden layers
    ([2, 256, 256, 256, 2], 3, 500),               # per-set weights (hypernetwork shape)
    ([2, 256, 256, 256, 256, 1], 5, 16384 + 31),   # per-set weights, several rounds
]


@pytest.mark.parametrize("dims,B,n", CASES)
def test_reg_forward_matches_oracle_and_staged(dims, B, n):
    params = _params(dims, B, seed=len(dims) + n)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(B or 1, n, dims[0], generator=g) * 2 - 1
    y_r, g_r = _run(x, params, reg=True, grad=True)
    y_s, g_s = _run(x, params, reg=False, grad=True)
    with torch.no_grad():
        y_ref = orc.siren_forward(x.double(), [(W.double(), b.double()) for W, b in params])
    e_r, e_s = orc.norm_rel(y_r, y_ref), orc.norm_rel(y_s, y_ref)
    assert torch.isfinite(y_r).all()
    assert e_r < 3e-3, (e_r, e_s)
    # the output layer multiplies f16 operands on the MFMA (the staged kernel: fp32 VALU), so y
    # may carry up to ~2x the staged kernel's (already 1e-4-level) error
    assert e_r <= 2.0 * e_s + 5e-5, (e_r, e_s)
    for (dWr, dbr), (dWs, dbs) in zip(g_r, g_s):
        assert orc.norm_rel(dWr, dWs) < 2e-2
        assert orc.norm_rel(dbr, dbs) < 2e-2


def test_reg_forward_gradients_match_oracle():
    """Metric architecture: parameter gradients through the reg forward's phase codes vs fp64."""
    dims = [2, 256, 256, 256, 256, 1]
    params = _params(dims, None, seed=11)
    x = orc.get_mgrid(64).unsqueeze(0)
    _, g_r = _run(x, params, reg=True, grad=True)
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    y = orc.siren_forward(x.double(), ps)
    (y.square().sum() * (1.0 / y.numel())).backward()
    for (dW, db), (W, b) in zip(g_r, ps):
        assert orc.norm_rel(dW.double(), W.grad) < 5e-2
        assert orc.norm_rel(db.double(), b.grad) < 5e-2


def test_reg_forward_no_grad_equals_training_forward():
    dims = [2, 256, 256, 256, 256, 1]
    params = _params(dims, None, seed=5)
    x = orc.get_mgrid(48).unsqueeze(0)
    y_t, _ = _run(x, params, reg=True, grad=True)
    y_n, _ = _run(x, params, reg=True, grad=False)
    assert torch.equal(y_t, y_n)


def test_reg_forward_sine_output():
    dims = [2, 256, 256, 256, 2]
    params = _params(dims, None, seed=9)
    x = orc.get_mgrid(40).unsqueeze(0)
    y_r, _ = _run(x, params, reg=True, grad=False, outermost_linear=False)
    with torch.no_grad():
        y_ref = orc.siren_forward(x.double(), [(W.double(), b.double()) for W, b in params],
                                  outermost_linear=False)
    assert orc.norm_rel(y_r, y_ref) < 2e-2


def test_reg_forward_is_deterministic():
    dims = [2, 256, 256, 256, 256, 1]
    params = _params(dims, None, seed=2)
    x = orc.get_mgrid(128).unsqueeze(0)
    y1, g1 = _run(x, params, reg=True, grad=True)
    y2, g2 = _run(x, params, reg=True, grad=True)
    assert torch.equal(y1, y2)
    for (a, b), (c, d) in zip(g1, g2):
        assert torch.equal(a, c) and torch.equal(b, d)


@pytest.mark.parametrize("dims,B,n", [([2, 256, 256, 256, 256, 1], 5, 16384 + 31),
                                      ([2, 256, 256, 256, 256, 1], None, 16384 + 1),
                                      ([2, 256, 256, 256, 2], 3, 500)])
def test_ragged_and_batched_are_deterministic(dims, B, n):
    """Ragged row counts (rows x C not a multiple of 4) and per-set weights (the hypernetwork
    shape): two identical runs give bit-identical outputs and parameter gradients (no atomics on
    the path, fixed reduction orders). Round 2 kept P_0 for such shapes and the register forward's
    layer-0 phase-code stores then varied from run to run (tools/det_saved.py)."""
    params = _params(dims, B, seed=3)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(B or 1, n, dims[0], generator=g) * 2 - 1
    y1, g1 = _run(x, params, reg=True, grad=True)
    y2, g2 = _run(x, params, reg=True, grad=True)
    assert torch.equal(y1, y2)
    for l, ((a, b), (c, d)) in enumerate(zip(g1, g2)):
        assert torch.equal(a, c), (l, (a - c).abs().max())
        assert torch.equal(b, d), (l, (b - d).abs().max())


@pytest.mark.parametrize("dims,B,n", [([2, 256, 256, 256, 256, 1], 3, 1001),
                                      ([3, 256, 256, 256, 2], None, 999),
                                      ([1, 256, 256, 256, 1], 2, 515)])
def test_ragged_rows_gradients_match_oracle(dims, B, n):
    """Ragged shapes (rows x C not a multiple of 4, so a weight set's x rows can start 8 bytes past
    a 16-byte boundary) rebuild P_0 from x by LDS-DMA in the backward: parameter gradients vs the
    fp64 oracle's autograd (bf16-mode tolerance)."""
    params = _params(dims, B, seed=n)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(B or 1, n, dims[0], generator=g) * 2 - 1
    _, g_r = _run(x, params, reg=True, grad=True)
    ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
    y = orc.siren_forward(x.double(), ps)
    (y.square().sum() * (1.0 / y.numel())).backward()
    for (dW, db), (W, b) in zip(g_r, ps):
        assert orc.norm_rel(dW.double(), W.grad) < 5e-2
        assert orc.norm_rel(db.double(), b.grad) < 5e-2
