"""The SIREN stack as registered PyTorch custom ops (siren_mri_amd::sine_mlp_fwd/bwd,
sine_mlp_jvp/jvp_bwd; SURVEY.md §8(b) 'Custom-op layer'): dispatcher registration, schemas and
fake (meta) kernels, checked on the CPU with FakeTensors (no kernel runs); the GPU part runs
torch.library.opcheck and the analytic gradient with grad_outputs."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import siren_mri_amd.data_consistency  # noqa: F401 - registers dc_forward / dc_backward
import siren_mri_amd.jvp  # noqa: F401 - registers the tangent-stream ops
import siren_mri_amd.loss_functions  # noqa: F401 - registers kspace_sse / kspace_sse_bwd
import siren_mri_amd.ops  # noqa: F401 - registers the stack ops
from oracle import siren_oracle as orc

OPS = ("sine_mlp_fwd", "sine_mlp_bwd", "sine_mlp_jvp", "sine_mlp_jvp_bwd", "dc_forward", "dc_backward",
       "kspace_sse", "kspace_sse_bwd")


def test_ops_registered_with_schemas():
    for name in OPS:
        op = getattr(torch.ops.siren_mri_amd, name)
        schema = str(op.default._schema)
        assert schema.startswith(f"siren_mri_amd::{name}("), schema
    s = str(torch.ops.siren_mri_amd.sine_mlp_fwd.default._schema)
    assert "Tensor[] weights" in s and "-> (Tensor, Tensor)" in s
    assert "Tensor[]" in str(torch.ops.siren_mri_amd.sine_mlp_bwd.default._schema).split("->")[1]


def _fake_args(B, N, dims, batched):
    lead = (B, N) if batched else (1, N)
    x = torch.empty(*lead, dims[0], device="cuda")
    ws = [torch.empty(*((B,) if batched else ()), dims[l + 1], dims[l], device="cuda") for l in range(len(dims) - 1)]
    bs = [torch.empty(*((B,) if batched else ()), dims[l + 1], device="cuda") for l in range(len(dims) - 1)]
    return x, ws, bs


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("prec", [0, 1])
def test_fake_kernels_shapes(batched, prec):
    dims = [2, 256, 256, 256, 256, 1] if not batched else [16, 256, 256, 256, 256, 2]
    with FakeTensorMode():
        x, ws, bs = _fake_args(3, 777, dims, batched)
        y, saved = torch.ops.siren_mri_amd.sine_mlp_fwd(x, ws, bs, 30.0, prec, True, batched, True)
        assert y.shape == x.shape[:-1] + (dims[-1],) and y.device.type == "cuda" and y.dtype == torch.float32
        assert saved.dtype == torch.uint8 and saved.numel() > 0
        _, nokeep = torch.ops.siren_mri_amd.sine_mlp_fwd(x, ws, bs, 30.0, prec, True, batched, False)
        assert nokeep.numel() == 0
        dx, dW, db = torch.ops.siren_mri_amd.sine_mlp_bwd(y, x, ws, bs, saved, 30.0, prec, True, batched, True)
        assert dx.shape == x.shape
        assert [t.shape for t in dW] == [w.shape for w in ws] and [t.shape for t in db] == [b.shape for b in bs]
        if not batched:
            g, s1 = torch.ops.siren_mri_amd.sine_mlp_jvp(x, ws, bs, 30.0, prec, batched, 1, True)
            lap, s2 = torch.ops.siren_mri_amd.sine_mlp_jvp(x, ws, bs, 30.0, prec, batched, 2, True)
            assert g.shape == x.shape and lap.shape == x.shape[:-1] + (1,) and s2.numel() >= s1.numel() > 0


def test_kspace_fake_kernels():
    with FakeTensorMode():
        pred = torch.empty(4, 16384, 2, device="cuda")
        k0 = torch.empty(4, 2, 128, 128, device="cuda")
        y = torch.ops.siren_mri_amd.dc_forward(pred, k0, k0, 0.0)
        assert y.shape == pred.shape
        loss, d = torch.ops.siren_mri_amd.kspace_sse(pred, k0, k0, pred, None, 0.0, 1.0 / 16384)
        assert loss.shape == () and d.shape == pred.shape
        assert torch.ops.siren_mri_amd.kspace_sse_bwd(d, k0, None, loss, 0.0, 2.0).shape == pred.shape


def test_fake_kernel_rejects_bad_shapes():
    with FakeTensorMode():
        x, ws, bs = _fake_args(1, 10, [2, 64, 1], False)
        ws[1] = torch.empty(1, 65, device="cuda")
        with pytest.raises(RuntimeError, match="does not take"):
            torch.ops.siren_mri_amd.sine_mlp_fwd(x, ws, bs, 30.0, 0, True, False, True)


@pytest.mark.gpu
def test_opcheck_on_gpu():
    dev = torch.device("cuda:0")
    dims = [2, 64, 64, 1]
    params = orc.siren_init(dims, seed=1)
    x = (torch.rand(1, 300, 2) * 2 - 1).to(dev).requires_grad_(True)
    ws = [W.to(dev).requires_grad_(True) for W, _ in params]
    bs = [b.to(dev).requires_grad_(True) for _, b in params]
    torch.library.opcheck(torch.ops.siren_mri_amd.sine_mlp_fwd.default, (x, ws, bs, 30.0, 0, True, False, True),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


@pytest.mark.gpu
def test_gradient_with_grad_outputs_is_analytic_and_matches_oracle():
    """diff_operators.gradient(y, x, grad_outputs=g) (diff_operators.py:39-43) for a SIREN output:
    the analytic path, differentiable (its parameter gradients against the oracle's double backward)."""
    from siren_mri_amd import diff_operators, modules
    dev = torch.device("cuda:0")
    torch.manual_seed(2)
    m = modules.SingleBVPNet(type="sine", hidden_features=64, num_hidden_layers=2, precision="fp32").to(dev)
    coords = orc.get_mgrid(16)[None]
    g = torch.rand(1, 256, 1, generator=torch.Generator().manual_seed(3)) + 0.5
    o = m({"coords": coords.to(dev)})
    gr = diff_operators.gradient(o["model_out"], o["model_in"], grad_outputs=g.to(dev))
    gr.square().sum().backward()
    sd = m.state_dict()
    ps = [(sd[f"net.net.{i}.0.weight"].double().cpu().requires_grad_(True),
           sd[f"net.net.{i}.0.bias"].double().cpu().requires_grad_(True)) for i in range(4)]
    x = coords.double().requires_grad_(True)
    ref = orc.gradient(orc.siren_forward(x, ps), x, grad_outputs=g.double())
    ref.square().sum().backward()
    assert orc.norm_rel(gr.detach().cpu(), ref.detach()) < 1e-5
    for i, (W, _) in enumerate(ps):
        assert orc.norm_rel(m.net.net[i][0].weight.grad.cpu(), W.grad) < 1e-4


@pytest.mark.gpu
def test_backward_twice_with_retain_graph():
    """The saved buffer is read-only for the backward: retain_graph=True works (as in the reference)."""
    from siren_mri_amd.ops import siren_mlp
    dev = torch.device("cuda:0")
    params = orc.siren_init([2, 256, 256, 256, 1], seed=4)
    ws = [W.to(dev).requires_grad_(True) for W, _ in params]
    bs = [b.to(dev).requires_grad_(True) for _, b in params]
    y = siren_mlp(orc.get_mgrid(32)[None].to(dev), ws, bs, precision="bf16")
    y.square().sum().backward(retain_graph=True)
    g1 = [w.grad.clone() for w in ws]
    y.square().sum().backward()
    for a, w in zip(g1, ws):
        assert torch.equal(2 * a, w.grad)
