"""GPU: the HyperNetwork's heads as grouped native GEMMs (siren_hyper_forward / _backward,
csrc/siren_hyper.hip; meta_modules.py:11-54 HyperNetwork, one ReLU FCBlock per hypo-parameter)
against the per-head Linear + ReLU chain of the same module in fp32 (the reference's arithmetic)
and against the fp64 chain.

Both fp32 paths differ only in summation order: outputs and every gradient agree to 1e-5
norm-relative, and the native path is no further from fp64 than the chain (within 2x + 1e-6).
"""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _hyper(hidden_layers=2, hyper_hidden=128, latent=128, seed=0):
    from siren_mri_amd import meta_modules, modules
    torch.manual_seed(seed)
    hypo = modules.SingleBVPNet(out_features=2, type="sine", in_features=16, hidden_features=256,
                                num_hidden_layers=3)
    return meta_modules.HyperNetwork(hyper_in_features=latent, hyper_hidden_layers=hidden_layers,
                                     hyper_hidden_features=hyper_hidden, hypo_module=hypo).to(DEV)


def _run(hn, z, gouts, native):
    from siren_mri_amd import meta_modules
    hn.zero_grad(set_to_none=True)
    zz = z.clone().requires_grad_(True)
    if native:
        assert hn._native_layers(zz) is not None
        out = hn(zz)
    else:
        saved = meta_modules.HyperNetwork._native_layers
        meta_modules.HyperNetwork._native_layers = lambda self, z: None
        try:
            out = hn(zz)
        finally:
            meta_modules.HyperNetwork._native_layers = saved
    loss = sum((o * g).sum() for o, g in zip(out.values(), gouts))
    loss.backward()
    return ([o.detach().clone() for o in out.values()], zz.grad.clone(),
            {n: p.grad.clone() for n, p in hn.named_parameters()})


@pytest.mark.parametrize("hidden_layers,rows", [(2, 32), (1, 5), (3, 70)])
def test_native_heads_match_the_per_head_chain(hidden_layers, rows):
    """Configs 4/5's heads (latent 128, hidden 128, two hidden layers, ten hypo-parameters up to
    65,536 outputs) and ragged variants (5 / 70 rows, one / three hidden layers)."""
    hn = _hyper(hidden_layers)
    g = torch.Generator().manual_seed(1)
    z = torch.randn(rows, 128, generator=g).to(DEV)
    shapes = [(rows,) + tuple(s) for s in hn.param_shapes]
    gouts = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    o_n, dz_n, g_n = _run(hn, z, gouts, True)
    o_c, dz_c, g_c = _run(hn, z, gouts, False)
    # fp64 chain
    hn64 = _hyper(hidden_layers).double()
    hn64.load_state_dict(hn.state_dict())
    o_r, dz_r, g_r = _run(hn64, z.double(), [t.double() for t in gouts], False)
    errs = {}
    for i, (a, b, r) in enumerate(zip(o_n, o_c, o_r)):
        errs[f"out{i}"] = orc.norm_rel(a.cpu(), b.cpu())
        assert orc.norm_rel(a.cpu(), r.cpu()) <= 2 * orc.norm_rel(b.cpu(), r.cpu()) + 1e-6
    errs["dz"] = orc.norm_rel(dz_n.cpu(), dz_c.cpu())
    assert orc.norm_rel(dz_n.cpu(), dz_r.cpu()) <= 2 * orc.norm_rel(dz_c.cpu(), dz_r.cpu()) + 1e-6
    for n in g_n:
        errs[n] = orc.norm_rel(g_n[n].cpu(), g_c[n].cpu())
        assert orc.norm_rel(g_n[n].cpu(), g_r[n].cpu()) <= 2 * orc.norm_rel(g_c[n].cpu(), g_r[n].cpu()) + 1e-6, n
    worst = max(errs, key=errs.get)
    print(f"\n[hyper heads L={hidden_layers} rows={rows}] worst {worst} {errs[worst]:.2e}")
    assert errs[worst] < 1e-5, (worst, errs[worst])


def test_native_heads_deterministic():
    hn = _hyper()
    g = torch.Generator().manual_seed(2)
    z = torch.randn(32, 128, generator=g).to(DEV)
    gouts = [torch.randn((32,) + tuple(s), generator=g).to(DEV) for s in hn.param_shapes]
    a = _run(hn, z, gouts, True)
    b = _run(hn, z, gouts, True)
    for x, y in zip(a[0], b[0]):
        assert torch.equal(x, y)
    assert torch.equal(a[1], b[1])
    for n in a[2]:
        assert torch.equal(a[2][n], b[2][n]), n


def test_hypo_weight_loss_native_sum_of_squares():
    """hypo_weight_loss (loss_functions.py:279-287) on CUDA fp32: the native sum of squares and its
    gradient against the fp64 torch formula (1e-6), deterministic, ragged tensor sizes."""
    from siren_mri_amd import loss_functions
    g = torch.Generator().manual_seed(5)
    shapes = [(32, 256, 16), (32, 256), (32, 256, 256), (32, 2, 256), (32, 2), (7, 1001)]
    ws = [torch.randn(s, generator=g).to(DEV).requires_grad_(True) for s in shapes]
    out = {"hypo_params": {f"p{i}": w for i, w in enumerate(ws)}}
    l1 = loss_functions.hypo_weight_loss(out)
    l1.backward()
    g1 = [w.grad.clone() for w in ws]
    for w in ws:
        w.grad = None
    l2 = loss_functions.hypo_weight_loss(out)
    l2.backward()
    assert torch.equal(l1, l2) and all(torch.equal(a, w.grad) for a, w in zip(g1, ws))
    wd = [w.detach().double().cpu().requires_grad_(True) for w in ws]
    total = sum(w.numel() for w in wd)
    ref = sum((w ** 2).sum() for w in wd) / total
    ref.backward()
    assert abs(l1.item() - ref.item()) <= 1e-6 * abs(ref.item())
    for a, w in zip(g1, wd):
        assert orc.norm_rel(a.cpu(), w.grad) < 1e-6


def test_create_graph_through_native_heads_and_sum_of_squares():
    """torch.autograd.grad(..., create_graph=True) over the native heads and the native
    hypo_weight_loss works as it did with the plain PyTorch modules (the heads recompute the
    per-head Linear + ReLU chain differentiably; the sum of squares' gradient is 2 g w): the first
    derivatives equal the chain's, and a second derivative (of the gradient norm) equals the
    chain's to fp32 summation order."""
    from siren_mri_amd import loss_functions, meta_modules
    hn = _hyper(2, hyper_hidden=32, latent=16)
    g = torch.Generator().manual_seed(5)
    z0 = torch.randn(4, 16, generator=g).to(DEV)

    def second(native):
        z = z0.clone().requires_grad_(True)
        saved = meta_modules.HyperNetwork._native_layers
        if not native:
            meta_modules.HyperNetwork._native_layers = lambda self, z: None
        try:
            if native:
                assert hn._native_layers(z) is not None
            hp = hn(z)
            loss = loss_functions.hypo_weight_loss({"hypo_params": hp})
            (gz,) = torch.autograd.grad(loss, [z], create_graph=True)
            (ggz,) = torch.autograd.grad((gz ** 2).sum(), [z])
        finally:
            meta_modules.HyperNetwork._native_layers = saved
        return loss.detach(), gz.detach(), ggz
    l_n, g_n, gg_n = second(True)
    l_c, g_c, gg_c = second(False)
    assert float(l_n) == pytest.approx(float(l_c), rel=1e-5)
    assert orc.norm_rel(g_n.cpu(), g_c.cpu()) < 1e-5
    assert orc.norm_rel(gg_n.cpu(), gg_c.cpu()) < 1e-4


def test_encoder_with_more_than_32_convolutions():
    """an encoder with 15 residual blocks (33 convolutions) takes the operand prep in
    launches of at most 32 filters; its forward equals the same node's per-convolution casts."""
    from siren_mri_amd import encoder, modules
    torch.manual_seed(0)
    enc = modules.ConvImgEncoder(2, (32, 32), hidden_size=64, kernel_size=3, num_conv_res_blocks=15,
                                 precision="bf16").to(DEV)
    convs = enc._layers()
    assert convs is not None and len(convs) > 32
    wbs, wfs, bbs = encoder._prep_operands(convs, DEV, torch.cuda.current_stream().cuda_stream)
    for i, c in enumerate(convs):
        assert torch.equal(wbs[i], encoder._w_bf16(c.weight))
        assert torch.equal(bbs[i], c.bias.detach().to(torch.bfloat16))
        if i:
            assert torch.equal(wfs[i], encoder._w_flip(wbs[i]))
    I = torch.randn(2, 2, 32, 32, device=DEV)
    e = enc(I)
    e.sum().backward()
    assert torch.isfinite(e).all() and all(torch.isfinite(p.grad).all() for p in enc.parameters())
