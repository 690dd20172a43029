"""GPU: the fused bf16 conv-encoder node (siren_mri_amd/encoder.py) against
the bf16 autocast chain it replaces and against the fp32 encoder (the reference's arithmetic,
modules.py:340-380 / 433-450), and its native passes (siren_encoder.hip) against torch.

Tolerances: on MIOpen's convolutions the node's forward has the autocast chain's roundings, so the
embedding agrees to fp32 summation order (1e-5); with the native 5x5 kernels (another summation
order inside each convolution) to the bf16 level (6e-3); parameter gradients agree to the bf16
level (2e-2 norm-relative; with every 2/64/128-channel convolution native, two bf16 paths each a
few % from fp32: 1e-1, measured 6.9e-2 on conv_theta's weight); against fp32 no further off than
the autocast chain (test_fused_node_against_fp32_encoder).
"""
import pytest
import torch

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _encoder(precision, seed=0, blocks=2, hidden=128, k=7):
    from siren_mri_amd import modules
    torch.manual_seed(seed)
    return modules.ConvImgEncoder(2, (128, 128), hidden_size=hidden, kernel_size=k, num_conv_res_blocks=blocks,
                                  precision=precision).to(DEV)


def _run(enc, I, ge):
    enc.zero_grad(set_to_none=True)
    e = enc(I)
    e.backward(ge)
    return e.detach().clone(), {n: p.grad.detach().clone() for n, p in enc.named_parameters()}


@pytest.mark.parametrize("native_conv", [False, True])
@pytest.mark.parametrize("blocks,hidden,k", [(2, 128, 7), (1, 64, 5)])
def test_fused_node_matches_autocast_chain(blocks, hidden, k, native_conv):
    """native_conv=False: the node on MIOpen's convolutions, the chain's own roundings (forward to
    fp32 summation order, 1e-5). True: every 2/64/128-channel convolution on the native kernels
    (another fp32 summation order inside each convolution, so activations may differ by a bf16
    rounding step, compounding over the layers from conv_theta on: measured 3.8e-3 / 4.6e-3
    forward, bound 6e-3); test_fused_node_against_fp32_encoder checks the native node is no
    further from fp32 than the chain."""
    from siren_mri_amd import encoder
    enc = _encoder("bf16", blocks=blocks, hidden=hidden, k=k)
    g = torch.Generator().manual_seed(1)
    I = torch.randn(3, 2, 128, 128, generator=g).to(DEV)
    ge = torch.randn(3, hidden, generator=g).to(DEV)
    assert enc._layers() is not None
    encoder._CONV_NATIVE[0] = encoder._WGRAD_NATIVE[0] = native_conv
    try:
        e_f, g_f = _run(enc, I, ge)
        encoder.set_fused(False)
        try:
            e_c, g_c = _run(enc, I, ge)
        finally:
            encoder.set_fused(True)
    finally:
        encoder._CONV_NATIVE[0] = encoder._WGRAD_NATIVE[0] = True
    assert orc.norm_rel(e_f.cpu(), e_c.cpu()) < (6e-3 if native_conv else 1e-5)
    assert g_f.keys() == g_c.keys()
    for n in g_f:
        # native: conv_theta's weight gradient sums the whole network's bf16 backward over every
        # pixel (chain and node each ~5 % from fp32 there: measured 6.9e-2 between them); the
        # accuracy bound is test_fused_node_against_fp32_encoder's (<= 1.25 x the chain's error)
        assert orc.norm_rel(g_f[n].cpu(), g_c[n].cpu()) < (1e-1 if native_conv else 2e-2), n


def test_fused_node_against_fp32_encoder():
    """Against the fp32 encoder (the reference's arithmetic): the bf16 gradients of the first layers
    sit ~5-10 % off after the ReLU masks and residual sums of a bf16 backward, for the autocast chain
    as for the node; the node must be no further off than the chain it replaces."""
    from siren_mri_amd import encoder
    enc = _encoder("bf16", seed=2)
    ref = _encoder("fp32", seed=2)
    ref.load_state_dict(enc.state_dict())
    g = torch.Generator().manual_seed(3)
    I = torch.randn(2, 2, 128, 128, generator=g).to(DEV)
    ge = torch.randn(2, 128, generator=g).to(DEV)
    torch.backends.cudnn.allow_tf32 = False
    e_f, g_f = _run(enc, I, ge)
    encoder.set_fused(False)
    try:
        e_c, g_c = _run(enc, I, ge)
    finally:
        encoder.set_fused(True)
    e_r, g_r = _run(ref, I, ge)
    assert orc.norm_rel(e_f.cpu(), e_r.cpu()) < 3e-2
    for n in g_f:
        ef = orc.norm_rel(g_f[n].cpu(), g_r[n].cpu())
        ec = orc.norm_rel(g_c[n].cpu(), g_r[n].cpu())
        print(f"{n}: node {ef:.2e} autocast chain {ec:.2e}")
        assert ef < 0.2 and ef <= 1.25 * ec + 5e-3, (n, ef, ec)


def test_native_passes_deterministic():
    """The passes' channel sums (block partials added in block order by the last block) repeat bit
    for bit. (The whole node does not: MIOpen's convolutions of the residual blocks differ between
    calls in the last bits, in the autocast chain as in the node.)"""
    from siren_mri_amd import _native
    lib = _native.lib()
    st = _native.stream_handle(DEV)
    ws = _ws()
    B, P, C = 4, 16384, 128
    g = torch.Generator().manual_seed(11)
    a = torch.randn(B * P, C, generator=g).to(DEV).to(torch.bfloat16)
    g1 = torch.randn(B * P, C, generator=g).to(DEV).to(torch.bfloat16)
    w = torch.randn(P, generator=g).to(DEV)
    bias = torch.zeros(1, device=DEV)
    gin = torch.randn(B, C, generator=g).to(DEV)
    res = []
    for _ in range(4):
        out = torch.empty_like(a)
        db = torch.empty(C, device=DEV)
        lib.siren_enc_relu_bwd(g1.data_ptr(), None, a.data_ptr(), out.data_ptr(), db.data_ptr(), B * P, C, ws.data_ptr(),
                               ws.numel(), st)
        e = torch.empty(B, C, device=DEV)
        lib.siren_enc_pixfc_fwd(a.data_ptr(), None, w.data_ptr(), bias.data_ptr(), e.data_ptr(), B, P, C,
                                ws.data_ptr(), ws.numel(), st)
        ga, db2, gw = torch.empty_like(a), torch.empty(C, device=DEV), torch.empty(P, device=DEV)
        lib.siren_enc_pixfc_bwd(gin.data_ptr(), a.data_ptr(), None, w.data_ptr(), ga.data_ptr(), db2.data_ptr(),
                                gw.data_ptr(), B, P, C, ws.data_ptr(), ws.numel(), st)
        res.append((db, e, db2, gw))
    torch.cuda.synchronize()
    for r in res[1:]:
        for x, y in zip(res[0], r):
            assert torch.equal(x, y)


def _ws():
    from siren_mri_amd import _native
    return _native.enc_workspace(DEV)


@pytest.mark.parametrize("C,P", [(128, 70000), (64, 4096), (8, 333)])
def test_relu_bwd_and_res_passes_against_torch(C, P):
    from siren_mri_amd import _native
    lib = _native.lib()
    st = _native.stream_handle(DEV)
    ws = _ws()
    g = torch.Generator().manual_seed(C + P)
    mk = lambda: torch.randn(P, C, generator=g).to(DEV).to(torch.bfloat16)  # noqa: E731
    g1, g2, y, a, x = mk(), mk(), mk(), mk(), mk()
    out = torch.empty_like(g1)
    db = torch.empty(C, device=DEV)
    _native.check(lib.siren_enc_relu_bwd(g1.data_ptr(), g2.data_ptr(), y.data_ptr(), out.data_ptr(), db.data_ptr(),
                                         P, C, ws.data_ptr(), ws.numel(), st), "relu_bwd")
    ref = ((g1 + g2) * (y > 0)).to(torch.bfloat16)
    assert torch.equal(out, ref)
    torch.testing.assert_close(db, ref.float().sum(0), rtol=1e-5, atol=1e-4)
    # res fwd / bwd
    o = torch.empty_like(a)
    cb = torch.randn(C, generator=g).to(DEV).to(torch.bfloat16)
    ab = a + cb  # bf16 add: the conv + bias-add chain's rounding
    _native.check(lib.siren_enc_res_fwd(a.data_ptr(), cb.data_ptr(), x.data_ptr(), o.data_ptr(), P, C, st), "res_fwd")
    assert torch.equal(o, torch.relu(torch.relu(ab) + x))
    gs, ga = torch.empty_like(a), torch.empty_like(a)
    _native.check(lib.siren_enc_res_bwd(g1.data_ptr(), None, o.data_ptr(), a.data_ptr(), cb.data_ptr(), gs.data_ptr(),
                                        ga.data_ptr(), db.data_ptr(), P, C, ws.data_ptr(), ws.numel(), st), "res_bwd")
    s_ref = g1 * (o > 0)
    assert torch.equal(gs, s_ref)
    assert torch.equal(ga, s_ref * (ab > 0))
    torch.testing.assert_close(db, ga.float().sum(0), rtol=1e-5, atol=1e-4)
    yb = a.clone()
    _native.check(lib.siren_enc_bias_relu(yb.data_ptr(), cb.data_ptr(), P, C, st), "bias_relu")
    assert torch.equal(yb, torch.relu(ab))


def test_pixel_linear_passes_against_torch():
    from siren_mri_amd import _native
    lib = _native.lib()
    st = _native.stream_handle(DEV)
    ws = _ws()
    B, H, C = 5, 128, 128
    P = H * H
    g = torch.Generator().manual_seed(9)
    a = torch.randn(B, H, H, C, generator=g).to(DEV).to(torch.bfloat16)
    a_raw = a
    w = (torch.randn(P, generator=g) / 128).to(DEV)
    bias = torch.randn(1, generator=g).to(DEV)
    e = torch.empty(B, C, device=DEV)
    cb = torch.randn(C, generator=g).to(DEV).to(torch.bfloat16)
    _native.check(lib.siren_enc_pixfc_fwd(a.data_ptr(), cb.data_ptr(), w.data_ptr(), bias.data_ptr(), e.data_ptr(), B,
                                          P, C, ws.data_ptr(), ws.numel(), st), "pixfc_fwd")
    a = a + cb  # the reference below sees the biased pre-activation
    r = torch.relu(a.float()).reshape(B, P, C)
    torch.testing.assert_close(e, torch.einsum("bpc,p->bc", r, w) + bias, rtol=1e-4, atol=1e-4)
    gin = torch.randn(B, C, generator=g).to(DEV)
    ga = torch.empty_like(a)
    db = torch.empty(C, device=DEV)
    gw = torch.empty(P, device=DEV)
    _native.check(lib.siren_enc_pixfc_bwd(gin.data_ptr(), a_raw.data_ptr(),
                                          cb.data_ptr(), w.data_ptr(), ga.data_ptr(), db.data_ptr(), gw.data_ptr(), B, P,
                                          C, ws.data_ptr(), ws.numel(), st), "pixfc_bwd")
    ga_ref = ((a.float() > 0) * gin[:, None, None, :] * w.reshape(1, H, H, 1)).to(torch.bfloat16)
    assert torch.equal(ga, ga_ref)
    torch.testing.assert_close(db, ga_ref.float().sum((0, 1, 2)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gw, torch.einsum("bc,bpc->p", gin, r), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N,H,W", [(2, 128, 128), (3, 7, 64), (1, 1, 192)])
def test_conv_weight_gradient_kernel_against_fp32(N, H, W):
    """siren_conv_wrw_k5 (the residual blocks' 128 -> 128 5x5 weight gradient) against the fp32
    weight gradient of the same bf16 operands (exact products; fp32 sums in another order)."""
    from siren_mri_amd import _native
    lib = _native.lib()
    g = torch.Generator().manual_seed(N * 1000 + H + W)
    x = torch.randn(N, 128, H, W, generator=g).to(torch.bfloat16)
    dy = torch.randn(N, 128, H, W, generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.double(), (128, 128, 5, 5), dy.double(), padding=2).float()
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    dyd = dy.to(DEV).contiguous(memory_format=torch.channels_last)
    ws = torch.empty(int(lib.siren_conv_wrw_workspace_bytes(N, H, W)), dtype=torch.uint8, device=DEV)
    prev = _native.get_option("wrw_dma")
    outs = {}
    try:
        for dma in (0, 1, 1, 2):  # register staging; LDS-DMA (option wrw_dma) twice: run-to-run equality;
            # 2: 128-pixel chunks (W a multiple of 128; else the 64-pixel form runs)
            _native.set_option("wrw_dma", dma)
            dw = torch.empty(128, 128, 5, 5, device=DEV).contiguous(memory_format=torch.channels_last)
            _native.check(lib.siren_conv_wrw_k5(xd.data_ptr(), dyd.data_ptr(), N, H, W, 128, dw.data_ptr(),
                                                ws.data_ptr(), ws.numel(), _native.stream_handle(DEV)), "conv_wrw")
            outs.setdefault(dma, []).append(dw)
    finally:
        _native.set_option("wrw_dma", prev)
    assert orc.norm_rel(outs[0][0].cpu(), ref) < 1e-6
    # the LDS-DMA form stages the same image: bit-identical, and deterministic
    assert torch.equal(outs[1][0], outs[0][0])
    assert torch.equal(outs[1][0], outs[1][1])
    # 128-pixel chunks: the same K steps in the same pixel order, so bit-identical too
    assert torch.equal(outs[2][0], outs[0][0])


@pytest.mark.parametrize("dma", [0, 1, 2])
@pytest.mark.parametrize("bias,relu", [(False, False), (True, False), (True, True)])
def test_conv_forward_kernel_against_fp32(bias, relu, dma):
    """siren_conv_fwd_k5 (128 -> 128, 5x5, W = 128) against the fp32 convolution of the same bf16
    operands (then the conv + bias-add chain's bf16 roundings), and bit-equal on a rerun; in each
    stage-fill form (option conv_dma: registers, LDS-DMA, LDS-DMA with per-workgroup offsets) on a
    6-row image, where most stages hold rows outside the image."""
    from siren_mri_amd import _native
    prev = _native.get_option("conv_dma")
    _native.set_option("conv_dma", dma)
    try:
        _conv_forward_case(bias, relu)
    finally:
        _native.set_option("conv_dma", prev)


def _conv_forward_case(bias, relu):
    from siren_mri_amd import _native
    import torch.nn.functional as F
    lib = _native.lib()
    N, H = 2, 6
    g = torch.Generator().manual_seed(17 + bias + 2 * relu)
    x = torch.randn(N, 128, H, 128, generator=g).to(torch.bfloat16)
    w = (torch.randn(128, 128, 5, 5, generator=g) / 40).to(torch.bfloat16)
    b = torch.randn(128, generator=g).to(torch.bfloat16)
    ref = F.conv2d(x.double(), w.double(), padding=2).to(torch.bfloat16)
    if bias:
        ref = ref + b.view(1, -1, 1, 1)
        if relu:
            ref = torch.relu(ref)
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    bd = b.to(DEV)
    outs = []
    for _ in range(2):
        y = torch.empty(N, 128, H, 128, dtype=torch.bfloat16, device=DEV).contiguous(memory_format=torch.channels_last)
        _native.check(lib.siren_conv_fwd_k5(xd.data_ptr(), wd.data_ptr(), bd.data_ptr() if bias else None, int(relu),
                                            y.data_ptr(), N, H, 128, 128, _native.stream_handle(DEV)), "conv_fwd")
        outs.append(y)
    assert torch.equal(outs[0], outs[1])
    d = (outs[0].float().cpu() - ref.float())
    # fp32 sums in another order: at most one bf16 rounding step apart
    assert orc.norm_rel(outs[0].float().cpu(), ref.float()) < 4e-3
    assert (d.abs() <= ref.float().abs() * 2 ** -7 + 1e-6).float().mean() > 0.999


@pytest.mark.parametrize("k,ci,co", [(7, 64, 128), (7, 128, 64), (3, 64, 128), (3, 128, 128), (5, 64, 64),
                                     (5, 128, 128), (7, 2, 64), (3, 2, 128), (5, 2, 32), (7, 2, 96)])
@pytest.mark.parametrize("bias,relu", [(False, False), (True, True)])
def test_generic_conv_forward_kernel_against_fp32(k, ci, co, bias, relu):
    """siren_conv_fwd (round 5: the encoder's other shapes — cnn[0]'s 64 -> 128 7x7, its input
    gradient 128 -> 64, the 3x3 forms; conv_theta's 2 input channels, with a ragged last
    workgroup of image rows) against the fp64 convolution of the same bf16 operands (then the
    conv + bias-add chain's bf16 roundings), bit-equal on a rerun and between the stage fills
    (option conv_dma)."""
    from siren_mri_amd import _native
    import torch.nn.functional as F
    lib = _native.lib()
    N, H = (2, 5) if ci == 2 else (2, 6)
    assert lib.siren_conv_check(0, N, H, 128, ci, co, k) == 0, _native.last_error()
    g = torch.Generator().manual_seed(k * 1000 + ci + co + bias)
    x = torch.randn(N, ci, H, 128, generator=g).to(torch.bfloat16)
    w = (torch.randn(co, ci, k, k, generator=g) / (ci * k)).to(torch.bfloat16)
    b = torch.randn(co, generator=g).to(torch.bfloat16)
    ref = F.conv2d(x.double(), w.double(), padding=k // 2).to(torch.bfloat16)
    if bias:
        ref = ref + b.view(1, -1, 1, 1)
        if relu:
            ref = torch.relu(ref)
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    bd = b.to(DEV)
    outs = []
    prev = _native.get_option("conv_dma")
    try:
        for dma in (2, 2, 0):  # the LDS-DMA stage fill twice (run-to-run), then register staging
            _native.set_option("conv_dma", dma)
            y = torch.empty(N, co, H, 128, dtype=torch.bfloat16, device=DEV).contiguous(memory_format=torch.channels_last)
            _native.check(lib.siren_conv_fwd(xd.data_ptr(), wd.data_ptr(), bd.data_ptr() if bias else None, int(relu),
                                             y.data_ptr(), N, H, 128, ci, co, k, _native.stream_handle(DEV)), "conv_fwd")
            outs.append(y)
    finally:
        _native.set_option("conv_dma", prev)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])  # the same stage image either way
    d = (outs[0].float().cpu() - ref.float())
    assert orc.norm_rel(outs[0].float().cpu(), ref.float()) < 4e-3
    assert (d.abs() <= ref.float().abs() * 2 ** -7 + 1e-6).float().mean() > 0.999


@pytest.mark.parametrize("k,ci,co", [(7, 64, 128), (3, 128, 64), (5, 64, 128), (7, 2, 64), (3, 2, 128), (5, 2, 96)])
@pytest.mark.parametrize("N,H,W", [(2, 128, 128), (3, 7, 64)])
def test_generic_conv_weight_gradient_kernel_against_fp32(k, ci, co, N, H, W):
    """siren_conv_wrw against the fp64 weight gradient of the same bf16 operands, bit-equal on a rerun."""
    from siren_mri_amd import _native
    lib = _native.lib()
    assert lib.siren_conv_check(1, N, H, W, ci, co, k) == 0, _native.last_error()
    g = torch.Generator().manual_seed(N * 1000 + H + W + k + ci)
    x = torch.randn(N, ci, H, W, generator=g).to(torch.bfloat16)
    dy = torch.randn(N, co, H, W, generator=g).to(torch.bfloat16)
    ref = torch.nn.grad.conv2d_weight(x.double(), (co, ci, k, k), dy.double(), padding=k // 2).float()
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    dyd = dy.to(DEV).contiguous(memory_format=torch.channels_last)
    ws = torch.empty(int(lib.siren_conv_wrw_ws_bytes(N, H, W, ci, co, k)), dtype=torch.uint8, device=DEV)
    outs = []
    prev = _native.get_option("wrw_dma")
    try:
        for dma in (prev, prev, 3):  # the default twice (run-to-run), then the 128-pixel LDS-DMA form
            _native.set_option("wrw_dma", dma)
            dw = torch.empty(co, ci, k, k, device=DEV).contiguous(memory_format=torch.channels_last)
            _native.check(lib.siren_conv_wrw(xd.data_ptr(), dyd.data_ptr(), N, H, W, ci, co, k, dw.data_ptr(),
                                             ws.data_ptr(), ws.numel(), _native.stream_handle(DEV)), "conv_wrw")
            outs.append(dw)
    finally:
        _native.set_option("wrw_dma", prev)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])  # the same K steps in the same pixel order
    assert orc.norm_rel(outs[0].cpu(), ref) < 1e-6


def test_c4_encoder_has_no_miopen_7x7():
    """Configs 4/5's encoder (kernel_size 7): cnn[0] and its gradients and conv_theta (2 input
    channels: forward and weight gradient; no input gradient) run on the native kernels."""
    from siren_mri_amd import encoder
    enc = _encoder("bf16", blocks=1, hidden=128, k=7)
    xi = torch.empty(2, 2, 128, 128, dtype=torch.bfloat16, device=DEV).contiguous(memory_format=torch.channels_last)
    wt = encoder._w_bf16(enc.conv_theta.weight)
    assert encoder._native_gen(0, xi, wt) and encoder._native_gen(1, xi, wt)
    x = torch.empty(2, 64, 128, 128, dtype=torch.bfloat16, device=DEV).contiguous(memory_format=torch.channels_last)
    wb = encoder._w_bf16(enc.cnn[0].weight)
    assert encoder._native_gen(0, x, wb) and encoder._native_gen(1, x, wb)
    g = torch.empty(2, 128, 128, 128, dtype=torch.bfloat16, device=DEV).contiguous(memory_format=torch.channels_last)
    assert encoder._native_gen(0, g, encoder._w_flip(wb))


def test_operand_prep_equals_the_casts():
    """siren_enc_prep (one launch per step) == _w_bf16 / _w_flip / .to(torch.bfloat16), bit for bit,
    for every convolution of the encoder (contiguous and channels-last fp32 filters)."""
    from siren_mri_amd import _native, encoder
    enc = _encoder("bf16", blocks=1, hidden=128, k=7)
    convs = enc._layers()
    convs[1].weight.data = convs[1].weight.data.contiguous(memory_format=torch.channels_last)
    wbs, wfs, bbs = encoder._prep_operands(convs, DEV, _native.stream_handle(DEV))
    for i, c in enumerate(convs):
        ref = encoder._w_bf16(c.weight)
        assert torch.equal(wbs[i], ref) and wbs[i].is_contiguous(memory_format=torch.channels_last), i
        assert torch.equal(bbs[i], c.bias.detach().to(torch.bfloat16)), i
        if i:
            rf = encoder._w_flip(ref)
            assert torch.equal(wfs[i], rf) and wfs[i].stride() == rf.stride(), i
        else:
            assert wfs[i] is None


def test_image_gradient_takes_the_autocast_chain():
    """An image that requires a gradient goes through the autocast chain (the fused node gives
    none): a real gradient, the chain's with the node switched off (MIOpen's convolutions are not
    bit-reproducible run to run: 1e-3)."""
    from siren_mri_amd import encoder
    enc = _encoder("bf16", blocks=1, hidden=64, k=5)
    I = torch.randn(2, 2, 128, 128, generator=torch.Generator().manual_seed(4)).to(DEV).requires_grad_(True)
    enc(I).square().sum().backward()
    g_on = I.grad.clone()
    assert g_on.abs().sum() > 0
    I.grad = None
    encoder.set_fused(False)
    try:
        enc(I).square().sum().backward()
    finally:
        encoder.set_fused(True)
    assert orc.norm_rel(g_on.cpu(), I.grad.cpu()) < 1e-3


@pytest.mark.parametrize("blocks,k", [(5, 7), (2, 3)])
def test_fused_dgrad_epilogues_match_the_passes(blocks, k):
    """The encoder's ReLU and residual-tail backward passes in the 5x5 input-gradient convolution's
    epilogue (siren_conv_dgrad_k5_fused, encoder._EPI_FUSED) against the separate passes
    (enc_relu_bwd / enc_res_bwd after siren_conv_fwd_k5): the same arithmetic element for element,
    so every weight gradient is bit-identical; the bias gradients are channel sums in another fixed
    order (1e-6). Run twice: deterministic."""
    from siren_mri_amd import encoder
    enc = _encoder("bf16", blocks=blocks, k=k, seed=4)
    g = torch.Generator().manual_seed(5)
    I = torch.randn(4, 2, 128, 128, generator=g).to(DEV)
    ge = torch.randn(4, 128, generator=g).to(DEV)
    assert enc._layers() is not None
    res = []
    for fused in (True, True, False):
        encoder._EPI_FUSED[0] = fused
        try:
            res.append(_run(enc, I, ge))
        finally:
            encoder._EPI_FUSED[0] = True
    (e1, g1), (e1b, g1b), (e0, g0) = res
    assert torch.equal(e1, e0)
    shapes = dict((n, p.shape) for n, p in enc.named_parameters())
    for n in g1:
        native_w = len(shapes[n]) == 4 and shapes[n][-1] > 1  # (the 1x1's weight gradient is MIOpen's)
        if native_w:
            assert torch.equal(g1[n], g1b[n]), n  # run to run
            assert torch.equal(g1[n], g0[n]), n
        elif len(shapes[n]) == 4:
            # the 1x1 convolution's weight gradient: MIOpen's, not bit-reproducible run to run
            # (measured 6e-6 between two identical calls); its input is bit-identical in all runs
            assert orc.norm_rel(g1[n].cpu(), g1b[n].cpu()) < 1e-4, n
            assert orc.norm_rel(g1[n].cpu(), g0[n].cpu()) < 1e-4, n
        else:
            assert orc.norm_rel(g1[n].cpu(), g1b[n].cpu()) < 1e-6, n
            assert orc.norm_rel(g1[n].cpu(), g0[n].cpu()) < 1e-6, n



def test_dma_staged_convolutions_equal_register_staged():
    """The 5x5 convolutions with their stages filled by LDS-DMA (options conv_dma, wrw_dma) against
    the register-staged kernels: the same LDS image and K order, so the encoder node's embedding and
    every gradient are bit-identical (the 1x1's MIOpen weight gradient aside, 1e-4)."""
    from siren_mri_amd import _native
    enc = _encoder("bf16", blocks=2, k=7, seed=8)
    g = torch.Generator().manual_seed(9)
    I = torch.randn(2, 2, 128, 128, generator=g).to(DEV)
    ge = torch.randn(2, 128, generator=g).to(DEV)
    res = {}
    prev, prev_w = _native.get_option("conv_dma"), _native.get_option("wrw_dma")
    for dma in (0, 1, 2):  # 2: the DMA source offsets computed once per workgroup
        _native.set_option("conv_dma", dma)
        _native.set_option("wrw_dma", 1 if dma else 0)  # the weight gradient's LDS-DMA form beside them
        try:
            res[dma] = _run(enc, I, ge)
        finally:
            _native.set_option("conv_dma", prev)
            _native.set_option("wrw_dma", prev_w)
    e0, g0 = res[0]
    shapes = dict((n, p.shape) for n, p in enc.named_parameters())
    for dma in (1, 2):
        e1, g1 = res[dma]
        assert torch.equal(e1, e0), dma
        for n in g1:
            if len(shapes[n]) == 4 and shapes[n][-1] == 1:
                assert orc.norm_rel(g1[n].cpu(), g0[n].cpu()) < 1e-4, (dma, n)
            elif n.startswith("fc") or len(shapes[n]) == 4:
                assert torch.equal(g1[n], g0[n]), (dma, n)
            else:
                assert orc.norm_rel(g1[n].cpu(), g0[n].cpu()) < 1e-6, (dma, n)
