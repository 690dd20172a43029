"""bf16 forward and backward of ConvImgEncoder (modules.py:340-380, Conv2dResBlock modules.py:433-450)
as ONE autograd node (configs 4/5).

The reference's autograd chain runs, around each convolution, a ReLU, its mask in the backward, a
bias-gradient reduction and the residual adds as separate passes over 134 MB planes (C4: 32 x 128^2
x 128 channels in bf16), and the final Linear over the 16,384 pixels as a cast copy + GEMV. Here:

  forward   the residual blocks' 128 -> 128 5x5 convolutions on a native implicit-GEMM MFMA
            kernel (siren_conv_fwd_k5: bias + ReLU in its epilogue), the other shapes on MIOpen
            bias-free (PyTorch would add a bias in a separate pass) + one bias/ReLU pass
            (siren_enc_bias_relu); each residual block's tail relu(relu(a + b) + x) in one pass
            (siren_enc_res_fwd); the 1x1 conv's bias + relu_2 + the pixel Linear as one reduction
            (siren_enc_pixfc_fwd, fp32 out).
  backward  the pixel Linear's three gradients and conv_1x1's ReLU mask + bias gradient in one pass
            (siren_enc_pixfc_bwd); each block's mask / skip / bias-gradient work in one pass
            (siren_enc_res_bwd, siren_enc_relu_bwd, the skip gradient added inside the next mask
            pass instead of by a separate add); conv input gradients as FORWARD convolutions with
            the flipped, transposed filter (stride 1, 'same' padding: the same GEMM, on the faster
            forward kernels); conv weight gradients alone (aten.convolution_backward, weight mask).

Arithmetic as the bf16 autocast path (modules.py ConvImgEncoder precision='bf16'): bf16 operands and
activations, fp32 accumulation, fp32 master weights and gradients; the conv bias gradients and the
pixel Linear are accumulated in fp32 (the autocast chain rounds them through bf16).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native

_CL = torch.channels_last
_FUSED = [True]


def set_fused(enabled: bool) -> None:
    """Process-wide switch: the fused node (default) or the autocast chain (A/B, tests)."""
    _FUSED[0] = bool(enabled)


def fused_enabled() -> bool:
    return _FUSED[0]


def _ok_channels(c: int) -> bool:
    return 8 <= c <= 256 and (c & (c - 1)) == 0


def supported(enc) -> bool:
    """The layer structure this node takes (ConvImgEncoder as modules.py builds it)."""
    convs = [m for m in enc.modules() if isinstance(m, torch.nn.Conv2d)]  # the residual blocks' too
    if not all(c.stride == (1, 1) and c.dilation == (1, 1) and c.groups == 1 and c.bias is not None
               and c.kernel_size[0] == c.kernel_size[1] and c.kernel_size[0] % 2 == 1
               and c.padding == (c.kernel_size[0] // 2,) * 2 for c in convs):
        return False
    return all(_ok_channels(c.out_channels) for c in convs)


def _w_bf16(w):
    return w.detach().to(torch.bfloat16).contiguous(memory_format=_CL)


ENC_PREP_MAX = 32  # filters per siren_enc_prep launch (csrc/siren_encoder.hip)


def _prep_operands(convs, dev, stream):
    """Every convolution's bf16 channels-last filter, its input gradient's flipped / transposed bf16
    filter (none for conv_theta: no gradient into the image) and its bf16 bias, in one launch
    (siren_enc_prep; the casts of _w_bf16 / _w_flip / .to(torch.bfloat16), bit for bit)."""
    import ctypes
    n = len(convs)
    wbs, wfs, bbs, geom = [], [], [], []
    for i, c in enumerate(convs):
        co, ci, kh, kw = c.weight.shape
        wbs.append(torch.empty((co, ci, kh, kw), dtype=torch.bfloat16, device=dev, memory_format=_CL))
        wfs.append(torch.empty((ci, co, kh, kw), dtype=torch.bfloat16, device=dev, memory_format=_CL) if i else None)
        bbs.append(torch.empty(co, dtype=torch.bfloat16, device=dev))
        geom += [co, ci, kh, *c.weight.stride()]
    # one launch per ENC_PREP_MAX filters (an encoder with more than 14 residual blocks has more
    # than 32 convolutions)
    for a in range(0, n, ENC_PREP_MAX):
        b = min(n, a + ENC_PREP_MAX)
        VP = ctypes.c_void_p * (b - a)
        _native.check(_native.lib().siren_enc_prep(
            b - a, VP(*[c.weight.data_ptr() for c in convs[a:b]]), VP(*[c.bias.data_ptr() for c in convs[a:b]]),
            (ctypes.c_int64 * (7 * (b - a)))(*geom[7 * a:7 * b]), VP(*[t.data_ptr() for t in wbs[a:b]]),
            VP(*[t.data_ptr() if t is not None else None for t in wfs[a:b]]), VP(*[t.data_ptr() for t in bbs[a:b]]),
            stream), "siren_enc_prep")
    return wbs, wfs, bbs


def _w_flip(wb):
    """Filter of the input gradient as a forward convolution: W'[ci][co] = W[co][ci] rotated 180."""
    return wb.flip(2, 3).transpose(0, 1).contiguous(memory_format=_CL)


_CONV_NATIVE = [True]
_CONV_OK = {}


def _native_conv(x, wb):
    co, ci, k, _ = wb.shape
    n, _, h, w = x.shape
    return _CONV_NATIVE[0] and co == ci == 128 and k == 5 and w == 128 and h % 2 == 0


def _native_gen(kind, x, wb):
    """Whether the generic native kernels (siren_conv_fwd / siren_conv_wrw: 3x3 / 5x5 / 7x7, 2, 64
    or 128 input channels) take this shape (kind 0 forward, 1 weight gradient)."""
    co, ci, k, _ = wb.shape
    n, _, h, w = x.shape
    key = (kind, n, h, w, ci, co, k)
    hit = _CONV_OK.get(key)
    if hit is None:
        hit = _CONV_OK[key] = _native.lib().siren_conv_check(kind, n, h, w, ci, co, k) == 0
    return _CONV_NATIVE[0] and hit


def _conv(x, wb, bb, pad, relu=False):
    """Stride-1 'same' convolution, bf16 NHWC out: the native MFMA kernels — the residual blocks'
    128 -> 128 5x5 shape (siren_conv_fwd_k5), the other 3x3 / 5x5 / 7x7 shapes with 2, 64 or 128
    input channels (siren_conv_fwd: conv_theta, cnn[0] and its input gradient), bias + ReLU in
    their epilogue — and MIOpen for the rest (the 1x1, other widths; relu=True needs a bias on that
    path and is applied by siren_enc_bias_relu)."""
    if _native_conv(x, wb):
        n, _, h, w = x.shape
        y = torch.empty((n, wb.shape[0], h, w), dtype=torch.bfloat16, device=x.device, memory_format=_CL)
        _native.check(_native.lib().siren_conv_fwd_k5(x.data_ptr(), wb.data_ptr(),
                                                      bb.data_ptr() if bb is not None else None, 1 if relu else 0,
                                                      y.data_ptr(), n, h, w, wb.shape[1],
                                                      _native.stream_handle(x.device)), "siren_conv_fwd_k5")
        return y
    if _native_gen(0, x, wb):
        n, ci, h, w = x.shape
        co, k = wb.shape[0], wb.shape[2]
        y = torch.empty((n, co, h, w), dtype=torch.bfloat16, device=x.device, memory_format=_CL)
        _native.check(_native.lib().siren_conv_fwd(x.data_ptr(), wb.data_ptr(), bb.data_ptr() if bb is not None else None,
                                                   1 if relu else 0, y.data_ptr(), n, h, w, ci, co, k,
                                                   _native.stream_handle(x.device)), "siren_conv_fwd")
        return y
    y = F.conv2d(x, wb, None if relu else bb, padding=pad).contiguous(memory_format=_CL)
    if relu:
        P, C = _plane(y)
        _native.check(_native.lib().siren_enc_bias_relu(y.data_ptr(), bb.data_ptr() if bb is not None else None, P, C,
                                                        _native.stream_handle(x.device)), "siren_enc_bias_relu")
    return y


# the encoder's backward passes in the input-gradient convolutions' epilogues (siren_conv_dgrad_k5_fused)
_EPI_FUSED = [True]


def _epilogue_ok(dy, wf):
    """The native 5x5 kernel takes this input gradient and the encoder workspace holds its
    per-workgroup channel sums (N H / 2 rows of 128)."""
    if not (_EPI_FUSED[0] and _native_conv(dy, wf)):
        return False
    n, _, h, _ = dy.shape
    return n * (h // 2) * 128 * 4 <= _native.enc_workspace(dy.device).numel()


def _dgrad_fused(mode, dy, wf, g2, m, pa, cb, db, ws):
    """The input gradient conv(dy, wf) with the next backward pass in its epilogue: mode 1 the ReLU
    backward (out = (g [+ g2]) (m > 0)), mode 2 the residual tail's (skip gradient out, and
    out2 = out (bf16(pa + cb) > 0)); db receives the channel sums (see siren_conv_dgrad_k5_fused)."""
    n, _, h, w = dy.shape
    out = torch.empty_like(m)
    out2 = torch.empty_like(m) if mode == 2 else None
    _native.check(_native.lib().siren_conv_dgrad_k5_fused(
        mode, dy.data_ptr(), wf.data_ptr(), g2.data_ptr() if g2 is not None else None, m.data_ptr(),
        pa.data_ptr() if pa is not None else None, cb.data_ptr() if cb is not None else None, out.data_ptr(),
        out2.data_ptr() if out2 is not None else None, db.data_ptr(), n, h, w, wf.shape[1], ws.data_ptr(),
        ws.numel(), _native.stream_handle(dy.device)), "siren_conv_dgrad_k5_fused")
    return out, out2


_WGRAD_NATIVE = [True]


def _wgrad(g, x, wb, pad):
    """dL/dW of a stride-1 'same' convolution: the native MFMA kernels for the residual blocks'
    128 -> 128 5x5 shape (siren_conv_wrw_k5) and the other 3x3 / 5x5 / 7x7 shapes with 2, 64 or
    128 input channels (siren_conv_wrw), fp32 out in the filter's channels-last layout; MIOpen's
    weight-gradient convolution otherwise (the 1x1)."""
    co, ci, k, _ = wb.shape
    n, _, h, w = x.shape
    if _WGRAD_NATIVE[0] and co == ci == 128 and k == 5 and w % 64 == 0:
        lib = _native.lib()
        dw = torch.empty(wb.shape, dtype=torch.float32, device=x.device, memory_format=_CL)
        ws = torch.empty(int(lib.siren_conv_wrw_workspace_bytes(n, h, w)), dtype=torch.uint8, device=x.device)
        _native.check(lib.siren_conv_wrw_k5(x.data_ptr(), g.data_ptr(), n, h, w, ci, dw.data_ptr(), ws.data_ptr(),
                                            ws.numel(), _native.stream_handle(x.device)), "siren_conv_wrw_k5")
        return dw
    if _WGRAD_NATIVE[0] and _native_gen(1, x, wb):
        lib = _native.lib()
        dw = torch.empty(wb.shape, dtype=torch.float32, device=x.device, memory_format=_CL)
        ws = torch.empty(int(lib.siren_conv_wrw_ws_bytes(n, h, w, ci, co, k)), dtype=torch.uint8, device=x.device)
        _native.check(lib.siren_conv_wrw(x.data_ptr(), g.data_ptr(), n, h, w, ci, co, k, dw.data_ptr(), ws.data_ptr(),
                                         ws.numel(), _native.stream_handle(x.device)), "siren_conv_wrw")
        return dw
    return torch.ops.aten.convolution_backward(g, x, wb, None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


def _plane(t):
    """(P, C) of an NHWC tensor (channels-last contiguous)."""
    n, c, h, w = t.shape
    return n * h * w, c


class _EncoderBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc, I, *params):
        dev = I.device
        lib = _native.lib()
        stream = _native.stream_handle(dev)
        ws = _native.enc_workspace(dev)
        convs = ctx.convs = enc._enc_layers
        wbs, wfs, bbs = _prep_operands(convs, dev, stream)
        ctx.wfs = wfs
        x0 = I.detach().to(torch.bfloat16).contiguous(memory_format=_CL)
        saved = [x0]

        # each convolution bias-free, its bias (+ ReLU) in the native kernel's epilogue or in one
        # pass after MIOpen's (PyTorch would add a bias in a separate pass)
        t = _conv(x0, wbs[0], bbs[0], convs[0].padding[0], relu=True)
        saved.append(t)
        t = _conv(t, wbs[1], bbs[1], convs[1].padding[0], relu=True)
        saved.append(t)
        k = 2
        for _ in range(enc._enc_nblocks):
            h = _conv(t, wbs[k], bbs[k], convs[k].padding[0], relu=True)
            if _EPI_FUSED[0] and _native_conv(h, wbs[k + 1]):
                # the block's tail in the second convolution's epilogue (siren_conv_fwd_k5_res)
                a = torch.empty_like(h)
                out = torch.empty_like(h)
                n_, _, h_, w_ = h.shape
                _native.check(lib.siren_conv_fwd_k5_res(h.data_ptr(), wbs[k + 1].data_ptr(), bbs[k + 1].data_ptr(),
                                                        t.data_ptr(), a.data_ptr(), out.data_ptr(), n_, h_, w_,
                                                        h.shape[1], stream), "siren_conv_fwd_k5_res")
            else:
                a = _conv(h, wbs[k + 1], None, convs[k + 1].padding[0])  # bias added in the tail pass
                out = torch.empty_like(a)
                P, C = _plane(a)
                _native.check(lib.siren_enc_res_fwd(a.data_ptr(), bbs[k + 1].data_ptr(), t.data_ptr(), out.data_ptr(),
                                                    P, C, stream), "siren_enc_res_fwd")
            saved += [h, a, out]
            t = out
            k += 2
        a = _conv(t, wbs[k], None, convs[k].padding[0])  # the 1x1 conv; its bias and relu_2 in the pixfc pass
        saved.append(a)
        B = a.shape[0]
        P = a.shape[2] * a.shape[3]
        C = a.shape[1]
        fc = enc.fc
        e = torch.empty(B, C, dtype=torch.float32, device=dev)
        _native.check(lib.siren_enc_pixfc_fwd(a.data_ptr(), bbs[k].data_ptr(), fc.weight.detach().contiguous().data_ptr(),
                                              fc.bias.detach().data_ptr(), e.data_ptr(), B, P, C, ws.data_ptr(),
                                              ws.numel(), stream), "siren_enc_pixfc_fwd")
        ctx.bbs = bbs
        ctx.enc = enc
        ctx.wbs = wbs
        ctx.save_for_backward(*saved)
        ctx.set_materialize_grads(False)
        return e

    @staticmethod
    def backward(ctx, ge):
        enc, convs, wbs, bbs = ctx.enc, ctx.convs, ctx.wbs, ctx.bbs
        nparams = 2 * len(convs) + 2
        if ge is None:
            return (None, None) + (None,) * nparams
        saved = list(ctx.saved_tensors)
        dev = ge.device
        lib = _native.lib()
        stream = _native.stream_handle(dev)
        ws = _native.enc_workspace(dev)
        wsp, wsn = ws.data_ptr(), ws.numel()
        fc = enc.fc
        gW = [None] * len(convs)
        gb = [None] * len(convs)
        # relu_2 + pixel Linear, and the 1x1 conv's mask / bias gradient
        a = saved.pop()
        B, C = a.shape[0], a.shape[1]
        P = a.shape[2] * a.shape[3]
        gec = ge.detach().to(torch.float32).contiguous()
        ga = torch.empty_like(a)
        k = len(convs) - 1
        gb[k] = torch.empty(C, dtype=torch.float32, device=dev)
        gfw = torch.empty(P, dtype=torch.float32, device=dev)
        _native.check(lib.siren_enc_pixfc_bwd(gec.data_ptr(), a.data_ptr(), bbs[k].data_ptr(),
                                              fc.weight.detach().contiguous().data_ptr(), ga.data_ptr(), gb[k].data_ptr(), gfw.data_ptr(), B, P, C, wsp, wsn,
                                              stream), "siren_enc_pixfc_bwd")
        g_fc_w = gfw.view_as(fc.weight)
        g_fc_b = gec.sum().reshape(fc.bias.shape)
        xin = saved[-1]  # the 1x1 conv's input (the last block's output, or cnn[0]'s)
        pad = convs[k].padding[0]
        gW[k] = _wgrad(ga, xin, wbs[k], pad)
        g1 = _conv(ga, ctx.wfs[k], None, pad)
        g2 = None
        # an input-gradient convolution not yet run: (its input, filter, padding); the pass that
        # consumes its output runs in its epilogue where the native 5x5 kernel takes it
        # (siren_conv_dgrad_k5_fused), else g1 is formed and the pass runs on its own
        pending = None

        def form_g1():
            return _conv(pending[0], pending[1], None, pending[2]) if pending is not None else g1

        # residual blocks, last to first
        for _ in range(enc._enc_nblocks):
            k -= 2
            out = saved.pop()
            a = saved.pop()
            h = saved.pop()
            t = saved[-1]  # the block's input
            P, C = _plane(a)
            gb[k + 1] = torch.empty(C, dtype=torch.float32, device=dev)
            if pending is not None and g2 is not None and _epilogue_ok(pending[0], pending[1]):
                gskip, ga = _dgrad_fused(2, pending[0], pending[1], g2, out, a, bbs[k + 1], gb[k + 1], ws)
            else:
                g1 = form_g1()
                gskip = torch.empty_like(a)
                ga = torch.empty_like(a)
                _native.check(lib.siren_enc_res_bwd(g1.data_ptr(), g2.data_ptr() if g2 is not None else None,
                                                    out.data_ptr(), a.data_ptr(), bbs[k + 1].data_ptr(),
                                                    gskip.data_ptr(), ga.data_ptr(), gb[k + 1].data_ptr(), P, C, wsp,
                                                    wsn, stream), "siren_enc_res_bwd")
            pending = None
            pad = convs[k + 1].padding[0]
            gW[k + 1] = _wgrad(ga, h, wbs[k + 1], pad)
            P, C = _plane(h)
            gb[k] = torch.empty(C, dtype=torch.float32, device=dev)
            if _epilogue_ok(ga, ctx.wfs[k + 1]):
                ghm, _ = _dgrad_fused(1, ga, ctx.wfs[k + 1], None, h, None, None, gb[k], ws)
            else:
                gh = _conv(ga, ctx.wfs[k + 1], None, pad)
                ghm = torch.empty_like(h)
                _native.check(lib.siren_enc_relu_bwd(gh.data_ptr(), None, h.data_ptr(), ghm.data_ptr(),
                                                     gb[k].data_ptr(), P, C, wsp, wsn, stream), "siren_enc_relu_bwd")
            pad = convs[k].padding[0]
            gW[k] = _wgrad(ghm, t, wbs[k], pad)
            pending = (ghm, ctx.wfs[k], pad)
            g2 = gskip
        # cnn[0] and conv_theta (each followed by a ReLU); no gradient into the image
        for k in (1, 0):
            y = saved.pop()
            xin = saved[-1]
            P, C = _plane(y)
            gb[k] = torch.empty(C, dtype=torch.float32, device=dev)
            if pending is not None and _epilogue_ok(pending[0], pending[1]):
                gm, _ = _dgrad_fused(1, pending[0], pending[1], g2, y, None, None, gb[k], ws)
            else:
                g1 = form_g1()
                gm = torch.empty_like(y)
                _native.check(lib.siren_enc_relu_bwd(g1.data_ptr(), g2.data_ptr() if g2 is not None else None,
                                                     y.data_ptr(), gm.data_ptr(), gb[k].data_ptr(), P, C, wsp, wsn,
                                                     stream), "siren_enc_relu_bwd")
            pending = None
            pad = convs[k].padding[0]
            gW[k] = _wgrad(gm, xin, wbs[k], pad)
            if k == 1:
                g1 = _conv(gm, ctx.wfs[k], None, pad)
                g2 = None
        grads = []
        for k, c in enumerate(convs):
            grads.append(gW[k].to(torch.float32).contiguous(memory_format=_CL)
                         if c.weight.is_contiguous(memory_format=_CL) else gW[k].to(torch.float32).contiguous())
            grads.append(gb[k])
        grads += [g_fc_w, g_fc_b]
        return (None, None, *grads)


def encoder_bf16(enc, I):
    """ConvImgEncoder.forward for precision='bf16' on the GPU (see the module docstring)."""
    params = []
    for c in enc._enc_layers:
        params += [c.weight, c.bias]
    params += [enc.fc.weight, enc.fc.bias]
    return _EncoderBF16.apply(enc, I, *params)
