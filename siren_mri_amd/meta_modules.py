"""Hypernetwork MRI models (meta_modules.py of jonbmartin/siren_mri) — the callers that feed the
SIREN stack batched, per-slice weights (configs 4/5).

  HyperNetwork                                          meta_modules.py:11-54
  ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures  meta_modules.py:175-237
  hyper_weight_init / hyper_bias_init                   meta_modules.py:303-321

The hypo-network is a SingleBVPNet whose forward receives the HyperNetwork's parameter dict
({'net.net.i.0.weight': [B, out, in], ...}); the native stack runs all B slices in one call with
batched weights. The HyperNetwork's heads (one ReLU MLP per hypo-parameter) run as grouped native
GEMMs on CUDA fp32 (siren_hyper_forward / _backward: every head's layer of one depth in one launch);
the encoder is ConvImgEncoder (modules.py).
Deviation (bug 0.5): constructors take no `device=` argument (the reference scripts pass one the
reference constructor does not accept).
"""
from __future__ import annotations

from collections import OrderedDict

import torch
from torch import nn

from . import data_consistency, fusion, modules


def hyper_weight_init(m, in_features_main_net):
    if hasattr(m, "weight"):
        nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity="relu", mode="fan_in")
        m.weight.data = m.weight.data / 1.0e2
    if hasattr(m, "bias"):
        with torch.no_grad():
            m.bias.uniform_(-1 / in_features_main_net, 1 / in_features_main_net)


def hyper_bias_init(m):
    if hasattr(m, "weight"):
        nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity="relu", mode="fan_in")
        m.weight.data = m.weight.data / 1.0e2
    if hasattr(m, "bias"):
        fan_in, _ = nn.init._calculate_fan_in_and_fan_out(m.weight)
        with torch.no_grad():
            m.bias.uniform_(-1 / fan_in, 1 / fan_in)


class HyperNetwork(nn.Module):
    """One ReLU FCBlock per hypo-parameter; output reshaped to (-1,) + param shape."""

    def __init__(self, hyper_in_features, hyper_hidden_layers, hyper_hidden_features, hypo_module):
        super().__init__()
        self.names = []
        self.nets = nn.ModuleList()
        self.param_shapes = []
        for name, param in hypo_module.meta_named_parameters():
            self.names.append(name)
            self.param_shapes.append(param.size())
            hn = modules.FCBlock(in_features=hyper_in_features, out_features=int(param.numel()),
                                 num_hidden_layers=hyper_hidden_layers,
                                 hidden_features=hyper_hidden_features, outermost_linear=True,
                                 nonlinearity="relu")
            self.nets.append(hn)
            in_main = param.size()[-1]
            if "weight" in name:
                hn.net[-1].apply(lambda m, n=in_main: hyper_weight_init(m, n))
            elif "bias" in name:
                hn.net[-1].apply(hyper_bias_init)

    def _native_layers(self, z):
        """Per head the Linear layers [hidden..., output] when the grouped native heads take this
        call (CUDA fp32 latent [B, in], plain ReLU FCBlocks of one hidden width); else None."""
        if not (z.is_cuda and z.dtype == torch.float32 and z.dim() == 2 and len(self.nets) <= _native_hyper_maxg()):
            return None
        heads = []
        for net in self.nets:
            if not (isinstance(net, modules.FCBlock) and net.nonlinearity == "relu" and net.outermost_linear):
                return None
            lins = [net.net[i][0] for i in range(len(net.net))]
            if not 2 <= len(lins) <= 5 or any(type(m) is not modules.BatchLinear or m.bias is None for m in lins):
                return None
            if any(p.dtype != torch.float32 or p.device != z.device for m in lins for p in (m.weight, m.bias)):
                return None
            heads.append(lins)
        hid = heads[0][0].weight.shape[0]
        depth = len(heads[0]) - 1
        for lins in heads:
            if len(lins) - 1 != depth or lins[0].weight.shape[1] != z.shape[1]:
                return None
            if any(m.weight.shape[0] != hid for m in lins[:-1]) or any(m.weight.shape[1] != hid for m in lins[1:]):
                return None
        return heads

    def forward(self, z):
        heads = self._native_layers(z)
        if heads is not None:
            flat = [t for lins in heads for m in lins for t in (m.weight, m.bias)]
            outs = _HyperHeads.apply(len(heads), len(heads[0]) - 1, z, *flat)
            return OrderedDict((name, o.reshape((-1,) + tuple(shape)))
                               for name, o, shape in zip(self.names, outs, self.param_shapes))
        params = OrderedDict()
        for name, net, shape in zip(self.names, self.nets, self.param_shapes):
            params[name] = net(z).reshape((-1,) + tuple(shape))
        return params


def _native_hyper_maxg():
    from . import _native
    return _native.HYPER_MAXG


class _HyperHeads(torch.autograd.Function):
    """All heads of a HyperNetwork (meta_modules.py:48-54) in grouped native launches: forward
    siren_hyper_forward (ReLU outputs kept), backward siren_hyper_backward (every dW / db and the
    latent's gradient summed over the heads in head order). Same fp32 arithmetic as the per-head
    Linear + ReLU chain up to summation order."""

    @staticmethod
    def _desc(G, D, z, params):
        from . import _native
        d = _native.SirenHyperDesc()
        d.heads, d.depth, d.rows, d.in_features = G, D, z.shape[0], z.shape[1]
        d.hidden = params[0].shape[0]
        for g in range(G):
            for l in range(D + 1):
                W, b = params[2 * (g * (D + 1) + l)], params[2 * (g * (D + 1) + l) + 1]
                d.weight[g * 5 + l] = W.data_ptr()
                d.bias[g * 5 + l] = b.data_ptr()
            d.out_features[g] = params[2 * (g * (D + 1) + D)].shape[0]
        return d

    @staticmethod
    def forward(ctx, G, D, z, *params):
        import ctypes
        from . import _native
        lib = _native.lib()
        zc = z.detach().contiguous()
        ps = [p.detach().contiguous() for p in params]
        d = _HyperHeads._desc(G, D, zc, ps)
        saved = torch.empty(int(lib.siren_hyper_saved_bytes(ctypes.byref(d))) // 4, dtype=torch.float32, device=z.device)
        outs = [torch.empty(zc.shape[0], d.out_features[g], dtype=torch.float32, device=z.device) for g in range(G)]
        VP = ctypes.c_void_p * G
        _native.check(lib.siren_hyper_forward(ctypes.byref(d), zc.data_ptr(), VP(*[o.data_ptr() for o in outs]),
                                              saved.data_ptr(), saved.numel() * 4, _native.stream_handle(z.device)),
                      "siren_hyper_forward")
        ctx.G, ctx.D = G, D
        # the inputs themselves are saved (not detached copies) so that a create_graph backward can
        # differentiate through them
        ctx.save_for_backward(z, saved, *params)
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def _eager_backward(G, D, z, params, douts, needs):
        """create_graph=True: the per-head Linear + ReLU chain of the reference (meta_modules.py:
        48-54 through modules.FCBlock), recomputed in differentiable PyTorch and differentiated with
        the graph kept, so higher derivatives exist."""
        with torch.enable_grad():
            outs, wrt = [], [z] + list(params)
            for g in range(G):
                h = z
                for l in range(D + 1):
                    W, b = params[2 * (g * (D + 1) + l)], params[2 * (g * (D + 1) + l) + 1]
                    h = torch.nn.functional.linear(h, W, b)
                    if l < D:
                        h = torch.relu(h)
                outs.append(h)
            pairs = [(o, g) for o, g in zip(outs, douts) if g is not None]
            want = [t for t, n in zip(wrt, needs) if n]
            got = iter(torch.autograd.grad([o for o, _ in pairs], want, [g for _, g in pairs], create_graph=True,
                                           allow_unused=True) if pairs and want else [None] * len(want))
            res = [next(got) if n else None for n in needs]
        return (None, None, *res)

    @staticmethod
    def backward(ctx, *douts):
        import ctypes
        from . import _native
        G, D = ctx.G, ctx.D
        t = ctx.saved_tensors
        if torch.is_grad_enabled():
            return _HyperHeads._eager_backward(G, D, t[0], list(t[2:]), douts, ctx.needs_input_grad[2:])
        z, saved, ps = t[0].detach().contiguous(), t[1], [p.detach().contiguous() for p in t[2:]]
        lib = _native.lib()
        d = _HyperHeads._desc(G, D, z, ps)
        gs = [g.contiguous() if g is not None else torch.zeros(z.shape[0], d.out_features[i], device=z.device)
              for i, g in enumerate(douts)]
        ws = torch.empty(int(lib.siren_hyper_workspace_bytes(ctypes.byref(d))), dtype=torch.uint8, device=z.device)
        grads = [torch.empty_like(p) for p in ps]
        NW = G * 5
        dWp = (ctypes.c_void_p * NW)()
        dbp = (ctypes.c_void_p * NW)()
        for g in range(G):
            for l in range(D + 1):
                k = 2 * (g * (D + 1) + l)
                dWp[g * 5 + l] = grads[k].data_ptr()
                dbp[g * 5 + l] = grads[k + 1].data_ptr()
        need_z = ctx.needs_input_grad[2]
        dz = torch.empty_like(z) if need_z else None
        _native.check(lib.siren_hyper_backward(ctypes.byref(d), z.data_ptr(), (ctypes.c_void_p * G)(*[g.data_ptr() for g in gs]),
                                               saved.data_ptr(), saved.numel() * 4, ws.data_ptr(), ws.numel(), dWp, dbp,
                                               dz.data_ptr() if need_z else None, _native.stream_handle(z.device)),
                      "siren_hyper_backward")
        return (None, None, dz, *grads)


class ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(nn.Module):
    """k-space neural process: conv encoder -> HyperNetwork -> SIREN (batched weights) -> DC.
    precision: the SIREN stack's arithmetic (native kernels); encoder_precision: the conv
    encoder's ('fp32' = reference, 'bf16' = MIOpen bf16 channels-last, see ConvImgEncoder)."""

    # takes model_input["fourier_B"] with raw coordinates (features.py model_input): the hypo net's
    # first layer forms the Fourier features
    fourier_input = True

    def __init__(self, in_features, out_features, image_resolution=None, partial_conv=False,
                 fourier_features_size=512, latent_dim=256, hidden_features=256, num_hidden_layers=5,
                 hyper_hidden_features=512, hyper_hidden_layers=1, conv_kernel_size=3,
                 num_conv_res_blocks=4, w0=30, precision=None, encoder_precision="fp32"):
        super().__init__()
        self.dc = data_consistency.DataConsistencyInKspace(noise_lvl=None)
        if partial_conv:
            raise NotImplementedError("PartialConvImgEncoder is outside the SIREN path")
        self.encoder = modules.ConvImgEncoder(channel=2, image_resolution=image_resolution,
                                              hidden_size=latent_dim, kernel_size=conv_kernel_size,
                                              num_conv_res_blocks=num_conv_res_blocks,
                                              precision=encoder_precision)
        self.hypo_net = modules.SingleBVPNet(out_features=out_features, type="sine",
                                             sidelength=image_resolution,
                                             in_features=fourier_features_size,
                                             hidden_features=hidden_features,
                                             num_hidden_layers=num_hidden_layers, w0=w0,
                                             precision=precision)
        self.hyper_net = HyperNetwork(hyper_in_features=latent_dim,
                                      hyper_hidden_layers=hyper_hidden_layers,
                                      hyper_hidden_features=hyper_hidden_features,
                                      hypo_module=self.hypo_net)

    def forward(self, model_input):
        if model_input.get("embedding", None) is None:
            embedding = self.encoder(model_input["img_sparse"])
        else:
            embedding = model_input["embedding"]
        hypo_params = self.hyper_net(embedding)
        if "img_sparse" in model_input:
            # the planes of the DC below, for a staged fused loss (fusion.py)
            fusion.stage_dc(model_input["img_sparse"], model_input["dc_mask"],
                            float(self.dc.noise_lvl) if self.dc.noise_lvl else 0.0)
        out = self.hypo_net(model_input, params=hypo_params)
        model_out = out["model_out"]
        if "img_sparse" in model_input:
            model_out = self.dc(model_out, model_input["img_sparse"], model_input["dc_mask"])
        return {"model_in": out["model_in"], "model_out": model_out, "latent_vec": embedding,
                "hypo_params": hypo_params}

    def get_hypo_net_weights(self, model_input):
        embedding = self.encoder(model_input["img_sparse"])
        return self.hyper_net(embedding), embedding

    def freeze_hypernet(self):
        for p in self.hyper_net.parameters():
            p.requires_grad = False
        for p in self.encoder.parameters():
            p.requires_grad = False
