"""Hypernetwork MRI models (meta_modules.py of jonbmartin/siren_mri) — the callers that feed the
SIREN stack batched, per-slice weights (configs 4/5).

  HyperNetwork                                          meta_modules.py:11-54
  ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures  meta_modules.py:175-237
  hyper_weight_init / hyper_bias_init                   meta_modules.py:303-321

The hypo-network is a SingleBVPNet whose forward receives the HyperNetwork's parameter dict
({'net.net.i.0.weight': [B, out, in], ...}); the native stack runs all B slices in one call with
batched weights. The encoder and the HyperNetwork's ReLU MLPs are plain PyTorch-ROCm modules.
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

    def forward(self, z):
        params = OrderedDict()
        for name, net, shape in zip(self.names, self.nets, self.param_shapes):
            params[name] = net(z).reshape((-1,) + tuple(shape))
        return params


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
