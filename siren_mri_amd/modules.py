"""Drop-in replacements for the reference's SIREN modules (modules.py of jonbmartin/siren_mri).

Same class names, constructor signatures, parameter names and init RNG order as:
  BatchLinear      modules.py:11-27      Sine           modules.py:30-38
  FCBlock          modules.py:40-119     SingleBVPNet   modules.py:122-170
  ImageDownsampling modules.py:192-223   ConvImgEncoder modules.py:340-380 (+ Conv2dResBlock :433-450)
  init functions   modules.py:600-654
so `state_dict`s and HyperNetwork parameter dicts interoperate with the reference.

What changes is where the work runs: an FCBlock with nonlinearity='sine' executes its whole
[BatchLinear -> Sine] stack as ONE native gfx950 forward call and ONE native backward call
(siren_mri_amd.ops.siren_mlp, libsiren_mri_amd.so). A CUDA tensor never falls back to anything
else (the ops raise if the library is missing). A CPU tensor — config 1 "on CPU (plumbing, no
GPU)" — runs the stack as plain PyTorch ops on the host (cpu_stack.py), selected by device only.
Non-sine FCBlocks (the HyperNetwork's ReLU MLPs) and the conv encoder are not on the SIREN hot
path and run as ordinary PyTorch(-ROCm) modules.

Deliberate deviations from the reference:
  * ImageDownsampling keeps `sidelength` as a device-agnostic buffer instead of calling
    `.cuda()` in __init__ (reference bug 0.4, modules.py:203).
  * SingleBVPNet mode 'rbf'/'nerf' (baselines outside the SIREN path) raise NotImplementedError.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from .meta import MetaModule, MetaSequential, get_subdict
from .ops import get_default_precision, siren_mlp


class BatchLinear(nn.Linear, MetaModule):
    """Linear layer whose weight may be replaced by a (batched) params dict (modules.py:11-27):
    out = input @ W^T + b, W either [out, in] or [B, out, in]. Used as-is only outside fused
    sine stacks (e.g. the HyperNetwork's ReLU MLPs)."""
    __doc__ = nn.Linear.__doc__

    def forward(self, input, params=None):
        if params is None:
            params = OrderedDict(self.named_parameters())
        bias = params.get("bias", None)
        weight = params["weight"]
        if (input.dim() == 2 and weight.dim() == 2 and bias is not None and bias.dim() == 1 and input.is_cuda
                and weight.shape[0] >= _WIDE_OUT and input.shape[0] <= 256):
            return _WideOutLinear.apply(input, weight, bias)
        out = input.matmul(weight.transpose(-1, -2))
        if bias is not None:
            out = out + bias.unsqueeze(-2)
        return out


_WIDE_OUT = 8192


class _WideOutLinear(torch.autograd.Function):
    """input @ W^T + b for few rows and many outputs (the HyperNetwork's heads that emit a 256x256
    hypo-weight: [B <= 256, 128] -> [B, 65536]). Same values as the matmul + add chain; its
    backward's input gradient g @ W ([B, 65536] x [65536, 128]) has a long K and a 32 x 128 output,
    which the library GEMM ran on 4 workgroups (0.24 ms); here it is split over K into a batched
    GEMM of 32 chunks and summed (a fixed order)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            n_out = w.shape[0]
            s = 32 if n_out % 32 == 0 else 1
            gs = g.reshape(g.shape[0], s, n_out // s).transpose(0, 1)      # [s, B, K/s]
            gx = torch.bmm(gs, w.reshape(s, n_out // s, w.shape[1])).sum(0)  # [B, in]
        if ctx.needs_input_grad[1]:
            gw = g.t().mm(x)
        if ctx.needs_input_grad[2]:
            gb = g.sum(0)
        return gx, gw, gb


class Sine(nn.Module):
    """sin(w0 * x) (modules.py:30-38). Inside an FCBlock it is fused into the native stack."""

    def __init__(self, w0=30):
        super().__init__()
        self.w0 = w0

    def forward(self, input):
        return torch.sin(self.w0 * input)


# ------------------------------------------------------------------------------ initialisers
def init_weights_normal(m):
    """modules.py:600-604 (ReLU): kaiming normal, fan_in."""
    if type(m) == BatchLinear or type(m) == nn.Linear:
        if hasattr(m, "weight"):
            nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity="relu", mode="fan_in")


def init_weights_selu(m):
    """modules.py:607-611."""
    if type(m) == BatchLinear or type(m) == nn.Linear:
        if hasattr(m, "weight"):
            n = m.weight.size(-1)
            nn.init.normal_(m.weight, std=1 / math.sqrt(n))


def init_weights_elu(m):
    """modules.py:614-618."""
    if type(m) == BatchLinear or type(m) == nn.Linear:
        if hasattr(m, "weight"):
            n = m.weight.size(-1)
            nn.init.normal_(m.weight, std=math.sqrt(1.5505188080679277) / math.sqrt(n))


def init_weights_xavier(m):
    """modules.py:621-624."""
    if type(m) == BatchLinear or type(m) == nn.Linear:
        if hasattr(m, "weight"):
            nn.init.xavier_normal_(m.weight)


def sine_init(m):
    """modules.py:641-646: W ~ U(+-sqrt(6/fan_in)/30)."""
    with torch.no_grad():
        if hasattr(m, "weight"):
            n = m.weight.size(-1)
            bound = np.sqrt(6 / n) / 30
            m.weight.uniform_(-bound, bound)


def first_layer_sine_init(m):
    """modules.py:649-654: W ~ U(+-1/fan_in) for the first layer."""
    with torch.no_grad():
        if hasattr(m, "weight"):
            n = m.weight.size(-1)
            m.weight.uniform_(-1 / n, 1 / n)


_NONLINEARITIES = {
    # name: (module factory, weight init, first-layer init)   (modules.py:53-59)
    "sine": (lambda w0: Sine(w0=w0), sine_init, first_layer_sine_init),
    "relu": (lambda w0: nn.ReLU(inplace=True), init_weights_normal, None),
    "sigmoid": (lambda w0: nn.Sigmoid(), init_weights_xavier, None),
    "tanh": (lambda w0: nn.Tanh(), init_weights_xavier, None),
    "selu": (lambda w0: nn.SELU(inplace=True), init_weights_selu, None),
    "softplus": (lambda w0: nn.Softplus(), init_weights_normal, None),
    "elu": (lambda w0: nn.ELU(inplace=True), init_weights_elu, None),
}


class FCBlock(MetaModule):
    """Fully connected block (modules.py:40-119), hypernetwork-compatible.

    Layout (and hence parameter names) is the reference's:
    net = MetaSequential(MetaSequential(BatchLinear, nl), ..., MetaSequential(BatchLinear[, nl])).
    With nonlinearity='sine' the forward is the fused native stack; `precision` selects its
    arithmetic ('fp32' — the reference's — or 'bf16' operands with fp32 accumulation).
    """

    def __init__(self, in_features, out_features, num_hidden_layers, hidden_features,
                 outermost_linear=False, nonlinearity="relu", weight_init=None, w0=30,
                 precision=None):
        super().__init__()
        self.first_layer_init = None
        make_nl, nl_weight_init, first_layer_init = _NONLINEARITIES[nonlinearity]
        self.weight_init = weight_init if weight_init is not None else nl_weight_init
        self.nonlinearity = nonlinearity
        self.outermost_linear = outermost_linear
        self.w0 = w0
        self.precision = precision

        layers = [MetaSequential(BatchLinear(in_features, hidden_features), make_nl(w0))]
        for _ in range(num_hidden_layers):
            layers.append(MetaSequential(BatchLinear(hidden_features, hidden_features), make_nl(w0)))
        if outermost_linear:
            layers.append(MetaSequential(BatchLinear(hidden_features, out_features)))
        else:
            layers.append(MetaSequential(BatchLinear(hidden_features, out_features), make_nl(w0)))
        self.net = MetaSequential(*layers)
        if self.weight_init is not None:
            self.net.apply(self.weight_init)
        if first_layer_init is not None:
            self.net[0].apply(first_layer_init)

    @property
    def num_linear(self) -> int:
        return len(self.net)

    def layer_params(self, params=None):
        """(weights, biases) lists of the linear layers, from `params` or the module's own."""
        if params is None:
            lin = self.__dict__.get("_linears")
            if lin is None or len(lin) != len(self.net) or any(
                    self.net[i][0] is not m for i, m in ((0, lin[0]), (len(lin) - 1, lin[-1]))):
                lin = [self.net[i][0] for i in range(self.num_linear)]  # (Sequential indexing is slow)
                self.__dict__["_linears"] = lin
            ws = [m.weight for m in lin]
            bs = [m.bias for m in lin]
        else:
            ws = [params[f"{i}.0.weight"] for i in range(self.num_linear)]
            bs = [params[f"{i}.0.bias"] for i in range(self.num_linear)]
        return ws, bs

    def forward(self, coords, params=None, ff_B=None, **kwargs):
        """ff_B: coords are raw coordinates whose Gaussian Fourier features (features.py:21-41) are
        the block's input (ops.siren_mlp forms them in the first layer where it can)."""
        sub = get_subdict(params, "net") if params is not None else None
        if self.nonlinearity == "sine":
            ws, bs = self.layer_params(sub)
            return siren_mlp(coords, ws, bs, w0=self.w0,
                             precision=self.precision or get_default_precision(),
                             outermost_linear=self.outermost_linear, ff_B=ff_B)
        if ff_B is not None:
            from .features import fourier_features
            coords = fourier_features(coords, ff_B)
        return self.net(coords, params=sub)

    def forward_with_activations(self, coords, params=None, retain_grad=False):
        """Per-layer activations (modules.py:99-119) — a diagnostics path (summaries), computed
        with plain device ops, not the fused kernels."""
        if params is None:
            params = OrderedDict(self.named_parameters())
        activations = OrderedDict()
        x = coords.clone().detach().requires_grad_(True)
        activations["input"] = x
        for i, layer in enumerate(self.net):
            sub = get_subdict(params, "net.%d" % i)
            for j, sublayer in enumerate(layer):
                if isinstance(sublayer, BatchLinear):
                    x = sublayer(x, params=get_subdict(sub, "%d" % j))
                else:
                    x = sublayer(x)
                if retain_grad:
                    x.retain_grad()
                activations["_".join((str(sublayer.__class__), "%d" % i))] = x
        return activations


class ImageDownsampling(nn.Module):
    """modules.py:192-223. `sidelength` is a buffer (no `.cuda()` at construction — bug 0.4)."""

    def __init__(self, sidelength, downsample=False):
        super().__init__()
        if isinstance(sidelength, int):
            sidelength = (sidelength, sidelength)
        if sidelength is None:
            assert downsample is False
            self.register_buffer("sidelength", None, persistent=False)
        else:
            self.register_buffer("sidelength", torch.tensor(sidelength, dtype=torch.float32),
                                 persistent=False)
        self.downsample = downsample

    def forward(self, coords):
        if self.downsample:
            return coords + self.forward_bilinear(coords)
        return coords

    def forward_box(self, coords):
        return 2 * (torch.rand_like(coords) - 0.5) / self.sidelength

    def forward_bilinear(self, coords):
        Y = torch.sqrt(torch.rand_like(coords)) - 1
        Z = 1 - torch.sqrt(torch.rand_like(coords))
        b = torch.rand_like(coords) < 0.5
        return (b * Y + ~b * Z) / self.sidelength


class SingleBVPNet(MetaModule):
    """Canonical SIREN representation network (modules.py:122-170), mode='mlp'."""

    def __init__(self, out_features=1, type="sine", in_features=2, mode="mlp", hidden_features=256,
                 num_hidden_layers=3, w0=30, **kwargs):
        super().__init__()
        self.mode = mode
        if mode != "mlp":
            raise NotImplementedError(
                f"SingleBVPNet mode={mode!r}: only the SIREN 'mlp' mode is on the MI355X path")
        self.image_downsampling = ImageDownsampling(sidelength=kwargs.get("sidelength", None),
                                                    downsample=kwargs.get("downsample", False))
        self.net = FCBlock(in_features=in_features, out_features=out_features,
                           num_hidden_layers=num_hidden_layers, hidden_features=hidden_features,
                           outermost_linear=True, nonlinearity=type, w0=w0,
                           precision=kwargs.get("precision", None))
        if kwargs.get("verbose", False):
            print(self)

    def forward(self, model_input, params=None):
        # grad leaf for derivatives w.r.t. coordinates (modules.py:151). The reference clones first;
        # a detached alias is the same leaf without a copy (nothing writes coordinates in place).
        ff_B = model_input.get("fourier_B")
        if ff_B is not None and not self.image_downsampling.downsample:
            # raw coordinates + B (features.py GaussianFourierFeatureTransform.model_input): the
            # SIREN's first layer forms the features; model_in is then the raw coordinates, and
            # derivatives w.r.t. the features need the materialised path (fusion off)
            coords = model_input["coords"]
            return {"model_in": coords, "model_out": self.net(coords, get_subdict(params, "net"), ff_B=ff_B)}
        if ff_B is not None:
            from .features import fourier_features
            model_input = dict(model_input, coords=fourier_features(model_input["coords"], ff_B))
        coords_org = model_input["coords"].detach().requires_grad_(True)
        coords = coords_org
        if self.image_downsampling.downsample:
            coords = self.image_downsampling(coords)
        output = self.net(coords, get_subdict(params, "net"))
        out = {"model_in": coords_org, "model_out": output}
        if self.net.nonlinearity == "sine" and not self.image_downsampling.downsample and output.is_cuda:
            # (on a CPU device the stack's autograd graph gives the derivatives, as in the reference)
            from .diff_operators import register_siren_output
            register_siren_output(output, coords_org, self.net, get_subdict(params, "net"))
        return out

    def forward_with_activations(self, model_input):
        coords = model_input["coords"].clone().detach().requires_grad_(True)
        activations = self.net.forward_with_activations(coords)
        return {"model_in": coords, "model_out": activations.popitem(), "activations": activations}


# ------------------------------------------------------------------------------ conv encoder
class Conv2dResBlock(nn.Module):
    """modules.py:433-450 (plain PyTorch-ROCm / MIOpen; not on the SIREN path)."""

    def __init__(self, in_channel, out_channel=128):
        super().__init__()
        self.convs = nn.Sequential(
            nn.Conv2d(in_channel, out_channel, 5, 1, 2),
            nn.ReLU(),
            nn.Conv2d(out_channel, out_channel, 5, 1, 2),
            nn.ReLU(),
        )
        self.final_relu = nn.ReLU()

    def forward(self, x):
        return self.final_relu(self.convs(x) + x)


class ConvImgEncoder(nn.Module):
    """modules.py:340-380: conv stem -> residual blocks -> 1x1 -> per-channel FC over pixels.
    Plain PyTorch-ROCm (MIOpen convolutions); the SIREN it feeds is the native path.

    precision='fp32' is the reference's arithmetic. precision='bf16'  runs
    the convolutions in bf16 on MIOpen with channels-last (NHWC) activations and weights — the
    layout MIOpen's bf16 implicit-GEMM kernels take without transposes — under autocast, with
    fp32 master weights and gradients; the final per-channel FC over the 128^2 pixels (a 16,384-term
    dot product per channel) stays fp32."""

    def __init__(self, channel, image_resolution, hidden_size=256, kernel_size=3, num_conv_res_blocks=4,
                 precision="fp32"):
        super().__init__()
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"ConvImgEncoder precision {precision!r}: 'fp32' or 'bf16'")
        self.hidden_size = hidden_size
        self.precision = precision
        padding = kernel_size // 2
        self.conv_theta = nn.Conv2d(channel, hidden_size // 2, kernel_size, 1, padding)
        self.relu = nn.ReLU(inplace=True)
        layers = [nn.Conv2d(hidden_size // 2, hidden_size, kernel_size, 1, padding), nn.ReLU()]
        layers += [Conv2dResBlock(hidden_size, hidden_size) for _ in range(num_conv_res_blocks)]
        layers.append(nn.Conv2d(hidden_size, hidden_size, 1, 1, 0))
        self.cnn = nn.Sequential(*layers)
        self.relu_2 = nn.ReLU(inplace=True)
        self.fc = nn.Linear(image_resolution[0] * image_resolution[1], 1)
        self.image_resolution = image_resolution
        self._nhwc = False

    def _layers(self):
        """The convolutions in order (conv_theta, cnn[0], each block's two, the 1x1) for the fused
        bf16 node (siren_mri_amd/encoder.py), or None when the structure is not the built one."""
        from . import encoder
        if "_enc_layers" not in self.__dict__:
            layers = None
            mods = list(self.cnn)
            blocks = [m for m in mods if isinstance(m, Conv2dResBlock)]
            if (len(mods) == len(blocks) + 3 and isinstance(mods[0], nn.Conv2d) and isinstance(mods[1], nn.ReLU)
                    and all(isinstance(m, Conv2dResBlock) for m in mods[2:-1]) and isinstance(mods[-1], nn.Conv2d)
                    and all(len(b.convs) == 4 and isinstance(b.convs[1], nn.ReLU) and isinstance(b.convs[3], nn.ReLU)
                            for b in blocks)):
                layers = [self.conv_theta, mods[0]]
                for b in blocks:
                    layers += [b.convs[0], b.convs[2]]
                layers.append(mods[-1])
            self.__dict__["_enc_layers"] = layers
            self.__dict__["_enc_nblocks"] = len(blocks)
            if layers is not None and not encoder.supported(self):
                self.__dict__["_enc_layers"] = None
        return self.__dict__["_enc_layers"]

    def forward(self, I):
        if self.precision == "bf16" and I.is_cuda:
            from . import encoder
            if not self._nhwc:
                # conv weights to channels-last once (their .grad follows the parameter's layout)
                for m in self.modules():
                    if isinstance(m, nn.Conv2d):
                        m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
                self._nhwc = True
            # the fused node gives no gradient into the image: an image that requires one takes
            # the autocast chain
            if encoder.fused_enabled() and self._layers() is not None and not I.requires_grad:
                return encoder.encoder_bf16(self, I)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                o = self.relu(self.conv_theta(I.contiguous(memory_format=torch.channels_last)))
                o = self.relu_2(self.cnn(o))
            o = o.float().contiguous().view(o.shape[0], self.hidden_size, -1)
            return self.fc(o).squeeze(-1)
        o = self.relu(self.conv_theta(I))
        o = self.cnn(o)
        return self.fc(self.relu_2(o).view(o.shape[0], self.hidden_size, -1)).squeeze(-1)
