"""Benchmark: SIREN fitting throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config m|c1|c2|c3|c4|c4_fp32|m_fp32|m_shard8]
                    [--scaling weak|strong] [--precision bf16|fp32] [--no-graph]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workloads (BASELINE.json configs); the default is M, the metric's:
  m   train_img.py fit step: 512^2 coordinate grid (262,144 coords per GPU per step, full batch),
      SingleBVPNet 2-256-256-256-256-1 (w0=30), image_mse + Adam(1e-4), bf16 kernels. Synthetic
      target: a smooth random image (sum of 32 sinusoids).
  c1  64^2 cameraman, 2-256-256-1 ("3x256" = num_hidden_layers 1), image_mse + Adam, bf16.
  c2  256^2 IRData slice 0 (/max, x2-1, bilinear 256^2), 5x256, image_mse + Adam, bf16.
  c3  512^2 + gradients_mse (analytic gradient and its double backward), 5x256, fp32.
  c4  hypernetwork MRI neural process (reference config hyperoptIV_homebrew): 32 k-space slices
      of 128^2 per GPU per step, conv encoder (bf16 channels-last) -> hypernetwork -> SIREN
      16-256-256-256-256-2 with per-slice weights (bf16) -> data consistency, image_hypernetwork_loss,
      clip_grad_norm_(1.0), Adam(5.57e-5).
  c4_fp32  the same step in the reference's arithmetic: fp32 encoder (MIOpen, immediate mode) and
      fp32 SIREN (tests/test_gpu_c4_precision.py checks the two at equal steps).
  m_fp32   the metric fit in fp32 (exact-fp32 MFMA), the reference's arithmetic.
  m_shard8 rank 0's 1/8 row shard of the metric grid without the exchange (the compute-only bound of
      the 8-GPU strong-scaling speed-up).
One step = forward + loss + backward (+ N>1: the gradient all-reduce over RCCL) + Adam.

Scaling: weak (default; every rank owns its own full-size problem: a 512^2 block of a 512 x 512N
image, or its own 32 slices) or strong (--scaling strong: ONE global grid split into contiguous
row blocks by training_ddp.shard_rows; the summed gradient all-reduce makes it the single-GPU fit).

Timed regions (each EXACTLY K steps between barrier + synchronize): one replay of a hipGraph
holding K captured steps, and K eager steps. --timing auto (default) runs both and reports the
faster as `value` (both in config.ms_per_step_by_region): graph replay removes the host's
per-step launch work, which decides small grids (C1, C2), while eager back-to-back launches are
faster for the 512^2 step on ROCm 7 (graph kernel nodes add a few us each). The dominant
kernel's launches are bracketed by HIP event pairs on its launch stream in the eager region (ROCm
reports no elapsed time between events recorded inside a graph).

Prints ONE JSON line on rank 0: value (coord-samples/s, whole job), roofline of the dominant
kernel (MFMA-bound per SURVEY.md §8(d): algorithmic FLOPs per launch / launch time / dense peak;
PMC HBM traffic from profiles/pmc_traffic.json), the step's FLOP roofline, cpu_baseline (the CPU
oracle on this host, rank 0, N=1 only), psnr (M: 64^2 cameraman, 500 steps vs the reference's
golden trajectory) and, for the default run, short measurements of configs c1..c4 ("configs").
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
T_START = time.perf_counter()

PEAK = {"bf16": 2.5e15, "fp32": 157.3e12}  # dense MFMA (MI355X_MICROARCH.md; no sparsity)
HBM_PEAK = 8.0e12
KCLASS_NAMES = {
    1: "nt_bf16_kernel<fwd> (per-layer forward GEMM + bias/w0/phase epilogue)",
    2: "nt_*_kernel<dx> (per-layer input-gradient GEMM + cos epilogue)",
    3: "tn_dw_kernel (per-layer weight-gradient split-K GEMM)",
    4: "fused_fwd_reg_kernel (whole forward, activations in registers: layer 0 on the f32 MFMA, "
       "hidden and output layers on the f16 MFMA)",
    5: "bwd_ring_bf16_kernel (middle layer dX + dW)",
    6: "dx_ring_bf16_kernel<0,false,false,0> (middle-layer input gradient)",
    7: "dw_ring_bf16_kernel<0,0> (middle-layer weight gradient)",
    8: "dx_ring_bf16_kernel<C,dx,rec,0> (layer-1 input gradient with layer 0 folded in)",
    9: "dw_ring_bf16_kernel<C,0> (layer-1 weight gradient, P_0 rebuilt from x)",
    10: "dx_ring_bf16_kernel<0,false,false,O> (top hidden layer with the output layer folded in)",
    11: "dw_ring_bf16_kernel<0,O> (top hidden layer weight gradient + output-layer dW/db)",
    12: "pair_ring_bf16_kernel<middle> (middle layer: dX and dW roles on XCD-paired workgroups)",
    13: "pair_ring_bf16_kernel<top> (top hidden layer + output layer: dX and dW roles)",
    14: "pair_ring_bf16_kernel<bottom> (layer 1 + first layer, P_0 rebuilt: dX and dW roles)",
}
# kernel symbol of each class at the M shape (C = 2 inputs, O = 1 output), as rocprofv3 names it (the
# M step's forward is the fused-loss form, siren_mri_amd/fusion.py)
KCLASS_SYMBOL = {
    "bf16": {1: "siren::nt_bf16_kernel<0, 256, false, false>", 2: "siren::nt_bf16_kernel<1, 256, false, false>",
             3: "siren::tn_dw_kernel<1, false, false>", 4: "siren::fused_fwd_reg_kernel<2, 1, 0, true>",
             5: "siren::bwd_ring_bf16_kernel", 6: "siren::dx_ring_bf16_kernel<0, false, false, 0>",
             7: "siren::dw_ring_bf16_kernel<0, 0>", 8: "siren::dx_ring_bf16_kernel<2, true, true, 0>",
             9: "siren::dw_ring_bf16_kernel<2, 0>", 10: "siren::dx_ring_bf16_kernel<0, false, false, 1>",
             11: "siren::dw_ring_bf16_kernel<0, 1>",
             12: "siren::pair_ring_bf16_kernel<0, false, false, 0, 0>",
             13: "siren::pair_ring_bf16_kernel<0, false, false, 1, 0>",
             14: "siren::pair_ring_bf16_kernel<2, true, true, 0, 2>"},
    "fp32": {1: "siren::nt_f32_kernel<0, 256>", 2: "siren::nt_f32_kernel<1, 256>", 3: "siren::tn_dw_kernel<0, false, false>"},
}
CONFIG_DEFAULT_STEPS = {"m": (50, 10), "c1": (50, 10), "c2": (50, 10), "c3": (20, 5), "c4": (10, 3), "c4_fp32": (5, 2),
                        "m_fp32": (10, 3), "m_shard8": (50, 10)}
C4 = dict(num_fourier_features=8, kl_weight=2.78e-8, fw_weight=6.4e-6, lr=5.57e-5, fourier_features_scale=21,
          latent_dim=128, hidden_features_hyper=128, hidden_layers_hyper=2, hidden_layers=3, hidden_features=256,
          conv_kernel_size=7, num_conv_res_blocks=5, w0=30, slices=32, res=128)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--config", default="m", choices=["m", "c1", "c2", "c3", "c4", "c4_fp32", "m_fp32", "m_shard8"])
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    p.add_argument("--precision", default=None, choices=["bf16", "fp32"],
                   help="SIREN arithmetic (default: bf16, fp32 for c3)")
    p.add_argument("--timing", default="auto", choices=["auto", "graph", "eager"],
                   help="timed region: a hipGraph replay of K captured steps, K eager steps, or (auto) both, "
                        "reporting the faster")
    p.add_argument("--no-graph", action="store_true", help="same as --timing eager")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-psnr", action="store_true")
    p.add_argument("--no-other-configs", action="store_true")
    p.add_argument("--cpu-budget-s", type=float, default=12.0, help="CPU seconds per config of the CPU baseline")
    a = p.parse_args()
    st, wu = CONFIG_DEFAULT_STEPS[a.config]
    a.steps = st if a.steps is None else a.steps
    a.warmup = wu if a.warmup is None else a.warmup
    if a.precision is None:
        a.precision = "fp32" if a.config in ("c3", "m_fp32", "c4_fp32") else "bf16"
    if a.no_graph:
        a.timing = "eager"
    return a


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    return world, rank, torch.device("cuda", local)


# ------------------------------------------------------------------------------ algorithmic counts
def siren_fwd_flops(dims):
    """Per coordinate: sum over layers of 2 in out (SURVEY.md §8(a) 'Algorithmic counts')."""
    return sum(2 * dims[i] * dims[i + 1] for i in range(len(dims) - 1))


def siren_grad_flops(dims):
    """Per coordinate, forward with C tangent streams (layer 0's tangent is W_0's column, no GEMM)."""
    C, S = dims[0], 1 + dims[0]
    return 2 * C * dims[1] + S * sum(2 * dims[i] * dims[i + 1] for i in range(1, len(dims) - 1))


def encoder_flops_fwd(k, res_blocks, latent, res):
    """ConvImgEncoder forward per slice (modules.py:340-380, 433-450): conv_theta 2->latent/2 (k),
    conv latent/2->latent (k), res_blocks x 2 convs latent->latent (5x5), 1x1, FC over pixels."""
    px = res * res
    f = 2 * k * k * 2 * (latent // 2) * px + 2 * k * k * (latent // 2) * latent * px
    f += res_blocks * 2 * (2 * 25 * latent * latent * px) + 2 * latent * latent * px + 2 * latent * px
    return f


# ------------------------------------------------------------------------------ workloads
class Workload:
    """step(): one training step; coords: coordinate samples per rank per step; flops: algorithmic
    FLOPs per rank per step of the SIREN (encoder separately); kdims: the SIREN dims."""

    def __init__(self, name, step, coords, flops, dims, precision, workload, data, extra=None):
        self.name, self.step, self.coords, self.flops, self.dims = name, step, coords, flops, dims
        self.precision, self.workload, self.data, self.extra = precision, workload, data, extra or {}


def build_fit(cfg, args, dev, rank, world, precision, shard_of=None):
    """M / C1 / C2: the train_img.py fit (image_mse, Adam 1e-4) of one image. shard_of=N: this
    process computes rank 0's row shard of an N-way strong-scaling split, without the exchange (the
    compute-only bound of the N-GPU speed-up)."""
    from siren_mri_amd import dataio, fusion, loss_functions, modules, training
    from siren_mri_amd.training_ddp import GradAllReducer, shard_rows
    side, nh = {"m": (512, 3), "c1": (64, 1), "c2": (256, 3)}[cfg]
    torch.manual_seed(0)
    model = modules.SingleBVPNet(type="sine", mode="mlp", hidden_features=256, num_hidden_layers=nh,
                                 sidelength=(side, side), precision=precision).to(dev)
    grid = dataio.get_mgrid(side)
    if cfg == "m":
        img = torch.from_numpy(dataio.smooth_random_image(side, seed=rank if args.scaling == "weak" else 0))
        data = f"synthetic (smooth random {side}^2 image: 32 sinusoids; coords = get_mgrid({side}))"
    elif cfg == "c1":
        img = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=side)[0][1]["img"]
        data = "cameraman 64^2 (PIL bilinear), coords = get_mgrid(64)"
    else:
        img = dataio.irdata_image(0, side)
        data = "IRData slice 0 (data/IRData.mat) / max, x2-1, bilinear 256^2; coords = get_mgrid(256)"
    img = img.reshape(-1, 1)
    if shard_of:
        lo, hi = shard_rows(grid.shape[0], 0, shard_of)
    elif args.scaling == "strong" and world > 1:
        lo, hi = shard_rows(grid.shape[0], rank, world)
    else:
        lo, hi = 0, grid.shape[0]
    coords = grid[lo:hi][None].to(dev)
    tgt = img[lo:hi][None].to(dev)
    opt = training.make_adam(model.parameters(), 1e-4)
    reducer = GradAllReducer(model.parameters(), op="sum") if world > 1 else None
    model_input = {"coords": coords}
    one = torch.ones((), device=dev)  # the backward's seed, allocated once (not a fill kernel per step)

    def step():
        # training.train's step: the target staged for the forward's fused loss epilogue
        # (siren_mri_amd/fusion.py), then model -> image_mse's reduction (sum / 128^2 over this
        # rank's coordinates: in a strong-scaling shard the partial sums over the ranks add up to
        # the whole image's loss) -> backward
        st = fusion.stage_image_loss(tgt, weight=loss_functions.KSPACE_WEIGHT)
        out = model(model_input)
        loss = loss_functions.weighted_sse(out["model_out"], tgt)
        fusion.clear(st)
        loss.backward(one)
        if reducer is not None:
            reducer()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dims = [2] + [256] * (nh + 1) + [1]
    n = hi - lo
    strong = shard_of or (args.scaling == "strong" and world > 1)
    wl = (f"train_img.py fit step: {side}x{side} grid{' (strong: this rank ' + str(n) + ' rows)' if strong else ''}"
          f"{' (1/' + str(shard_of) + ' shard, no exchange)' if shard_of else ''}, "
          f"SingleBVPNet {'-'.join(map(str, dims))} (w0=30), image_mse + Adam(1e-4), full batch")
    return Workload(cfg, step, n, 3 * siren_fwd_flops(dims) * n, dims, precision, wl, data,
                    {"optimizer": opt, "side": side})


def build_c3(args, dev, rank, world, precision):
    """C3: train_poisson_grad_img.py-style fit, gradients_mse at 512^2, fp32."""
    from siren_mri_amd import dataio, loss_functions, modules, training
    from siren_mri_amd.training_ddp import GradAllReducer, shard_rows
    side = 512
    torch.manual_seed(0)
    model = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=3, precision=precision).to(dev)
    _, gt = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=side, compute_diff="gradients")[0]
    grid = dataio.get_mgrid(side)
    lo, hi = shard_rows(grid.shape[0], rank, world) if (args.scaling == "strong" and world > 1) else (0, grid.shape[0])
    coords = grid[lo:hi][None].to(dev)
    gtg = {"gradients": gt["gradients"][lo:hi][None].to(dev)}
    opt = training.make_adam(model.parameters(), 1e-4)
    reducer = GradAllReducer(model.parameters(), op="mean") if world > 1 else None
    model_input = {"coords": coords}

    def step():
        out = model(model_input)
        loss = loss_functions.gradients_mse(out, gtg)["gradients_loss"]
        loss.backward()
        if reducer is not None:
            reducer()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dims = [2, 256, 256, 256, 256, 1]
    n = hi - lo
    return Workload("c3", step, n, 3 * siren_grad_flops(dims) * n, dims, precision,
                    f"train_poisson_grad_img.py-style fit step: {side}x{side} grid, SingleBVPNet 5x256, "
                    "gradients_mse (analytic gradient + its double backward) + Adam(1e-4)",
                    "cameraman 512^2, gt gradients = sobel(10 img) along axes 1, 2 (dataio.py:779-782)",
                    {"optimizer": opt})


def c4_batch(dev, n_slices, seed=0):
    from siren_mri_amd import dataio
    ds = dataio.SyntheticMRIKspace(n_slices=max(n_slices, 1), image_resolution=(C4["res"],) * 2, seed=seed)
    coord = dataio.Implicit2DWrapper(ds, sidelength=(C4["res"],) * 2, image=False)
    gen = dataio.ImageGeneralizationWrapper(coord, test_sparsity="CS_cartesian", generalization_mode="conv_cnp")
    items = [gen[i] for i in range(n_slices)]
    inp = {k: torch.stack([it[0][k] for it in items]).to(dev) for k in items[0][0]}
    gt = {k: torch.stack([it[1][k] for it in items]).to(dev) for k in items[0][1]}
    return inp, gt


def build_c4(args, dev, rank, world, precision, encoder_precision="bf16"):
    # MIOpen's find (autotuned) convolution algorithms for the bf16 encoder's 1x1 convolution: searched
    # once during the warm-up steps. The fp32 encoder (c4_fp32: every convolution on MIOpen) takes
    # MIOpen's immediate-mode choice: a find over its fp32 shapes runs for minutes
    torch.backends.cudnn.benchmark = encoder_precision == "bf16"
    from functools import partial
    from siren_mri_amd import fusion, loss_functions, meta_modules, training
    from siren_mri_amd.features import GaussianFourierFeatureTransform
    from siren_mri_amd.training_ddp import GradAllReducer
    torch.manual_seed(0)
    nff = C4["num_fourier_features"]
    model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=2 * nff, out_features=2, image_resolution=(C4["res"],) * 2, fourier_features_size=2 * nff,
        latent_dim=C4["latent_dim"], hidden_features=C4["hidden_features"],
        hyper_hidden_features=C4["hidden_features_hyper"], hyper_hidden_layers=C4["hidden_layers_hyper"],
        num_hidden_layers=C4["hidden_layers"], conv_kernel_size=C4["conv_kernel_size"],
        num_conv_res_blocks=C4["num_conv_res_blocks"], w0=C4["w0"], precision=precision,
        encoder_precision=encoder_precision).to(dev)
    torch.manual_seed(0)
    ff = GaussianFourierFeatureTransform(2, nff, scale=C4["fourier_features_scale"], device=dev)
    inp, gt = c4_batch(dev, C4["slices"], seed=rank)
    loss_fn = partial(loss_functions.image_hypernetwork_loss, None, C4["kl_weight"], C4["fw_weight"])
    opt = training.make_adam(model.parameters(), C4["lr"])
    reducer = GradAllReducer(model.parameters(), op="mean") if world > 1 else None
    params = [p for p in model.parameters() if p.requires_grad]

    def step():
        # training.train's transform step: raw coordinates + B for the hypernetwork, whose SIREN forms
        # the Fourier features in its first layer (features.py model_input)
        mi = ff.model_input(model, dict(inp))
        st = fusion.stage_image_loss(gt["img"])  # as training.train: the fused DC + loss epilogue
        out = model(mi)
        losses = loss_fn(out, gt)
        fusion.clear(st)
        loss = sum(v.mean() for v in losses.values())
        if reducer is not None:
            reducer.begin()
        loss.backward()
        if reducer is not None:
            reducer()
        torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dims = [2 * nff] + [C4["hidden_features"]] * (C4["hidden_layers"] + 1) + [2]
    n = C4["slices"] * C4["res"] ** 2
    enc = 3 * encoder_flops_fwd(C4["conv_kernel_size"], C4["num_conv_res_blocks"], C4["latent_dim"], C4["res"]) * C4["slices"]
    return Workload("c4", step, n, 3 * siren_fwd_flops(dims) * n, dims, precision,
                    f"train_mri_neural_process step (reference config hyperoptIV_homebrew): {C4['slices']} slices "
                    f"of {C4['res']}^2 k-space per GPU, conv encoder ({encoder_precision}, k=7, 5 res blocks) -> "
                    f"hypernetwork -> SIREN {'-'.join(map(str, dims))} per-slice weights ({precision}) -> DC, "
                    "image_hypernetwork_loss, clip 1.0, Adam(5.57e-5)",
                    "synthetic k-space (IRData slices x flips/rotations + seeded ellipses, fftshift(fft2)), "
                    "seeded CS-Cartesian masks, FF B = randn(2, 8) * 21 (seed 0)",
                    {"optimizer": opt, "encoder_flops_per_step": enc, "encoder_precision": encoder_precision,
                     "model": model, "inp": inp, "ff": ff, "loss_fn": loss_fn,
                     "conv_algorithms": ("MIOpen find (torch.backends.cudnn.benchmark)" if encoder_precision == "bf16"
                                         else "MIOpen immediate mode")})


def build(cfg, args, dev, rank, world, precision=None):
    precision = precision or ("fp32" if cfg in ("c3", "m_fp32", "c4_fp32") else args.precision)
    if cfg in ("m", "c1", "c2"):
        return build_fit(cfg, args, dev, rank, world, precision)
    if cfg == "m_fp32":  # the metric fit in the reference's arithmetic (fp32 operands, exact-fp32 MFMA)
        return build_fit("m", args, dev, rank, world, precision)
    if cfg == "m_shard8":  # rank 0's 1/8 row shard of the metric grid (strong scaling at 8 GPUs)
        return build_fit("m", args, dev, rank, world, precision, shard_of=8)
    if cfg == "c3":
        return build_c3(args, dev, rank, world, precision)
    if cfg == "c4_fp32":  # config 4 in the reference's arithmetic: fp32 encoder (MIOpen) and fp32 SIREN
        return build_c4(args, dev, rank, world, "fp32", encoder_precision="fp32")
    return build_c4(args, dev, rank, world, precision)


# ------------------------------------------------------------------------------ timing
def enable_graph_mode(wl):
    opt = wl.extra.get("optimizer")
    if opt is not None and hasattr(opt, "enable_graph_mode"):
        opt.enable_graph_mode()


def capture(step, nsteps):
    """A hipGraph of `nsteps` consecutive steps (captured on a side stream, torch's private pool)."""
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(nsteps):
                step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return g


def timed(fn, world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def max_over_ranks(v, dev, world):
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_timed(wl, args, dev, world, kclass=None, max_launches=4096):
    """Warm-up, then timed regions of EXACTLY args.steps steps each: one replay of a hipGraph
    holding the K captured steps (--timing graph/auto), and K eager steps (--timing eager/auto),
    during which the dominant kernel class (kclass) is timed by HIP event pairs on its launch
    stream around each launch (ROCm reports no elapsed time between events recorded inside a
    graph). Returns (elapsed_s of the reported region, region name, KernelTimer or None,
    {region: elapsed_s})."""
    from siren_mri_amd import _native
    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    regions = {}
    if args.timing in ("graph", "auto"):
        try:
            enable_graph_mode(wl)
            wl.step()  # an eager step in graph mode creates the optimizer's device step counter
            g1 = capture(wl.step, 1)
            for _ in range(2):
                g1.replay()
            torch.cuda.synchronize()
            gk = capture(wl.step, args.steps)
            regions["graph"] = timed(gk.replay, world)
            del gk, g1
        except Exception as e:  # noqa: BLE001 - reported, then timed eagerly
            print(f"bench: hipGraph capture failed ({type(e).__name__}: {e}); timing eager steps", file=sys.stderr)
            opt = wl.extra.get("optimizer")
            if opt is not None and hasattr(opt, "_native_reject"):
                for g in opt.param_groups:
                    r = opt._native_reject(g)
                    if r:
                        print(f"bench:   optimizer group not native: {r}", file=sys.stderr)
            torch.cuda.synchronize()
    kt = None
    if kclass is not None:
        kt = _native.KernelTimer(kclass, max_launches=max_launches)
        kt.__enter__()

    def loop():
        for _ in range(args.steps):
            wl.step()
    regions["eager"] = timed(loop, world)
    if kt is not None:
        kt.__exit__(None, None, None)
    # the same choice on every rank: the max over ranks of each region
    regions = {k: max_over_ranks(v, dev, world) for k, v in regions.items()}
    name = min(regions, key=regions.get) if args.timing == "auto" else (
        "graph" if "graph" in regions and args.timing == "graph" else "eager")
    return regions[name], name, kt, regions


def dominant_class(wl):
    """The kernel class with the largest time per step (3 eager steps per class; every class is one
    template instantiation at a given shape, so its average launch is one rocprofv3 row)."""
    from siren_mri_amd import _native
    totals = {}
    for kc in sorted(KCLASS_NAMES):
        with _native.KernelTimer(kc) as t:
            for _ in range(3):
                wl.step()
        if t.launches:
            totals[kc] = (t.total_ms / 3, t.launches // 3)
    return totals


def kernel_flops(wl, kclass):
    """Algorithmic FLOPs of ONE launch of a kernel class (bf16 fused path): R rows
    of the launch's weight sets, F = hidden width, C inputs, O outputs, nh hidden 256x256 layers."""
    d = wl.dims
    R, C, F, O, nh = wl.coords, d[0], d[1], d[-1], len(d) - 3
    gemm = 2.0 * R * F * F
    table = {
        1: gemm, 2: gemm, 3: gemm, 5: 2 * gemm, 6: gemm, 7: gemm, 12: 2 * gemm,
        4: 2.0 * R * (C * F + nh * F * F + F * O),                  # the whole forward
        8: gemm + 3 * 2.0 * R * C * F, 9: gemm + 2.0 * R * C * F,
        10: gemm + 2.0 * R * F * O, 11: gemm + 4.0 * R * F * O,
        13: 2 * gemm + 6.0 * R * F * O,                              # top pair: dZ, dW + output layer
        14: 2 * gemm + 4 * 2.0 * R * C * F,                          # bottom pair: dZ_1, dW_1 + layer 0
    }
    return table[kclass]


HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md §HBM (spec)


def kernel_bytes(wl, kclass):
    """Algorithmic HBM bytes of ONE launch of a kernel class (every input read once,
    every output written once; split-K partial slabs, an implementation artefact, excluded), or
    None for a class without a stated count. R rows per launch, F hidden width, C inputs, O outputs;
    phases / gradients 2 B each in bf16 mode, 4 B in fp32."""
    d = wl.dims
    R, C, F, O = wl.coords, d[0], d[1], d[-1]
    ps = 2 if wl.precision == "bf16" else 4
    table = {
        4: R * (4 * C + 3 * 2 * F + 3 * 4 * O),   # x; P_1..P_3 codes; y, the loss target, dL/dy
        12: R * (3 * 2 * F),                      # dZ_l, P_{l-1} in; dZ_{l-1} out
        13: R * (3 * 2 * F + 4 * O),              # P_top, dy, P_{top-1} in; dZ_{top-1} out
        14: R * (2 * F + 2 * 4 * C),              # dZ_1, x in; dx out
        1: R * (2 * ps * F),                      # P_{l-1} in, P_l out
        2: R * (3 * ps * F),                      # dZ_l, P_{l-1} in, dZ_{l-1} out
        3: R * (2 * ps * F),                      # dZ_l, P_{l-1} in
    }
    return table.get(kclass)


def traffic_key(wl):
    """profiles/pmc_traffic.json key of a workload: precision, rows of ONE launch (the coordinate
    rows this GPU processes per step), hidden width and hidden-layer count."""
    return f"{wl.precision}:rows{wl.coords}:{wl.dims[1]}:{len(wl.dims) - 3}"


def traffic_from_profile(kclass, wl):
    """HBM bytes per launch of the kernel from the committed PMC passes (profiles/pmc_traffic.json:
    FETCH_SIZE x 2 + WRITE_SIZE per launch, the gfx950 correction applied by tools/pmc_summary.py),
    keyed by the launch's rows (traffic_key) and the kernel symbol, or None when this exact
    workload / kernel was not profiled. Keyed by rows, not by the grid's side: a row shard of the
    512^2 grid is a different launch."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    sym = KCLASS_SYMBOL.get(wl.precision, {}).get(kclass)
    if sym is None or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        ent = d.get(traffic_key(wl), {}).get(sym)
        return None if ent is None else round(ent["bytes"] / 1e9, 4)
    except (OSError, ValueError, KeyError):
        return None


def step_traffic_from_profile(wl):
    """HBM bytes of one whole step of the workload (every kernel's bytes per launch x launches per
    step) from the same PMC record, or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            v = json.load(f).get(traffic_key(wl), {}).get("_step_bytes")
        return None if v is None else int(v)
    except (OSError, ValueError):
        return None


# ------------------------------------------------------------------------------ CPU baseline
def cpu_threads():
    """Threads for the CPU baseline: os.cpu_count(), bounded by what this process
    may actually run on (its affinity mask and its cgroup CPU quota — on the GPU box os.cpu_count()
    reports the whole machine while the job owns a share of it)."""
    n = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    use = min(n, aff, quota or n)
    return use, {"os_cpu_count": n, "affinity": aff, "cgroup_quota_cpus": quota}


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return platform.processor() or "unknown"


def _cpu_time(step, budget_s, warm=3, timed_n=5):
    """3 warm-ups + 5 timed steps, fewer when a step exceeds budget_s / 8."""
    t0 = time.perf_counter()
    step()
    first = time.perf_counter() - t0
    w = 1 + (warm - 1 if first * (warm + timed_n) <= budget_s else 0)
    for _ in range(w - 1):
        step()
    times = []
    t_start = time.perf_counter()
    while len(times) < timed_n and (len(times) < 2 or time.perf_counter() - t_start + first <= budget_s):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    return float(np.median(times)), w, len(times)


def cpu_step(cfg):
    """The CPU oracle (oracle/siren_oracle.py: the reference algorithm on PyTorch-CPU fp32) running
    one training step of config cfg; returns (step, coords per step, sample description)."""
    from oracle import siren_oracle as orc
    from siren_mri_amd import dataio
    if cfg in ("m", "c1", "c2"):
        side, nh = {"m": (512, 3), "c1": (64, 1), "c2": (256, 3)}[cfg]
        model = orc.OracleSiren(hidden_features=256, num_hidden_layers=nh, seed=0)
        coords = orc.get_mgrid(side)[None]
        img = (torch.from_numpy(dataio.smooth_random_image(side, seed=0)) if cfg == "m" else
               dataio.Implicit2DWrapper(dataio.Camera(), sidelength=side)[0][1]["img"] if cfg == "c1" else
               dataio.irdata_image(0, side))
        gt = {"img": img.reshape(1, -1, 1)}
        opt = torch.optim.Adam(lr=1e-4, params=model.parameters())

        def step():
            loss = orc.image_mse(None, model({"coords": coords}), gt, high_freq=False)["img_loss"]
            loss.backward()
            opt.step()
            opt.zero_grad()
        return step, side * side, f"full {side}^2 step, {nh + 2} linear layers"
    if cfg == "c3":
        model = orc.OracleSiren(hidden_features=256, num_hidden_layers=3, seed=0)
        coords = orc.get_mgrid(512)[None]
        _, gt = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=512, compute_diff="gradients")[0]
        gtg = {"gradients": gt["gradients"][None]}
        opt = torch.optim.Adam(lr=1e-4, params=model.parameters())

        def step():
            loss = orc.gradients_mse(model({"coords": coords}), gtg)["gradients_loss"]
            loss.backward()
            opt.step()
            opt.zero_grad()
        return step, 512 * 512, "full 512^2 gradients_mse step (autograd double backward)"
    # c4: the encoder + hypernetwork modules on the CPU, the hypo-net SIREN through the oracle
    from functools import partial
    from siren_mri_amd import meta_modules
    nff, ns = C4["num_fourier_features"], 2
    torch.manual_seed(0)
    model = meta_modules.ConvolutionalNeuralProcessImplicit2DHypernetFourierFeatures(
        in_features=2 * nff, out_features=2, image_resolution=(C4["res"],) * 2, fourier_features_size=2 * nff,
        latent_dim=C4["latent_dim"], hidden_features=C4["hidden_features"],
        hyper_hidden_features=C4["hidden_features_hyper"], hyper_hidden_layers=C4["hidden_layers_hyper"],
        num_hidden_layers=C4["hidden_layers"], conv_kernel_size=C4["conv_kernel_size"],
        num_conv_res_blocks=C4["num_conv_res_blocks"], w0=C4["w0"])
    B = torch.randn(2, nff) * C4["fourier_features_scale"]
    inp, gt = c4_batch(torch.device("cpu"), ns)
    L = C4["hidden_layers"] + 2
    opt = torch.optim.Adam(lr=C4["lr"], params=model.parameters())
    loss_fn = partial(orc.image_hypernetwork_loss, None, C4["kl_weight"], C4["fw_weight"])

    def step():
        emb = model.encoder(inp["img_sparse"])
        hp = model.hyper_net(emb)
        x = orc.fourier_features(inp["coords"], B)
        y = orc.siren_forward(x, [(hp[f"net.net.{i}.0.weight"], hp[f"net.net.{i}.0.bias"]) for i in range(L)])
        y = orc.data_consistency(y, inp["img_sparse"], inp["dc_mask"])
        losses = loss_fn({"model_out": y, "latent_vec": emb, "hypo_params": hp}, gt)
        sum(v.mean() for v in losses.values()).backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad()
    return step, ns * C4["res"] ** 2, f"{ns} of the 32 slices per step (rate per coordinate sample), fp32"


def cpu_baseline(cfg, budget_s):
    threads, cpus = cpu_threads()
    torch.set_num_threads(threads)
    step, coords, what = cpu_step(cfg)
    med, warm, n = _cpu_time(step, budget_s)
    return {"value": coords / med, "unit": "coord-samples/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle restatement (PyTorch-CPU fp32, autograd, Adam): {what}; {warm} warm-up + {n} timed "
                      f"steps, median {med:.3f} s/step; {torch.get_num_threads()} threads",
            "cpu_model": cpu_model(), **cpus}


# ------------------------------------------------------------------------------ PSNR leg
def psnr_check(args, dev):
    """64^2 cameraman, 3 hidden layers, Adam 1e-4, seed 0: PSNR at steps 0/50/100/200/500 vs the
    reference's trajectory recorded in tests/golden/psnr_c1.npz (image_mse, high_freq=False)."""
    from siren_mri_amd import dataio, loss_functions, modules, training, utils
    gold = np.load(os.path.join(ROOT, "tests", "golden", "psnr_c1.npz"), allow_pickle=False)
    steps = list(gold["steps"])
    img = dataio.Implicit2DWrapper(dataio.Camera(), sidelength=64)[0][1]["img"][None].to(dev)
    coords = dataio.get_mgrid(64)[None].to(dev)
    res = {}
    for prec in (args.precision, "fp32") if args.precision != "fp32" else ("fp32",):
        torch.manual_seed(0)
        m = modules.SingleBVPNet(type="sine", hidden_features=256, num_hidden_layers=3, sidelength=(64, 64),
                                 precision=prec).to(dev)
        opt = training.make_adam(m.parameters(), 1e-4)
        vals = []
        for s in range(max(steps) + 1):
            out = m({"coords": coords})
            if s in steps:
                vals.append(utils.psnr(dataio.lin2img(out["model_out"].detach()).cpu().numpy()[0],
                                       dataio.lin2img(img).cpu().numpy()[0]))
            loss = loss_functions.image_mse(None, out, {"img": img}, high_freq=False)["img_loss"]
            loss.backward()
            opt.step()
            opt.zero_grad()
        res[prec] = [round(v, 3) for v in vals]
    return {"steps": [int(s) for s in steps], "reference": [round(float(v), 3) for v in gold["nh3_psnr"]],
            **{f"siren_mri_amd_{k}": v for k, v in res.items()},
            "config": "64x64 cameraman, SingleBVPNet 3 hidden x 256, Adam 1e-4, seed 0"}


# ------------------------------------------------------------------------------ per-config line
def measure(cfg, args, dev, rank, world, with_kernels=True):
    from siren_mri_amd import _native
    wl = build(cfg, args, dev, rank, world)
    for _ in range(2):
        wl.step()
    torch.cuda.synchronize()
    totals = dominant_class(wl) if (with_kernels and wl.precision == "bf16") else {}
    dom = max(totals, key=lambda k: totals[k][0]) if totals else None
    per_step = totals[dom][1] if dom else 0
    elapsed, region, kt, regions = run_timed(wl, args, dev, world, kclass=dom,
                                             max_launches=max(64, (per_step + 1) * args.steps))
    graph = region == "graph"
    ms = elapsed / args.steps * 1e3
    step_flops = wl.flops
    peak = PEAK[wl.precision]
    res = {"config": cfg, "ms_per_step": ms, "coords_per_gpu_step": wl.coords,
           "value": world * wl.coords * args.steps / elapsed, "graph": graph, "precision": wl.precision,
           "ms_per_step_by_region": {k: round(v / args.steps * 1e3, 4) for k, v in regions.items()},
           "workload": wl.workload, "data": wl.data,
           "step_roofline": {"bound": "mfma", "flops_per_step_per_gpu": step_flops,
                             "achieved_tflops": round(step_flops / (ms * 1e-3) / 1e12, 2),
                             "peak_tflops": peak / 1e12, "frac": round(step_flops / (ms * 1e-3) / peak, 4)}}
    if "encoder_flops_per_step" in wl.extra:
        res["encoder"] = {"flops_per_step_per_gpu": wl.extra["encoder_flops_per_step"],
                          "precision": wl.extra["encoder_precision"],
                          "share_of_step_flops": round(wl.extra["encoder_flops_per_step"] /
                                                       (wl.extra["encoder_flops_per_step"] + step_flops), 4)}
        res["encoder"].update(time_encoder(wl, args))
    if dom is not None and kt is not None and kt.launches:
        avg_s = kt.avg_ms * 1e-3
        flops = kernel_flops(wl, dom)
        traffic = traffic_from_profile(dom, wl)
        traffic_note = None
        if traffic and traffic / avg_s > HBM_PEAK_GBPS:
            # a recorded byte count above what HBM can move in the measured launch time is not this
            # launch's traffic (a stale or mismatched profile): refuse it rather than print it
            traffic_note = (f"rejected: {traffic} GB per launch over {avg_s * 1e3:.4f} ms would be "
                            f"{traffic / avg_s:.0f} GB/s, above the {HBM_PEAK_GBPS:.0f} GB/s HBM peak")
            traffic = None
        nbytes = kernel_bytes(wl, dom)
        mfma_frac = flops / avg_s / peak
        # the path is a dense contraction (~12 B of algorithmic I/O per coordinate,
        # ~1e5 FLOP/B), so the roofline that bounds it is the MFMA peak and `frac` is the dominant
        # kernel's algorithmic FLOPs / its launch time / the dense peak. The bytes the design itself
        # stores between kernels (phase codes, dZ planes) are NOT algorithmic: their HBM rate is
        # reported under a separate key only, never as `frac`.
        design_hbm_frac = nbytes / avg_s / HBM_PEAK if nbytes else None
        res["roofline"] = {
            "bound": "mfma", "kernel": KCLASS_NAMES[dom],
            "kernel_symbol": KCLASS_SYMBOL.get(wl.precision, {}).get(dom),
            "achieved": round(flops / avg_s / 1e12, 2), "peak": round(peak / 1e12, 1), "unit": "TFLOP/s",
            "frac": round(mfma_frac, 4),
            "basis": "SURVEY.md §8(d): algorithmic FLOPs per launch / HIP-event launch time / dense MFMA peak",
            "design_bytes_per_launch": nbytes,
            "hbm_frac_of_design_bytes": round(design_hbm_frac, 4) if design_hbm_frac else None,
            "design_bytes_note": "bytes the design materialises between kernels (phase codes, dZ planes), "
                                 "each read once / written once, over 8 TB/s; not algorithmic I/O",
            "flops_per_launch": flops,
            "avg_launch_ms": round(kt.avg_ms, 4), "launches": kt.launches,
            "timing": "HIP event pairs on the launch stream around every launch of the kernel over a timed "
                      "region of K eager steps" + (" (the reported value is the hipGraph region's)" if graph else ""),
            "traffic": traffic, "traffic_unit": "GB per launch (HBM, rocprofv3 PMC FETCH_SIZE + WRITE_SIZE)",
            "hbm_gbps_of_traffic": round(traffic * 1e9 / avg_s / 1e9, 1) if traffic else None,
            "traffic_key": traffic_key(wl), **({"traffic_note": traffic_note} if traffic_note else {}),
            "kernel_ms_per_step": {KCLASS_NAMES[k].split(" ")[0] + f"[{k}]": round(v[0], 4) for k, v in totals.items()}}
        step_bytes = step_traffic_from_profile(wl)
        if traffic or step_bytes:
            # algorithmic I/O of the whole path: 12 B per coordinate (coords 8 B,
            # target 4 B) + parameters, gradients and Adam state once each (5 x 4 B per parameter)
            nparam = sum(wl.dims[i] * wl.dims[i + 1] + wl.dims[i + 1] for i in range(len(wl.dims) - 1))
            alg = 12 * wl.coords + 20 * nparam
            res["roofline"]["traffic_vs_algorithmic_io"] = {
                "algorithmic_io_bytes_per_step": alg,
                "dominant_kernel_traffic_over_step_io": round(traffic * 1e9 / alg, 1) if traffic else None,
                "step_traffic_bytes": step_bytes,
                "step_traffic_over_step_io": round(step_bytes / alg, 1) if step_bytes else None}
    return res, wl, dom, totals


def time_encoder(wl, args):
    """The conv encoder's forward + backward alone on the same batch (HIP events), for the C4 split."""
    model, inp = wl.extra["model"], wl.extra["inp"]
    enc = model.encoder
    for _ in range(2):
        enc(inp["img_sparse"]).sum().backward()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(3, min(args.steps, 10))
    e0.record()
    for _ in range(n):
        enc(inp["img_sparse"]).sum().backward()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    model.zero_grad(set_to_none=False)
    f = wl.extra["encoder_flops_per_step"]
    return {"fwd_bwd_ms": round(ms, 3), "achieved_tflops": round(f / (ms * 1e-3) / 1e12, 1),
            "frac_of_bf16_peak" if wl.extra["encoder_precision"] == "bf16" else "frac_of_fp32_peak":
                round(f / (ms * 1e-3) / PEAK[wl.extra["encoder_precision"]], 4)}


def main():
    args = parse()
    world, rank, dev = setup_dist()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    from siren_mri_amd import _native
    _native.load_library()

    res, wl, dom, totals = measure(args.config, args, dev, rank, world)
    nparams = sum(p.numel() for p in wl.extra["optimizer"].param_groups[0]["params"])
    result = {
        "metric": "coord-samples/sec/step, 5x256 SIREN on 512^2 grid; PSNR vs ref",
        "value": res["value"],
        "unit": "coord-samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["ms_per_step"],
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": wl.precision,
        "precision_detail": ("forward hidden GEMMs fp16 x fp16 -> fp32, backward GEMMs bf16 x bf16 -> fp32, "
                             "phases stored as 16-bit revolutions, weights / loss / Adam fp32"
                             if wl.precision == "bf16" else "fp32 throughout"),
        "data": res["data"],
        "config": {"workload": res["workload"], "config": args.config,
                   "coords_per_gpu_step": wl.coords, "global_batch": world * wl.coords,
                   "parallelism": f"dp{world} ({'strong: one grid split by rows' if args.scaling == 'strong' else 'weak: one problem per GPU'}"
                                  f", one gradient all-reduce per step)",
                   "params": nparams, "timed_region": ("hipGraph replay of K captured steps" if res["graph"] else "K eager steps")
                   + (" (--timing auto: the faster of the two regions)" if args.timing == "auto" else ""),
                   "ms_per_step_by_region": res["ms_per_step_by_region"]},
        "step_roofline": res["step_roofline"],
    }
    if "roofline" in res:
        result["roofline"] = res["roofline"]
    if "encoder" in res:
        result["encoder"] = res["encoder"]
    # north_star's per-kernel target: bf16-MFMA utilisation of the fused SineLayer GEMM (the whole
    # forward: every layer's GEMM + bias + sine in one launch), from the same HIP-event timer
    if wl.precision == "bf16" and 4 in totals:
        if dom == 4 and "roofline" in res:
            f_ms, f_n = res["roofline"]["avg_launch_ms"], res["roofline"]["launches"]
        else:
            with _native.KernelTimer(4, max_launches=64) as ft:
                for _ in range(10):
                    wl.step()
            f_ms, f_n = ft.avg_ms, ft.launches
        f_flops = kernel_flops(wl, 4)
        result["fused_sine_gemm"] = {
            "kernel": KCLASS_NAMES[4], "kernel_symbol": KCLASS_SYMBOL["bf16"][4], "flops_per_launch": f_flops,
            "avg_launch_ms": round(f_ms, 4), "launches": f_n, "achieved_tflops": round(f_flops / (f_ms * 1e-3) / 1e12, 2),
            "mfma_peak_tflops": PEAK["bf16"] / 1e12, "mfma_frac": round(f_flops / (f_ms * 1e-3) / PEAK["bf16"], 4)}
    del wl
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_psnr and args.config == "m":
        result["psnr"] = psnr_check(args, dev)
    if world == 1 and not args.no_other_configs and args.config == "m":
        oargs = argparse.Namespace(**vars(args))
        others = {}
        for cfg in ("c1", "c2", "c3", "c4", "c4_fp32", "m_fp32", "m_shard8"):
            oargs.steps, oargs.warmup = CONFIG_DEFAULT_STEPS[cfg]
            print(f"bench: config {cfg} ({time.perf_counter() - T_START:.0f} s)", file=sys.stderr, flush=True)
            try:
                r, owl, _, _ = measure(cfg, oargs, dev, rank, world, with_kernels=not cfg.startswith("c4"))
                others[cfg] = r
                del owl
            except Exception as e:  # noqa: BLE001 - a failing side config must not lose the metric line
                others[cfg] = {"error": f"{type(e).__name__}: {e}"}
            torch.cuda.empty_cache()
        sh = others.get("m_shard8", {})
        if "ms_per_step" in sh:
            # compute-only bound of the 8-GPU strong-scaling speed-up: the full step over one rank's
            # 1/8 shard (no all-reduce; SURVEY.md §8(d) target >= 6.5x)
            others["m_shard8"]["strong_scaling_bound_8gpu"] = round(res["ms_per_step"] / sh["ms_per_step"], 2)
        result["configs"] = others
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the metric config's CPU sample: 3 warm-up + 5 timed full steps need ~20 s
        result["cpu_baseline"] = cpu_baseline(args.config, max(args.cpu_budget_s, 24.0 if args.config == "m" else 0.0))
        if args.config == "m" and not args.no_other_configs:
            result["cpu_baselines"] = {c: cpu_baseline(c, args.cpu_budget_s) for c in ("c1", "c2", "c3", "c4")}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
