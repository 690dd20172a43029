"""Benchmark: SIREN fitting throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision bf16|fp32]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]'s metric configuration): the train_img.py
fit — a 512x512 coordinate grid (262,144 coords per GPU per step, full batch) through a
5x256 SIREN (SingleBVPNet: 2-256-256-256-256-1, w0=30), image_mse + Adam(lr=1e-4). One step =
forward + loss + backward + (N>1: one RCCL all-reduce of the 198,401 grads) + Adam. Synthetic
target: a smooth random image (sum of 32 sinusoids). Multi-GPU is weak scaling: every rank owns
its own 512^2 block of coordinates (a 512 x 512N image), one gradient all-reduce per step.

Prints ONE JSON line on rank 0 with: value (coord-samples/s, whole job), roofline of the
dominant kernel (HIP events around each of its launches inside the timed region; algorithmic
FLOPs / bytes per launch from kernel_model), cpu_baseline (the CPU oracle timed on this host, rank 0, N=1 only),
and psnr (64^2 cameraman, 500 steps, this path vs the reference's golden trajectory).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK = {"bf16": (2.5e15, "TFLOP/s"), "fp32": (157.3e12, "TFLOP/s")}
HBM_PEAK = 8.0e12
KCLASS_NAMES = {
    1: "nt_bf16_kernel<fwd> (per-layer forward GEMM + bias/w0/phase epilogue)",
    2: "nt_*_kernel<dx> (per-layer input-gradient GEMM + cos epilogue)",
    3: "tn_dw_kernel (per-layer weight-gradient split-K GEMM)",
    4: "fused_fwd_pipe_kernel (whole forward: layer 0, hidden MFMA layers, output layer)",
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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--side", type=int, default=512)
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--num-hidden-layers", type=int, default=3)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-psnr", action="store_true")
    p.add_argument("--cpu-budget-s", type=float, default=20.0)
    return p.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    return world, rank, torch.device("cuda", local)


def build_step(args, dev, rank, world):
    from siren_mri_amd import dataio, loss_functions, modules, training
    from siren_mri_amd.training_ddp import GradAllReducer
    torch.manual_seed(0)
    model = modules.SingleBVPNet(type="sine", mode="mlp", hidden_features=args.hidden,
                                 num_hidden_layers=args.num_hidden_layers, sidelength=(args.side, args.side),
                                 precision=args.precision).to(dev)
    coords = dataio.get_mgrid(args.side)[None].to(dev)
    img = dataio.smooth_random_image(args.side, seed=rank)
    gt = {"img": torch.from_numpy(img).reshape(1, -1, 1).to(dev)}
    opt = training.make_adam(model.parameters(), 1e-4)
    reducer = GradAllReducer(model.parameters(), op="sum") if world > 1 else None
    model_input = {"coords": coords}

    def step():
        out = model(model_input)
        loss = loss_functions.image_mse(None, out, gt, high_freq=False)["img_loss"]
        loss.backward()
        if reducer is not None:
            reducer()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    return step, model


def kernel_model(args, kclass, p0_recompute):
    """Algorithmic FLOPs and HBM bytes of ONE launch of a kernel class at the bench workload
    (DESIGN.md §5): R rows, F = hidden width, e = bytes per stored activation element (2 in bf16
    mode: 16-bit phases / bf16 gradients; 4 in fp32 mode), C = 2 inputs, O = 1 output. Bytes are
    the kernel's essential inputs and outputs once each (split-K partial slabs are not counted:
    they are an implementation choice, visible in the PMC traffic)."""
    R = args.side * args.side
    F, nh = args.hidden, args.num_hidden_layers
    e = 2 if args.precision == "bf16" else 4
    C, O = 2, 1
    gemm = 2.0 * R * F * F
    dw_out = 4 * (F * F + F)
    if kclass == 1:            # P_l = enc(w0 (sin(P_{l-1}) W^T + b)): read P_{l-1}, write P_l
        return gemm, R * F * 2 * e
    if kclass in (2, 6):       # dZ_{l-1} = (dZ_l W) cos(P_{l-1}) w0: read dZ_l, P_{l-1}; write dZ_{l-1}
        return gemm, R * F * 3 * e
    if kclass in (3, 7):       # dW_l = dZ_l^T sin(P_{l-1}), db_l: read dZ_l, P_{l-1}; write dW_l, db_l
        return gemm, R * F * 2 * e + dw_out
    if kclass == 4:            # x in, the kept sine layers' phases out, y out
        planes = nh if p0_recompute else nh + 1
        return 2.0 * R * (C * F + nh * F * F + F * O), R * (4 * C + planes * F * e + 4 * O)
    if kclass == 5:            # 6 + 7 in one pass
        return 2 * gemm, R * F * 3 * e + dw_out
    if kclass == 8:            # read dZ_1, x (P_0 rebuilt from x, or read); write dx, dW_0/db_0
        return (gemm + 3 * 2.0 * R * C * F,
                R * (F * e + 4 * C + 4 * C + (0 if p0_recompute else F * e)) + 4 * (F * C + F))
    if kclass == 9:            # read dZ_1, x; write dW_1, db_1
        return gemm + 2.0 * R * C * F, R * (F * e + 4 * C) + dw_out
    if kclass == 10:           # read P_top, dy, P_{top-1}; write dZ_{top-1}
        return gemm + 2.0 * R * F * O, R * (3 * F * e + 4 * O)
    if kclass == 11:           # read P_top, dy, P_{top-1}; write dW, db, dW_L, db_L
        return gemm + 4.0 * R * F * O, R * (2 * F * e + 4 * O) + dw_out + 4 * (F * O + O)
    if kclass == 12:           # 6 + 7 with dZ_l and P_{l-1} read once per pair
        return 2 * gemm, R * F * 3 * e + dw_out
    if kclass == 13:           # 10 + 11: read P_top, dy, P_{top-1} once; write dZ_{top-1}, dW, dW_L
        return (2 * gemm + 6.0 * R * F * O,
                R * (3 * F * e + 4 * O) + dw_out + 4 * (F * O + O))
    if kclass == 14:           # 8 + 9: read dZ_1, x once; write dx, dW_1, dW_0
        return (2 * gemm + 4 * 2.0 * R * C * F,
                R * (F * e + 4 * C + 4 * C) + dw_out + 4 * (F * C + F))
    raise ValueError(kclass)


def timed_region(step, steps, world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def cpu_baseline(args, budget_s):
    """The CPU oracle (oracle/siren_oracle.py, the reference algorithm on PyTorch-CPU fp32)
    running the same 512^2 5x256 fit step, timed on this host's cores."""
    from oracle import siren_oracle as orc
    torch.manual_seed(0)
    model = orc.OracleSiren(hidden_features=args.hidden, num_hidden_layers=args.num_hidden_layers, seed=0)
    coords = orc.get_mgrid(args.side)[None]
    from siren_mri_amd import dataio
    gt = {"img": torch.from_numpy(dataio.smooth_random_image(args.side, seed=0)).reshape(1, -1, 1)}
    opt = torch.optim.Adam(lr=1e-4, params=model.parameters())

    def step():
        out = model({"coords": coords})
        loss = orc.image_mse(None, out, gt, high_freq=False)["img_loss"]
        loss.backward()
        opt.step()
        opt.zero_grad()

    step()  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 and (time.perf_counter() - t_start) < budget_s:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": args.side * args.side / med, "unit": "coord-samples/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle SingleBVPNet restatement (PyTorch-CPU fp32, autograd, Adam), 1 warm-up + "
                      f"{len(times)} timed full {args.side}x{args.side} steps, median {med:.3f} s/step, "
                      f"{torch.get_num_threads()} threads on {os.cpu_count()} visible CPUs"}


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


# kernel symbol of each class at the bench shape (C = 2 inputs, O = 1 output), as rocprofv3 names it
KCLASS_SYMBOL = {
    "bf16": {1: "siren::nt_bf16_kernel<0, 256, false, false>", 2: "siren::nt_bf16_kernel<1, 256, false, false>",
             3: "siren::tn_dw_kernel<1, false, false>", 4: "siren::fused_fwd_pipe_kernel<2, 1>",
             5: "siren::bwd_ring_bf16_kernel", 6: "siren::dx_ring_bf16_kernel<0, false, false, 0>",
             7: "siren::dw_ring_bf16_kernel<0, 0>", 8: "siren::dx_ring_bf16_kernel<2, true, true, 0>",
             9: "siren::dw_ring_bf16_kernel<2, 0>", 10: "siren::dx_ring_bf16_kernel<0, false, false, 1>",
             11: "siren::dw_ring_bf16_kernel<0, 1>",
             12: "siren::pair_ring_bf16_kernel<0, false, false, 0, 0>",
             13: "siren::pair_ring_bf16_kernel<0, false, false, 1, 0>",
             14: "siren::pair_ring_bf16_kernel<2, true, true, 0, 2>"},
    "fp32": {1: "siren::nt_f32_kernel<0>", 2: "siren::nt_f32_kernel<1>", 3: "siren::tn_dw_kernel<0, false, false>"},
}


def traffic_from_profile(kclass, args):
    """HBM bytes per launch of the kernel from the committed PMC pass (profiles/pmc_traffic.json,
    written by tools/pmc_bench.sh + tools/pmc_summary.py: FETCH_SIZE x2 (gfx950 correction) +
    WRITE_SIZE, KB -> bytes), or None when this workload/kernel was not profiled."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    sym = KCLASS_SYMBOL.get(args.precision, {}).get(kclass)
    if sym is None or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        ent = d.get(f"{args.precision}:{args.side}:{args.hidden}:{args.num_hidden_layers}", {}).get(sym)
        return None if ent is None else round(ent["bytes"] / 1e9, 4)
    except (OSError, ValueError, KeyError):
        return None


def main():
    args = parse()
    world, rank, dev = setup_dist(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    from siren_mri_amd import _native
    _native.load_library()

    step, model = build_step(args, dev, rank, world)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # pick the dominant kernel (largest time per step) from a short untimed probe (3 steps per
    # class; every class is one kernel template instantiation, so its average launch duration is
    # the rocprofv3 row of that kernel)
    totals = {}
    for kc in sorted(KCLASS_NAMES):
        with _native.KernelTimer(kc) as t:
            for _ in range(3):
                step()
        if t.launches:
            totals[kc] = t.total_ms
    dom = max(totals, key=totals.get)
    p0_recompute = args.precision == "bf16" and bool(_native.get_option("fused_forward"))
    if bool(_native.get_option("fused_forward_reg")):  # class 4 is the register-resident forward
        KCLASS_NAMES[4] = ("fused_fwd_reg_kernel (whole forward, activations in registers: layer 0 on the "
                           "f32 MFMA, hidden and output layers on the f16 MFMA)")
        KCLASS_SYMBOL["bf16"][4] = "siren::fused_fwd_reg_kernel<2, 1>"

    with _native.KernelTimer(dom, max_launches=max(64, 8 * args.steps)) as kt:
        elapsed = timed_region(step, args.steps, world)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    coords_per_rank = args.side * args.side
    value = world * coords_per_rank * args.steps / elapsed
    avg_s = kt.avg_ms * 1e-3
    flops, nbytes = kernel_model(args, dom, p0_recompute)
    mfma_peak, _ = PEAK[args.precision]
    # the binding roofline: whichever resource the algorithmic work needs longer on at peak
    if nbytes / HBM_PEAK >= flops / mfma_peak:
        bound, work, peak, unit, scale = "hbm", nbytes, HBM_PEAK, "GB/s", 1e9
    else:
        bound, work, peak, unit, scale = "mfma", flops, mfma_peak, "TFLOP/s", 1e12
    achieved = work / avg_s if avg_s > 0 else float("nan")
    roofline = {"bound": bound, "kernel": KCLASS_NAMES[dom], "kernel_symbol": KCLASS_SYMBOL.get(args.precision, {}).get(dom),
                "achieved": round(achieved / scale, 2),
                "peak": round(peak / scale, 1), "unit": unit, "frac": round(achieved / peak, 4),
                "traffic": traffic_from_profile(dom, args),
                "traffic_unit": "GB per launch (HBM, PMC)",
                "algorithmic_bytes_per_launch": nbytes, "flops_per_launch": flops,
                "achieved_tflops": round(flops / avg_s / 1e12, 2) if avg_s > 0 else None,
                "avg_launch_ms": round(kt.avg_ms, 4), "launches": kt.launches,
                "kernel_ms_per_step": {KCLASS_NAMES[k].split(" ")[0] + f"[{k}]": round(v / 3, 4)
                                       for k, v in totals.items()}}
    result = {
        "metric": "coord-samples/sec/step, 5x256 SIREN on 512^2 grid; PSNR vs ref",
        "value": value,
        "unit": "coord-samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "precision_detail": ("forward hidden GEMMs fp16 x fp16 -> fp32, backward GEMMs bf16 x bf16 -> fp32, "
                             "phases stored as 16-bit revolutions, weights / loss / Adam fp32"
                             if args.precision == "bf16" else "fp32 throughout"),
        "data": "synthetic (smooth random 512^2 image per rank: 32 sinusoids; coords = get_mgrid(512))",
        "config": {"workload": f"train_img.py fit step: {args.side}x{args.side} coordinate grid per GPU, "
                               f"SingleBVPNet 2-{'-'.join([str(args.hidden)] * (args.num_hidden_layers + 1))}-1 "
                               f"(w0=30), image_mse + Adam(1e-4), full batch",
                   "coords_per_gpu_step": coords_per_rank, "global_batch": world * coords_per_rank,
                   "parallelism": f"dp{world} (coordinate-sharded, one gradient all-reduce per step)"},
        "roofline": roofline,
    }
    # north_star's per-kernel target: bf16-MFMA utilisation of the fused SineLayer GEMM (the whole
    # forward: every layer's GEMM + bias + sine in one launch) = its algorithmic FLOPs / its average
    # launch time / the dense bf16 peak, from the same HIP-event timer, measured after the timed region
    if 4 in totals and dom != 4:
        with _native.KernelTimer(4, max_launches=64) as ft:
            for _ in range(10):
                step()
        f_flops, f_bytes = kernel_model(args, 4, p0_recompute)
        f_s = ft.avg_ms * 1e-3
        result_fwd = {"kernel": KCLASS_NAMES[4], "kernel_symbol": KCLASS_SYMBOL.get(args.precision, {}).get(4),
                      "flops_per_launch": f_flops, "avg_launch_ms": round(ft.avg_ms, 4), "launches": ft.launches,
                      "achieved_tflops": round(f_flops / f_s / 1e12, 2), "mfma_peak_tflops": mfma_peak / 1e12,
                      "mfma_frac": round(f_flops / f_s / mfma_peak, 4),
                      "hbm_gbps": round(f_bytes / f_s / 1e9, 1), "hbm_frac": round(f_bytes / f_s / HBM_PEAK, 4)}
    elif dom == 4:
        result_fwd = {"kernel": KCLASS_NAMES[4], "mfma_frac": round(flops / avg_s / mfma_peak, 4),
                      "achieved_tflops": round(flops / avg_s / 1e12, 2), "avg_launch_ms": round(kt.avg_ms, 4)}
    else:
        result_fwd = None
    if result_fwd is not None:
        result["fused_sine_gemm"] = result_fwd
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, args.cpu_budget_s)
    if rank == 0 and world == 1 and not args.no_psnr:
        result["psnr"] = psnr_check(args, dev)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
