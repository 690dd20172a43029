"""A/B a runtime option on one box: bench steps alternating option values, per-kernel-class times.

    python tools/ab_option.py NAME V1,V2 [--rounds 3] [--steps 100] [--config m|c1|..|c4]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from siren_mri_amd import _native  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("name")
    p.add_argument("values")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--kclass", type=int, default=0, help="also time this kernel class (bench.KCLASS_NAMES)")
    p.add_argument("--config", default="m", help="bench workload (bench.py --config)")
    cli = p.parse_args()
    sys.argv = [sys.argv[0], "--no-psnr", "--no-cpu-baseline", "--config", cli.config]
    args = bench.parse()
    _native.load_library()
    dev = torch.device("cuda", 0)
    step = bench.build(args.config, args, dev, 0, 1).step
    vals = [int(v) for v in cli.values.split(",")]
    default = _native.get_option(cli.name)
    for _ in range(10):
        step()
    for r in range(cli.rounds):
        for v in vals:
            _native.set_option(cli.name, v)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(cli.steps):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / cli.steps * 1e3
            kt = ""
            if cli.kclass:
                with _native.KernelTimer(cli.kclass) as t:
                    for _ in range(20):
                        step()
                kt = f", kernel class {cli.kclass}: {t.avg_ms * 1e3:.1f} us/launch"
            print(f"round {r} {cli.name}={v}: {ms:.4f} ms/step{kt}", flush=True)
    _native.set_option(cli.name, default)


if __name__ == "__main__":
    main()
