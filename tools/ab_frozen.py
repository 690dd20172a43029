"""A/B a runtime option per kernel class with the model state restored before every step (debug
timing switches whose results are wrong then cannot drift the weights into another regime).

    python tools/ab_frozen.py NAME V1,V2 [--kclass 13] [--reps 20] [--rounds 2]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from siren_mri_amd import _native  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("name")
    p.add_argument("values")
    p.add_argument("--kclass", type=int, nargs="*", default=[12, 13, 14])
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--rounds", type=int, default=2)
    cli = p.parse_args()
    sys.argv = [sys.argv[0], "--no-psnr", "--no-cpu-baseline", "--no-other-configs"]
    args = bench.parse()
    _native.load_library()
    dev = torch.device("cuda", 0)
    wl = bench.build("m", args, dev, 0, 1)
    opt = wl.extra["optimizer"]
    for _ in range(5):
        wl.step()
    torch.cuda.synchronize()
    params = [q for g in opt.param_groups for q in g["params"]]
    snap = [(q, q.detach().clone()) for q in params]
    for q in params:
        for k, v in opt.state.get(q, {}).items():
            if torch.is_tensor(v):
                snap.append((v, v.detach().clone()))

    def restore():
        with torch.no_grad():
            for t, s in snap:
                t.copy_(s)

    default = _native.get_option(cli.name)
    for r in range(cli.rounds):
        for v in [int(x) for x in cli.values.split(",")]:
            _native.set_option(cli.name, v)
            row = []
            for kc in cli.kclass:
                with _native.KernelTimer(kc) as t:
                    for _ in range(cli.reps):
                        restore()
                        wl.step()
                row.append(f"{kc}: {t.total_ms / max(1, t.launches) * 1e3:7.1f} us")
            print(f"round {r} {cli.name}={v}  " + "  ".join(row), flush=True)
    _native.set_option(cli.name, default)
    restore()


if __name__ == "__main__":
    main()
