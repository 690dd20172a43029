"""Time each pair_ring_bf16_kernel role alone (debug_pair_roles 1 / 2) against both (3) at the
bench workload: which role bounds the paired launch, and what the shared tiles save.

    python tools/pair_roles.py   (the bench's metric configuration)
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
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--roles", type=int, nargs="*", default=[3, 1, 2, 3])
    p.add_argument("--option", default=None, help="NAME=V1,V2: repeat every role set per option value")
    cli = p.parse_args()
    sys.argv = [sys.argv[0], "--no-psnr", "--no-cpu-baseline", "--no-other-configs"]
    args = bench.parse()
    _native.load_library()
    dev = torch.device("cuda", 0)
    step = bench.build("m", args, dev, 0, 1).step
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    opts = [(None, None)]
    if cli.option:
        name, vals = cli.option.split("=")
        opts = [(name, int(v)) for v in vals.split(",")]
    for (oname, oval), roles in [(o, r) for o in opts for r in cli.roles]:
        if oname:
            _native.set_option(oname, oval)
        _native.set_option("debug_pair_roles", roles)
        row = []
        for kc in (_native.KCLASS_PAIR_RING, _native.KCLASS_PAIR_RING_TOP, _native.KCLASS_PAIR_RING_BOT):
            with _native.KernelTimer(kc) as t:
                for _ in range(cli.reps):
                    step()
            row.append(f"{kc}: {t.total_ms / max(1, t.launches) * 1e3:7.1f} us")
        print((f"{oname}={oval} " if oname else "") + f"roles={roles}  " + "  ".join(row), flush=True)
    _native.set_option("debug_pair_roles", 3)


if __name__ == "__main__":
    main()
