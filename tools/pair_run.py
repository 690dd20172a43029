"""Run N bench steps with only some pair_ring roles active (PMC / trace target).

    python tools/pair_run.py ROLES [steps]     # ROLES: 3 both, 1 input-gradient, 2 weight-gradient
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from siren_mri_amd import _native  # noqa: E402

roles = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
sys.argv = sys.argv[:1]
args = bench.parse()
_native.load_library()
dev = torch.device("cuda", 0)
step, _ = bench.build_step(args, dev, 0, 1)
for _ in range(3):
    step()
_native.set_option("debug_pair_roles", roles)
for _ in range(steps):
    step()
torch.cuda.synchronize()
_native.set_option("debug_pair_roles", 3)
print("done", roles, steps)
