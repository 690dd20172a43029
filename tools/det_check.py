"""Determinism check: gradients of the metric stack, REPS runs on the same inputs; prints how many
repeats differ from the first and, for those, the max abs difference per layer."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from oracle import siren_oracle as orc  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402

DEV = torch.device("cuda:0")


def run(n, dims, seed):
    params = [orc.siren_init(dims, seed=seed + l)[l] for l in range(len(dims) - 1)]
    x = torch.rand(1, n, dims[0], generator=torch.Generator().manual_seed(n + 1)) * 2 - 1
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    y = siren_mlp(x.to(DEV), ws, bs, precision="bf16")
    y.square().sum().backward()
    torch.cuda.synchronize()
    return [(w.grad.cpu(), b.grad.cpu()) for w, b in zip(ws, bs)]


REPS = int(os.environ.get("REPS", "8"))
for n in (int(a) for a in (sys.argv[1:] or ["65613", "4096"])):
    dims = [2, 256, 256, 256, 256, 1]
    res = [run(n, dims, n) for _ in range(REPS)]
    bad = []
    for k, r in enumerate(res[1:], 1):
        d = [max((x - y).abs().max().item(), (u - v).abs().max().item()) for (x, u), (y, v) in zip(res[0], r)]
        if any(v != 0 for v in d):
            bad.append((k, d))
    print(f"n={n}: {len(bad)} of {REPS - 1} repeats differ from the first {bad[:3]}")
