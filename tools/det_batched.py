"""Run-to-run determinism of the per-set-weights (hypernetwork-shape) backward under option
settings: python tools/det_batched.py  (prints the max |difference| per parameter gradient)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from siren_mri_amd import _native  # noqa: E402
from test_gpu_fwdreg import _params  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402

DEV = torch.device("cuda:0")


def _run(xd, params):
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    y = siren_mlp(xd, ws, bs, precision="bf16")
    (y.square().sum() * (1.0 / y.numel())).backward()
    torch.cuda.synchronize()
    return [(w.grad.cpu(), b.grad.cpu()) for w, b in zip(ws, bs)]

cases = [([2, 256, 256, 256, 256, 1], 5, 16384 + 31, False), ([2, 256, 256, 256, 256, 1], 5, 16384, False),
         ([2, 256, 256, 256, 256, 1], None, 16384 + 31, False), ([2, 256, 256, 256, 256, 1], 2, 16384 + 32, False),
         ([2, 256, 256, 256, 256, 1], None, 16384, True), ([2, 256, 256, 256, 256, 1], 5, 16384 + 32, True),
         ([2, 256, 256, 1], None, 16384 + 31, False), ([2, 256, 256, 256, 1], None, 16384 + 31, False),
         ([2, 256, 256, 256, 256, 1], None, 16384 + 1, False), ([2, 256, 256, 256, 256, 1], None, 16384 + 16, False)]
if len(sys.argv) > 1:
    cases = [cases[int(i)] for i in sys.argv[1:]]
OPTS = [{}]
for spec in os.environ.get("DET_OPTS", "").split(";"):
    if spec:
        OPTS.append({kv.split("=")[0]: int(kv.split("=")[1]) for kv in spec.split(",")})
for (dims, B, n, misalign), opts in [(c, o) for c in cases for o in OPTS]:
    old = {k: _native.get_option(k) for k in opts}
    for k, v in opts.items():
        _native.set_option(k, v)
    params = _params(dims, B, seed=3)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(B or 1, n, dims[0], generator=g) * 2 - 1
    xd = x.to(DEV)
    if misalign:  # x starting 8 bytes past a 16-byte boundary
        buf = torch.zeros(x.numel() + 2, device=DEV)
        buf[2:] = x.flatten().to(DEV)
        xd = buf[2:].view(B or 1, n, dims[0])
    ref = None
    diffs = []
    for rep in range(4):
        gr = _run(xd, params)
        if ref is None:
            ref = gr
        else:
            diffs.append([max(float((a - c).abs().max()), float((b - d).abs().max())) for (a, b), (c, d) in zip(ref, gr)])
    for k, v in old.items():
        _native.set_option(k, v)
    print(f"{opts} dims={dims} B={B} rows={n} misaligned={misalign}:", [max(d[l] for d in diffs) for l in range(len(dims) - 1)], flush=True)
