"""Run-to-run comparison of the forward's saved buffer (prepared weights + phase codes) at a
ragged row count: python tools/det_saved.py [rows]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_fwdreg import _params  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402

DEV = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16385
dims = [2, 256, 256, 256, 256, 1]
params = _params(dims, None, seed=3)
g = torch.Generator().manual_seed(n)
x = (torch.rand(1, n, 2, generator=g) * 2 - 1).to(DEV)
ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
bs = [b.to(DEV).requires_grad_(True) for _, b in params]
bufs = []
for rep in range(3):
    junk = torch.full((64 << 20,), rep + 7, dtype=torch.uint8, device=DEV)  # dirty the allocator's pool
    del junk
    y, saved = siren_mlp(x, ws, bs, precision="bf16", return_saved=True)
    torch.cuda.synchronize()
    bufs.append(saved.clone())
total = bufs[0].numel()
pbytes = n * 256 * 2
preg = (pbytes + 255) // 256 * 256
nph = 4 if total >= 4 * preg else 3
pstart = total - nph * preg
print("saved bytes", total, "phase regions", nph, "starting at", pstart)
edges = [("w_op[1]", 0), ("wt[1]", 131072), ("w_op[2]", 262144), ("wt[2]", 393216), ("w_op[3]", 524288),
         ("wt[3]", 655360), ("frag", 786432)] + [(f"P_{4 - nph + i}", pstart + i * preg) for i in range(nph)] + [("end", total)]
for k in (1, 2):
    diff = bufs[0] != bufs[k]
    print(f"run 0 vs {k}:")
    for (name, a), (_, b) in zip(edges[:-1], edges[1:]):
        d = diff[a:b].nonzero().flatten()
        if d.numel():
            msg = f"  {name}: {d.numel()} bytes differ"
            if name.startswith("P_"):
                rows = sorted(set((d // 512).tolist()))
                msg += f", rows {rows[:6]}{'...' if len(rows) > 6 else ''} (valid rows < {n}), cols {sorted(set(((d % 512) // 2).tolist()))[:8]}"
            print(msg)
