"""Run-to-run comparison of every gradient of the metric stack (bf16, default kernels):
    python tools/det_bwd.py [rows] [runs]
Prints, per layer, whether dW / db / dx differ from run 0 and by how much (norm-relative)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import siren_oracle as orc  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402

DEV = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dims = [2, 256, 256, 256, 256, 1]
params = orc.siren_init(dims, seed=5)
x = (torch.rand(1, n, 2, generator=torch.Generator().manual_seed(6)) * 2 - 1).to(DEV)
lw = torch.randn(1, n, 1, generator=torch.Generator().manual_seed(9)).to(DEV)
res = []
for r in range(runs):
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    xd = x.clone().requires_grad_(True)
    (siren_mlp(xd, ws, bs, precision="bf16") * lw).sum().backward()
    torch.cuda.synchronize()
    res.append(([w.grad.cpu() for w in ws], [b.grad.cpu() for b in bs], xd.grad.cpu()))
lib = os.environ.get("SIREN_MRI_AMD_LIB", "default")
bad = 0
for r in range(1, runs):
    msg = []
    for l in range(len(dims) - 1):
        for name, a, b in (("dW", res[r][0][l], res[0][0][l]), ("db", res[r][1][l], res[0][1][l])):
            if not torch.equal(a, b):
                msg.append(f"{name}{l} {orc.norm_rel(a, b):.1e}")
    if not torch.equal(res[r][2], res[0][2]):
        msg.append(f"dx {orc.norm_rel(res[r][2], res[0][2]):.1e}")
    bad += bool(msg)
    print(f"[{lib}] run {r} vs 0: {'equal' if not msg else ' '.join(msg)}")
print(f"[{lib}] {bad} of {runs - 1} runs differ")
