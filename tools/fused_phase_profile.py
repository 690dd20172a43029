"""Debug: where the fused forward spends its time (per-workgroup clock64 phase counters).

    PYTHONPATH=. python tools/fused_phase_profile.py [side] [hidden] [nh]
"""
import sys

import torch

from oracle import siren_oracle as orc
from siren_mri_amd import _native
from siren_mri_amd.ops import siren_mlp

side = int(sys.argv[1]) if len(sys.argv) > 1 else 512
F = int(sys.argv[2]) if len(sys.argv) > 2 else 256
nh = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda:0")
dims = orc.siren_dims(2, F, nh, 1)
params = orc.siren_init(dims, seed=0)
ws = [W.to(dev).requires_grad_(True) for W, _ in params]
bs = [b.to(dev).requires_grad_(True) for _, b in params]
x = orc.get_mgrid(side).unsqueeze(0).to(dev)


def fwd(grad):
    with torch.set_grad_enabled(grad):
        return siren_mlp(x, ws, bs, precision="bf16")


for grad in (True, False):
    for _ in range(3):
        fwd(grad)
    torch.cuda.synchronize()
    with _native.KernelTimer(_native.KCLASS_FWD_FUSED) as kt:
        for _ in range(10):
            fwd(grad)
    print(f"grad={grad}: fused forward {kt.avg_ms * 1e3:.1f} us/launch")

prof = torch.zeros(256 * 4, dtype=torch.int64, device=dev)
_native.set_option("debug_fused_profile", prof.data_ptr())
fwd(True)
torch.cuda.synchronize()
_native.set_option("debug_fused_profile", 0)
p = prof.view(256, 4).double().cpu()
names = ["layer0 pass", "K loop (+barrier)", "epilogue", "convert/output"]
tot = p.sum(1).mean().item()
for k in range(4):
    print(f"{names[k]:20s} mean {p[:, k].mean().item():10.0f} cycles  ({100 * p[:, k].mean().item() / tot:.1f} %)")
print(f"total per workgroup {tot:.0f} cycles")
