import os, sys, torch
sys.path.insert(0, os.getcwd())
from oracle import siren_oracle as orc
from siren_mri_amd import _native
from siren_mri_amd.ops import siren_mlp
dev = torch.device("cuda:0")
params = orc.siren_init(orc.siren_dims(2, 256, 3, 1), seed=0)
ws = [W.to(dev).requires_grad_(True) for W, _ in params]
bs = [b.to(dev).requires_grad_(True) for _, b in params]
x = orc.get_mgrid(512).unsqueeze(0).to(dev)
for dbg in [int(v) for v in (sys.argv[1:] or (0, 1, 2, 3, 0))]:
    _native.set_option("debug_fwd_skip", dbg)
    for _ in range(3): siren_mlp(x, ws, bs, precision="bf16")
    torch.cuda.synchronize()
    with _native.KernelTimer(_native.KCLASS_FWD_FUSED) as kt:
        for _ in range(10): siren_mlp(x, ws, bs, precision="bf16")
    print(f"skip={dbg}: fused forward {kt.avg_ms * 1e3:.1f} us", flush=True)
_native.set_option("debug_fwd_skip", 0)
