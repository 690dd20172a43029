"""Forward-kernel timing at the metric shape (512^2, 5x256, bf16) for debug skip bits of the
register-resident forward (needs a library built with -DSIREN_FREG_DEBUG, via SIREN_MRI_AMD_LIB):
  python tools/freg_probe.py 0 1 2 4 8 16 ...   (bits: see siren_fwdreg.hip)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import siren_oracle as orc  # noqa: E402
from siren_mri_amd import _native  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402

dev = torch.device("cuda:0")
params = orc.siren_init(orc.siren_dims(2, 256, 3, 1), seed=0)
ws = [W.to(dev).requires_grad_(True) for W, _ in params]
bs = [b.to(dev).requires_grad_(True) for _, b in params]
x = orc.get_mgrid(512).unsqueeze(0).to(dev)
for dbg in [int(v) for v in (sys.argv[1:] or (0,))]:
    _native.set_option("debug_fwd_skip", dbg)
    for _ in range(3):
        siren_mlp(x, ws, bs, precision="bf16")
    torch.cuda.synchronize()
    with _native.KernelTimer(_native.KCLASS_FWD_FUSED) as kt:
        for _ in range(20):
            siren_mlp(x, ws, bs, precision="bf16")
    print(f"dbg={dbg}: forward {kt.avg_ms * 1e3:.1f} us", flush=True)
_native.set_option("debug_fwd_skip", 0)
