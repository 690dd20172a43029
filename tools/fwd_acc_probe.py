"""Forward accuracy of the fused (pipe) vs the per-layer bf16 forward against the fp64 oracle
(norm-relative error of y), for the metric architecture and a few widths."""
import os, sys
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import test_gpu_fused as T
from oracle import siren_oracle as orc

for dims, B, n in T.CASES:
    params = T._params(dims, B, seed=len(dims) + n)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(B or 1, n, dims[0], generator=g) * 2 - 1
    y_f, _ = T._forward(x, params, fused=True, grad=False)
    y_u, _ = T._forward(x, params, fused=False, grad=False)
    y_ref = orc.siren_forward(x.double(), [(W.double(), b.double()) for W, b in params])
    print(dims, B, n, "fused-vs-ref %.3e  perlayer-vs-ref %.3e  fused-vs-perlayer %.3e" % (
        orc.norm_rel(y_f, y_ref), orc.norm_rel(y_u, y_ref), orc.norm_rel(y_f, y_u)), flush=True)
