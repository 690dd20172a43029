"""Debug: per-row / per-column error pattern of dx for the wide-input first layer."""
import torch
from oracle import siren_oracle as orc
from siren_mri_amd.ops import siren_mlp

DEV = torch.device("cuda:0")
for prec in ("fp32", "bf16"):
    for C, rows in ((20, 64), (20, 700), (120, 700)):
        dims = [C, 256, 256, 2]
        params = orc.siren_init(dims, seed=C)
        g = torch.Generator().manual_seed(C)
        x = torch.sin(torch.rand(1, rows, C, generator=g) * 6.28)
        lw = torch.randn(1, rows, 2, generator=g)
        ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
        xx = x.double().requires_grad_(True)
        (orc.siren_forward(xx, ps) * lw.double()).sum().backward()
        ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
        bs = [b.to(DEV).requires_grad_(True) for _, b in params]
        xd = x.to(DEV).requires_grad_(True)
        (siren_mlp(xd, ws, bs, precision=prec) * lw.to(DEV)).sum().backward()
        dx, ref = xd.grad.cpu().double()[0], xx.grad[0]
        err = (dx - ref).abs()
        scale = ref.abs().mean()
        bad_rows = (err.max(1).values > 0.05 * scale).nonzero().flatten()
        bad_cols = (err.max(0).values > 0.05 * scale).nonzero().flatten()
        print(prec, C, rows, "rel", float(err.norm() / ref.norm()), "bad rows", bad_rows[:20].tolist(),
              len(bad_rows), "bad cols", bad_cols.tolist()[:40])
        if len(bad_rows):
            r = int(bad_rows[0])
            print("  row", r, "dx", dx[r, :6].tolist(), "ref", ref[r, :6].tolist())
