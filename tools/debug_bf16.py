import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from oracle import siren_oracle as orc
from siren_mri_amd.ops import siren_mlp
dev = torch.device("cuda:0")

def grads(x, params, prec, lw):
    ws = [W.to(dev).requires_grad_(True) for W, _ in params]
    bs = [b.to(dev).requires_grad_(True) for _, b in params]
    y = siren_mlp(x.to(dev), ws, bs, precision=prec)
    (y * lw.to(dev)).sum().backward()
    return y.detach().cpu(), [(w.grad.cpu(), b.grad.cpu()) for w, b in zip(ws, bs)]

for side, hidden, nh in [(32, 256, 3), (8, 256, 2), (64, 64, 2), (16, 128, 1)]:
    dims = orc.siren_dims(2, hidden, nh, 1)
    params = orc.siren_init(dims, seed=1)
    x = orc.get_mgrid(side).unsqueeze(0)
    lw = torch.randn(1, side * side, 1)
    y32, g32 = grads(x, params, "fp32", lw)
    y16, g16 = grads(x, params, "bf16", lw)
    print(f"side {side} hidden {hidden} nh {nh}: y {orc.norm_rel(y16, y32):.2e}")
    for l, ((a, b), (c, d)) in enumerate(zip(g16, g32)):
        print(f"   layer {l}: dW {orc.norm_rel(a, c):.2e} db {orc.norm_rel(b, d):.2e}")
    if side == 8:
        a, c = g16[1][0], g32[1][0]
        print("   dW1 bf16[:4,:4]", a[:4, :4]); print("   dW1 fp32[:4,:4]", c[:4, :4])

# first timings at the metric size
dims = orc.siren_dims(2, 256, 3, 1)
params = orc.siren_init(dims, seed=0)
x = orc.get_mgrid(512).unsqueeze(0).to(dev)
ws = [W.to(dev).requires_grad_(True) for W, _ in params]
bs = [b.to(dev).requires_grad_(True) for _, b in params]
gt = torch.randn(1, 512 * 512, 1, device=dev)
for prec in ("bf16", "fp32"):
    for it in range(13):
        if it == 3:
            torch.cuda.synchronize(); t0 = time.perf_counter()
        y = siren_mlp(x, ws, bs, precision=prec)
        loss = ((y - gt) ** 2).mean()
        loss.backward()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 10
    print(f"{prec}: fwd+bwd {dt*1e3:.2f} ms/step -> {512*512/dt:.3e} coord-samples/s")
