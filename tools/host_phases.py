"""Host (CPU) time per phase of the bench step at a tiny grid (GPU work << host work), to find
the launch-path overhead: python tools/host_phases.py [side]"""
import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
import bench
from siren_mri_amd import dataio, loss_functions, modules, training

side = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = modules.SingleBVPNet(type="sine", mode="mlp", hidden_features=256, num_hidden_layers=3,
                             sidelength=(side, side), precision="bf16").to(dev)
coords = dataio.get_mgrid(side)[None].to(dev)
gt = {"img": torch.rand(1, side * side, 1, device=dev)}
opt = training.make_adam(model.parameters(), 1e-4)
mi = {"coords": coords}
T = {k: 0.0 for k in ("forward", "loss", "backward", "step", "zero_grad")}
from siren_mri_amd import ops
INNER = {}


def _timed(name, fn):
    def wrap(*a, **k):
        t = time.perf_counter()
        r = fn(*a, **k)
        INNER[name] = INNER.get(name, 0.0) + time.perf_counter() - t
        return r
    return wrap


ops._SirenMLPFunction.backward = staticmethod(_timed("mlp_bwd", ops._SirenMLPFunction.backward))
ops._SirenMLPFunction.forward = staticmethod(_timed("mlp_fwd", ops._SirenMLPFunction.forward))
loss_functions._WeightedSSE.backward = staticmethod(_timed("sse_bwd", loss_functions._WeightedSSE.backward))
loss_functions._WeightedSSE.forward = staticmethod(_timed("sse_fwd", loss_functions._WeightedSSE.forward))
N = 400
for it in range(N + 50):
    t0 = time.perf_counter()
    out = model(mi)
    t1 = time.perf_counter()
    loss = loss_functions.image_mse(None, out, gt, high_freq=False)["img_loss"]
    t2 = time.perf_counter()
    loss.backward()
    t3 = time.perf_counter()
    opt.step()
    t4 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    t5 = time.perf_counter()
    if it == 49:
        INNER.clear()
    if it >= 50:
        for k, a, b in (("forward", t0, t1), ("loss", t1, t2), ("backward", t2, t3), ("step", t3, t4),
                        ("zero_grad", t4, t5)):
            T[k] += b - a
torch.cuda.synchronize()
tot = sum(T.values())
print("host us/step:", {k: round(v / N * 1e6, 1) for k, v in T.items()}, "total", round(tot / N * 1e6, 1))
print("inside autograd functions us/step:", {k: round(v / N * 1e6, 1) for k, v in INNER.items()})
