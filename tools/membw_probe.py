"""Achievable HBM write / copy bandwidth on this GPU (PyTorch fill / copy of a 403 MB buffer,
the forward's phase-tensor volume)."""
import torch

dev = torch.device("cuda:0")
n = 403 * 1024 * 1024 // 4
a = torch.empty(n, dtype=torch.float32, device=dev)
b = torch.empty(n, dtype=torch.float32, device=dev)
for name, fn, nbytes in [("fill", lambda: a.fill_(1.0), n * 4), ("copy", lambda: b.copy_(a), 2 * n * 4),
                         ("zero", lambda: a.zero_(), n * 4)]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name}: {ms * 1e3:.1f} us, {nbytes / ms / 1e9:.2f} TB/s", flush=True)

# pure read: reduction over a 268 MB buffer (the middle pair kernel's dZ + P volume)
m = 268 * 1024 * 1024 // 4
c = torch.ones(m, dtype=torch.float32, device=dev)
for _ in range(3):
    c.sum()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    c.sum()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"sum(268MB): {ms * 1e3:.1f} us, {m * 4 / ms / 1e9:.2f} TB/s", flush=True)
