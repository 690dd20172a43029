"""Run-to-run check of the wide-input (C = 16) shared-weight stack of
tests/test_gpu_wide.py::test_wide_inputs_shared_ragged[16]:
    python tools/det_wide.py [runs] [C] [N]
Between runs the caching allocator is filled with different byte patterns (a read of memory the
path never wrote shows up as a run-to-run difference); prints which saved regions / gradients
differ from run 0 and every run's gradient error against the fp64 oracle."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import siren_oracle as orc  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402
from tests.test_gpu_wide import _params  # noqa: E402

DEV = torch.device("cuda:0")
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
C = int(sys.argv[2]) if len(sys.argv) > 2 else 16
N = int(sys.argv[3]) if len(sys.argv) > 3 else 70000 + C
dims = [C, 256, 256, 256, 1]
params = _params(dims, None, C)
g = torch.Generator().manual_seed(C + 100)
x = torch.sin(torch.rand(1, N, C, generator=g) * 6.28)
lw = torch.randn(1, N, 1, generator=g)
ps = [(W.double().requires_grad_(True), b.double().requires_grad_(True)) for W, b in params]
y_ref = orc.siren_forward(x.double(), ps)
(y_ref * lw.double()).sum().backward()

res = []
for r in range(runs):
    junk = [torch.full((s << 20,), (0x11 * (r + 3)) & 0xFF, dtype=torch.uint8, device=DEV) for s in (8, 32, 128)]
    del junk
    ws = [W.to(DEV).requires_grad_(True) for W, _ in params]
    bs = [b.to(DEV).requires_grad_(True) for _, b in params]
    y, saved = siren_mlp(x.to(DEV), ws, bs, precision="bf16", return_saved=True)
    torch.cuda.synchronize()
    sv_fwd = saved.cpu()
    (y * lw.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    if not torch.equal(sv_fwd, saved.cpu()):
        print(f"run {r}: the backward changed the saved buffer", flush=True)
    gw = [w.grad.cpu() for w in ws]
    gb = [b.grad.cpu() for b in bs]
    res.append((y.detach().cpu(), saved.cpu(), gw, gb))
    errs = " ".join(f"dW{l}={orc.norm_rel(gw[l], ps[l][0].grad):.2e}" for l in range(len(gw)))
    print(f"run {r}: y={orc.norm_rel(y.detach().cpu(), y_ref.detach()):.2e} {errs}", flush=True)

for r in range(1, runs):
    y, sv, gw, gb = res[r]
    msg = []
    if not torch.equal(y, res[0][0]):
        msg.append("y")
    d = (sv != res[0][1]).nonzero().flatten()
    if d.numel():
        msg.append(f"saved bytes differ: {d.numel()} (first {d[:4].tolist()}, last {d[-1].item()}, of {sv.numel()})")
        nsine = len(dims) - 2
        front = sv.numel() - nsine * N * 512
        fd = d[d < front]
        if fd.numel():
            msg.append(f"front (prepared weights, {front} B): {fd.numel()} bytes, range [{fd.min().item()}, {fd.max().item()}]")
        for l in range(nsine):
            o = front + l * N * 512
            ld = d[(d >= o) & (d < o + N * 512)] - o
            if ld.numel():
                rows_ = torch.unique(ld // 512)
                feats = torch.unique((ld % 512) // 2)
                blocks = torch.unique(rows_ // 256)
                msg.append(f"P_{l}: {ld.numel()} bytes, {rows_.numel()} rows [{rows_.min().item()}, {rows_.max().item()}], "
                           f"features [{feats.min().item()}, {feats.max().item()}] ({feats.numel()}), "
                           f"256-row blocks {blocks.tolist()[:12]}{'...' if blocks.numel() > 12 else ''}, "
                           f"rows mod 32: {torch.unique(rows_ % 32).tolist()}")
                # the first few differing dwords: this run, run 0, the dwords 32 B later / earlier,
                # and the row's x values (float bits) that a stray load could have delivered
                dw = torch.unique(ld // 4)[:6]
                for q in dw.tolist():
                    base = o + 4 * q
                    cur = sv[base:base + 4].view(torch.int32).item()
                    ref = res[0][1][base:base + 4].view(torch.int32).item()
                    nxt = res[0][1][base + 32:base + 36].view(torch.int32).item()
                    prv = res[0][1][base - 32:base - 28].view(torch.int32).item()
                    row = (4 * q) // 512
                    xb = x[0, row].view(torch.int32).tolist()
                    msg.append(f"  dword@row {row} byte {(4 * q) % 512}: run {r} {cur & 0xffffffff:08x} run0 {ref & 0xffffffff:08x} "
                               f"(+32B {nxt & 0xffffffff:08x}, -32B {prv & 0xffffffff:08x}); "
                               f"in x row: {any((cur & 0xffffffff) == (v & 0xffffffff) for v in xb)}")
    for l in range(len(gw)):
        if not torch.equal(gw[l], res[0][2][l]):
            msg.append(f"dW{l} {orc.norm_rel(gw[l], res[0][2][l]):.1e}")
    print(f"run {r} vs 0: {'equal' if not msg else chr(10).join(msg)}", flush=True)
