"""Diagnostic: run-to-run comparison of the stored P_0 phase codes (option debug_keep_p0 = 1,
the round-2 path for ragged shapes) of the register-resident forward. Prints, for every
differing 16-byte store chunk: tile, wave, lane row j, block pfb, half, lane half hh.
    python tools/det_p0.py [rows] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import siren_oracle as orc  # noqa: E402
from siren_mri_amd import _native  # noqa: E402
from siren_mri_amd.ops import siren_mlp  # noqa: E402

DEV = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16385
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dims = [2, 256, 256, 256, 256, 1]
params = orc.siren_init(dims, seed=3)
x = (torch.rand(1, n, 2, generator=torch.Generator().manual_seed(n)) * 2 - 1).to(DEV)
ws = [W.to(DEV) for W, _ in params]
bs = [b.to(DEV) for _, b in params]
_native.set_option("debug_keep_p0", 1)
bufs, ys = [], []
for rep in range(reps):
    junk = torch.full((64 << 20,), rep + 7, dtype=torch.uint8, device=DEV)
    del junk
    wsr = [w.clone().requires_grad_(True) for w in ws]
    y, saved = siren_mlp(x, wsr, bs, precision="bf16", return_saved=True)
    torch.cuda.synchronize()
    bufs.append(saved.clone().cpu())
    ys.append(y.detach().cpu())
_native.set_option("debug_keep_p0", 0)
total = bufs[0].numel()
preg = (n * 512 + 255) // 256 * 256
p0 = total - 4 * preg
print(f"rows {n}: saved {total} B, P_0 region at {p0}")
for k in range(1, reps):
    print(f"run 0 vs {k}: y equal {torch.equal(ys[0], ys[k])}")
    for name, a, b in [("weights", 0, p0)] + [(f"P_{i}", p0 + i * preg, p0 + (i + 1) * preg) for i in range(4)]:
        d = (bufs[0][a:b] != bufs[k][a:b]).nonzero().flatten()
        if d.numel() == 0:
            continue
        print(f"  {name}: {d.numel()} bytes differ")
        if name.startswith("P_"):
            chunks = sorted(set((d // 16).tolist()))
            desc = []
            for c in chunks[:40]:
                byte = c * 16
                row, col = byte // 512, byte % 512
                desc.append(f"t{row // 256}w{(row % 256) // 32}j{row % 32}:fb{col // 64}h{(col % 64) // 32}hh{(col % 32) // 16}")
            print("   chunks:", len(chunks), " ".join(desc))
            # for each differing dword: both runs' values and the first dword of the chunk 32 B on
            # (the codes of elements 8, 9: what the next part of the epilogue writes)
            dw = sorted(set((d // 4).tolist()))[:8]
            for q in dw:
                b0 = a + q * 4
                v0 = bufs[0][b0:b0 + 4].view(torch.int32).item()
                vk = bufs[k][b0:b0 + 4].view(torch.int32).item()
                nx0 = bufs[0][b0 + 32:b0 + 36].view(torch.int32).item()
                nxk = bufs[k][b0 + 32:b0 + 36].view(torch.int32).item()
                print(f"   dword@{(b0 - a) % 512}: run0 {v0:#010x} run{k} {vk:#010x} | +32B run0 {nx0:#010x} run{k} {nxk:#010x}")
            r = d[0].item() // 512
            print("   row", r, "run0", bufs[0][a + r * 512:a + r * 512 + 512].view(torch.int16)[:16].tolist())
            print("   row", r, f"run{k}", bufs[k][a + r * 512:a + r * 512 + 512].view(torch.int16)[:16].tolist())
