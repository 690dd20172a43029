"""Debug: where the pair_ring_bf16_kernel roles spend their cycles (s_memtime segment counters,
one training step of the bench workload; the counters themselves cost ~10 %).

    python tools/ring_profile.py [--side 512]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from siren_mri_amd import _native  # noqa: E402

NPROF = 6
DX_SEG = ["vm_wait", "barrier", "dma issue", "mfma+epi1", "barrier2", "epi2 stores"]
DW_SEG = ["vm_wait", "barrier", "dma issue", "mfma+convert", "-", "-"]
BOT_SEG = ["vm_wait", "barrier", "dma+dx store", "late epi", "mfma", "epi"]


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    _native.load_library()
    dev = torch.device("cuda", 0)
    step = bench.build(args.config, args, dev, 0, 1).step
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    nl = 8
    buf = torch.zeros(nl * 256 * 8 * NPROF, dtype=torch.int64, device=dev)
    _native.set_option("debug_ring_profile", buf.data_ptr())
    step()
    torch.cuda.synchronize()
    _native.set_option("debug_ring_profile", 0)
    p = buf.view(nl, 256, 8, NPROF).double().cpu()
    names = ["top (13)", "middle (12)", "bottom (14)"]
    for li in range(3):
        blk = p[li]
        if blk.abs().sum() == 0:
            continue
        role = torch.tensor([(b >> 3) & 1 for b in range(256)])
        for r, segs in ((0, DX_SEG if li < 2 else BOT_SEG), (1, DW_SEG)):
            sel = blk[role == r]  # [128, 8, NPROF]
            for wl, ws in (("w0-7", slice(0, 8)), ("w0-3", slice(0, 4)), ("w4-7", slice(4, 8))):
                m = sel[:, ws].mean(dim=(0, 1))
                tot = m.sum().item()
                parts = "  ".join(f"{segs[k]} {m[k].item():7.0f} ({100 * m[k].item() / max(tot, 1):4.1f}%)"
                                  for k in range(NPROF) if segs[k] != "-")
                print(f"{names[li]:12s} {'dx' if r == 0 else 'dw'} {wl}: total {tot:9.0f} | {parts}", flush=True)


if __name__ == "__main__":
    main()
