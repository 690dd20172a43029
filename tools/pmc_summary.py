"""Per-kernel mean of rocprofv3 PMC counters over the dispatches of tools/pmc_bench.sh passes.

FETCH_SIZE is reported in KB and, on gfx950, counts half the bytes of 16-B/lane streaming reads
(MI355X_MICROARCH.md §HBM): HBM read bytes = 2 x FETCH_SIZE x 1024. WRITE_SIZE (KB) is exact.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(pattern):
    out = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
            cname = r.get("Counter_Name") or r.get("Counter-Name")
            val = r.get("Counter_Value") or r.get("Counter-Value")
            disp = r.get("Dispatch_Id") or r.get("Dispatch-Id")
            if name is None or cname is None:
                continue
            out[name][cname].append((disp, float(val)))
    return out


def main(prefix, json_out=None):
    merged = defaultdict(dict)
    for k in (1, 2, 3):
        data = load(f"{prefix}_pmc{k}/**/*counter_collection.csv")
        for name, counters in data.items():
            for c, vals in counters.items():
                # sum per dispatch (counters may be reported per XCD / instance), then mean
                per = defaultdict(float)
                for disp, v in vals:
                    per[disp] += v
                merged[name][c] = sum(per.values()) / max(1, len(per))
    # SQ_VALU_MFMA_BUSY_CYCLES is a cycle count summed over the SIMDs (32 per 32x32x16 MFMA);
    # GRBM_GUI_ACTIVE is the kernel's active cycles summed over the 8 XCDs (MI355X_MICROARCH.md):
    # MFMA busy % = busy / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
    print("| kernel | HBM read MB (2xFETCH) | HBM write MB | MFMA busy cycles (sum over SIMDs) | MFMA busy % | "
          "VALU active % | wait % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    rows = []
    for name, c in merged.items():
        short = name.split("(")[0].replace("void ", "")[-60:]
        rd = 2 * c.get("FETCH_SIZE", float("nan")) * 1024 / 1e6
        wr = c.get("WRITE_SIZE", float("nan")) * 1024 / 1e6
        wc = c.get("SQ_WAVE_CYCLES", float("nan"))
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan"))
        valu = c.get("SQ_ACTIVE_INST_VALU", float("nan"))
        wait = c.get("SQ_WAIT_ANY", float("nan"))
        gui = c.get("GRBM_GUI_ACTIVE", float("nan"))
        mpct = 100 * mfma / (1024 * gui / 8) if gui == gui and gui > 0 else float("nan")
        rows.append((rd + (wr if wr == wr else 0), name, short, rd, wr, (mfma, mpct), valu, wait, wc, c))
    rows.sort(key=lambda r: -r[0] if r[0] == r[0] else 0)
    for _, name, short, rd, wr, mfma, valu, wait, wc, c in rows:
        print(f"| `{short}` | {rd:.1f} | {wr:.1f} | {mfma[0]:.3g} | {mfma[1]:.1f} | "
              f"{100 * valu / wc if wc else float('nan'):.1f} | {100 * wait / wc if wc else float('nan'):.1f} |")
    if json_out:
        # per-kernel HBM bytes per launch, keyed by the kernel symbol without `void ` and arguments
        d = {}
        for _, name, short, rd, wr, *_r in rows:
            sym = name.split("(")[0].replace("void ", "").strip()
            d[sym] = {"read_bytes": rd * 1e6, "write_bytes": wr * 1e6, "bytes": (rd + wr) * 1e6}
        import json
        with open(json_out, "w") as f:
            json.dump(d, f, indent=1)
    print()
    print("raw means per dispatch:")
    for _, name, short, *_r, c in rows:
        print(f"- `{short}`: " + ", ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
