"""Mean PMC counters of one kernel (name substring) per library variant, from tools/pmc_probe.sh."""
import csv
import glob
import sys
from collections import defaultdict


def main(prefix, kname, names):
    for n in names:
        acc = defaultdict(list)
        for path in glob.glob(f"{prefix}_{n}_pmc*/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                if kname not in (r.get("Kernel_Name") or ""):
                    continue
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        vals = {k: sum(v) / len(v) for k, v in acc.items()}
        print(f"== {n}")
        for k in sorted(vals):
            print(f"  {k:28s} {vals[k]:.4g}")
        if "GRBM_GUI_ACTIVE" in vals and "SQ_WAVE_CYCLES" in vals:
            print(f"  waves-cycles/GUI_ACTIVE      {vals['SQ_WAVE_CYCLES'] / vals['GRBM_GUI_ACTIVE']:.3g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
