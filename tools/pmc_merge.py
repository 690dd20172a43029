"""Merge one workload's PMC passes (tools/pmc_bench.sh TAG ...) into profiles/pmc_traffic.json.

    python tools/pmc_merge.py gpurun_out/TAG KEY [STEP_KERNEL]

KEY is bench.traffic_key of the workload ("bf16:rows262144:256:3"). Per kernel symbol: HBM read
bytes per launch = 2 x FETCH_SIZE x 1024 (the gfx950 correction of MI355X_MICROARCH.md §HBM),
write bytes = WRITE_SIZE x 1024, each the mean over that kernel's dispatches. The whole-step
traffic is the sum over kernels of bytes per launch x launches per step, with launches per step =
a kernel's dispatch count / STEP_KERNEL's (default: the Adam kernel, one launch per step; the
forward is two launches, its two epilogue forms).
"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(prefix):
    means, counts = defaultdict(dict), {}
    for k, counter in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
        for name, cs in load(f"{prefix}_pmc{k}/**/*counter_collection.csv").items():
            vals = cs.get(counter)
            if not vals:
                continue
            per = defaultdict(float)
            for disp, v in vals:
                per[disp] += v  # summed over XCD / instance rows of one dispatch
            sym = name.split("(")[0].replace("void ", "").strip()
            means[sym][counter] = sum(per.values()) / len(per)
            if k == 1:
                counts[sym] = len(per)
    return means, counts


def main(prefix, key, step_kernel="siren::adam_kernel"):
    means, counts = per_kernel(prefix)
    entry = {}
    for sym, c in means.items():
        rd = 2 * c.get("FETCH_SIZE", 0.0) * 1024
        wr = c.get("WRITE_SIZE", 0.0) * 1024
        entry[sym] = {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr, "dispatches": counts.get(sym, 0)}
    steps = sum(n for s, n in counts.items() if s.startswith(step_kernel))
    if steps:
        entry["_step_bytes"] = sum(e["bytes"] * e["dispatches"] / steps for s, e in entry.items()
                                   if isinstance(e, dict) and e.get("dispatches"))
        entry["_steps_profiled"] = steps
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[key] = entry
    d["_note"] = ("HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_bench.sh, "
                  "tools/pmc_merge.py): read = 2 x FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md), KB -> bytes; "
                  "keyed precision:rows<rows per launch>:hidden:num_hidden_layers, then kernel symbol; _step_bytes = "
                  "the whole step's traffic (launches per step from dispatch counts)")
    with open(path, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in entry.items() if k.startswith("_step")}))
    for sym, e in sorted(((s, e) for s, e in entry.items() if not s.startswith("_")), key=lambda t: -t[1]["bytes"]):
        print(f"{e['bytes'] / 1e6:10.1f} MB  x{e['dispatches']:5d}  {sym}")


if __name__ == "__main__":
    main(*sys.argv[1:])
