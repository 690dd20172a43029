"""Per-step kernel breakdown of a rocprofv3 kernel trace (CSV): the last N steps, a step delimited
by launches of a marker kernel (default: the SIREN forward).

    python tools/step_kernels.py run_kernel_trace.csv [N] [marker]
"""
import collections
import csv
import sys

path = sys.argv[1]
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 3
marker = sys.argv[3] if len(sys.argv) > 3 else "fused_fwd_reg_kernel"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(marks) < nlast + 1:
    sys.exit(f"only {len(marks)} marker launches")
lo, hi = marks[-nlast - 1], marks[-1]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[lo:hi]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += d
wall = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3 / nlast
busy = sum(v[1] for v in agg.values()) / nlast
print(f"# last {nlast} steps (marker {marker}): wall {wall:.0f} us/step, kernels {busy:.0f} us/step")
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t / nlast:9.1f} us/step {n / nlast:5.1f}/step  {name[:130]}")
