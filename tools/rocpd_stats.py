"""Kernel statistics (name, calls, average / total duration, share) from a rocprofv3 SQLite
results database (the default output format of ROCm 7), in the CSV layout of --stats
(`Name,Calls,TotalDurationNs,AverageNs,Percentage`) so tools/rocprof_summary.py reads it.

    python tools/rocpd_stats.py run_results.db out_kernel_stats.csv"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = list(c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels group by {name} "
                          "order by sum(end - start) desc"))
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for n, calls, total, avg in rows:
            w.writerow([n, calls, total, f"{avg:.1f}", f"{100.0 * total / tot:.4f}"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
