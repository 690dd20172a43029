"""Summarise a rocprofv3 --kernel-trace --stats CSV into a per-step kernel table (markdown).

    python tools/rocprof_summary.py run_kernel_stats.csv [steps_total|auto] [out.md]

With `auto` (default) the number of training steps is the call count of the optimizer kernel
(`adam_kernel`, one launch per step)."""
import csv
import sys


def main(path, steps_total="auto", out=None):
    rows = list(csv.DictReader(open(path)))
    if steps_total == "auto":
        adam = [int(r["Calls"]) for r in rows if "adam_kernel" in r["Name"]]
        steps_total = adam[0] if adam else 1
    steps_total = int(steps_total)
    lines = [f"steps in the profiled run: {steps_total}", "",
             "| kernel | calls | avg us | us/step | % |", "|---|---:|---:|---:|---:|"]
    for r in rows:
        name = r["Name"].replace("|", "/")
        if len(name) > 90:
            name = name[:87] + "..."
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                     f"{float(r['TotalDurationNs'])/1e3/steps_total:.1f} | {float(r['Percentage']):.2f} |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "auto", sys.argv[3] if len(sys.argv) > 3 else None)
