"""Summarise a rocprofv3 --kernel-trace --stats CSV into a per-step kernel table (markdown)."""
import csv
import sys


def main(path, steps_total, out=None):
    rows = list(csv.DictReader(open(path)))
    lines = ["| kernel | calls | avg us | us/step | % |", "|---|---:|---:|---:|---:|"]
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
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None)
