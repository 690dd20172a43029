#!/bin/bash
# One-box A/B of two source trees' M step (the same bench command, rocprofv3 kernel stats each),
# run alternately: bash tools/ab_tree.sh TAG OTHER_TREE [rounds]
#   -> gpurun_out/TAG_{head,other}_<i>/run_kernel_stats.csv and TAG_summary.txt
set -e
TAG=$1; OTHER=$2; N=${3:-2}
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 "$N"); do
  for side in head other; do
    T=$R; [ "$side" = other ] && T=$R/$OTHER
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_${side}_$i" -o run --output-format csv -- \
      python "$T/bench.py" --steps 50 --warmup 10 --no-psnr --no-cpu-baseline --no-other-configs \
      > "$R/gpurun_out/${TAG}_${side}_$i.json" 2> "$R/gpurun_out/${TAG}_${side}_$i.err"
  done
done
cd "$R"
python - "$R/gpurun_out/$TAG" "$N" > "$R/gpurun_out/${TAG}_summary.txt" <<'PY'
import csv, glob, json, sys
tag, n = sys.argv[1], int(sys.argv[2])
for i in range(1, n + 1):
    for side in ("head", "other"):
        d = f"{tag}_{side}_{i}"
        ms = json.load(open(d + ".json"))["ms_per_step"]
        rows = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0])))
        top = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]
        print(f"{side} {i}: {ms:.4f} ms/step")
        for r in top:
            print(f"   {float(r['AverageNs'])/1e3:8.1f} us  x{r['Calls']:>5}  {r['Name'][:80]}")
PY
cat "$R/gpurun_out/${TAG}_summary.txt"
