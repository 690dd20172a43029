#!/bin/bash
# Usage (on the GPU box, from the repo root): bash tools/profile_bench.sh TAG [bench args...]
# 1) plain bench line -> gpurun_out/TAG_bench.json
# 2) rocprofv3 kernel trace + stats of the same command -> gpurun_out/TAG_prof/
set -e
TAG=$1; shift
R=$(pwd)
mkdir -p "$R/gpurun_out"
timeout -k 10 300 python bench.py "$@" > "$R/gpurun_out/${TAG}_bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run --output-format csv -- \
    python "$R/bench.py" "$@" > "$R/gpurun_out/${TAG}_prof.log" 2>&1
cd "$R"
STATS=$(find "$R/gpurun_out/${TAG}_prof" -name 'run_kernel_stats.csv' | head -1)
cp "$STATS" "$R/gpurun_out/${TAG}_kernel_stats.csv"
python tools/rocprof_summary.py "$STATS" auto "$R/gpurun_out/${TAG}_summary.md" > /dev/null
