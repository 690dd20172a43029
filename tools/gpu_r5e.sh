#!/bin/bash
# PMC traffic passes (M and the 1/8 shard), the shard's kernel stats, and the default bench line
set -e
mkdir -p gpurun_out/r5e
bash tools/pmc_bench.sh r5e/m --steps 10 --warmup 3 --no-psnr --no-cpu-baseline --no-other-configs
bash tools/pmc_bench.sh r5e/s8 --config m_shard8 --steps 10 --warmup 3 --no-psnr --no-cpu-baseline --no-other-configs
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5e/s8prof" -o run --output-format csv -- \
  python "$R/bench.py" --config m_shard8 --steps 50 --warmup 10 --no-psnr --no-cpu-baseline --no-other-configs \
  > "$R/gpurun_out/r5e/s8prof.json" 2> "$R/gpurun_out/r5e/s8prof.err"
cd "$R"
timeout -k 10 600 python bench.py > gpurun_out/r5e/bench.json 2> gpurun_out/r5e/bench.err
