#!/bin/bash
# A/B step time of two builds of the library: tools/ab_bench.sh <A.so> <B.so> [rounds]
# (alternating bench.py runs without the CPU baseline / PSNR legs; prints ms/step and kernel times)
set -e
A=$1; B=$2; N=${3:-3}
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for lib in "$A" "$B"; do
    out=$(SIREN_MRI_AMD_LIB=$lib timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-psnr 2>/dev/null)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['ms_per_step'],4), d['roofline']['kernel_ms_per_step'])" "$(basename $lib)" "$out"
  done
done
