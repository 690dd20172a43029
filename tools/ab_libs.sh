#!/bin/bash
# A/B step time of several builds of the library on one box:
#   tools/ab_libs.sh ROUNDS A.so B.so [C.so ...]
# (alternating bench.py runs without the CPU baseline / PSNR legs; prints ms/step and kernel times)
set -e
N=$1; shift
for i in $(seq 1 "$N"); do
  for lib in "$@"; do
    out=$(SIREN_MRI_AMD_LIB=$lib timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-psnr 2>/dev/null)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['ms_per_step'],4), d['roofline']['kernel_ms_per_step'])" "$(basename $lib)" "$out"
  done
done
