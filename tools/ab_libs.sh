#!/bin/bash
# A/B step time of several builds of the library on one box:
#   tools/ab_libs.sh ROUNDS A.so B.so [C.so ...]
# (bench.py runs without the CPU baseline / PSNR legs; prints ms/step and kernel times). Rounds
# alternate the library order (A B .. then .. B A): a run's clock depends on what the GPU ran just
# before it (measured: the same code object 106 vs 131 us per forward after different predecessors)
set -e
N=$1; shift
libs=("$@")
for i in $(seq 1 "$N"); do
  if (( i % 2 == 0 )); then order=$(printf '%s\n' "${libs[@]}" | tac); else order=$(printf '%s\n' "${libs[@]}"); fi
  for lib in $order; do
    sleep 3
    out=$(SIREN_MRI_AMD_LIB=$lib timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-psnr --no-other-configs --timing eager 2>/dev/null)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['ms_per_step'],4), d['roofline']['kernel_ms_per_step'])" "$(basename $lib)" "$out"
  done
done
