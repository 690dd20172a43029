#!/bin/bash
# full GPU suite, then the r3-vs-HEAD one-box A/B of the M step
mkdir -p gpurun_out/r5d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5d/gpu_tests.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/r5d/gpu_tests.txt
bash tools/ab_tree.sh r5d/ab build/r3copy 2 > /dev/null 2>&1 || exit 1
for i in 1 2; do for v in d0 vmn26 d4 d4_vmn2 d32 nt sc1 all; do echo "== $v"; timeout -k 5 60 build/fwd_f0_$v 200 || exit 1; done; done > gpurun_out/r5d/fwd_var.txt 2>&1
