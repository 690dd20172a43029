#!/bin/bash
# slab reduction with 16 loads in flight: pair / metric tests, then a one-box M A/B (old vs new lib)
mkdir -p gpurun_out/r6q
timeout -k 10 500 python -u -m pytest tests/test_gpu_metric_parity.py tests/test_gpu_fused.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6q/tests.txt 2>&1 || { tail -30 gpurun_out/r6q/tests.txt; exit 1; }
timeout -k 10 600 bash tools/ab_libs.sh 3 ablib/libA.so ablib/libB.so > gpurun_out/r6q/ab.txt 2>&1 || exit 1
tail -2 gpurun_out/r6q/tests.txt; cat gpurun_out/r6q/ab.txt
