#!/bin/bash
# last check of the final tree: the whole GPU suite and smoke
mkdir -p gpurun_out/r6t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6t/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r6t/gpu_tests.txt; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6t/smoke.txt 2>&1 || exit 1
tail -2 gpurun_out/r6t/gpu_tests.txt; tail -1 gpurun_out/r6t/smoke.txt
