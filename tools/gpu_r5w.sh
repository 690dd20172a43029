#!/bin/bash
# the whole GPU suite and smoke at the final tree
mkdir -p gpurun_out/r5w
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5w/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5w/smoke.txt 2>&1
