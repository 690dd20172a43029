#!/bin/bash
# full GPU suite, then the default bench with its kernel profile
mkdir -p gpurun_out/r5o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5o/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r5o/bench.json 2> gpurun_out/r5o/bench.err
