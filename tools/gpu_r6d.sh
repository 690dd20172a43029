#!/bin/bash
# round 6: encoder tests (residual tail forward in the conv epilogue), C4 bench, C4 bf16-vs-fp32 at
# equal steps, c4_fp32
mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -v --timeout 300 --timeout-method thread > gpurun_out/r6d/tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --no-psnr --no-cpu-baseline > gpurun_out/r6d/c4.json 2> gpurun_out/r6d/c4.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4_precision.py -v -s --timeout 880 --timeout-method thread > gpurun_out/r6d/c4_precision.txt 2>&1
timeout -k 10 400 python bench.py --config c4_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6d/c4_fp32.json 2> gpurun_out/r6d/c4_fp32.err || exit 1
