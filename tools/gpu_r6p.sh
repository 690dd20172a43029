#!/bin/bash
# hypernetwork heads' GEMM with 16-byte LDS reads: hyper + encoder tests, C4 step kernels
mkdir -p gpurun_out/r6p
timeout -k 10 400 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6p/tests.txt 2>&1 || { tail -30 gpurun_out/r6p/tests.txt; exit 1; }
bash tools/prof_config.sh r6p/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
python tools/step_kernels.py gpurun_out/r6p/c4_prof/run_kernel_trace.csv 3 > gpurun_out/r6p/c4_step_kernels.txt
rm -f gpurun_out/r6p/c4_prof/run_kernel_trace.csv
tail -3 gpurun_out/r6p/tests.txt; head -3 gpurun_out/r6p/c4_step_kernels.txt; grep hy_ gpurun_out/r6p/c4_step_kernels.txt
