#!/bin/bash
# encoder passes with more loads in flight (pixel-Linear passes, block-sum tails), wrw_dma on:
# encoder tests, then the C4 step's kernels
mkdir -p gpurun_out/r6k
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_hyper.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6k/enc_tests.txt 2>&1 || { tail -30 gpurun_out/r6k/enc_tests.txt; exit 1; }
bash tools/prof_config.sh r6k/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
python tools/step_kernels.py gpurun_out/r6k/c4_prof/run_kernel_trace.csv 3 > gpurun_out/r6k/c4_step_kernels.txt
rm -f gpurun_out/r6k/c4_prof/run_kernel_trace.csv
tail -3 gpurun_out/r6k/enc_tests.txt; head -30 gpurun_out/r6k/c4_step_kernels.txt
