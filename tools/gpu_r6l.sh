#!/bin/bash
# generic-shape convolution LDS-DMA form (conv_dma 2) + pixel-Linear block counts: encoder tests,
# the C4 step's kernels, and a one-box A/B of conv_dma 1 vs 2 on C4
mkdir -p gpurun_out/r6l
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6l/enc_tests.txt 2>&1 || { tail -30 gpurun_out/r6l/enc_tests.txt; exit 1; }
bash tools/prof_config.sh r6l/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
python tools/step_kernels.py gpurun_out/r6l/c4_prof/run_kernel_trace.csv 3 > gpurun_out/r6l/c4_step_kernels.txt
rm -f gpurun_out/r6l/c4_prof/run_kernel_trace.csv
timeout -k 10 400 python -u tools/ab_option.py conv_dma 1,2,1,2 --rounds 2 --steps 60 --config c4 > gpurun_out/r6l/ab.txt 2>&1 || exit 1
tail -3 gpurun_out/r6l/enc_tests.txt; head -16 gpurun_out/r6l/c4_step_kernels.txt; cat gpurun_out/r6l/ab.txt
