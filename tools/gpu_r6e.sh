#!/bin/bash
# round 6: fp32 hidden layers on the row-stacked tile (forward and input gradient): parity, C3 and
# m_fp32 bench lines and kernel profiles
mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest tests/test_gpu_siren_stack.py tests/test_gpu_jvp.py tests/test_gpu_metric_parity.py -v --timeout 300 --timeout-method thread > gpurun_out/r6e/tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --no-psnr --no-cpu-baseline > gpurun_out/r6e/c3.json 2> gpurun_out/r6e/c3.err || exit 1
timeout -k 10 300 python bench.py --config m_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6e/m_fp32.json 2> gpurun_out/r6e/m_fp32.err || exit 1
bash tools/prof_config.sh r6e/c3 --config c3 --timing eager --steps 10 --warmup 3 --no-psnr --no-cpu-baseline || exit 1
bash tools/prof_config.sh r6e/m_fp32 --config m_fp32 --timing eager --steps 10 --warmup 3 --no-psnr --no-cpu-baseline || exit 1
