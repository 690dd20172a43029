#!/bin/bash
# round 6: row-stacked tangents (C3), fused encoder epilogues (C4), C4 bf16-vs-fp32 at equal steps,
# the C3 kernel profile, c3 / c4 / c4_fp32 bench lines
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -v --timeout 300 --timeout-method thread > gpurun_out/r6b/tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --no-psnr --no-cpu-baseline > gpurun_out/r6b/c3.json 2> gpurun_out/r6b/c3.err || exit 1
timeout -k 10 300 python bench.py --config c4 --no-psnr --no-cpu-baseline > gpurun_out/r6b/c4.json 2> gpurun_out/r6b/c4.err || exit 1
bash tools/prof_config.sh r6b/c3 --config c3 --timing eager --steps 10 --warmup 3 --no-psnr --no-cpu-baseline || exit 1
bash tools/prof_config.sh r6b/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4_precision.py -v -s --timeout 880 --timeout-method thread > gpurun_out/r6b/c4_precision.txt 2>&1
timeout -k 10 400 python bench.py --config c4_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6b/c4_fp32.json 2> gpurun_out/r6b/c4_fp32.err || exit 1
