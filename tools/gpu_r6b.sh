#!/bin/bash
# round 6: C4 bf16-vs-fp32 at equal steps, the C3 kernel profile, c4_fp32 and the default bench line
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4_precision.py -v -s --timeout 880 --timeout-method thread > gpurun_out/r6b/c4_precision.txt 2>&1
timeout -k 10 300 python bench.py --config c3 --no-psnr --no-cpu-baseline > gpurun_out/r6b/c3.json 2> gpurun_out/r6b/c3.err || exit 1
bash tools/prof_config.sh r6b/c3 --config c3 --timing eager --steps 10 --warmup 3 --no-psnr --no-cpu-baseline || exit 1
timeout -k 10 400 python bench.py --config c4_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6b/c4_fp32.json 2> gpurun_out/r6b/c4_fp32.err || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err || exit 1
