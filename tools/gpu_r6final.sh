#!/bin/bash
# end of round 6: the whole GPU suite, smoke, the default bench line, the headline kernel profile
# and the M step's PMC passes (traffic per launch for bench.py's roofline.traffic)
mkdir -p gpurun_out/r6f
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6f/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r6f/bench.json 2> gpurun_out/r6f/bench.err || exit 1
bash tools/prof_config.sh r6f/m --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-other-configs || exit 1
bash tools/pmc_bench.sh r6f/m --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-other-configs --timing eager || exit 1
