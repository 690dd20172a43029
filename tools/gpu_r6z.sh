#!/bin/bash
# end of round 6: the whole GPU suite, smoke, the default bench line, the headline kernel profile,
# the M step's PMC passes and the C4 kernel profile (large traces summarised here and deleted:
# gpurun copies back at most 64 MiB)
mkdir -p gpurun_out/r6z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6z/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z/smoke.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r6z/bench.json 2> gpurun_out/r6z/bench.err || exit 1
bash tools/prof_config.sh r6z/m --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-other-configs || exit 1
python tools/rocprof_summary.py gpurun_out/r6z/m_prof/run_kernel_stats.csv auto gpurun_out/r6z/m_kernel_stats.md > /dev/null
rm -f gpurun_out/r6z/m_prof/run_kernel_trace.csv
bash tools/pmc_bench.sh r6z/m --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-other-configs --timing eager || exit 1
find gpurun_out/r6z -name '*counter_collection.csv' -size +4M -delete
bash tools/prof_config.sh r6z/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
python tools/step_kernels.py gpurun_out/r6z/c4_prof/run_kernel_trace.csv 3 > gpurun_out/r6z/c4_step_kernels.txt
rm -f gpurun_out/r6z/c4_prof/run_kernel_trace.csv
du -sh gpurun_out/r6z
