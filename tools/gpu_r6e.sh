#!/bin/bash
# round 6: fp32 hidden layers on the row-stacked tile (forward and input gradient): parity, C3 and
# m_fp32 bench lines and kernel profiles; C4 PMC passes. Large traces are summarised on the box and
# deleted (gpurun copies back at most 64 MiB).
mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest tests/test_gpu_siren_stack.py tests/test_gpu_jvp.py tests/test_gpu_metric_parity.py -v --timeout 300 --timeout-method thread > gpurun_out/r6e/tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c3 --no-psnr --no-cpu-baseline > gpurun_out/r6e/c3.json 2> gpurun_out/r6e/c3.err || exit 1
timeout -k 10 300 python bench.py --config m_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6e/m_fp32.json 2> gpurun_out/r6e/m_fp32.err || exit 1
for c in c3 m_fp32; do
  bash tools/prof_config.sh r6e/$c --config $c --timing eager --steps 10 --warmup 3 --no-psnr --no-cpu-baseline || exit 1
  python tools/step_kernels.py gpurun_out/r6e/${c}_prof/run_kernel_trace.csv 3 $([ $c = c3 ] && echo first_fwd_kernel || echo first_fwd_kernel) > gpurun_out/r6e/${c}_step_kernels.txt
  python tools/rocprof_summary.py gpurun_out/r6e/${c}_prof/run_kernel_stats.csv auto gpurun_out/r6e/${c}_kernel_stats.md > /dev/null
  rm -f gpurun_out/r6e/${c}_prof/run_kernel_trace.csv
done
bash tools/pmc_step.sh r6e/c4 --config c4 --timing eager > gpurun_out/r6e/c4_pmc.log 2>&1 || exit 1
find gpurun_out/r6e -name '*counter_collection.csv' -size +2M -delete
du -sh gpurun_out/r6e
