# round-3 session-5 final GPU batch: tests + smoke, default bench, rocprof kernel stats, PMC passes
set -e
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3s5_gpu_tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r3s5_gpu_tests.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r3s5_bench.json 2> gpurun_out/r3s5_bench.err
bash tools/profile_bench.sh r3s5 --no-other-configs --no-cpu-baseline --no-psnr --timing eager --steps 100
bash tools/pmc_bench.sh r3s5 --no-other-configs --no-cpu-baseline --no-psnr --timing eager --steps 10 --warmup 3
