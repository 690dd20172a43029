# round-3 session-5 GPU batch: one-box step A/B of the epilogue forms, C4 kernel profile
set -e
R=$(pwd)
timeout -k 10 400 python tools/ab_option.py freg_magic 0,1 --rounds 3 > gpurun_out/ab_opt_magic.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/c4_prof" -o run --output-format csv -- \
    python "$R/bench.py" --config c4 --no-cpu-baseline --no-psnr --steps 5 --warmup 2 > "$R/gpurun_out/c4_prof.log" 2>&1
