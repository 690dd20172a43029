# rocprofv3 kernel trace + stats of one bench config: bash tools/prof_config.sh TAG bench-args...
set -e
TAG=$1; shift
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run --output-format csv -- \
    python "$R/bench.py" "$@" > "$R/gpurun_out/${TAG}_prof.log" 2>&1
