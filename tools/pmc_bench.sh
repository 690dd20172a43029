#!/bin/bash
# PMC passes over a short bench run (separate rocprofv3 runs, counters only + kernel trace):
#   bash tools/pmc_bench.sh TAG [bench args...]   -> gpurun_out/TAG_pmc{1,2,3}/ and TAG_pmc.md
set -e
TAG=$1; shift
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d "$R/gpurun_out/${TAG}_pmc1" -o run --output-format csv -- \
    python "$R/bench.py" "$@" > "$R/gpurun_out/${TAG}_pmc1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/${TAG}_pmc2" -o run --output-format csv -- \
    python "$R/bench.py" "$@" > "$R/gpurun_out/${TAG}_pmc2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES \
    -d "$R/gpurun_out/${TAG}_pmc3" -o run --output-format csv -- \
    python "$R/bench.py" "$@" > "$R/gpurun_out/${TAG}_pmc3.log" 2>&1
cd "$R"
python tools/pmc_summary.py "$R/gpurun_out/${TAG}" "$R/gpurun_out/${TAG}_pmc.json" > "$R/gpurun_out/${TAG}_pmc.md"
