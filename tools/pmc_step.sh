#!/bin/bash
# PMC counter groups over a short bench run (one group per rocprofv3 run), per-kernel means:
#   bash tools/pmc_step.sh TAG   -> gpurun_out/TAG_g*/ and gpurun_out/TAG_pmc.txt
R=$(pwd)
TAG=$1; shift
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
k=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"; do
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/${TAG}_g$k" -o run --output-format csv -- \
    python "$R/bench.py" --steps 5 --warmup 2 --no-psnr --no-cpu-baseline "$@" > "$R/gpurun_out/${TAG}_g$k.log" 2>&1 || echo "group $k failed"
done
cd "$R"
python - "$TAG" > "gpurun_out/${TAG}_pmc.txt" <<'PY'
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for p in glob.glob(f"gpurun_out/{tag}_g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k in sorted(acc):
    d = {c: sum(v.values()) / len(v) for c, v in acc[k].items()}
    if d.get("SQ_WAVE_CYCLES", 0) < 1e6 and d.get("WRITE_SIZE", 0) < 1e4:
        continue
    print("==", k)
    for c in sorted(d):
        print(f"   {c:34s} {d[c]:.4g}")
    if "GRBM_GUI_ACTIVE" in d:
        cyc = d["GRBM_GUI_ACTIVE"] / 8
        print(f"   kernel cycles (GUI_ACTIVE/8)       {cyc:.4g}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            print(f"   MFMA busy per SIMD / cycles        {d['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.3f}")
PY
cat "gpurun_out/${TAG}_pmc.txt"
