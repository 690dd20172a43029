#!/bin/bash
# TA / TCP counters of torch's fill kernel (tools/membw_probe.py), for comparison with pmc_ta.sh
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
k=0
for grp in "TA_BUSY_avr TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
  k=$((k + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$R/gpurun_out/r2fill_pmc$k" -o run --output-format csv -- \
    python "$R/tools/membw_probe.py" > "$R/gpurun_out/r2fill_pmc$k.log" 2>&1 || echo "pass $k failed"
done
cd "$R"
python - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for p in glob.glob("gpurun_out/r2fill_pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: f"{sum(v)/len(v):.4g}" for c, v in d.items()})
PY
