#!/bin/bash
# Effective shader clock and MFMA busy fraction of the tile-sweep GEMMs (rocprofv3 PMC pass).
#   effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md, DVFS give-back)
set -e
export TMPDIR=/tmp
rm -rf /tmp/prof_clk
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --kernel-trace -d /tmp/prof_clk -o run --output-format csv -- python3 tools/tile_sweep.py > gpurun_out/clock_probe_run.log 2>&1
C=$(find /tmp/prof_clk -name "*counter_collection.csv")
K=$(find /tmp/prof_clk -name "*kernel_trace.csv")
cp "$C" gpurun_out/clock_counters.csv
cp "$K" gpurun_out/clock_trace.csv
python3 - "$C" "$K" <<'PY'
import csv, sys, collections
cnt = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(sys.argv[1])):
    d = int(r["Dispatch_Id"]); cnt[d][r["Counter_Name"]] = cnt[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    names[d] = r["Kernel_Name"]
dur = {}
for r in csv.DictReader(open(sys.argv[2])):
    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for d in sorted(cnt):
    if "gemm" not in names[d] or d not in dur or dur[d] < 1e-4:
        continue
    c = cnt[d]
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / dur[d] / 1e9
    print(f"{names[d][:60]:60s} {dur[d]*1e6:8.1f} us  clk {clk:5.2f} GHz  mfma_busy/gui {c.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/max(1,c.get('GRBM_GUI_ACTIVE',1)):.3f}  busy_cu {c.get('SQ_BUSY_CU_CYCLES',0):.3g}")
PY
