#!/bin/bash
# SQ stall counters of one conv GEMM (tools/gemm_micro.py args) -- where the MFMA pipe idles.
set -e
export TMPDIR=/tmp
rm -rf /tmp/prof_sq
CTRS=${SQ_COUNTERS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"}
timeout -s KILL 90 rocprofv3 --pmc $CTRS -d /tmp/prof_sq -o run --output-format csv -- python3 tools/gemm_micro.py "$@" > gpurun_out/sq_probe_run.log 2>&1
C=$(find /tmp/prof_sq -name "*counter_collection.csv")
python3 - "$C" <<'PY'
import csv, sys, collections
cnt = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
for r in csv.DictReader(open(sys.argv[1])):
    d = int(r["Dispatch_Id"]); cnt[d][r["Counter_Name"]] += float(r["Counter_Value"]); names[d] = r["Kernel_Name"]
for d in sorted(cnt)[-3:]:
    print(names[d][:70]); print({k: f"{v:.4g}" for k, v in cnt[d].items()})
PY
