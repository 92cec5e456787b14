#!/bin/bash
# PMC counters for one micro-benchmarked GEMM shape.  usage: tools/pmc.sh TAG gemm_micro-args...
set -e
TAG=$1; shift
export TMPDIR=/tmp
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  rm -rf /tmp/pmc_$TAG
  timeout -k 10 300 rocprofv3 --pmc $grp -d /tmp/pmc_$TAG -o run --output-format csv -- python3 tools/gemm_micro.py "$@" --reps 3 > /dev/null 2>&1
  F=$(find /tmp/pmc_$TAG -name "*counter_collection.csv")
  python3 - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if "gemm" not in k and "patch" not in k: continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
disp = len({r["Dispatch_Id"] for r in rows if "gemm" in r["Kernel_Name"] or "patch" in r["Kernel_Name"]})
print(" ".join(f"{k}={v / max(disp,1):.4g}" for k, v in sorted(agg.items())), f"(per dispatch, {disp} dispatches)")
PY
done
