#!/bin/bash
# Effective shader clock and MFMA utilisation of one conv shape (tools/gemm_micro.py args), for the
# gather GEMM (GANAMD_PATCH=0) and the LDS-patch conv (GANAMD_PATCH=1), one rocprofv3 PMC pass each:
#   clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md, DVFS give-back)
#   util  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x clock)   (fp32 32x32x2: 64 cycles per MFMA)
# TF/s = 157.3 x util x clock / 2.4 GHz: a kernel below peak is either clock-held (util high) or
# issue-starved (util low).      usage: tools/clock_probe.sh TAG gemm_micro-args...
set -e
TAG=$1; shift
export TMPDIR=/tmp
for P in 0 1; do
  rm -rf /tmp/prof_clk_$TAG$P
  GANAMD_PATCH=$P timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --kernel-trace -d /tmp/prof_clk_$TAG$P -o run --output-format csv -- python3 tools/gemm_micro.py "$@" > /dev/null 2>&1
  C=$(find /tmp/prof_clk_$TAG$P -name "*counter_collection.csv")
  K=$(find /tmp/prof_clk_$TAG$P -name "*kernel_trace.csv")
  python3 - "$C" "$K" "$P" <<'PY'
import csv, sys, collections
cnt = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(sys.argv[1])):
    d = int(r["Dispatch_Id"]); cnt[d][r["Counter_Name"]] = cnt[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    names[d] = r["Kernel_Name"]
dur = {}
for r in csv.DictReader(open(sys.argv[2])):
    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
rows = []
for d in sorted(cnt):
    if not ("gemm" in names[d] or "patch" in names[d]) or d not in dur or dur[d] < 1e-4:
        continue
    c = cnt[d]
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / dur[d]
    util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * dur[d] * clk)
    rows.append((names[d][:48], dur[d] * 1e6, clk / 1e9, util))
for n, us, clk, u in rows[-3:]:
    print(f"PATCH={sys.argv[3]} {n:48s} {us:8.1f} us  clk {clk:4.2f} GHz  mfma util {u:.3f}")
PY
done
