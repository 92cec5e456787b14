# SQ counter diagnosis of the probe conv launch at 3 waves/SIMD (default) and 2 (LDS padding)
set -e
export TMPDIR=/tmp
ARGS="--op fwd --B 96 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 5"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
for pad in 0 28672; do
  rm -rf /tmp/sq_$pad
  GANAMD_CONV_LDS_PAD=$pad timeout -s KILL 120 rocprofv3 --pmc $C -d /tmp/sq_$pad -o run --output-format csv -- python3 tools/gemm_micro.py $ARGS > gpurun_out/sq_$pad.log 2>&1
  python3 - $pad <<'PY'
import csv, glob, collections, sys
f = glob.glob(f"/tmp/sq_{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "conv_gemm_kernel" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
last = list(per.values())[-1]
print("pad", sys.argv[1], {k: f"{v:.3e}" for k, v in sorted(last.items())})
PY
done
