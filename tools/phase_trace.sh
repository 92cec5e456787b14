#!/bin/bash
# Kernel-time breakdown of ONE eager generator step and ONE critic step at the bench batch
# (tools/gen_step_trace.py under rocprofv3 --kernel-trace; tools/trace_summary.py over the traced
# step's window).   usage: tools/phase_trace.sh TAG   -> gpurun_out/TAG_{gen,critic}_summary.txt
set -e
export TMPDIR=/tmp
TAG=$1
for PH in gen critic; do
  rm -rf /tmp/ptr_$PH
  PHASE=$PH timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ptr_$PH -o run --output-format csv -- python3 tools/gen_step_trace.py > gpurun_out/${TAG}_${PH}_trace.log 2>&1
  T=$(find /tmp/ptr_$PH -name "*kernel_trace.csv")
  S=$(grep -o 'step [0-9.]*' gpurun_out/${TAG}_${PH}_trace.log | awk '{print $2}')
  python3 tools/trace_summary.py "$T" --last $S --top 60 > gpurun_out/${TAG}_${PH}_summary.txt
done
