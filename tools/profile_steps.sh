#!/bin/bash
# Kernel-trace profile of one critic-step graph and one generator-step graph (B=64), each
# summarised over its last replay (tools/trace_summary.py).  usage: tools/profile_steps.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-steps}
for W in ${STEPS:-critic generator}; do
  rm -rf /tmp/prof_$W
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_$W -o run --output-format csv -- python3 tools/step_probe.py $W > gpurun_out/${TAG}_${W}_probe.log 2>&1
  T=$(find /tmp/prof_$W -name "*kernel_trace.csv")
  MS=$(grep "graph replay" gpurun_out/${TAG}_${W}_probe.log | awk '{print $5}')
  python3 tools/trace_summary.py "$T" --last $(python3 -c "print($MS/1000*0.98)") --top 70 > gpurun_out/${TAG}_${W}_summary.txt
  head -3 gpurun_out/${TAG}_${W}_summary.txt
done
