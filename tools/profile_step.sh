#!/bin/bash
# usage: tools/profile_step.sh critic|generator
set -e
W=$1
export TMPDIR=/tmp
rm -rf /tmp/prof_$W
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$W -o run --output-format csv -- python3 tools/step_probe.py $W > gpurun_out/${W}_probe.log 2>&1
T=$(find /tmp/prof_$W -name "*kernel_trace.csv")
MS=$(grep "graph replay" gpurun_out/${W}_probe.log | awk '{print $5}')
python3 tools/trace_summary.py "$T" --last $(python3 -c "print($MS/1000*0.98)") --top 60 > gpurun_out/${W}_summary.txt
