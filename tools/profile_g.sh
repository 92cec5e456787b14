#!/bin/bash
set -e
export TMPDIR=/tmp
rm -rf /tmp/prof_g
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_g -o run --output-format csv -- python3 tools/g_forward_probe.py > gpurun_out/g_probe.log 2>&1
T=$(find /tmp/prof_g -name "*kernel_trace.csv")
MS=$(grep "graph replay" gpurun_out/g_probe.log | awk '{print $3}')
python3 tools/trace_summary.py "$T" --last $(python3 -c "print($MS/1000*0.98)") --top 50 > gpurun_out/g_summary.txt
