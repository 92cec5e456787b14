#!/bin/bash
# Kernel-trace profile of one timed bench iteration (graph mode by default); summaries only go to
# gpurun_out/ (the raw trace stays in /tmp).   usage: tools/profile.sh TAG [bench args...]
set -e
TAG=$1; shift
export TMPDIR=/tmp
rm -rf /tmp/prof_$TAG
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.log 2>&1
T=$(find /tmp/prof_$TAG -name "*kernel_trace.csv")
S=$(find /tmp/prof_$TAG -name "*kernel_stats.csv")
MS=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith(\"{\\\"metric\")][-1][\"ms_per_step\"])" gpurun_out/${TAG}_bench.log)
python3 tools/trace_summary.py "$T" --last $(python3 -c "print($MS/1000*0.98)") > gpurun_out/${TAG}_summary.txt
cp "$S" gpurun_out/${TAG}_kernel_stats.csv
