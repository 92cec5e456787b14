#!/bin/bash
# One rocprofv3 kernel trace of the default bench (no extras); per-iteration breakdown of the last
# timed iteration.   usage: tools/prof_iter.sh TAG [extra bench args]
set -e
T=$1; shift
export TMPDIR=/tmp
rm -rf /tmp/prof_$T
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_$T -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1 "$@" > gpurun_out/${T}_bench_prof.log 2>&1
TR=$(find /tmp/prof_$T -name "*kernel_trace.csv")
MS=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric')][-1]['ms_per_step'])" gpurun_out/${T}_bench_prof.log)
python3 tools/trace_summary.py "$TR" --last $(python3 -c "print($MS/1000*0.98)") --top 80 > gpurun_out/${T}_iteration_summary.txt
gzip -c "$TR" > gpurun_out/${T}_trace.csv.gz
head -30 gpurun_out/${T}_iteration_summary.txt
