#!/bin/bash
# The round's committed evidence: the bench line, a rocprofv3 kernel-trace/stats run of the SAME
# bench command (summaries only leave /tmp), the roofline-probe launches' average from that trace,
# and the PMC traffic of the probe launch.   usage: tools/round_profile.sh rNN [1|2]
# (part 1: PMC traffic + the traced bench + the probe launches; part 2: the iteration trace + the
# plain bench -- each part fits one gpurun call; no part: both)
set -e
R=$1
P=${2:-12}
export TMPDIR=/tmp
if [[ $P == *1* ]]; then
timeout -k 10 300 tools/pmc_traffic.sh > gpurun_out/${R}_pmc_traffic.log 2>&1
cp gpurun_out/roofline_traffic.json profiles/roofline_traffic.json
rm -rf /tmp/prof_$R
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_$R -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${R}_bench_prof.log 2>&1
T=$(find /tmp/prof_$R -name "*kernel_trace.csv")
S=$(find /tmp/prof_$R -name "*kernel_stats.csv")
cp "$S" gpurun_out/${R}_bench_kernel_stats.csv
gzip -c "$T" > gpurun_out/${R}_bench_trace.csv.gz
python3 tools/probe_from_trace.py "$T" > gpurun_out/${R}_roofline_probe.txt
fi
[[ $P == *2* ]] || exit 0
# the per-iteration breakdown comes from a second trace without the post-run extras (its last
# ms_per_step window is exactly the final timed iteration)
rm -rf /tmp/prof_${R}b
timeout -k 10 900 rocprofv3 --kernel-trace -d /tmp/prof_${R}b -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/${R}_bench_prof2.log 2>&1
T2=$(find /tmp/prof_${R}b -name "*kernel_trace.csv")
MS2=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric')][-1]['ms_per_step'])" gpurun_out/${R}_bench_prof2.log)
python3 tools/trace_summary.py "$T2" --last $(python3 -c "print($MS2/1000*0.98)") --top 60 > gpurun_out/${R}_iteration_summary.txt
timeout -k 10 900 python3 bench.py > gpurun_out/${R}_bench.log 2>&1
