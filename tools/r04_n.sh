#!/bin/bash
# Round-4 GPU call: A/B of the penalty sweeps on a second stream (bench --gp-overlap on/off), then the
# round's committed evidence (tools/round_profile.sh r04: PMC traffic, rocprofv3 stats + trace of the
# bench command, iteration breakdown, roofline-probe check, bench line with the CPU baseline).
set -o pipefail
mkdir -p gpurun_out
for O in on off on off; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-extras --gp-overlap $O >> gpurun_out/r04n_gp_ab.json 2>> gpurun_out/r04n_gp_ab.log || exit 1
done
timeout -k 10 1000 bash tools/round_profile.sh r04 > gpurun_out/r04n_profile.log 2>&1
