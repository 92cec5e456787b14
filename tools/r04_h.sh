#!/bin/bash
# Round-4 GPU call: SQ stall counters of the largest conv launches (patch conv 96/48 channels, the
# critic's 128-channel gather GEMM, the row-blocked wgrad), full GEMM census of one iteration.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r04h_sq.log
timeout -k 10 200 python -u tools/g16_map_diag.py > gpurun_out/r04h_map.log 2>&1 || exit 1
for A in "--op fwd --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 5" \
         "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 3 --pad 1 --scaled --reps 5" \
         "--op fwd --B 128 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 5" \
         "--op wgrad --B 64 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled --reps 5" \
         "--op wgrad --B 128 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 5" \
         "--op dgrad --B 128 --cin 64 --H 64 --cout 64 --k 3 --pad 1 --reps 5"; do
  echo "== $A" >> gpurun_out/r04h_sq.log
  timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04h_sq.log 2>&1 || exit 1
  timeout -k 10 120 bash tools/sq_probe.sh $A >> gpurun_out/r04h_sq.log 2>&1 || exit 1
done
GANAMD_CENSUS_OUT=gpurun_out/r04h_census.txt timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.log
