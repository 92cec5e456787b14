#!/bin/bash
# Round-4 GPU call: per-fragment LDS layouts -- kernel tests, SQ counters of the 16x16 launches, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_ops_gpu.py tests/test_abi.py > gpurun_out/r04j_ops.log 2>&1 || exit 1
: > gpurun_out/r04j_sq.log
for A in "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 3 --pad 1 --scaled --reps 5" \
         "--op wgrad --B 64 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled --reps 5" \
         "--op fwd --B 64 --cin 48 --H 16 --cout 48 --k 3 --pad 1 --scaled --reps 5"; do
  echo "== $A" >> gpurun_out/r04j_sq.log
  timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04j_sq.log 2>&1 || exit 1
  timeout -k 10 120 bash tools/sq_probe.sh $A >> gpurun_out/r04j_sq.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.log
