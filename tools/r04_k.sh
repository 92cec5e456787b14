#!/bin/bash
# Round-4 GPU call: A/B of the unrolled patch-conv tap loop (tools/variants/unroll.so) on the patch
# shapes it changes, then its kernel tests and bench.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r04k_ab.log
for A in "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 3 --pad 1 --scaled --reps 10" \
         "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 256 --cin 96 --H 32 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op dgrad --B 64 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 256 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10"; do
  for SO in -gan-_amd/libganamd.so tools/variants/unroll.so; do
    echo "== $SO $A" >> gpurun_out/r04k_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04k_ab.log 2>&1 || exit 1
  done
done
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
GANAMD_SO=$(realpath tools/variants/unroll.so) timeout -k 10 300 $T tests/test_ops_gpu.py -k "patch or split6 or modconv or conv_fwd" > gpurun_out/r04k_ops.log 2>&1 &&
GANAMD_SO=$(realpath tools/variants/unroll.so) timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.log
