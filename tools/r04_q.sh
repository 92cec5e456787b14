#!/bin/bash
# Round-4 GPU call: (1) patch conv B-fragment look-ahead and (2) unconditional conv-GEMM prefetch
# loads -- A/B of tools/variants/base.so (before both), x3ld.so (2 only) and the tree's library (both)
# on patch and gather-GEMM shapes; kernel tests; headline bench per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r04q_ab.log
for A in "--op fwd --B 256 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 3 --pad 1 --scaled --reps 10" \
         "--op dgrad --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 64 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 64 --cin 256 --H 16 --cout 256 --k 3 --pad 1 --reps 10" \
         "--op dgrad --B 64 --cin 256 --H 16 --cout 256 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 256 --cin 192 --H 16 --cout 192 --k 5 --pad 2 --scaled --reps 10"; do
  for SO in tools/variants/base.so tools/variants/x3ld.so -gan-_amd/libganamd.so; do
    echo "== $SO $A" >> gpurun_out/r04q_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04q_ab.log 2>&1 || exit 1
  done
done
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_ops_gpu.py tests/test_abi.py > gpurun_out/r04q_ops.log 2>&1 &&
STEPS=3 timeout -k 10 700 bash tools/ab_lib.sh r04q tools/variants/base.so -gan-_amd/libganamd.so tools/variants/base.so -gan-_amd/libganamd.so > /dev/null 2>&1
