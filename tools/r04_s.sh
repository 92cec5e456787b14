#!/bin/bash
# Round-4 GPU call: (1) row-blocked wgrad with two 32-column blocks per wave for 3x3 convs with
# M <= 64 (tools/variants/wrow2.so = head + 1), (2) the 96-row patch conv on v_mfma_f32_16x16x32_bf16
# (8 waves, 2 along M) -- the tree's library = head + 1 + 2; A/B against tools/variants/head.so;
# kernel tests; headline bench per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r04s_ab.log
for A in "--op fwd --B 256 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 64 --cin 96 --H 64 --cout 96 --k 3 --pad 1 --scaled --reps 10" \
         "--op dgrad --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 128 --cin 64 --H 64 --cout 64 --k 3 --pad 1 --reps 10" \
         "--op wgrad --B 64 --cin 64 --H 64 --cout 64 --k 3 --pad 1 --reps 10" \
         "--op wgrad --B 128 --cin 64 --H 64 --cout 64 --k 3 --pad 1 --reps 10"; do
  for SO in tools/variants/head.so tools/variants/wrow2.so -gan-_amd/libganamd.so; do
    echo "== $SO $A" >> gpurun_out/r04s_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04s_ab.log 2>&1 || exit 1
  done
done
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_ops_gpu.py tests/test_abi.py tests/test_rng.py > gpurun_out/r04s_ops.log 2>&1 &&
STEPS=3 timeout -k 10 700 bash tools/ab_lib.sh r04s tools/variants/head.so -gan-_amd/libganamd.so tools/variants/head.so -gan-_amd/libganamd.so > /dev/null 2>&1
