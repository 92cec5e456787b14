#!/bin/bash
# Round-4 GPU call: (1) the split6 LDS conv body on 16x16 blocks (paired v_mfma_f32_16x16x32_bf16, 2 waves/SIMD:
# tools/variants/x3mb16.so) vs 32x32 blocks (the tree's library) on the critic's gather-GEMM shapes, (2) the
# bf16 scaled conv kernels without register spills (tree) vs tools/variants/head.so on config 4 (lazy);
# kernel tests; headline bench per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r04t_ab.log
for A in "--op fwd --B 64 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 128 --cin 256 --H 16 --cout 256 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 64 --cin 512 --H 8 --cout 512 --k 3 --pad 1 --reps 10" \
         "--op dgrad --B 64 --cin 256 --H 16 --cout 256 --k 3 --pad 1 --reps 10" \
         "--op dgrad --B 64 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 256 --cin 192 --H 16 --cout 192 --k 5 --pad 2 --scaled --reps 10"; do
  for SO in -gan-_amd/libganamd.so tools/variants/x3mb16.so; do
    echo "== $SO $A" >> gpurun_out/r04t_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04t_ab.log 2>&1 || exit 1
  done
done
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_ops_gpu.py tests/test_abi.py tests/test_rng.py > gpurun_out/r04t_ops.log 2>&1 &&
STEPS=3 timeout -k 10 700 bash tools/ab_lib.sh r04t -gan-_amd/libganamd.so tools/variants/x3mb16.so -gan-_amd/libganamd.so tools/variants/x3mb16.so > /dev/null 2>&1 &&
: > gpurun_out/r04t_lazy.txt &&
for SO in tools/variants/head.so -gan-_amd/libganamd.so; do
  echo "== $SO" >> gpurun_out/r04t_lazy.txt
  GANAMD_SO=$(realpath -- $SO) timeout -k 10 300 python3 bench.py --config lazy --steps 3 --warmup 1 --no-extras --no-cpu-baseline >> gpurun_out/r04t_lazy.txt 2>> gpurun_out/r04t_lazy.log || exit 1
done
