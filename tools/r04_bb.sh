#!/bin/bash
# Round-4 GPU call: conv GEMM kernels at 2 waves/SIMD (tools/variants/wpe2.so: amdgpu_waves_per_eu 2 -- the
# 32x32x16 form's measured ceiling is 236 split6 TF/s at 2 waves/SIMD against 202 at 3) vs the tree's 3.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r04bb_ab.log
for A in "--op fwd --B 96 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 128 --cin 256 --H 16 --cout 256 --k 3 --pad 1 --reps 10" \
         "--op dgrad --B 64 --cin 256 --H 16 --cout 256 --k 3 --pad 1 --reps 10" \
         "--op fwd --B 256 --cin 192 --H 16 --cout 192 --k 5 --pad 2 --scaled --reps 10"; do
  for SO in -gan-_amd/libganamd.so tools/variants/wpe2.so; do
    echo "== $SO $A" >> gpurun_out/r04bb_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04bb_ab.log 2>&1 || exit 1
  done
done
STEPS=3 timeout -k 10 700 bash tools/ab_lib.sh r04bb -gan-_amd/libganamd.so tools/variants/wpe2.so -gan-_amd/libganamd.so tools/variants/wpe2.so > /dev/null 2>&1
