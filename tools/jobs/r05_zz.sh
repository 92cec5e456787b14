#!/bin/bash
# r05zz: the all-kernel-rows wgrad with by-value loaders (variant): determinism (race tool + the
# pytest determinism gates under GANAMD_SO) and the wgrad A/B against the in-tree round-4 kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=tools/variants/allk_byval.so
: > gpurun_out/r05zz_race.txt
for s in "8 96 96 64 3 1" "8 96 96 64 5 1" "8 96 54 64 3 1" "32 64 64 64 3 0" "128 64 64 64 3 0" "16 48 48 64 5 1"; do
  echo "== $s" >> gpurun_out/r05zz_race.txt
  GANAMD_SO=$L timeout -k 10 120 python3 -u tools/wgrad_race.py $s 50 2>&1 | grep -v amdgpu.ids | tail -n 1 >> gpurun_out/r05zz_race.txt || exit $?
done
GANAMD_SO=$L timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "deterministic or wgrad_row or split6" > gpurun_out/r05zz_tests.log 2>&1 || { tail -n 5 gpurun_out/r05zz_tests.log; exit 1; }
AB_SET=wgrad timeout -k 10 400 python3 -u tools/ab_shapes.py ./-gan-_amd/libganamd.so $L > gpurun_out/r05zz_ab.txt 2>&1
cat gpurun_out/r05zz_race.txt; tail -n 1 gpurun_out/r05zz_tests.log; grep weighted gpurun_out/r05zz_ab.txt
