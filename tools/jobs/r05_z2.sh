#!/bin/bash
# r05z2: bisect -- the round-4 wgrad with compute(abuf, bbuf) (b_comp), with the stage store split into A and B stores (b_store)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r05z2_race.txt
for v in b_comp b_store; do
  for s in "8 96 96 64 3 1" "8 96 96 64 5 1" "32 64 64 64 3 0"; do
    echo "== $v $s" >> gpurun_out/r05z2_race.txt
    GANAMD_SO=tools/variants/$v.so timeout -k 10 120 python3 -u tools/wgrad_race.py $s 30 2>&1 | grep -v amdgpu.ids | tail -n 4 >> gpurun_out/r05z2_race.txt || exit $?
  done
done
cat gpurun_out/r05z2_race.txt
