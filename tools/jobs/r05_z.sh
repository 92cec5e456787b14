#!/bin/bash
# r05z: bisect -- the round-4 wgrad with only the KStep struct of the rewrite (b_kstep), with only the rewrite's accumulator shape acc[1][TN][KK] (b_acc)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r05z_race.txt
for v in b_kstep b_acc; do
  for s in "8 96 96 64 3 1" "8 96 96 64 5 1" "32 64 64 64 3 0"; do
    echo "== $v $s" >> gpurun_out/r05z_race.txt
    GANAMD_SO=tools/variants/$v.so timeout -k 10 120 python3 -u tools/wgrad_race.py $s 30 2>&1 | grep -v amdgpu.ids | tail -n 4 >> gpurun_out/r05z_race.txt || exit $?
  done
done
cat gpurun_out/r05z_race.txt
