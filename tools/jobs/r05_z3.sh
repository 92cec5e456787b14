#!/bin/bash
# r05z3: bisect -- the round-4 wgrad with the K-step load split into an A load and a B-row load taking the kernel row (b_split)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r05z3_race.txt
for v in b_split; do
  for s in "8 96 96 64 3 1" "8 96 96 64 5 1" "32 64 64 64 3 0"; do
    echo "== $v $s" >> gpurun_out/r05z3_race.txt
    GANAMD_SO=tools/variants/$v.so timeout -k 10 120 python3 -u tools/wgrad_race.py $s 30 2>&1 | grep -v amdgpu.ids | tail -n 4 >> gpurun_out/r05z3_race.txt || exit $?
  done
done
cat gpurun_out/r05z3_race.txt
