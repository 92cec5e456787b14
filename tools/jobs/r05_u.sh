#!/bin/bash
# r05u: the round-4 row-blocked wgrad under many repetitions (200 per shape): is it deterministic
# beyond the 30-run check?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r05u_race.txt
for s in "8 96 96 64 3 1" "8 96 96 64 5 1" "8 96 54 64 3 1" "16 48 48 64 5 1" "16 64 64 64 3 0" "32 64 64 64 3 0" \
         "8 128 128 32 3 0" "64 96 96 32 3 1" "64 48 48 64 3 1" "128 64 64 64 3 0"; do
  echo "== $s" >> gpurun_out/r05u_race.txt
  timeout -k 10 120 python3 -u tools/wgrad_race.py $s 200 2>&1 | grep -v amdgpu.ids | tail -n 3 >> gpurun_out/r05u_race.txt || exit $?
done
cat gpurun_out/r05u_race.txt
