#!/bin/bash
# Round-4 GPU call: fake-batch group schedules at B = 64 (bench --fake-groups), configs 4 and 5 at the
# final build, then the round's committed evidence (tools/round_profile.sh r04).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r04v_groups.txt
for FG in 4,1 3,2 4,1 3,2; do
  echo "== --fake-groups $FG" >> gpurun_out/r04v_groups.txt
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --fake-groups $FG >> gpurun_out/r04v_groups.txt 2>> gpurun_out/r04v_groups.log || exit 1
done
timeout -k 10 300 python3 bench.py --config lazy --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04v_lazy.json 2> gpurun_out/r04v_lazy.log &&
timeout -k 10 300 python3 bench.py --config progan --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04v_progan.json 2> gpurun_out/r04v_progan.log &&
timeout -k 10 1000 bash tools/round_profile.sh r04 > gpurun_out/r04v_profile.log 2>&1
