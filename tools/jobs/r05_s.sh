#!/bin/bash
# r05s: a root block's shortcut StyleBlock as a fifth branch beside rir_3 -- generator tests, then
# bench A/B (GANAMD_SHORTCUT_BRANCH=1 / 0, alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py \
  tests/test_headline_gpu.py tests/test_models_gpu.py > gpurun_out/r05s_tests.log 2>&1 || exit $?
: > gpurun_out/r05s_ab.txt
for v in 1 0 1 0; do
  GANAMD_SHORTCUT_BRANCH=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r05s_b.log 2>&1 || exit $?
  echo "branch=$v $(grep -o 'ms per phase graph: .*' gpurun_out/r05s_b.log) $(grep '^{"metric' gpurun_out/r05s_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/r05s_ab.txt
done
cat gpurun_out/r05s_ab.txt
