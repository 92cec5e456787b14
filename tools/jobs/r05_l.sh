#!/bin/bash
# r05l: the round-4 row-blocked wgrad restored -- determinism re-check, G-step determinism, pipeline
# graph==eager and DP graph tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 1 30 > gpurun_out/r05l_race.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad_deterministic or wgrad_row" > gpurun_out/r05l_wgrad.log 2>&1 &&
timeout -k 10 300 python3 -u tools/determinism.py 8 > gpurun_out/r05l_det.log 2>&1 &&
timeout -k 10 700 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py \
  tests/test_dp_gpu.py > gpurun_out/r05l_pipe_dp.log 2>&1
rc=$?
tail -n 1 gpurun_out/r05l_race.log
grep -E "FAILED|passed|failed" gpurun_out/r05l_wgrad.log gpurun_out/r05l_pipe_dp.log
grep "G step twice" gpurun_out/r05l_det.log
exit $rc
