#!/bin/bash
# r05j: the pad mode as a template argument of the row-blocked wgrad -- determinism re-check, then
# the G-step determinism, the pipeline graph==eager tests and the DP graph tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 1 20 > gpurun_out/r05j_race.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad_deterministic or wgrad_row" > gpurun_out/r05j_wgrad.log 2>&1 &&
timeout -k 10 300 python3 -u tools/determinism.py 8 > gpurun_out/r05j_det.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py \
  tests/test_dp_gpu.py > gpurun_out/r05j_pipe_dp.log 2>&1
rc=$?
tail -3 gpurun_out/r05j_race.log; grep -E "FAILED|passed|failed" gpurun_out/r05j_wgrad.log gpurun_out/r05j_pipe_dp.log
grep "G step twice" gpurun_out/r05j_det.log
exit $rc
