#!/bin/bash
# r05k: row-blocked wgrad with the vmcnt drain before its LDS stores vs without it (variant)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 1 30 > gpurun_out/r05k_race.log 2>&1 &&
GANAMD_SO=tools/variants/novmwait.so timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 1 30 > gpurun_out/r05k_race_novm.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad_deterministic or wgrad_row" > gpurun_out/r05k_wgrad.log 2>&1 &&
timeout -k 10 300 python3 -u tools/determinism.py 8 > gpurun_out/r05k_det.log 2>&1
rc=$?
tail -1 gpurun_out/r05k_race.log gpurun_out/r05k_race_novm.log; grep -E "FAILED|passed|failed" gpurun_out/r05k_wgrad.log
grep "G step twice" gpurun_out/r05k_det.log
exit $rc
