#!/bin/bash
# r05d: the whole GPU suite at the round-5 defaults (64-row patch tile, wide critic tiles, all-rows
# 3x3 wgrad for 64 channels, sized-workspace ABI), then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GANAMD_HEARTBEAT=gpurun_out/r05d_heartbeat
timeout -k 10 1080 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05d_tests.log 2>&1 &&
timeout -k 10 100 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05d_smoke.log 2>&1
