#!/bin/bash
# r05h: wgrad determinism, the round-5 row-blocked kernel vs the round-4 one (variant build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base wrow_r04; do
  lib=""; [ $v != base ] && lib=tools/variants/$v.so
  GANAMD_SO=$lib timeout -k 10 200 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
    -k "wgrad_deterministic" > gpurun_out/r05h_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "FAILED|^E .*Assert" gpurun_out/r05h_$v.log | cut -c1-160
  [ $rc -gt 1 ] && exit $rc
done
exit 0
