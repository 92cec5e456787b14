#!/bin/bash
# r05p: costed wide/narrow tile choice -- conv op tests, the wide A/B set against the narrow-only
# build, then the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py > gpurun_out/r05p_ops.log 2>&1 &&
AB_SET=wide timeout -k 10 600 python3 -u tools/ab_shapes.py ./-gan-_amd/libganamd.so tools/variants/nowide.so > gpurun_out/r05p_wide.txt 2>&1 &&
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r05p_bench.log 2>&1
rc=$?
tail -n 2 gpurun_out/r05p_ops.log; grep weighted gpurun_out/r05p_wide.txt; tail -n 1 gpurun_out/r05p_bench.log | cut -c1-200
exit $rc
