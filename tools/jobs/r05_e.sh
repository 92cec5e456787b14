#!/bin/bash
# r05e: which round-5 default moves the 2-rank graph-mode generator gradient off the shard mean
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$(pwd)/tools/variants
T="tests/test_dp_gpu.py::test_dp_graph_iteration_matches_shard_mean"
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # tag, lib
  GANAMD_SO=$2 timeout -k 10 240 python3 -u -m pytest -x -v -s --timeout 220 --timeout-method thread "$T[overlap-8]" > gpurun_out/r05e_dp_$1.log 2>&1
  rc=$?
  grep "graph-mode DP" gpurun_out/r05e_dp_$1.log >> gpurun_out/r05e_summary.txt
  echo "$1 rc=$rc" >> gpurun_out/r05e_summary.txt
  if fatal $rc; then exit $rc; fi
}
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py > gpurun_out/r05e_pipeline.log 2>&1
rc=$?
echo "pipeline rc=$rc" >> gpurun_out/r05e_summary.txt
if fatal $rc; then exit $rc; fi
run base $(pwd)/-gan-_amd/libganamd.so
run noallk $V/noallk.so
run nowide $V/nowide.so
run nop64 $V/nop64.so
exit 0
