#!/bin/bash
# r05f: run-to-run determinism of the generator step (B=8) under four configurations
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/determinism.py 8 > gpurun_out/r05f_det.log 2>&1
