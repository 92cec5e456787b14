#!/bin/bash
# progan 4-rank DP test with the rounding-order-aware bar; then the full GPU suite + smoke.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dp_gpu.py -k progan > gpurun_out/r04z_dp.log 2>&1 &&
bash tools/round_final.sh
