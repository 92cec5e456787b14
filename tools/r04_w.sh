#!/bin/bash
# Round-4 GPU call: diagnosis of the progan 4-rank DP test failure (replay vs eager vs the test's loop,
# one process, with and without the fake-batch overlap).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/progan_dp_diag.py 1 > gpurun_out/r04w_diag.log 2>&1 &&
timeout -k 10 300 python3 -u tools/progan_dp_diag.py 0 >> gpurun_out/r04w_diag.log 2>&1
