#!/bin/bash
# Round-4 GPU call: the penalty sweeps on a second stream -- critic / pipeline / DP / headline tests, bench.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 500 $T tests/test_models_gpu.py tests/test_pipeline_gpu.py tests/test_critic_gpu.py > gpurun_out/r04l_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.log
