#!/bin/bash
# Round-4 GPU call: kernel tests, the headline bench (full extras), the B=16 G-step diagnosis, the
# model + pipeline tests, a one-iteration kernel profile.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_ops_gpu.py tests/test_abi.py > gpurun_out/r04f_ops.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.log &&
timeout -k 10 200 python -u tools/g16_grad_diag.py gpu > gpurun_out/r04f_g16.log 2>&1 &&
timeout -k 10 400 $T tests/test_models_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r04f_models.log 2>&1 &&
timeout -k 10 300 tools/prof_iter.sh r04f > gpurun_out/r04f_prof.log 2>&1
