#!/bin/bash
# Round-4 (re-entry) first GPU call: every kernel test (incl. the split6 LDS-patch conv and the
# row-blocked wgrad, never yet run on hardware; route / modconv_sd_bwd), the model + pipeline tests.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_ops_gpu.py tests/test_abi.py > gpurun_out/r04d_ops.log 2>&1 &&
timeout -k 10 500 $T tests/test_models_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r04d_models.log 2>&1
