# GPU tests of the round-3 changes, the headline bench, and the 48x256-tile A/B (GANAMD_W48).
set -e
export GANAMD_HEARTBEAT=gpurun_out/heartbeat
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_critic_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1
tail -2 gpurun_out/r03b_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --steps 5 > gpurun_out/r03b_bench.log 2>&1
tail -1 gpurun_out/r03b_bench.log | cut -c1-200
GANAMD_W48=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --steps 5 > gpurun_out/r03b_bench_w48.log 2>&1
tail -1 gpurun_out/r03b_bench_w48.log | cut -c1-200
timeout -k 10 300 python3 tools/ab_shapes.py ./-gan-_amd/libganamd.so:GANAMD_W48=0 ./-gan-_amd/libganamd.so:GANAMD_W48=1 > gpurun_out/r03b_ab_w48.txt 2>&1 || true
