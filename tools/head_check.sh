# HEAD on one MI355X: the headline bench, then the GPU tests (FILES= to run a subset).
set -e
export GANAMD_HEARTBEAT=gpurun_out/heartbeat
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r03_head_bench.log 2>&1
tail -1 gpurun_out/r03_head_bench.log
timeout -k 10 1000 python -u -m pytest ${FILES:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_head_tests.log 2>&1
tail -3 gpurun_out/r03_head_tests.log
