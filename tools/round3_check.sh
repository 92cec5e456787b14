# GPU tests of a round-3 change (FILES=...), then the headline bench with and without an env knob
# (KNOB="VAR=value" runs the bench a second time with it).
set -e
export GANAMD_HEARTBEAT=gpurun_out/heartbeat
timeout -k 10 900 python -u -m pytest ${FILES:-tests/test_critic_gpu.py tests/test_pipeline_gpu.py tests/test_models_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
tail -2 gpurun_out/r03c_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/r03c_bench.log 2>&1
grep 'ms per phase' gpurun_out/r03c_bench.log; tail -1 gpurun_out/r03c_bench.log | cut -c1-200
if [ -n "$KNOB" ]; then
  env $KNOB timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/r03c_bench_knob.log 2>&1
  grep 'ms per phase' gpurun_out/r03c_bench_knob.log; tail -1 gpurun_out/r03c_bench_knob.log | cut -c1-200
fi
