set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k "bf16" > gpurun_out/tests_bf16.log 2>&1 || (tail -40 gpurun_out/tests_bf16.log; exit 1)
grep -E "PASS|FAIL|passed|failed|bf16" gpurun_out/tests_bf16.log | tail -20
timeout -k 10 600 python -u bench.py --config lazy --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_lazy.log 2>&1
tail -3 gpurun_out/bench_lazy.log | cut -c1-1500
