set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k "transpose or progan or g_forward or g_step or abi or plan" > gpurun_out/tests_convt.log 2>&1 || (tail -40 gpurun_out/tests_convt.log; exit 1)
grep -E "PASS|FAIL|passed|failed" gpurun_out/tests_convt.log | tail -30
timeout -k 10 600 python -u bench.py --config progan --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_progan.log 2>&1
tail -3 gpurun_out/bench_progan.log
