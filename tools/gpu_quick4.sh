set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "models or dp or critic" > gpurun_out/tests_q.log 2>&1 || (grep -E "FAIL|Error" gpurun_out/tests_q.log | head; tail -30 gpurun_out/tests_q.log; exit 1)
tail -1 gpurun_out/tests_q.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/bench_q.log 2>&1
tail -1 gpurun_out/bench_q.log | cut -c1-250
