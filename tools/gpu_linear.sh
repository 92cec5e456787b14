set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1 || (grep -E "FAIL|Error|error" gpurun_out/tests.log | head -20; tail -30 gpurun_out/tests.log; exit 1)
tail -2 gpurun_out/tests.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1
grep "ms per phase" gpurun_out/bench.log; tail -1 gpurun_out/bench.log | cut -c1-400
