set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pb_tests.log 2>&1
tail -2 gpurun_out/pb_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline 2>&1 | grep -E '^\{|ms per phase' | cut -c1-200
