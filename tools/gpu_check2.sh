set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1 || (tail -40 gpurun_out/tests.log; exit 1)
tail -2 gpurun_out/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
tail -6 gpurun_out/bench.log
