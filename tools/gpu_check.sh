# GPU tests (all, or a -k filter) + smoke + a short bench; stops at the first failure.
set -e
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -k "$K" > gpurun_out/tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1
fi
tail -3 gpurun_out/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
tail -8 gpurun_out/bench.log
