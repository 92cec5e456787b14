# The round-3 engine on the other configs: headline-batch parity module, smoke(), the lazy (config 4)
# and progan (config 5) benches.
set -e
export GANAMD_HEARTBEAT=gpurun_out/heartbeat
timeout -k 10 900 python -u -m pytest tests/test_headline_gpu.py tests/test_gan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03t_tests.log 2>&1
tail -2 gpurun_out/r03t_tests.log
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03t_smoke.log 2>&1
tail -2 gpurun_out/r03t_smoke.log
timeout -k 10 200 python3 bench.py --config lazy --steps 2 --no-extras > gpurun_out/r03t_lazy.log 2>&1
tail -1 gpurun_out/r03t_lazy.log | cut -c1-200
timeout -k 10 200 python3 bench.py --config progan --steps 3 --no-extras > gpurun_out/r03t_progan.log 2>&1
tail -1 gpurun_out/r03t_progan.log | cut -c1-200
