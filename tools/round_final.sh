# Round-end check on one MI355X: GPU tests, smoke(), then the committed profile evidence.
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
tail -3 gpurun_out/final_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
tail -2 gpurun_out/final_smoke.log
bash tools/round_profile.sh r01
echo profile done
