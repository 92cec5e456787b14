# Round-end check on one MI355X: the whole GPU suite, then smoke().  (The committed profile evidence,
# tools/round_profile.sh rNN, is a separate call: together they exceed one call's time limit.)
set -e
export GANAMD_HEARTBEAT=gpurun_out/heartbeat
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
tail -3 gpurun_out/final_tests.log
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
tail -2 gpurun_out/final_smoke.log
