set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "models or modconv or stylebank" > gpurun_out/tests_q.log 2>&1 || (grep -E "FAIL|Error|assert" gpurun_out/tests_q.log | head; tail -30 gpurun_out/tests_q.log; exit 1)
tail -1 gpurun_out/tests_q.log
bash tools/gpu_ab_overlap.sh
