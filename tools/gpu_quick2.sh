set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "pack or transpose or d_step or abi or progan" > gpurun_out/tests_q.log 2>&1 || (grep -E "FAIL|Error" gpurun_out/tests_q.log | head; tail -30 gpurun_out/tests_q.log; exit 1)
tail -1 gpurun_out/tests_q.log
bash tools/prof_iter.sh r02c > /dev/null
head -24 gpurun_out/r02c_iteration_summary.txt
grep '"value"' gpurun_out/r02c_bench_prof.log | cut -c1-200
