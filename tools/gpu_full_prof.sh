set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1 || (grep -E "FAIL|Error|assert" gpurun_out/tests.log | head; tail -30 gpurun_out/tests.log; exit 1)
tail -1 gpurun_out/tests.log
bash tools/prof_iter.sh $1 > /dev/null
head -4 gpurun_out/$1_iteration_summary.txt
grep -E "pack_batch|split_reduce|dgrad_fold|linear" gpurun_out/$1_iteration_summary.txt | head
grep '"value"' gpurun_out/$1_bench_prof.log | cut -c1-200
