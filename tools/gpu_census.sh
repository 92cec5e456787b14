set -e
GANAMD_CENSUS_OUT=gpurun_out/census_full.txt timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_census.log 2>&1
head -5 gpurun_out/census_full.txt
