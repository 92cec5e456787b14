set -e
for r in 3 6 10 16; do echo "GANAMD_REDUCE_US=$r"; GANAMD_REDUCE_US=$r timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras 2>&1 | grep -E "phase graph|^\{" | cut -c1-160; done
