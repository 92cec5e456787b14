set -e
for v in lds direct; do echo "kernel [$v]"; GANAMD_CONV_KERNEL=$v timeout -k 10 100 python -u tools/tile_sweep.py; done
