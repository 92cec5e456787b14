set -e
for t in 0 128x128 128x256 256x128; do GANAMD_CONV_TILE=$t timeout -k 10 100 python -u tools/tile_sweep.py; done
for t in 0 128x256; do GANAMD_SO=$PWD/-gan-_amd/libganamd_bk32.so GANAMD_CONV_TILE=$t timeout -k 10 100 python -u tools/tile_sweep.py; done
