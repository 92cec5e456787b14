set -e
for KS in 16 32; do
 export GANAMD_CONV_KS=$KS
 timeout -k 10 60 python tools/gemm_micro.py --op fwd --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled
 timeout -k 10 60 python tools/gemm_micro.py --op fwd --B 64 --cin 128 --H 32 --cout 128 --k 3 --pad 1
 timeout -k 10 60 python tools/gemm_micro.py --op dgrad --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled
 timeout -k 10 60 python tools/gemm_micro.py --op fwd --B 64 --cin 1025 --H 4 --cout 1025 --k 3 --pad 1
 timeout -k 10 60 python tools/gemm_micro.py --op fwd --B 64 --cin 64 --H 64 --cout 64 --k 3 --pad 1
done
