set -e
for a in "--op wgrad --cin 64 --H 64 --cout 64 --k 3 --pad 1" "--op wgrad --cin 128 --H 32 --cout 128 --k 3 --pad 1" \
   "--op wgrad --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled" "--op wgrad --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" \
   "--op wgrad --cin 256 --H 16 --cout 256 --k 3 --pad 1" "--op wgrad --cin 512 --H 8 --cout 512 --k 3 --pad 1" \
   "--op fwd --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" "--op dgrad --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" \
   "--op fwd --cin 512 --H 8 --cout 512 --k 3 --pad 1" "--op dgrad --cin 256 --H 16 --cout 256 --k 3 --pad 1" \
   "--op fwd --cin 192 --H 1 --cout 192 --k 1 --pad 0" "--op fwd --cin 4100 --H 1 --cout 4100 --k 1 --pad 0"; do
   timeout -k 10 60 python tools/gemm_micro.py $a --B 128; done
