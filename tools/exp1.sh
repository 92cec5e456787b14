# wgrad split-K target sweep
set -e
for T in 1024 2048 4096; do
 export GANAMD_WGRAD_BLOCKS=$T
 for a in "--op wgrad --cin 64 --H 64 --cout 64 --k 3 --pad 1" "--op wgrad --cin 128 --H 32 --cout 128 --k 3 --pad 1" \
   "--op wgrad --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled" "--op wgrad --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" \
   "--op wgrad --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled" "--op wgrad --cin 512 --H 8 --cout 512 --k 3 --pad 1" \
   "--op wgrad --cin 3 --H 64 --cout 48 --k 3 --pad 1"; do
   timeout -k 10 60 python tools/gemm_micro.py $a --B 64; done
done
