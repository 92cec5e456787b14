set -e
for a in "--B 128 --cin 64 --H 64 --cout 64 --k 3 --pad 1" "--B 128 --cin 128 --H 32 --cout 128 --k 3 --pad 1" \
         "--B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled" "--B 64 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled" \
         "--B 128 --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" "--B 128 --cin 256 --H 16 --cout 256 --k 3 --pad 1"; do
  timeout -k 10 60 python tools/gemm_micro.py --op wgrad $a --reps 10 2>&1 | grep -v amdgpu.ids
done
