# A/B of GEMM shapes between the current tree and ./_old (a git worktree, possibly built with other flags)
set -e
for d in . _old; do
 echo "== $d"
 (cd $d && for a in "--op fwd --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled" "--op fwd --cin 128 --H 32 --cout 128 --k 3 --pad 1" \
   "--op dgrad --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled" "--op fwd --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" \
   "--op dgrad --cin 1025 --H 4 --cout 1025 --k 3 --pad 1" "--op fwd --cin 64 --H 64 --cout 64 --k 3 --pad 1" \
   "--op dgrad --cin 64 --H 64 --cout 64 --k 3 --pad 1" "--op dgrad --cin 256 --H 16 --cout 256 --k 3 --pad 1" \
   "--op fwd --cin 192 --H 1 --cout 192 --k 1 --pad 0" "--op dgrad --cin 512 --H 16 --cout 512 --k 3 --stride 2 --pad 1"; do
   timeout -k 10 60 python tools/gemm_micro.py $a --B 64; done)
done
