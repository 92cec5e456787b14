set -e
for d in . _old; do
echo "== $d"
(cd $d && for a in "--op fwd --cin 1024 --H 32 --cout 1024 --k 1 --pad 0" "--op fwd --cin 256 --H 64 --cout 256 --k 3 --pad 1" \
   "--op fwd --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled" "--op fwd --cin 64 --H 64 --cout 64 --k 3 --pad 1"; do
   timeout -k 10 60 python tools/gemm_micro.py $a --B 64; done)
done
