# Small conv GEMMs (the SK/SE attention convs and linears): time per launch with and without split-K.
set -e
for sk in ${SKS:-1 0}; do
  echo "GANAMD_SPLITK=$sk"
  for a in "--op fwd --B 64 --cin 192 --H 5 --cout 192 --k 3 --pad 1" "--op fwd --B 64 --cin 96 --H 5 --cout 96 --k 3 --pad 1" \
           "--op fwd --B 64 --cin 1025 --H 1 --cout 1025 --k 1 --pad 0" "--op fwd --B 64 --cin 96 --H 1 --cout 96 --k 1 --pad 0" \
           "--op fwd --B 64 --cin 4100 --H 1 --cout 4100 --k 1 --pad 0"; do
    GANAMD_SPLITK=$sk timeout -k 10 60 python tools/gemm_micro.py $a --reps 50 2>&1 | grep -v amdgpu.ids
  done
done
