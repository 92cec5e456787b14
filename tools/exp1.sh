set -e
timeout -k 10 60 python tools/gemm_micro.py --op wgrad --B 64 --cin 48 --H 64 --cout 48 --k 5 --pad 2
timeout -k 10 60 python tools/gemm_micro.py --op wgrad --B 64 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled
timeout -k 10 60 python tools/gemm_micro.py --op wgrad --B 64 --cin 64 --H 64 --cout 64 --k 3 --pad 1
timeout -k 10 60 python tools/gemm_micro.py --op wgrad --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled
