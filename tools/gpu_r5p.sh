set -uo pipefail
O=gpurun_out/r5p; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "sort or radix or order" > $O/pytest_sort.log 2>&1 || { echo pytest failed; exit 1; }
AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_SPLIT=1;WX_RS_SPLIT=1,WX_RS_LBW=4;WX_RS_SPLIT=1,WX_RS_NT_STORE=0" > $O/ab_split_keys.txt 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 300 python3 -u tools/ab_sort_rank.py 1e9 pairs 0 ";WX_RS_LBW=3" > $O/ab_pairs.txt 2>&1 || exit 1
