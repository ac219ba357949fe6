set -uo pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "sort or radix or order" > $O/pytest_sort.log 2>&1 || { echo pytest failed; exit 1; }
AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_LB_LANES=1;WX_RS_LBW=2;WX_RS_LBW=4" > $O/ab_lanes_keys.txt 2>&1 || exit 1
AB_ROUNDS=3 timeout -k 10 300 python3 -u tools/ab_sort_rank.py 1e9 pairs 0 ";WX_RS_LB_LANES=1" > $O/ab_lanes_pairs.txt 2>&1 || exit 1
AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_SPLIT=1;WARPDB_RS_LEAD=auto" > $O/ab_split_lead.txt 2>&1 || exit 1
bash tools/ab_env_bench.sh $O/ab_compact_dw.txt 2 "--workload project --no-secondary --no-cpu-baseline --steps 40" ";WX_COMPACT_DWAVES=11;WX_COMPACT_DWAVES=10" > /dev/null || exit 1
