# Partial sort tests + ORDER BY LIMIT timing (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/sort; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_warpdb_api.py -x -q -k "sort or order" --timeout 120 --timeout-method thread > $O/pytest11.log 2>&1
timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 > $O/bench11.txt 2>&1
echo ok
