# Radix sort tests + timing + profile (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/sort; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_warpdb_api.py -x -q -k "sort or order" --timeout 120 --timeout-method thread > $O/pytest9.log 2>&1
timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 > $O/bench9.txt 2>&1
WARPDB_EXTRA_DEFINES=WX_RS_HUNROLL=8 timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 >> $O/bench9.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof9 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_sort.py 1e9 0 > $O/prof9.log 2>&1
echo ok
