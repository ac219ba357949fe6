# Full GPU tests + radix sort timing and kernel profile (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/sort; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest8.log 2>&1
timeout -k 10 300 python3 tools/bench_sort.py 1e8,1e9 0 > $O/bench8.txt 2>&1
timeout -k 10 200 ./tools/rocprim_sort_bench 1e9 >> $O/bench8.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_sort.py 1e9 0 > $O/prof8.log 2>&1
echo ok
