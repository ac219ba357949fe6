# Radix sort tests, timing and geometry sweep (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/sort; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "sort" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 > $O/bench_sort3.txt 2>&1
WARPDB_EXTRA_DEFINES=WX_RS_DIAG_NO_LOOKBACK=1 timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 > $O/bench_sort3_nolb.txt 2>&1
for G in "256 16" "256 32" "512 8" "512 24" "1024 8"; do
  set -- $G
  echo "== block $1 items $2" >> $O/sweep.txt
  WARPDB_RS_BLOCK=$1 WARPDB_RS_ITEMS=$2 timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 >> $O/sweep.txt 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_sort.py 1e9 0 > $O/prof3.log 2>&1
echo ok
