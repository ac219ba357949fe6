# Radix look-back A/B (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/sort; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "sort" --timeout 120 --timeout-method thread > $O/pytest10.log 2>&1
for V in 1 0 1 0; do
  echo "== WX_RS_LB_BLOCK=$V" >> $O/lbblock.txt
  WARPDB_EXTRA_DEFINES=WX_RS_LB_BLOCK=$V timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 >> $O/lbblock.txt 2>&1
done
echo ok
