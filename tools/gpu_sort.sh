# Sort workload bench + look-back window A/B (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/sort; mkdir -p $O
timeout -k 10 300 python3 bench.py --workload sort > $O/bench_sort_wl.log 2>&1
for W in 1 2 4 1 2 4; do
  echo "== LBW $W" >> $O/lbw.txt
  WARPDB_EXTRA_DEFINES=WX_RS_LBW=$W timeout -k 10 300 python3 tools/bench_sort.py 1e9 0 >> $O/lbw.txt 2>&1
done
echo ok
