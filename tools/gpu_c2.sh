# C2 size (1e8 rows): compaction schedules (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/c2; mkdir -p $O
for S in deep static deep static; do
  echo "== $S" >> $O/sched.txt
  WARPDB_COMPACT_SCHED=$S timeout -k 10 200 python3 bench.py --rows 1e8 --steps 50 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ' >> $O/sched.txt
  echo >> $O/sched.txt
done
for R in 2e8 5e8; do
  for S in deep static; do
    echo "== $S $R" >> $O/sched.txt
    WARPDB_COMPACT_SCHED=$S timeout -k 10 200 python3 bench.py --rows $R --steps 30 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' | tr '\n' ' ' >> $O/sched.txt
    echo >> $O/sched.txt
  done
done
echo ok
