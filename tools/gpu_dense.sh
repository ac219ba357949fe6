# Dense projection + compaction store ablations (GPU box).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "dense or compact" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 tools/ablate_compact.py 1e9 7 deep,deep_ntst,deep_nolookback,deep_nostore > $O/ablate_compact.txt 2>&1
ABL_GRIDS=1,2,4 ABL_UNROLLS=8 timeout -k 10 300 python3 tools/ablate_stream.py 1e9 dense > $O/ablate_dense.txt 2>&1
timeout -k 10 300 python3 bench.py --workload dense > $O/bench_dense.log 2>&1
timeout -k 10 300 python3 bench.py --workload project --rows 1e8 --cpu-sample 2e7 > $O/bench_project_1e8.log 2>&1
echo ok
