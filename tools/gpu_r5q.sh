set -uo pipefail
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "sort or radix or order" > $O/pytest_sort.log 2>&1 || { echo pytest failed; exit 1; }
AB_ROUNDS=3 timeout -k 10 400 python3 -u tools/ab_sort_rank.py 1e9 keys 0 ";WX_RS_SPLIT=0;WX_RS_SPLIT=0,WX_RS_NT_STORE=1;WX_RS_NT_STORE=1" > $O/ab_split_store.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/bench_sort.py 1e8,1e9 0 > $O/sort_sizes.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_sort -o run --output-format csv -- python3 $R/bench.py --workload sort --steps 5 --no-cpu-baseline > $R/$O/sort.json 2> $R/$O/sort.err || exit 1
cd $R && bash tools/pmc_run.sh sort 1e9 "" sort5 > $O/pmc_sort.log 2>&1
