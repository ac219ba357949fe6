#!/usr/bin/env bash
# Round 3 checkpoint: exchange / group / workload-golden GPU tests, the
# exchange kernels' own cost, the default bench line (wall time) and its
# rocprofv3 kernel stats.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r3chk
mkdir -p "$O"
PYT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_exchange.py tests/test_workload_golden.py tests/test_gpu_group_wide.py \
  tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_fuzz.py tests/test_gpu_max_sizes.py -k "group or exchange or slots or topk or workload or partitioned or fuzz or virtual" > "$O/pytest.log" 2>&1
timeout -k 10 200 python3 tools/exchange_kernels.py > "$O/exchange_kernels.txt" 2>&1
s=$(date +%s)
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"
e=$(date +%s)
echo "bench.py wall seconds: $((e - s))" > "$O/bench_wall.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_default" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_default.log" 2>&1
echo done
