#!/usr/bin/env bash
# The one GPU-session runner (GPU box).  Usage:
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
# Every step runs under its own time limit, writes under gpurun_out/TAG/ and
# stops the session on failure (set -e); steps:
#   smoke                      __graft_entry__.smoke()
#   suite[:PYTEST ARGS]        pytest -m gpu (--durations=25), e.g. suite:-k group
#   pytest:NAME:FILES          pytest FILES -m gpu -v > NAME.log
#   bench:NAME[:BENCH ARGS]    python3 bench.py ARGS > NAME.json
#   prof:NAME[:BENCH ARGS]     the same bench under rocprofv3 --kernel-trace --stats
#                              (NAME_kernel_stats.csv is the summary to keep)
#   pmc:NAME[:BENCH ARGS]      FETCH_SIZE and WRITE_SIZE passes (one counter block
#                              each) over 3 steps, summarised to NAME_pmc.json and
#                              recorded in profiles/pmc_<workload>.json (copied
#                              under gpurun_out/TAG/: copy it back into profiles/)
#   sq:NAME[:BENCH ARGS]       SQ wave-cycle accounting (WAIT_ANY / WAIT_INST_ANY /
#                              ACTIVE_INST_ANY / LDS counters) in one pass, NAME_sq.json
#   py:NAME:SCRIPT [ARGS]      python3 SCRIPT ARGS > NAME.txt
#   pyprof:NAME:SCRIPT [ARGS]  the same under rocprofv3 --kernel-trace --stats
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for STEP in "$@"; do
  KIND=${STEP%%:*}
  REST=""
  [[ "$STEP" == *:* ]] && REST=${STEP#*:}
  NAME=${REST%%:*}
  ARGS=""
  [[ "$REST" == *:* ]] && ARGS=${REST#*:}
  echo "[$(date +%T)] $STEP" | tee -a "$O/steps.log"
  case "$KIND" in
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    suite)
      # shellcheck disable=SC2086
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        --durations=25 $REST > "$O/pytest_gpu.log" 2>&1 ;;
    pytest)
      # shellcheck disable=SC2086
      timeout -k 10 900 python3 -u -m pytest $ARGS -m gpu -x -v --timeout 300 --timeout-method thread \
        --durations=15 > "$O/$NAME.log" 2>&1 ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 400 python3 bench.py $ARGS > "$O/$NAME.json" 2> "$O/$NAME.err" ;;
    prof)
      # shellcheck disable=SC2086
      (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/prof_$NAME" -o run --output-format csv \
        -- python3 "$R/bench.py" $ARGS > "$O/$NAME.json" 2> "$O/$NAME.err")
      S=$(find "$O/prof_$NAME" -name "*kernel_stats.csv" | head -n 1 || true)
      if [ -n "$S" ]; then cp "$S" "$O/${NAME}_kernel_stats.csv"; fi ;;
    pmc)
      mkdir -p "$O/pmc_$NAME"
      for C in FETCH_SIZE WRITE_SIZE; do
        # shellcheck disable=SC2086
        (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C -d "$O/pmc_$NAME/$C" -o run --output-format csv -- \
          python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-secondary $ARGS \
          > "$O/pmc_$NAME/$C.log" 2>&1)
      done
      python3 tools/pmc_summary.py $(find "$O/pmc_$NAME" -name "*counter_collection.csv") > "$O/${NAME}_pmc.json"
      # the tracked profiles/pmc_<workload>.json bench.py reads (date + kernel-source sha)
      PW=$(echo " $ARGS " | sed -n 's/.* --workload \([a-z_]*\) .*/\1/p')
      PW=${PW:-project}
      [[ "$PW" == group && "$ARGS" == *--keys* ]] && PW=group_wide
      PR=$(echo " $ARGS " | sed -n 's/.* --rows \([0-9.e]*\) .*/\1/p')
      python3 tools/pmc_record.py "$PW" "${PR:-1e9}" "$O/${NAME}_pmc.json" "gpu_run.sh $TAG/$NAME"
      cp "profiles/pmc_$PW.json" "$O/" ;;
    sq)
      # wave-cycle accounting of the bench's kernels in one pass (8 SQ slots + 1 GRBM):
      # WAIT_ANY (parked: s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) +
      # ACTIVE_INST_ANY ~= WAVE_CYCLES; summarised per kernel to NAME_sq.json
      mkdir -p "$O/sq_$NAME"
      # shellcheck disable=SC2086
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        -d "$O/sq_$NAME" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-secondary $ARGS \
        > "$O/sq_$NAME/run.log" 2>&1)
      python3 tools/pmc_summary.py $(find "$O/sq_$NAME" -name "*counter_collection.csv") > "$O/${NAME}_sq.json" ;;
    pyprof)
      # the script under rocprofv3 --kernel-trace --stats (NAME_kernel_stats.csv, prof_NAME/)
      SCRIPT=${ARGS%% *}
      SARGS=""
      [[ "$ARGS" == *" "* ]] && SARGS=${ARGS#* }
      # shellcheck disable=SC2086
      (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/prof_$NAME" -o run --output-format csv \
        -- python3 "$R/$SCRIPT" $SARGS > "$O/$NAME.txt" 2>&1)
      S=$(find "$O/prof_$NAME" -name "*kernel_stats.csv" | head -n 1 || true)
      if [ -n "$S" ]; then cp "$S" "$O/${NAME}_kernel_stats.csv"; fi ;;
    py)
      SCRIPT=${ARGS%% *}
      SARGS=""
      [[ "$ARGS" == *" "* ]] && SARGS=${ARGS#* }
      # shellcheck disable=SC2086
      timeout -k 10 400 python3 "$SCRIPT" $SARGS > "$O/$NAME.txt" 2>&1 ;;
    *)
      echo "unknown step $STEP" >&2
      exit 2 ;;
  esac
done
echo "[$(date +%T)] done" | tee -a "$O/steps.log"
