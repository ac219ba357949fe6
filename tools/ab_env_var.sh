#!/usr/bin/env bash
# A/B of one environment variable through bench.py, one process per run,
# values alternating for ROUNDS rounds (GPU box).  One line per run: value,
# kernel ms (HIP events), frac, ms per step.
#   usage: bash tools/ab_env_var.sh OUT ROUNDS VAR "BENCH ARGS" "value;value;..."
set -uo pipefail
OUT=$1; ROUNDS=$2; VAR=$3; ARGS=$4; IFS=';' read -r -a VALS <<< "$5"
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "${VALS[@]}"; do
    line=$(env "$VAR=$v" timeout -k 10 300 python3 bench.py $ARGS 2>/dev/null | grep '^{') || { echo "round $r [$VAR=$v] FAILED" >> "$OUT"; exit 1; }
    python3 - "$r" "$VAR=$v" "$line" >> "$OUT" <<'PY'
import json, sys
d = json.loads(sys.argv[3]); r = d["roofline"]
print(f"round {sys.argv[1]} [{sys.argv[2]}] kernel {r['kernel_ms']:.4f} ms frac {r['frac']:.4f} step {d['ms_per_step']:.4f} ms check {d.get('check', '')[:40]}")
PY
  done
done
cat "$OUT"
