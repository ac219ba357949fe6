#!/usr/bin/env bash
# A/B of WARPDB_EXTRA_DEFINES variants through bench.py, one process per run,
# variants alternating for ROUNDS rounds (GPU box).  Prints one line per run:
# variant, kernel ms (HIP events), frac, ms per step.
#   usage: bash tools/ab_env_bench.sh OUT ROUNDS "BENCH ARGS" "variant;variant;..."
set -uo pipefail
OUT=$1; ROUNDS=$2; ARGS=$3; IFS=';' read -r -a VARS <<< "$4"
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "${VARS[@]}"; do
    line=$(WARPDB_EXTRA_DEFINES="$v" timeout -k 10 300 python3 bench.py $ARGS 2>/dev/null | grep '^{') || { echo "round $r [$v] FAILED" >> "$OUT"; exit 1; }
    python3 - "$r" "$v" "$line" >> "$OUT" <<'PY'
import json, sys
d = json.loads(sys.argv[3]); r = d["roofline"]
print(f"round {sys.argv[1]} [{sys.argv[2] or 'default'}] kernel {r['kernel_ms']:.4f} ms frac {r['frac']:.4f} step {d['ms_per_step']:.4f} ms check {d.get('check', '')[:40]}")
PY
  done
done
cat "$OUT"
