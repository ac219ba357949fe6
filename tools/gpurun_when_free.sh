#!/usr/bin/env bash
# Host-side helper (not run on the GPU box): submit one gpurun call, and
# resubmit it only while the pool answers "no box / slot free" (exit 3, or a
# transient back-off) -- nothing ran and nothing was charged then.  Any
# other outcome (the command ran, failed, or was refused) ends the loop.
# usage: tools/gpurun_when_free.sh LOG TIMEOUT 'COMMAND'
LOG=$1
TO=$2
CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    echo "[attempt $i: no box ($rc), waiting]" >> "$LOG.attempts"
    sleep 120
    continue
  fi
  echo "[attempt $i: rc=$rc]" >> "$LOG.attempts"
  exit $rc
done
