#!/bin/bash
# Host side (this container): submit one gpurun call, re-submitting it only while the pool
# answers "no box free / backing off" (status=transient: nothing ran, nothing charged).
# Any call that ran - whatever its result - is final.
# usage: bash tools/gpurun_wait.sh <timeout-s> <out-file> '<command>'
T=$1; OUT=$2; CMD=$3
for attempt in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient\|slot(s) on this pod are busy\|no free box" "$OUT" && ! grep -q "status=ok\|status=fail" "$OUT"; then
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
