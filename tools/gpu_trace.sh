#!/bin/bash
# GPU box: kernel trace of a short C3 bench (gap analysis) + host phase timers
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o bench -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$OUT/kt.log" 2>&1 || exit $?
cd "$ROOT"
PERSON_CAPTURE_AMD_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/ht.log" 2>&1 || exit $?
tail -3 "$OUT/ht.log" | cut -c1-300
