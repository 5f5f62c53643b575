#!/bin/bash
# GPU box: C3 bench at embed-stream priorities (HIP: lower = higher priority), alternating.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
: > gpurun_out/prio.txt
for p in "" -1 1 "" -1 1; do
  PERSON_CAPTURE_AMD_EMBED_PRIORITY=$p timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prio_one.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at prio '$p'"; tail -5 gpurun_out/prio_one.log; exit $rc; }
  v=$(tail -1 gpurun_out/prio_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
  echo "embed priority '${p:-default}': $v" | tee -a gpurun_out/prio.txt
done
