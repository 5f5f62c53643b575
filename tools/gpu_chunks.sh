#!/bin/bash
# GPU box: C3 bench under different detection-chunk pipelines
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
for cfg in "32 2" "16 4" "16 2" "8 8"; do
  set -- $cfg
  PERSON_CAPTURE_AMD_PIPE_CHUNK=$1 PERSON_CAPTURE_AMD_PIPE_AHEAD=$2 timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/chunks_$1_$2.log 2>&1 || exit $?
  echo "chunk $1 ahead $2: $(tail -1 gpurun_out/chunks_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
