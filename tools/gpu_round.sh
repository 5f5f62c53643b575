#!/bin/bash
# GPU box: full -m gpu suite + smoke, then the C3 bench line.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_full.sh || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c3.log; exit $rc
