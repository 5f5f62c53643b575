#!/bin/bash
# GPU-box check: GPU parity tests, then (only if they ended normally: pass or plain test
# failures) the bench and the ArcFace b256 probe. Any abort/fault/timeout stops the script.
# usage (GPU box): bash tools/gpu_check.sh [pytest -k expr]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
K=${1:-}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${K:+-k "$K"} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe_arcface.py 256 > gpurun_out/arc.log 2>&1
rc=$?; echo "arc rc=$rc"; cat gpurun_out/arc.log | tail -3
exit $rc
