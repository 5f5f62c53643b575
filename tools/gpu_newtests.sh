#!/bin/bash
# GPU box: the given test files only (fast iteration on new parity tests).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/newtests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|C3 |passed|failed" gpurun_out/newtests.log | tail -40
exit $rc
