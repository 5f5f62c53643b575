#!/bin/bash
# GPU box: the whole -m gpu suite, then smoke(). Any abort/fault/timeout stops the script.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
exit $rc
