#!/bin/bash
# GPU box: 2-D block conv parity, then the single-conv probe (t2d vs fast, dbg splits)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_t2d.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2d_tests.log 2>&1
rc=$?; echo "t2d tests rc=$rc"; tail -3 gpurun_out/t2d_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_t2d_dbg.sh
