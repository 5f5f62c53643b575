#!/bin/bash
# GPU box: 2-D block conv parity, then per-layer tables of both trunks (t2d on / off).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_t2d.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2d_tests.log 2>&1
rc=$?; echo "t2d tests rc=$rc"; tail -15 gpurun_out/t2d_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/probe_layers.py scrfd 64 > gpurun_out/layers_scrfd_t2d.txt 2>&1 || exit $?
PC_CONV_T2D=0 timeout -k 10 120 python -u tools/probe_layers.py scrfd 64 > gpurun_out/layers_scrfd_fast.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/probe_layers.py arc 256 > gpurun_out/layers_arc_t2d.txt 2>&1 || exit $?
PC_CONV_T2D=0 timeout -k 10 120 python -u tools/probe_layers.py arc 256 > gpurun_out/layers_arc_fast.txt 2>&1 || exit $?
head -12 gpurun_out/layers_scrfd_t2d.txt gpurun_out/layers_scrfd_fast.txt gpurun_out/layers_arc_t2d.txt gpurun_out/layers_arc_fast.txt
