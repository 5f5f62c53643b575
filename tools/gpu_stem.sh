#!/bin/bash
# GPU box: fused stem parity + layer tables of both trunks
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_conv.py -k "stem or fused" -x -q --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1
rc=$?; echo "stem tests rc=$rc"; tail -3 gpurun_out/stem_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/probe_layers.py scrfd 64 > gpurun_out/layers_scrfd.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/probe_layers.py arc 256 > gpurun_out/layers_arc.txt 2>&1 || exit $?
head -14 gpurun_out/layers_scrfd.txt gpurun_out/layers_arc.txt | grep -v amdgpu.ids
