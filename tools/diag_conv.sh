#!/bin/bash
# GPU box: conv engine diagnosis on the dominant ArcFace shapes
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"; mkdir -p gpurun_out
export PROBE_SHAPES=s3_3x3_256,s2_3x3_128,s1_3x3_64,gemm_1x1_2304
for dbg in 0 1 2 3; do
  echo "== PC_CONV_DBG=$dbg"
  PC_CONV_DBG=$dbg timeout -k 10 120 python -u tools/probe_conv.py auto f0:64 f1:64 f2:64 f3:64 f6:64 || exit $?
done
echo "== halo"
timeout -k 10 120 python -u tools/probe_conv.py h0 h1 h2 h3 || exit $?
