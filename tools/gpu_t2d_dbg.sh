#!/bin/bash
# GPU box: where the 2-D block conv's time goes (PC_CONV_DBG: 1 no DMA, 2 no K loop, 4 no stores)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
export PROBE_SHAPES=sc_320_32,sc_320_32_64,sc_160_64,s0_3x3_64_112,s1_3x3_64
out=gpurun_out/t2d_dbg.txt
: > $out
timeout -k 10 120 python -u tools/probe_conv.py not2d >> $out 2>&1 || exit $?
for d in ${T2D_DBGS:-0 1 2 4 6}; do
  echo "== dbg $d" >> $out
  PC_CONV_DBG=$d timeout -k 10 120 python -u tools/probe_conv.py t2d >> $out 2>&1 || exit $?
done
cat $out | grep -v amdgpu.ids
