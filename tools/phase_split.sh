#!/bin/bash
# Phase split of one split (f16x3) conv shape on two kernels (PC_CONV_DBG: 0 full, 2 no MFMAs, 4 no
# epilogue, 8 prologue only, 16 no output stores), single-conv probe, HIP events. usage (GPU box):
#   bash tools/phase_split.sh <probe shape> <VAR> <valA> <valB> [dbg values]   e.g. s3_3x3_256 PC_CONV_HXI 1 0
set -o pipefail
SHAPE=$1; VAR=$2; A=$3; B=$4; DBGS=$(echo "${5:-0,2,4,8,16}" | tr "," " ")
for v in "$A" "$B"; do
  for d in $DBGS; do
    echo "== $VAR=$v PC_CONV_DBG=$d"
    env "$VAR=$v" PC_CONV_DBG=$d PROBE_SHAPES=$SHAPE PROBE_SPLIT=1 timeout -k 10 120 python -u tools/probe_conv.py auto || exit $?
  done
done
