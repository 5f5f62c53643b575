#!/bin/bash
# Phase split of the small-batch conv_hxi forms (PC_CONV_HXI=59) at PROBE_N images on a 512-image net
# (PC_CONV_DBG 0 full, 2 no MFMAs, 4 no epilogue, 8 prologue only, 16 no stores). usage (GPU box):
#   bash tools/hxs_phase.sh <N> <shape> [<shape> ...]
set -o pipefail
N=$1; shift
for sh in "$@"; do
  for d in 0 2 4 8 16; do
    echo "== $sh N=$N PC_CONV_DBG=$d"
    PC_CONV_HXI=59 PC_CONV_DBG=$d PROBE_N=$N PROBE_MAXB=512 PROBE_SHAPES=$sh PROBE_SPLIT=1 \
      timeout -k 10 120 python -u tools/probe_conv.py auto || exit $?
  done
done
