#!/bin/bash
# GPU box: kernel-trace durations of the s3 conv at full / skeleton-only (no HIP events involved)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
for dbg in 0 1 2 3 7; do
  PC_CONV_DBG=$dbg PROBE_SHAPES=${SHAPE:-s3_3x3_256} timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $ROOT/gpurun_out/prof_dbg$dbg -o p -- python3 $ROOT/tools/probe_conv.py auto > $ROOT/gpurun_out/prof_dbg$dbg.log 2>&1 || exit $?
  f=$(find $ROOT/gpurun_out/prof_dbg$dbg -name "*kernel_stats.csv" | head -1)
  echo "== dbg $dbg"; cut -d, -f1-8 "$f" | head -6
done
