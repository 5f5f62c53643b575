#!/bin/bash
# C2 (ArcFace-r100 b256) evidence: wall-clock probe, rocprofv3 kernel-trace summary, and an MFMA
# PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE: counters only, no trace
# domains), reduced per conv kernel by tools/mfma_util.py.
# usage (GPU box): bash tools/profile_arcface.sh <tag>
set -eo pipefail
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/arc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 "$ROOT/tools/probe_arcface.py" 256 > "$OUT/probe.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o arc -- \
  python3 "$ROOT/tools/probe_arcface.py" 256 > "$OUT/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$OUT/pmc_mfma" -o arc -- python3 "$ROOT/tools/probe_arcface.py" 256 > "$OUT/pmc.log" 2>&1
KS=$(find "$OUT/kt" -name "*kernel_stats.csv" | head -1)
cp "$KS" "$OUT/${TAG}_arcface_b256_kernel_stats.csv"
python3 "$ROOT/tools/mfma_util.py" "$OUT/pmc_mfma" "$OUT/${TAG}_arcface_b256_mfma.json" --stats "$KS"
tail -1 "$OUT/probe.txt"
