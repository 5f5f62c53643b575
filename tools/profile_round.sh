#!/bin/bash
# Round profile: rocprofv3 kernel-trace summary of the bench, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (no trace domains beside counters), reduced
# to HBM bytes per conv launch in profiles/traffic.json.
# usage (GPU box): bash tools/profile_round.sh <tag>
set -eo pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o bench -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-parity > "$OUT/kt.log" 2>&1
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o bench -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-parity > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o bench -- \
  python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-parity > "$OUT/pmc_write.log" 2>&1
KS=$(find "$OUT/kt" -name "*kernel_stats.csv" | head -1)
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/traffic.json" --stats "$KS"
find "$OUT" -name "*kernel_stats.csv" | head -5
mkdir -p "$ROOT/profiles"
for f in $(find "$OUT/kt" -name "*kernel_stats.csv"); do cp "$f" "$ROOT/gpurun_out/prof_${TAG}/${TAG}_bench_kernel_stats.csv"; done
grep -v "^[WIE]20" "$OUT/kt.log" | tail -2 > "$OUT/${TAG}_bench_under_rocprof.json" || true
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$OUT/pmc_mfma" -o bench -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu --no-parity > "$OUT/pmc_mfma.log" 2>&1
python3 "$ROOT/tools/mfma_util.py" "$OUT/pmc_mfma" "$OUT/${TAG}_bench_mfma.json" --stats "$KS"
cp "$OUT/traffic.json" "$ROOT/gpurun_out/prof_${TAG}/${TAG}_traffic.json"
