#!/bin/bash
# PMC passes over one single-conv probe (tools/probe_conv.py), one counter group per run.
# usage (GPU box): bash tools/pmc_probe.sh <shape> <cfg> [tag]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
SHAPE=$1; CFG=$2; TAG=${3:-pmc}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export PROBE_SHAPES=$SHAPE
[ -f "$OUT/counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/tools/probe_conv.py" $CFG > "$OUT/p$i.log" 2>&1
  echo "pass $i rc=$?"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "conv" not in r.get("Kernel_Name", ""): continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for k in sorted(agg): print(f"{k:28s} {agg[k] / max(cnt[k],1):16.1f}  (per dispatch, {cnt[k]} rows)")
PY
