#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a python command; prints the
# per-dispatch mean of every counter for kernels whose name contains MATCH.
# usage (GPU box): bash tools/pmc_cmd.sh <tag> <match> <python script> [args...]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; MATCH=$2; shift 2
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr" \
  "TCC_EA0_RDREQ_sum TCP_PENDING_STALL_CYCLES_sum TD_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_REQ_sum TCC_READ_sum" \
  "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TCR_TCP_STALL_CYCLES_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/$@" > "$OUT/p$i.log" 2>&1
  echo "pass $i rc=$?"
done
python3 - "$OUT" "$MATCH" <<'PY'
import csv, glob, sys, collections
out, match = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(collections.Counter)
tot = collections.defaultdict(float); cntall = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if match not in name: continue
        c, v = r["Counter_Name"], float(r["Counter_Value"])
        agg[name][c] += v; cnt[name][c] += 1
        tot[c] += v; cntall[c] += 1
with open(out + "/summary.txt", "w") as fo:
    def emit(line):
        print(line); fo.write(line + "\n")
    emit(f"== all kernels matching '{match}' (per dispatch)")
    for k in sorted(tot):
        emit(f"{k:32s} {tot[k] / max(cntall[k], 1):18.1f}  ({cntall[k]} rows)")
    for name in sorted(agg, key=lambda n: -max(cnt[n].values())):
        emit(f"== {name} (per dispatch)")
        for k in sorted(agg[name]):
            emit(f"{k:32s} {agg[name][k] / max(cnt[name][k], 1):18.1f}  ({cnt[name][k]} rows)")
PY
