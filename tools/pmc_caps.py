"""Per-kernel limiter table from a tools/pmc_cmd.sh counter directory.

usage: python tools/pmc_caps.py <pmc_dir> [--runs R] [--match conv_] > table.txt

For every kernel (counters averaged per dispatch) it reports, with T = GRBM_GUI_ACTIVE / 8
(GRBM is summed over the 8 XCDs, MI355X_MICROARCH.md) the dispatch's shader cycles:
  mfma   SQ_VALU_MFMA_BUSY_CYCLES / (T x 1024 SIMDs)          MFMA pipe busy fraction
  issue  SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES                   wave time issuing
  stall  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES                     issue-stalled (MFMA RAW / pipe busy)
  park   SQ_WAIT_ANY / SQ_WAVE_CYCLES                          parked in s_waitcnt / s_barrier
         (the three are disjoint and sum to ~1: MI355X_MICROARCH.md PMC table)
  waves  SQ_WAVE_CYCLES x 4 / (T x 256)                        resident waves per CU (quad-cycles)
  ldsC   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE              LDS cycles lost to bank conflicts
  l2hit  TCC_HIT / (TCC_HIT + TCC_MISS)
  l2lat  TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ            average L2 read latency (cycles)
  hbmRd  TCC_EA0_RDREQ x 128 B / (T / 2.4 GHz)                  fabric read rate (x128: gfx950
         tallies a 128-B request as 64 B in FETCH_SIZE, MI355X_MICROARCH.md HBM section)
and names the cap: the largest of {park, stall} when MFMA is below 60 %, with the LDS
conflict share and the fabric rate as qualifiers.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

FMAX = 2.4e9


def short(name):
    for t in ("conv_fast", "conv_t2d", "conv_chain", "conv_igemm", "conv_halo", "stem_fused", "maxpool"):
        if t in name:
            if name.startswith("_ZN2pc9conv_fast"):   # <T, BC, BP, ROWB, WC, WP, NSTAGE, OCC, SPLIT, SX>
                ints = re.findall(r"L[ib](\d+)E", name)
                tag = f"conv_fast {ints[0]}x{ints[1]} rowb{ints[2]} s{ints[5]}"
                return tag + (" split" if ints[7] == "1" else "") + (" sx" if ints[8] == "1" else "")
            if "<" in name:
                return t + "<" + name.split("<", 1)[1].split(">")[0] + ">"
            return t
    return name[:48]


def main():
    args = sys.argv[1:]
    runs, match = 1, ""
    if "--runs" in args:
        i = args.index("--runs")
        runs = int(args[i + 1])
        args = args[:i] + args[i + 2:]
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        args = args[:i] + args[i + 2:]
    rows = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(args[0], "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                try:
                    v = float(r.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                rows[r.get("Kernel_Name", "")][r.get("Counter_Name", "")].append(v)
    out = []
    for name, c in rows.items():
        if match and match not in name:
            continue
        m = {k: sum(v) / len(v) for k, v in c.items() if v}
        disp = max(len(v) for v in c.values())
        T = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if T <= 0 or wc <= 0:
            continue
        e = dict(kernel=short(name), per_run=disp / max(1, runs), us=T / FMAX * 1e6,
                 mfma=m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (T * 1024),
                 issue=m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, stall=m.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                 park=m.get("SQ_WAIT_ANY", 0.0) / wc, waves=wc * 4 / (T * 256),
                 ldsc=m.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, m.get("SQ_LDS_IDX_ACTIVE", 0.0)),
                 l2hit=m.get("TCC_HIT_sum", 0.0) / max(1.0, m.get("TCC_HIT_sum", 0.0) + m.get("TCC_MISS_sum", 0.0)),
                 l2lat=m.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / max(1.0, m.get("TCP_TCC_READ_REQ_sum", 0.0)),
                 hbm=m.get("TCC_EA0_RDREQ_sum", 0.0) * 128 / (T / FMAX) / 1e9)
        if e["mfma"] >= 0.6:
            cap = "MFMA"
        else:
            cap = "waits (waitcnt/barrier)" if e["park"] >= e["stall"] else "issue stalls (MFMA dep/pipe)"
            if e["ldsc"] > 0.08:
                cap += f" + LDS conflicts {e['ldsc']:.0%}"
            if e["hbm"] > 4000:
                cap += " + HBM"
            if e["waves"] < 4.5:
                cap += f" ; {e['waves']:.1f} waves/CU"
        e["cap"] = cap
        out.append(e)
    tot = sum(e["us"] * e["per_run"] for e in out) or 1.0
    print(f"{'kernel':34s} {'/run':>5s} {'us':>8s} {'time%':>6s} {'mfma':>5s} {'issue':>5s} {'stall':>5s} {'park':>5s}"
          f" {'waves':>5s} {'ldsC':>5s} {'l2hit':>5s} {'l2lat':>6s} {'hbmGB/s':>8s}  cap")
    for e in sorted(out, key=lambda e: -e["us"] * e["per_run"]):
        print(f"{e['kernel'][:34]:34s} {e['per_run']:5.1f} {e['us']:8.1f} {e['us'] * e['per_run'] / tot:6.1%}"
              f" {e['mfma']:5.1%} {e['issue']:5.1%} {e['stall']:5.1%} {e['park']:5.1%} {e['waves']:5.1f}"
              f" {e['ldsc']:5.1%} {e['l2hit']:5.1%} {e['l2lat']:6.0f} {e['hbm']:8.0f}  {e['cap']}")
    w = sum(e["mfma"] * e["us"] * e["per_run"] for e in out) / tot
    print(f"time-weighted MFMA busy over these kernels: {w:.1%} (us from GRBM cycles at the 2.4 GHz cap)")


if __name__ == "__main__":
    main()
