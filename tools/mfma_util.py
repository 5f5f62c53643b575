"""MFMA utilisation of the conv kernels from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (+ SQ_BUSY_CYCLES), per kernel.

usage: python tools/mfma_util.py <pmc_dir> <out.json> [--stats kernel_stats.csv] [--flops F]

MfmaUtil (rocprofv3's derived formula) = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs x 4).
On MI355X GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS note), so the
busy fraction of the 1024 SIMDs is MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 256 x 4), and the
effective clock of a dispatch is GRBM_GUI_ACTIVE / 8 / its duration. MFMA_BUSY counts
per-SIMD cycles: 16 per v_mfma_f32_16x16x32_f16, so MFMA_BUSY x 1024 FLOP/cycle is the
FLOP count the counters saw (a check against the algorithmic FLOPs).

Clock: the GRBM quotient reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md,
DVFS note: r02's 3.69 GHz readings), so the effective clock is capped at the 2.4 GHz maximum
and, below 0.3 ms, the busy fraction is taken against the kernel wall time at that clock
(MFMA_BUSY / (avg_ns x 2.4 x 1024 SIMDs): a lower bound of the true busy fraction).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS = 256
FMAX_GHZ = 2.4


def main():
    args = sys.argv[1:]
    stats = None
    if "--stats" in args:
        i = args.index("--stats")
        stats = args[i + 1]
        args = args[:i] + args[i + 2:]
    pmc, out = args
    rows = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(pmc, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                try:
                    v = float(r.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                rows[r.get("Kernel_Name", "")][r.get("Counter_Name", "")].append(v)
    dur = {}
    if stats:
        with open(stats) as fh:
            for r in csv.DictReader(fh):
                dur[r.get("Name", "")] = float(r.get("AverageNs", 0) or 0)
    res = {}
    for name, c in rows.items():
        if not any(t in name for t in ("conv_fast", "conv_igemm", "conv_halo", "conv_hx", "conv_t2d", "conv_chain", "stem")):
            continue
        busy = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])) / max(1, len(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])))
        gui = sum(c.get("GRBM_GUI_ACTIVE", [])) / max(1, len(c.get("GRBM_GUI_ACTIVE", [])))
        e = {"dispatches": len(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])), "mfma_busy_cycles": busy,
             "grbm_gui_active": gui}
        if gui:
            e["mfma_util_simd_busy"] = round(busy / (gui / 8.0 * CUS * 4), 4)
            e["mfma_util_rocprof_formula"] = round(busy / (gui * CUS * 4), 4)
        e["counted_tflop_per_dispatch"] = round(busy * 1024 / 1e12, 6)
        if name in dur and dur[name] > 0:
            e["avg_ns"] = dur[name]
            q = gui / 8.0 / dur[name]
            e["grbm_clock_quotient_ghz"] = round(q, 3)
            e["effective_clock_ghz"] = round(min(q, FMAX_GHZ), 3)
            if dur[name] < 3e5 or q > FMAX_GHZ:
                # short dispatch: wall time at the maximum clock (lower bound of the busy fraction)
                e["mfma_util_simd_busy"] = round(busy / (dur[name] * FMAX_GHZ * CUS * 4), 4)
                e["clock_source"] = "wall time x 2.4 GHz (GRBM quotient unreliable below 0.3 ms)"
            else:
                e["clock_source"] = "GRBM_GUI_ACTIVE / 8"
            e["counted_tflops"] = round(busy * 1024 / dur[name] / 1e3, 1)
        res[name] = e
    # time-weighted total over the conv kernels that have durations
    tb = tc = 0.0
    for name, e in res.items():
        if "avg_ns" not in e:
            continue
        clk = e["effective_clock_ghz"] if e["clock_source"].startswith("GRBM") else FMAX_GHZ
        tb += e["mfma_busy_cycles"] * e["dispatches"]
        tc += e["avg_ns"] * clk * CUS * 4 * e["dispatches"]
    summary = {"conv_mfma_util_simd_busy": round(tb / tc, 4) if tc else None,
               "note": "time-weighted over the kernels with durations; SIMD-cycles at the capped effective clock",
               "per_kernel": res}
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({"conv_mfma_util_simd_busy": summary["conv_mfma_util_simd_busy"]}))


if __name__ == "__main__":
    main()
