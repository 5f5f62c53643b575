"""MFMA utilisation of the conv kernels from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (+ SQ_BUSY_CYCLES), per kernel.

usage: python tools/mfma_util.py <pmc_dir> <out.json> [--stats kernel_stats.csv] [--flops F]

MfmaUtil (rocprofv3's derived formula) = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs x 4).
On MI355X GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS note), so the
busy fraction of the 1024 SIMDs is MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 256 x 4), and the
effective clock of a dispatch is GRBM_GUI_ACTIVE / 8 / its duration. MFMA_BUSY counts
per-SIMD cycles: 16 per v_mfma_f32_16x16x32_f16, so MFMA_BUSY x 1024 FLOP/cycle is the
FLOP count the counters saw (a check against the algorithmic FLOPs).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS = 256


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
        if not any(t in name for t in ("conv_fast", "conv_igemm", "conv_halo")):
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
            e["effective_clock_ghz"] = round(gui / 8.0 / dur[name], 3)
            e["counted_tflops"] = round(busy * 1024 / dur[name] / 1e3, 1)
        res[name] = e
    # time-weighted total over the conv kernels that have durations
    tb = tg = 0.0
    for name, e in res.items():
        tb += e["mfma_busy_cycles"] * e["dispatches"]
        tg += e["grbm_gui_active"] * e["dispatches"]
    summary = {"conv_mfma_util_simd_busy": round(tb / (tg / 8.0 * CUS * 4), 4) if tg else None,
               "per_kernel": res}
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({"conv_mfma_util_simd_busy": summary["conv_mfma_util_simd_busy"]}))


if __name__ == "__main__":
    main()
