"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to HBM bytes per conv launch.

usage: python tools/pmc_traffic.py <pmc_dir> [<pmc_dir> ...] <out.json> [--stats kernel_stats.csv]

With --stats (the rocprofv3 --kernel-trace --stats summary of the same command) the
dominant conv instantiation (largest total time) is reported on its own as well:
its counter bytes per launch, average duration and the HBM rate they imply.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read (16 B/lane
global_load / LDS-DMA), so it is doubled; WRITE_SIZE is exact for 16-B stores.
The conv epilogue stores 8 B (f16x4) or 16 B per lane, so WRITE_SIZE is taken
as-is and flagged uncalibrated for the 8-B form.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# every conv kernel family of the engine (pc_conv*.hip)
CONV_KERNELS = ("conv_igemm", "conv_fast", "conv_halo", "conv_hx", "conv_t2d", "conv_chain")


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))   # counter -> kernel -> [values]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    ctr = row.get("Counter_Name", "")
                    try:
                        v = float(row.get("Counter_Value", "nan"))
                    except ValueError:
                        continue
                    vals[ctr][name].append(v)
    return vals


def dominant_kernel(stats_csv, per_kernel):
    best = None
    with open(stats_csv) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Name") or row.get("KernelName") or ""
            if not any(t in name for t in CONV_KERNELS):
                continue
            tot = float(row.get("TotalDurationNs", 0) or 0)
            if best is None or tot > best[1]:
                best = (name, tot, float(row.get("AverageNs", 0) or 0), int(float(row.get("Calls", 0) or 0)))
    if best is None:
        return None
    name, tot, avg_ns, calls = best
    k = per_kernel.get(name, {})
    f = k.get("FETCH_SIZE", (None, 0))[0]
    w = k.get("WRITE_SIZE", (None, 0))[0]
    res = {"kernel": name, "calls": calls, "avg_us": round(avg_ns / 1e3, 2), "total_ms": round(tot / 1e6, 3)}
    if f is not None and w is not None:
        hb = 2.0 * 1024.0 * f + 1024.0 * w
        res.update(fetch_bytes_per_launch=2.0 * 1024.0 * f, write_bytes_per_launch=1024.0 * w,
                   hbm_bytes_per_launch=hb, hbm_gbps=round(hb / avg_ns, 1) if avg_ns else None)
    return res


def main():
    args = sys.argv[1:]
    stats = None
    if "--stats" in args:
        i = args.index("--stats")
        stats = args[i + 1]
        args = args[:i] + args[i + 2:]
    *dirs, out = args
    vals = load(dirs)
    per_kernel = {}
    for ctr, kern in vals.items():
        for name, v in kern.items():
            per_kernel.setdefault(name, {})[ctr] = (sum(v) / len(v), len(v))
    conv = {k: v for k, v in per_kernel.items() if any(t in k for t in CONV_KERNELS)}
    fetch = sum(v.get("FETCH_SIZE", (0, 0))[0] * v.get("FETCH_SIZE", (0, 0))[1] for v in conv.values())
    nf = sum(v.get("FETCH_SIZE", (0, 0))[1] for v in conv.values())
    write = sum(v.get("WRITE_SIZE", (0, 0))[0] * v.get("WRITE_SIZE", (0, 0))[1] for v in conv.values())
    nw = sum(v.get("WRITE_SIZE", (0, 0))[1] for v in conv.values())
    res = {
        "source": [os.path.relpath(d) for d in dirs],
        "conv_launches_fetch": nf, "conv_launches_write": nw,
        "conv_fetch_bytes_per_launch": 2.0 * 1024.0 * fetch / nf if nf else None,
        "conv_write_bytes_per_launch": 1024.0 * write / nw if nw else None,
        "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16-B/lane reads); WRITE_SIZE KiB x1024",
        "per_kernel": {k: {c: {"mean_kib": round(m, 1), "dispatches": n} for c, (m, n) in v.items()}
                       for k, v in sorted(per_kernel.items())},
    }
    if nf and nw:
        res["conv_hbm_bytes_per_launch"] = res["conv_fetch_bytes_per_launch"] + res["conv_write_bytes_per_launch"]
    if stats:
        res["dominant"] = dominant_kernel(stats, per_kernel)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}))


if __name__ == "__main__":
    main()
