"""GPU busy / idle of the last part of a rocprofv3 kernel trace (rocpd SQLite output).

usage: python tools/trace_window.py <results.db> [fraction=0.25] [top=25]
Takes the last `fraction` of the dispatches (e.g. the timed loop at the end of a probe),
reports the window's wall time, the union of kernel busy time (all streams), the idle
gaps, and per-kernel totals / counts / average duration in that window.
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    rows = rows[int(len(rows) * (1 - frac)):]
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for _, s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = defaultdict(lambda: [0, 0])
    for n, s, e, _ in rows:
        k = n.split("(")[0][:90]
        tot[k][0] += e - s
        tot[k][1] += 1
    wall = t1 - t0
    print(f"{len(rows)} dispatches, window {wall / 1e6:.3f} ms, GPU busy (union) {busy / 1e6:.3f} ms "
          f"({busy / wall:.1%}), idle {(wall - busy) / 1e6:.3f} ms in {len(gaps)} gaps "
          f"(>20us: {sum(1 for g in gaps if g > 20000)} totalling {sum(g for g in gaps if g > 20000) / 1e6:.3f} ms)")
    print(f"{'kernel':90s} {'n':>6s} {'total ms':>9s} {'avg us':>8s}")
    for k, (d, n) in sorted(tot.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{k:90s} {n:6d} {d / 1e6:9.3f} {d / n / 1e3:8.1f}")


if __name__ == "__main__":
    main()
