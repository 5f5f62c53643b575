"""Per-layer profile of the two trunks (HIP events around every launch, pc_net_profile_ops).
usage: python tools/probe_layers.py [arc|arcx3|scrfd|scrfdx3] [batch]   -> table grouped by conv shape.
scrfdx3 / arcx3: the f16x3 split programs.
PROBE_MAXB=N: create the net for N images (the small-batch plans then serve batch <= min(16, N/4)).
PROBE_D=D: the SCRFD det size (default 640)."""
import sys
from collections import defaultdict

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import models
from person_capture_amd import program as pg
import os
from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F32
from person_capture_amd.runtime import GpuContext, Net


def describe(P, w):
    if w[0] == pg.OP_CONV:
        segs = []
        for i in range(w[2]):
            t, kh, kw, s, p = w[3 + 5 * i: 8 + 5 * i]
            H, W, Cc = P.dims(t)
            segs.append(f"{H}x{W}x{Cc} k{kh}s{s}")
        Ho, Wo, _ = P.dims(w[1])
        return f"conv {'+'.join(segs)} -> {Ho}x{Wo}x{w[14]}" + (f" sk{w[24]}" if w[24] > 1 else "")
    return {pg.OP_STEM: "stem", pg.OP_MAXPOOL: "maxpool"}.get(w[0], f"op{w[0]}")


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "arc"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else (256 if which.startswith("arc") else 64)
    ctx = GpuContext(0)
    if which in ("arc", "arcx3"):
        P = models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100, split=which == "arcx3")
    else:
        P = models.compile_scrfd(models.synth_scrfd("10g", seed=0, calibrate=False), "10g",
                                 int(os.environ.get("PROBE_D", 640)), split=which == "scrfdx3")
    prec = PC_PREC_F32 if os.environ.get('PROBE_F32') else PC_PREC_F16
    net = Net(ctx, P.serialize(), prec, max_batch=int(os.environ.get('PROBE_MAXB', B)))   # FaceEmbedder: 512 for arc
    H, W, Cc = P.dims(P.input)
    x = np.zeros((B, H, W, Cc), np.float32 if prec == PC_PREC_F32 else np.float16)
    x[..., :3] = np.random.default_rng(0).standard_normal((B, H, W, 3)) * (127.5 if P.input_centered else 1.0)
    d = ctx.upload(x)
    for _ in range(3):
        net.run(d.ptr, B)
    net.profile(True)
    reps = 5
    for _ in range(reps):
        net.run(d.ptr, B)
    recs = net.profile_ops()
    net.profile(False)
    agg = defaultdict(lambda: [0, 0.0, 0.0, ""])
    tot_ms = tot_fl = 0.0
    for op, kind, ms, fl, halo, cfg in recs:
        if 100 <= halo < 200:
            cfg = -1   # (the conv_fast form, not a generic tile)
        key = describe(P, P.ops[int(op)])
        a = agg[key]
        a[0] += 1; a[1] += ms; a[2] += fl
        a[3] = (f"i{int(halo) - 400}" if halo >= 400 else "c" if halo == 300 else f"t{int(halo) - 200}" if halo >= 200 else f"f{int(halo) - 100}" if halo >= 100 else f"h{int(halo)}") \
            if halo >= 0 else \
            (f"g{int(cfg)}" if cfg >= 0 else "-")
        tot_ms += ms; tot_fl += fl
    print(f"{which} batch {B}: {tot_ms / reps:.3f} ms/run, {tot_fl / (tot_ms * 1e-3) / 1e12:.1f} TFLOP/s overall")
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    for key, (n, ms, fl, plan) in rows:
        n //= reps
        print(f"{key:48s} {plan:4s} x{n:3d} {ms / reps:8.3f} ms  {ms / reps / max(n, 1) * 1e3:8.1f} us/launch  "
              f"{(fl / (ms * 1e-3) / 1e12) if ms else 0:7.1f} TF/s  {100 * ms / tot_ms:5.1f}%")


if __name__ == "__main__":
    main()
