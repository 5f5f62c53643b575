"""Single-conv microbenchmark of the implicit-GEMM engine (HIP-event timed).
usage: python tools/probe_conv.py [cfg[:rowb] ...]   (cfg "auto" = planner's choice)
env PROBE_SHAPES=name1,name2 restricts the shapes; PROBE_N=n overrides their batch; PROBE_SPLIT=1 probes the f16x3 split form
(split input and output, DESIGN.md §3.6: a 1x1 conv writes the split input first; only the
probed conv is timed)."""
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import program as pg
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import GpuContext, Net

SHAPES = [
    # name, N, H, cin, cout, k, stride
    ("s3_3x3_256", 256, 14, 256, 256, 3, 1),
    ("gemm_1x1_2304", 256, 14, 2304, 256, 1, 1),
    ("s2_3x3_128", 256, 28, 128, 128, 3, 1),
    ("s1_3x3_64", 256, 56, 64, 64, 3, 1),
    ("s0_3x3_64_112", 256, 112, 64, 64, 3, 1),
    ("s4_3x3_512", 256, 7, 512, 512, 3, 1),
    ("sc_160_64", 64, 160, 64, 64, 3, 1),
    ("sc_320_32", 64, 320, 32, 32, 3, 1),
    ("sc_320_32_64", 64, 320, 32, 64, 3, 1),
    ("sc_80_96", 64, 80, 96, 96, 3, 1),
    ("sc_40_96", 64, 40, 96, 96, 3, 1),
    ("sc_20_224", 64, 20, 224, 224, 3, 1),
]


def build(N, H, cin, cout, k, s):
    split = bool(os.environ.get("PROBE_SPLIT"))
    P = pg.Program(split=split)
    x = P.input_tensor(H, H, cin)
    if split:   # split copy of the input (identity 1x1 conv), then the probed conv reads it
        t = P.act(H, H, cin)
        P.conv(t, [(x, 1, 1, 1, 0, cin)], pg.pack_conv_weights([np.eye(cin)[:, :, None, None]], [cin], cin), cin)
        x = t
    Ho = (H + 2 * (k // 2) - k) // s + 1
    y = P.act(Ho, Ho, cout)
    rng = np.random.default_rng(0)
    w = rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (cin * k * k))
    P.conv(y, [(x, k, k, s, k // 2, cin)], pg.pack_conv_weights([w], [cin], cout), cout,
           bias=np.zeros(cout), act=pg.ACT_RELU)
    P.outputs = [y]
    return P


def main():
    cfgs = sys.argv[1:] or ["auto"]
    ctx = GpuContext(0)
    only = [x for x in os.environ.get("PROBE_SHAPES", "").split(",") if x]
    for name, N, H, cin, cout, k, s in SHAPES:
        if only and name not in only:
            continue
        N = int(os.environ.get("PROBE_N", N))
        P = build(N, H, cin, cout, k, s)
        x = np.random.default_rng(1).standard_normal((N, H, H, cin)).astype(np.float16)
        d = ctx.upload(x)
        for spec in cfgs:
            c, _, rowb = spec.partition(":")
            if rowb:
                os.environ["PC_CONV_ROWB"] = rowb
            else:
                os.environ.pop("PC_CONV_ROWB", None)
            os.environ.pop("PC_CONV_HALO", None)
            os.environ.pop("PC_CONV_FAST", None)
            os.environ.pop("PC_CONV_T2D", None)
            if c.startswith("f"):
                os.environ.pop("PC_CONV_CFG", None)
                os.environ["PC_CONV_FAST"] = str(int(c[1:]) + 1)
            elif c == "auto":
                os.environ.pop("PC_CONV_CFG", None)
            elif c == "t2d":          # 2-D block kernel (pc_conv_t2d.hip) where it can run
                os.environ.pop("PC_CONV_CFG", None)
                os.environ["PC_CONV_T2D"] = "2"
            elif c == "not2d":
                os.environ.pop("PC_CONV_CFG", None)
                os.environ["PC_CONV_T2D"] = "0"
            elif c.startswith("h"):
                os.environ.pop("PC_CONV_CFG", None)
                os.environ["PC_CONV_HALO"] = str(int(c[1:]) + 1)
            else:
                os.environ["PC_CONV_CFG"] = c
            try:
                net = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=int(os.environ.get("PROBE_MAXB", N)))
            except RuntimeError as e:
                print(f"{name:16s} cfg {spec:6s} n/a ({e})", flush=True)
                continue
            for _ in range(3):
                net.run(d.ptr, N)
            net.profile(True)
            for _ in range(10):
                net.run(d.ptr, N)
            last = len(P.ops) - 1   # the probed conv (the split form has the input copy first)
            recs = [r for r in net.profile_ops() if int(r[0]) == last]
            net.profile(False)
            ms = sum(r[2] for r in recs)
            us = ms * 1e3 / len(recs)
            tf = sum(r[3] for r in recs) / (ms * 1e-3) / 1e12
            code = int(recs[0][4])
            ran = f"i{code - 400}" if code >= 400 else "chain" if code == 300 else f"t{code - 200}" if code >= 200 else (f"f{code - 100}" if code >= 100 else
                                                         (f"h{code}" if code >= 0 else f"g{int(recs[0][5])}"))
            print(f"{name:16s} cfg {spec:6s} ran {ran:4s} {us:9.1f} us/launch  {tf:7.1f} TFLOP/s", flush=True)
            net.close()


if __name__ == "__main__":
    main()
