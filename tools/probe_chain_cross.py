"""Chain-on / chain-off crossover of the whole IResNet-100 forward (f16) per batch size:
wall time of `reps` back-to-back runs after a device sync, interleaved rounds.
usage: python tools/probe_chain_cross.py [B,B,...] [rounds]"""
import os
import sys
import time

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import GpuContext, Net


def net_ms(ctx, net, d, B, reps=5):
    net.run(d.ptr, B)
    ctx.sync()
    t = time.perf_counter()
    for _ in range(reps):
        net.run(d.ptr, B)
    ctx.sync()
    return (time.perf_counter() - t) * 1e3 / reps


def main():
    bs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "8,16,32,48,64,128,256").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = GpuContext(0)
    P = models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100)
    mb = max(bs)
    os.environ["PC_CHAIN_MIN"] = "1"
    on = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=mb)
    os.environ["PC_CHAIN"] = "0"
    off = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=mb)
    os.environ.pop("PC_CHAIN", None)
    x = np.zeros((mb, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(0).standard_normal((mb, 112, 112, 3))
    d = ctx.upload(x)
    res = {}
    for _ in range(rounds):
        for B in bs:
            res.setdefault((B, 1), []).append(net_ms(ctx, on, d, B))
            res.setdefault((B, 0), []).append(net_ms(ctx, off, d, B))
    for B in bs:
        a, b = np.median(res[(B, 1)]), np.median(res[(B, 0)])
        print(f"B {B}: chain {a:.3f} ms  per-conv {b:.3f} ms  ratio {a / b:.3f}", flush=True)


if __name__ == "__main__":
    main()
