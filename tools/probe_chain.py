"""ArcFace-r100 f16 at batch B with the resident chain on and off: wall ms per forward
(synced, 10 reps) and the per-op HIP-event split (chain launch vs the other convs).
usage: python tools/probe_chain.py [batch ...]"""
import os
import sys
import time

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import GpuContext, Net


def build(ctx, P, B, chain):
    if chain:
        os.environ.pop("PC_CHAIN", None)
        os.environ["PC_CHAIN_MIN"] = "1"
    else:
        os.environ["PC_CHAIN"] = "0"
    return Net(ctx, P.serialize(), PC_PREC_F16, max_batch=B)


def main():
    batches = [int(a) for a in sys.argv[1:]] or [256]
    ctx = GpuContext(0)
    P = models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100)
    for B in batches:
        x = np.zeros((B, 112, 112, 4), np.float16)
        x[..., :3] = np.random.default_rng(0).standard_normal((B, 112, 112, 3))
        d = ctx.upload(x)
        for chain in (False, True):
            net = build(ctx, P, B, chain)
            for _ in range(3):
                net.run(d.ptr, B)
            ctx.sync()
            t = time.perf_counter()
            n = 10
            for _ in range(n):
                net.run(d.ptr, B)
            ctx.sync()
            dt = (time.perf_counter() - t) / n
            net.profile(True)
            net.run(d.ptr, B)
            recs = net.profile_ops()
            net.profile(False)
            ch = recs[recs[:, 4] == 300]
            chain_ms = ch[:, 2].sum()
            chain_fl = ch[:, 3].sum()
            s3 = [r for r in recs if r[4] != 300]
            fl = net.flops_per_image * B
            print(f"B {B} chain {'on ' if chain else 'off'}: {dt * 1e3:7.3f} ms/fwd  {fl / dt / 1e12:7.1f} TF/s "
                  f"({fl / dt / 2.5e15 * 100:4.1f}% of 2.5 PF)"
                  + (f"  chain launch {chain_ms:.3f} ms = {chain_fl / (chain_ms * 1e-3) / 1e12:.1f} TF/s "
                     f"({len(ch)} launch)" if len(ch) else ""), flush=True)
            net.close()
        d.free()


if __name__ == "__main__":
    main()
