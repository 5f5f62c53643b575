"""A/B of resident-chain variants in one process (interleaved rounds, HIP-event time of
the chain launch): weight layouts PC_CHAIN_WL = 0/1/2, each with and without the
weight stream (PC_CONV_DBG 1). usage: python tools/probe_chain_ab.py [B] [rounds]"""
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import GpuContext, Net


def chain_ms(net, d, B, dbg):
    os.environ["PC_CONV_DBG"] = str(dbg)
    net.run(d.ptr, B)
    net.profile(True)
    for _ in range(3):
        net.run(d.ptr, B)
    recs = net.profile_ops()
    net.profile(False)
    os.environ.pop("PC_CONV_DBG", None)
    ch = recs[recs[:, 4] == 300]
    return float(ch[:, 2].mean())


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    variants = [v for v in os.environ.get("AB_WL", "0,2").split(",")]
    wds = [v for v in os.environ.get("AB_MODE", "0,1").split(",")]
    ctx = GpuContext(0)
    P = models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100)
    os.environ["PC_CHAIN_MIN"] = "1"
    nets = {}
    for wl in variants:
        os.environ["PC_CHAIN_WL"] = wl
        nets[wl] = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=B)
    os.environ.pop("PC_CHAIN_WL", None)
    x = np.zeros((B, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(0).standard_normal((B, 112, 112, 3))
    d = ctx.upload(x)
    res = {}
    for r in range(rounds):
        for wl, net in nets.items():
            for wd in wds:
                os.environ["PC_CHAIN_MODE"] = wd
                for dbg in (0, 1):
                    res.setdefault((wl, wd, dbg), []).append(chain_ms(net, d, B, dbg))
    for (wl, wd, dbg), v in sorted(res.items()):
        v = np.array(v)
        print(f"B {B} WL {wl} MODE {wd} dbg {dbg}: chain median {np.median(v):.3f} ms min {v.min():.3f} "
              f"({np.median(v) * 1e3 / 58:.1f} us per conv)", flush=True)


if __name__ == "__main__":
    main()
