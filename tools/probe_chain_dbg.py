"""Ablation of the resident chain kernel (tuning only): HIP-event time of the chain launch
of ArcFace-r100 at batch B with PC_CONV_DBG = 0 (full), 1 (no weight DMA), 2 (no MFMA),
3 (neither), 4 (no epilogue). usage: python tools/probe_chain_dbg.py [B]"""
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import GpuContext, Net


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ctx = GpuContext(0)
    P = models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100)
    os.environ["PC_CHAIN_MIN"] = "1"
    net = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=B)
    x = np.zeros((B, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(0).standard_normal((B, 112, 112, 3))
    d = ctx.upload(x)
    for rep in range(2):
        for dbg in (0, 1, 2, 3, 4, 0):
            os.environ["PC_CONV_DBG"] = str(dbg)
            for _ in range(2):
                net.run(d.ptr, B)
            net.profile(True)
            for _ in range(5):
                net.run(d.ptr, B)
            recs = net.profile_ops()
            net.profile(False)
            ch = recs[recs[:, 4] == 300]
            ms = ch[:, 2].mean()
            print(f"B {B} dbg {dbg}: chain {ms:.3f} ms ({ms * 1e3 / 58:.1f} us per conv), "
                  f"{ch[:, 3].mean() / (ms * 1e-3) / 1e12:.0f} TF/s", flush=True)
    os.environ.pop("PC_CONV_DBG", None)


if __name__ == "__main__":
    main()
