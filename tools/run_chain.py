"""Run ArcFace-r100 f16 at batch B with the resident chain forced on (profiling target).
env PC_CHAIN_WL / PC_CHAIN_PF pick the kernel variant."""
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import GpuContext, Net

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
os.environ["PC_CHAIN_MIN"] = "1"
ctx = GpuContext(0)
P = models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100)
net = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=B)
x = np.zeros((B, 112, 112, 4), np.float16)
x[..., :3] = np.random.default_rng(0).standard_normal((B, 112, 112, 3))
d = ctx.upload(x)
for _ in range(reps):
    net.run(d.ptr, B)
ctx.sync()
print("ok")
