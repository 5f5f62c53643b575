"""Quick device probe: ArcFace r100 forward throughput at batch B (wall clock, synced).
usage: probe_arcface.py [B] [PC_CONV_CFG] [f16|f16x3|f16c8]   (f16c8 calibrates its scales first)"""
import sys, time
sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
from person_capture_amd import models
from person_capture_amd.runtime import GpuContext, Net
from person_capture_amd._lib import PC_PREC_F16

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
import os
if len(sys.argv) > 2: os.environ['PC_CONV_CFG'] = sys.argv[2]
mode = sys.argv[3] if len(sys.argv) > 3 else "f16"
if len(sys.argv) > 2 and sys.argv[2] == "auto":
    os.environ.pop('PC_CONV_CFG', None)
ctx = GpuContext(0)
p = models.synth_iresnet(100, seed=0)
P = models.compile_iresnet(p, 100, split=mode == "f16x3", c8=mode == "f16c8")
net = Net(ctx, P.serialize(), PC_PREC_F16, max_batch=B)
x = np.zeros((B, 112, 112, 4), np.float16)
x[..., :3] = np.random.default_rng(0).standard_normal((B, 112, 112, 3)) * (127.5 if P.input_centered else 1.0)
d = ctx.upload(x)
if mode == "f16c8":
    net.calibrate(d.ptr, B)
for _ in range(3):
    net.run(d.ptr, B)
ctx.sync()
n = 10
t = time.perf_counter()
for _ in range(n):
    net.run(d.ptr, B)
ctx.sync()
dt = (time.perf_counter() - t) / n
fl = net.flops_per_image * B
print(f"cfg {os.environ.get('PC_CONV_CFG','auto')} batch {B}: {dt*1e3:.3f} ms/batch  {B/dt:.0f} fwd/s  {fl/dt/1e12:.1f} TFLOP/s  ({fl/dt/2.5e15*100:.1f}% of 2.5 PF)")
