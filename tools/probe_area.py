"""INTER_AREA 4K -> 416 batch probe: pc_resize_area_batch over N resident 4K frames, wall clock per call
(back to back, synchronised at the ends). usage: python tools/probe_area.py [N=32] [reps=20]
(run under rocprofv3 --kernel-trace --stats for the kernel's own duration)."""
import ctypes as C
import sys
import time

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

from person_capture_amd import imageops
from person_capture_amd._lib import check
from person_capture_amd.runtime import GpuContext


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    H, W = 2160, 3840
    ctx = GpuContext(0)
    frames = [ctx.upload(np.random.default_rng(i).integers(0, 256, (H, W, 3), dtype=np.uint8)) for i in range(N)]
    nh = int(round(H * 416 / W))
    p = imageops.resize_plan(H, W, (416, nh), 0.0, 0.0, True)
    (xt, xs), (yt, ys) = imageops.area_tables(W, p["new_w"], p["scale_x"]), imageops.area_tables(H, p["new_h"], p["scale_y"])
    outs = [ctx.alloc(p["new_w"] * p["new_h"] * 3) for _ in range(N)]
    srcs = (C.c_void_p * N)(*[f.ptr for f in frames])
    dsts = (C.c_void_p * N)(*[o.ptr for o in outs])

    def call():
        check(ctx.lib.pc_resize_area_batch(ctx.handle, srcs, dsts, N, W * 3, xt, xs, len(xt), yt, ys, len(yt),
                                           p["new_h"], p["new_w"]), ctx.handle, "resize_area_batch")
    call()
    ctx.sync()
    t = time.perf_counter()
    for _ in range(reps):
        call()
    ctx.sync()
    sec = (time.perf_counter() - t) / reps
    nbytes = N * (H * W * 3 + p["new_h"] * p["new_w"] * 3)
    print(f"area {N} x 4K -> {p['new_h']}x{p['new_w']}: {sec * 1e6:.1f} us per call, {nbytes / sec / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
