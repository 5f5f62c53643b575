"""ArcFace launches inside the C3 step (bench.py's setup): per kernel kind, launches, rows
per launch (from the FLOP records) and HIP-event time, to see how the batches of a step map
onto the kernels (resident chain or per-conv). usage: python tools/probe_c3_arc.py [steps]"""
import os
import sys
from collections import defaultdict

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np

import bench
from person_capture_amd.program import OP_CONV


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    os.environ.setdefault("PERSON_CAPTURE_AMD_DET_BATCH", "64")
    os.environ.setdefault("PERSON_CAPTURE_AMD_ARC_BATCH", "512")
    from person_capture_amd.face_embedder import FaceEmbedder, _DevImage
    from person_capture_amd.match import DeviceBank
    fe = FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5)
    frames = bench.synth_frames(0, 64)
    ctx = fe._ctx
    d = ctx.alloc(frames.nbytes)
    ctx.upload(frames, d)
    fsz = frames[0].nbytes
    devs = [_DevImage(d.ptr + i * fsz, 1080, 1920, 1920 * 3) for i in range(64)]
    bank = DeviceBank(ctx, bench.synth_bank(32))
    for _ in range(2):
        fe.extract_batch([None] * 64, dev_frames=devs, bank=bank)
    net = fe._arc.net
    fpi = net.flops_per_image
    net.profile(True)
    for _ in range(steps):
        fe.extract_batch([None] * 64, dev_frames=devs, bank=bank)
    ctx.sync()
    fe._ectx.sync()
    recs = net.profile_ops()
    net.profile(False)
    print("chain info", net.chain_info(), "embed quantum", fe._embed_quantum)
    agg = defaultdict(lambda: [0, 0.0, []])
    for r in recs:
        if int(r[1]) != OP_CONV:   # convs and chains only
            continue
        k = int(r[4])
        agg[k][0] += 1
        agg[k][1] += float(r[2])
    tot = sum(v[1] for v in agg.values())
    for k, (n, ms, _) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"code {k:4d}: {n:5d} launches {ms / steps:8.3f} ms/step ({ms / tot * 100:5.1f} %)")
    print(f"conv total {tot / steps:.3f} ms/step")
    # rows of each ArcFace run: the stem op's FLOPs over its per-image FLOPs
    stem = [r for r in recs if int(r[0]) == 0]
    if stem:
        per = min(float(r[3]) for r in stem) / max(1, min(1, 1))
        print("runs per step", len(stem) / steps, "stem FLOPs per run (relative):",
              sorted(round(float(r[3]) / per, 2) for r in stem)[:12])


if __name__ == "__main__":
    main()
