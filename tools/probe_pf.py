"""Per-frame extract() probe: the bench's C3 per-frame setup (FaceEmbedder with det batch 64,
ArcFace batch 512, 1080p synthetic frames from host memory), one extract(imgsz=D) per frame,
with a line per frame and the Python stack every 30 s (faulthandler) so a stall names itself.

usage: python tools/probe_pf.py [D] [frames] [reps]
"""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(30, repeat=True)

D = int(sys.argv[1]) if len(sys.argv) > 1 else 640
NF = int(sys.argv[2]) if len(sys.argv) > 2 else 8
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
os.environ.setdefault("PERSON_CAPTURE_AMD_DET_BATCH", "64")
os.environ.setdefault("PERSON_CAPTURE_AMD_ARC_BATCH", "512")

import bench  # noqa: E402
from person_capture_amd.face_embedder import FaceEmbedder  # noqa: E402

t = time.perf_counter()
fe = FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5)
print(f"embedder {time.perf_counter() - t:.1f} s, det precision {fe.det_precision}", flush=True)
frames = list(bench.synth_frames(0, NF))
for rep in range(REPS):
    for i, f in enumerate(frames):
        t = time.perf_counter()
        faces = fe.extract(f, imgsz=D)
        dt = time.perf_counter() - t
        if rep == 0 or i == 0:
            print(f"rep {rep} frame {i}: {len(faces)} faces {dt * 1e3:.2f} ms, engines {sorted(fe._scrfd_engines)}",
                  flush=True)
    t = time.perf_counter()
    for f in frames:
        fe.extract(f, imgsz=D)
    print(f"rep {rep}: {(time.perf_counter() - t) / NF * 1e3:.2f} ms/frame", flush=True)
faulthandler.cancel_dump_traceback_later()
