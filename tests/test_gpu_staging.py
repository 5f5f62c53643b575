"""Host frame staging (pc_frame_stage: pinned ring + H2D on a copy stream the detection
stream waits on): byte-exact transfers of contiguous, row-strided and multi-threaded frames,
and FaceEmbedder.extract_batch over host frames equal to the same frames resident in HBM
(the staged path must change nothing but where the bytes come from)."""
import numpy as np
import pytest

import bench
from person_capture_amd import face_embedder as fe_mod

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W,threads", [(1, 1, 1), (37, 53, 4), (1080, 1920, 1), (1080, 1920, 8),
                                         (2160, 3840, 4)])
def test_stage_frame_bytes(gpu_ctx, H, W, threads):
    rng = np.random.default_rng(H * 7 + W)
    big = rng.integers(0, 256, (H + 9, W + 13, 3), dtype=np.uint8)
    views = [big[:H, :W].copy(), big[5:5 + H, 7:7 + W]]   # contiguous, row-strided slice
    h2d = fe_mod.get_context(0, "h2d")
    for v in views:
        d = gpu_ctx.alloc(H * W * 3)
        for _ in range(6):   # more frames than ring slots: slot reuse waits on its last copy
            h2d.stage_frame(v, d.ptr, threads)
        gpu_ctx.wait_fence(h2d.fence("t"))
        got = gpu_ctx.download(d.ptr, (H, W, 3), np.uint8)
        assert np.array_equal(got, v)
        d.free()


def test_extract_batch_host_frames_equal_resident(gpu_ctx):
    frames = bench.synth_frames(0, 6)
    fe_a = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5)
    fe_b = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5)
    fe_a._pipe_chunk = fe_b._pipe_chunk = 2   # several staged chunks
    H, W = frames.shape[1:3]
    d = gpu_ctx.alloc(frames.nbytes)
    gpu_ctx.upload(frames, d)
    gpu_ctx.sync()
    fsz = frames[0].nbytes
    devs = [fe_mod._DevImage(d.ptr + i * fsz, H, W, W * 3) for i in range(len(frames))]
    host = [frames[0], frames[1][:, :], None, np.ascontiguousarray(frames[3]), frames[4], frames[5]]
    a = fe_a.extract_batch(host)
    dv = [x for i, x in enumerate(devs) if i != 2]
    b = fe_b.extract_batch([None] * len(dv), dev_frames=dv)
    b.insert(2, [])
    assert sum(len(r) for r in a) > 0
    for ra_, rb in zip(a, b):
        assert len(ra_) == len(rb)
        for x, y in zip(ra_, rb):
            assert np.array_equal(x["bbox"], y["bbox"]) and np.array_equal(x["feat"], y["feat"])
    # a row-strided crop through extract() equals the same crop uploaded contiguously
    crop = frames[0][100:700, 300:1100]
    x = fe_a.extract(crop)
    y = fe_b.extract(np.ascontiguousarray(crop))
    assert len(x) == len(y) and all(np.array_equal(p["feat"], q["feat"]) for p, q in zip(x, y))
