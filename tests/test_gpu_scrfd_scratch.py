"""SCRFD candidate scratch shared by every ScrfdEngine of one context (pc_scrfd_detect:
cand / cand_count / det_scale): a large det size at a small batch followed by a small det
size at a larger batch needs fewer candidate rows but more per-image counters. The counters
are regrown by image count, so the second call must give exactly what the same
engine gives on a fresh context."""
import numpy as np
import pytest

from person_capture_amd import face_embedder as fe_mod
from person_capture_amd.engines import ScrfdEngine
from person_capture_amd.runtime import GpuContext

pytestmark = pytest.mark.gpu


def test_small_det_size_after_large_one_regrows_counters(gpu_ctx):
    p = fe_mod.synthetic_weights("scrfd_2.5g", 0)
    frames = np.random.default_rng(11).integers(0, 256, (48, 120, 160, 3), dtype=np.uint8)
    fsz = frames[0].nbytes
    d = gpu_ctx.upload(frames)
    views = [(d.ptr + i * fsz, 120, 160, 160 * 3) for i in range(len(frames))]
    big = ScrfdEngine(gpu_ctx, p, "2.5g", D=1536, max_batch=2)
    big.detect_frames(views[:2], thresh=0.5)             # 2 images x 96768 candidate rows
    small = ScrfdEngine(gpu_ctx, p, "2.5g", D=320, max_batch=48)
    got = small.detect_frames(views, thresh=0.5)         # 48 images x 4200 rows: fewer rows, more counters
    ctx2 = GpuContext(0)
    d2 = ctx2.upload(frames)
    ref = ScrfdEngine(ctx2, p, "2.5g", D=320, max_batch=48).detect_frames(
        [(d2.ptr + i * fsz, 120, 160, 160 * 3) for i in range(len(frames))], thresh=0.5)
    for (b1, k1), (b2, k2) in zip(got, ref):
        assert np.array_equal(b1, b2) and np.array_equal(k1, k2)
    ctx2.close()
