"""Bulk host helpers of the align step equal their per-face forms bit for bit
(FaceEmbedder._canon_5pts, face_embedder.py:1431-1463; cv2.invertAffineTransform)."""
import numpy as np

from person_capture_amd import imageops


def test_canon_5pts_batch_matches_scalar():
    rng = np.random.default_rng(7)
    base = np.array([[30, 40], [70, 40], [50, 60], [35, 80], [65, 80]], np.float32)
    sets = [base + rng.normal(0, s, (5, 2)).astype(np.float32) for s in np.linspace(0, 40, 3000)]
    sets += [rng.permutation(base) for _ in range(200)]           # any landmark order
    sets += [np.round(base + rng.normal(0, 6, (5, 2))).astype(np.float32) for _ in range(500)]  # ties
    nan = base.copy()
    nan[2, 0] = np.nan
    inf = base.copy()
    inf[4, 1] = np.inf
    flat = base.copy()
    flat[:, 1] = 50
    sets += [nan, inf, flat]
    pts = np.stack(sets)
    got, ok = imageops.canon_5pts_batch(pts)
    n_valid = 0
    for i in range(len(pts)):
        ref = imageops.canon_5pts(pts[i])
        assert (ref is None) == (not ok[i]), i
        if ref is not None:
            n_valid += 1
            assert np.array_equal(ref, got[i]), i
    assert 0 < n_valid < len(pts)
    assert imageops.canon_5pts_batch(np.zeros((0, 5, 2), np.float32))[1].shape == (0,)


def test_warp_descs_match_scalar():
    rng = np.random.default_rng(8)
    M = rng.normal(0, 1, (300, 6))
    M[5, [0, 1, 3, 4]] = 0.0        # singular: inverse is all-zero linear part
    src = np.arange(300, dtype=np.int64) * 4099 + (1 << 40)
    dst = np.arange(300, dtype=np.int64) * 37632 + (1 << 41)
    d = imageops.warp_descs(src, 5760, 123, 97, M, dst)
    assert d.itemsize == 96
    for i in range(300):
        ref = imageops.warp_desc(int(src[i]), 5760, 123, 97, M[i], int(dst[i]))
        assert bytes(ref) == d[i].tobytes(), i


def test_accumulate0_matches_scalar_policy_step():
    """FaceEmbedder._accumulate0 == the per-box 0-degree accumulate() of
    _scrfd_policy (face_embedder.py:2214-2239)."""
    from person_capture_amd.face_embedder import FaceEmbedder
    rng = np.random.default_rng(3)
    W0, H0 = 1920, 1080
    for _ in range(200):
        n = int(rng.integers(0, 12))
        bb = np.concatenate([rng.uniform(-50, 2000, (n, 4)), rng.uniform(0, 1, (n, 1))], 1).astype(np.float32)
        kp = rng.uniform(-20, 2000, (n, 5, 2)).astype(np.float32)
        ref = []
        for i in range(n):
            x1, y1, x2, y2 = [int(v) for v in bb[i, :4]]
            xa1, ya1, xa2, ya2 = min(x1, x2), min(y1, y2), max(x1, x2), max(y1, y2)
            xa1 = max(0, min(W0 - 1, xa1))
            ya1 = max(0, min(H0 - 1, ya1))
            xa2 = max(xa1 + 1, min(W0, xa2))
            ya2 = max(ya1 + 1, min(H0, ya2))
            if xa2 - xa1 <= 2 or ya2 - ya1 <= 2:
                continue
            pts = np.asarray([[float(px) - xa1, float(py) - ya1] for px, py in kp[i]], np.float32)
            ref.append(((xa1, ya1, xa2, ya2), pts, float(bb[i, 4])))
        got = FaceEmbedder._accumulate0(bb, kp, W0, H0)
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            assert a[0] == b[0] and all(type(v) is int for v in a[0])
            assert np.array_equal(a[1], b[1]) and a[2] == b[2]


def test_resize_plan_dispatch():
    """imageops.resize_plan picks OpenCV 4.9's kernel (resize.cpp dispatch)."""
    from person_capture_amd.imageops import resize_plan
    assert resize_plan(224, 224, (112, 112), area=True)["kind"] == "area_fast"
    assert resize_plan(224, 224, (112, 112), area=False)["kind"] == "area_fast"     # LINEAR at exactly 2x2
    assert resize_plan(336, 336, (112, 112), area=False)["kind"] == "linear"        # LINEAR 3x stays linear
    p = resize_plan(130, 100, (112, 112), area=True)
    assert p["kind"] == "linear" and p["area_mode"] == 1
    assert resize_plan(112, 112, (112, 112), area=True)["kind"] == "copy"
    p = resize_plan(720, 1280, None, 0.75, 0.75, area=True)
    assert p["kind"] == "area" and (p["new_w"], p["new_h"]) == (960, 540) and p["scale_x"] == 1 / 0.75
    # scale is 1/(new/old), which can differ from old/new in the last bit
    assert resize_plan(130, 130, (112, 112), area=True)["scale_x"] == 1.0 / (112 / 130)


def test_accumulate0_boxes_keep_their_float_source():
    """The int boxes of _accumulate0 are plain 4-tuples to every consumer (equality, unpacking,
    pickling across the pre-scan shard gather) and carry the detector's float box (`f`) that the
    parity reports use to locate one-pixel box differences at the int() boundary."""
    import pickle
    from person_capture_amd.face_embedder import FaceEmbedder, _IBox
    bb = np.array([[10.7, 20.2, 80.9, 99.99, 0.9]], np.float32)
    kp = np.zeros((1, 5, 2), np.float32)
    (box, _pts, _sc), = FaceEmbedder._accumulate0(bb, kp, 1920, 1080)
    assert box == (10, 20, 80, 99) and isinstance(box, tuple) and tuple(box) == (10, 20, 80, 99)
    assert np.allclose(box.f, bb[0, :4])
    x1, y1, x2, y2 = box
    assert (x1, y1, x2, y2) == (10, 20, 80, 99)
    c = pickle.loads(pickle.dumps(box))
    assert c == box and np.array_equal(c.f, box.f)
    assert _IBox((1, 2, 3, 4)).f is None
