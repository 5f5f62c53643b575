"""Pins the oracle (and the product's host-side restatements) to golden vectors
produced by running the reference's own functions (tools/gen_golden.py):
Processor._fd_min / _stream_ref_bank_update (gui_app.py), FaceEmbedder._arcface_encode
/ _arcface_preprocess / _canon_5pts / _iou / _nms_boxes / best_face (face_embedder.py),
utils.cosine_distance / l2_normalize / expand_box_to_ratio, main.combine_scores."""
import os

import numpy as np
import pytest

from oracle import ref_algos as ra
from person_capture_amd import imageops, match

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


@pytest.mark.parametrize("impl", [ra.fd_min, match.fd_min])
def test_fd_min(impl):
    d = _load("fd_min.npz")
    off = 0
    for i, B in enumerate(d["bank_sizes"]):
        bank = d["banks"][off:off + B]
        off += B
        assert impl(d["feats"][i], bank) == d["fd"][i]
    e = d["fd_edge"]
    assert impl(None, d["banks"][:1]) == e[0] == 9.0
    assert impl(d["feats"][0], None) == e[1] == 9.0
    assert impl(d["feats"][0], np.zeros((0, 512), np.float32)) == e[2] == 9.0
    assert impl(d["feats"][0], d["banks"][0]) == e[3]


@pytest.mark.parametrize("impl", ["oracle", "product"])
def test_stream_ref_bank_update(impl):
    d = _load("bank_update.npz")
    names = ["skip", "added", "dup", "replaced"]
    for case in range(3):
        cap = int(d[f"case{case}_cap"])
        lst, arr = [], None
        for v, q, act, idx in zip(d[f"case{case}_vecs"], d[f"case{case}_quals"], d[f"case{case}_actions"],
                                  d[f"case{case}_idx"]):
            if impl == "oracle":
                arr, a, i = ra.stream_ref_bank_update(lst, arr, v, float(q), cap=cap)
            else:
                arr, a, i = match.stream_ref_bank_update(lst, arr, v, float(q), cap=cap)
            assert a == names[act]
            assert (-1 if i is None else i) == idx
        assert np.array_equal(np.asarray(arr, np.float32), d[f"case{case}_final"])


def test_arcface_encode_post():
    d = _load("arcface_encode.npz")
    chips = d["chips"]
    assert np.array_equal(ra.arcface_preprocess(chips[0]), d["pre0"])

    def sess(X):   # the weight-free linear "network" of tools/gen_golden.py
        n = X.shape[0]
        flat = X.reshape(n, -1)[:, : 64 * 588].reshape(n, 64, 588)
        return (flat.sum(axis=2) * np.float32(0.01)).astype(np.float32)

    X = np.concatenate([ra.arcface_preprocess(c) for c in chips])
    Xf = np.concatenate([ra.arcface_preprocess(np.ascontiguousarray(c[:, ::-1])) for c in chips])
    assert np.array_equal(ra.arcface_postprocess(sess(X), sess(Xf)), d["feat_fast0_esc0"])
    assert np.array_equal(ra.arcface_postprocess(sess(X), None), d["feat_fast1_esc0"])      # prescan: no flip
    assert np.array_equal(ra.arcface_postprocess(sess(X), sess(Xf)), d["feat_fast1_esc1"])  # escalated


@pytest.mark.parametrize("impl", [ra.canon_5pts, imageops.canon_5pts])
def test_canon_5pts(impl):
    d = _load("landmarks_boxes.npz")
    for p, ok, c in zip(d["pts"], d["canon_ok"], d["canon"]):
        r = impl(p)
        assert (r is not None) == bool(ok)
        if ok:
            assert np.array_equal(r, c)
    assert np.array_equal(ra.ARC_DST, d["arc_dst"])
    assert np.array_equal(imageops.ARC_DST, d["arc_dst"])


def test_iou_nms_best_face():
    from person_capture_amd.face_embedder import FaceEmbedder
    d = _load("landmarks_boxes.npz")
    b = d["boxes"]
    for i in range(len(b) - 1):
        assert ra.iou(b[i], b[i + 1]) == d["ious"][i]
        assert FaceEmbedder._iou(b[i], b[i + 1]) == d["ious"][i]
    inp = [tuple(int(v) for v in x) for x in b[:60]]
    assert np.array_equal(np.array(ra.nms_boxes(inp, 0.5)), d["nms_out"])
    assert np.array_equal(np.array(FaceEmbedder._nms_boxes(inp, 0.5)), d["nms_out"])
    faces = [{"bbox": np.array(x, np.int32), "quality": float(q)} for x, q in zip(b[:20], d["bf_quality"])]
    assert ra.best_face(faces) is faces[int(d["bf_idx"])]
    assert FaceEmbedder.best_face(faces) is faces[int(d["bf_idx"])]
    assert FaceEmbedder.best_face([]) is None


def test_utils_main():
    d = _load("utils_main.npz")
    for i in range(len(d["a"])):
        assert ra.cosine_distance(d["a"][i], d["b"][i]) == d["cosdist"][i]
        assert np.array_equal(ra.l2_normalize(d["a"][i]), d["l2"][i])
    from person_capture_amd import utils as pu
    for row, out in zip(d["ebr_in"], d["ebr_out"]):
        x1, y1, x2, y2, rw, rh, W, H, ax, ay, hb = row
        anchor = None if ax == -1 and ay == -1 else (ax, ay)
        r = ra.expand_box_to_ratio(x1, y1, x2, y2, rw, rh, int(W), int(H), anchor=anchor, head_bias=hb)
        assert tuple(r) == tuple(out)
        assert tuple(pu.expand_box_to_ratio(x1, y1, x2, y2, rw, rh, int(W), int(H), anchor=anchor,
                                            head_bias=hb)) == tuple(out)
    k = 0
    for fd_, rd_ in [(0.2, 0.5), (None, 0.3), (0.4, None), (None, None), (0.1, 0.1)]:
        for mode in ("min", "avg", "face_priority"):
            v = ra.combine_scores(fd_, rd_, mode)
            exp = d["combine"][k]
            assert (v is None and np.isnan(exp)) or v == exp
            k += 1
