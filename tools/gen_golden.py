#!/usr/bin/env python3
"""Generate golden vectors by running the reference's OWN functions (xmarre/person_capture
snapshot at /root/reference, read-only) on seeded inputs. Outputs only data files
(tests/golden/*.npz) — no reference source or bytecode is written anywhere.

Importable pieces: with a stub `cv2` module (channel/column
reversals only; OpenCV is not installed) person_capture.utils, .face_embedder and
.main import; Processor helpers are taken from gui_app.py by AST (PySide6 is absent)
and executed with numpy.

Run: python tools/gen_golden.py  (in the container that has /root/reference)
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def _stub_cv2():
    cv2 = types.ModuleType("cv2")
    cv2.COLOR_BGR2RGB, cv2.COLOR_BGR2GRAY = 4, 6
    cv2.INTER_AREA, cv2.INTER_LINEAR, cv2.LMEDS = 3, 1, 4
    cv2.BORDER_REFLECT, cv2.BORDER_REPLICATE = 2, 1
    cv2.setNumThreads = lambda n: None

    def cvt(img, code):
        if code == 4:
            return np.ascontiguousarray(img[..., ::-1])
        if code == 6:   # BGR2GRAY: only called on B == G == R frames below, where it is exactly channel 0
            assert np.array_equal(img[..., 0], img[..., 1]) and np.array_equal(img[..., 0], img[..., 2])
            return np.ascontiguousarray(img[..., 0])
        raise NotImplementedError(code)
    cv2.cvtColor = cvt
    cv2.flip = lambda img, f: np.ascontiguousarray(img[:, ::-1])
    sys.modules["cv2"] = cv2


def _processor_helpers():
    src = open(os.path.join(REF, "person_capture", "gui_app.py"), encoding="utf-8").read()
    tree = ast.parse(src)
    want = {"_fd_min", "_prescan_weights", "_stream_ref_bank_update", "_combine_scores"}
    body = []
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == "Processor":
            for item in node.body:
                if isinstance(item, ast.FunctionDef) and item.name in want:
                    body.append(item)
    cls = ast.ClassDef(name="Processor", bases=[], keywords=[], body=body, decorator_list=[])
    mod = ast.Module(body=[cls], type_ignores=[])
    ast.fix_missing_locations(mod)
    import ast as _ast
    import json
    from typing import List, Optional, Tuple
    ns = {"np": np, "json": json, "ast": _ast, "List": List, "Optional": Optional, "Tuple": Tuple}
    exec(compile(mod, "<gui_app.Processor subset>", "exec"), ns)
    return ns["Processor"]


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def main():
    _stub_cv2()
    sys.path.insert(0, REF)
    import person_capture.utils as U
    from person_capture.face_embedder import FaceEmbedder as FE
    import person_capture.main as M
    P = _processor_helpers()
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20260501)

    # ---- _fd_min ----
    feats, banks, fds = [], [], []
    for B, reps in ((1, 3), (32, 4), (64, 4), (1024, 1)):
        for t in range(reps):
            f = rng.standard_normal(512).astype(np.float32) * rng.uniform(0.1, 10)
            b = rng.standard_normal((B, 512)).astype(np.float32)
            b /= np.linalg.norm(b, axis=1, keepdims=True)
            if t == 1 or B == 1024:
                b[rng.integers(B)] = f / np.linalg.norm(f)
            fds.append(P._fd_min(f, b))
            feats.append(f)
            banks.append(b)
    fd_edge = np.array([P._fd_min(None, banks[0]), P._fd_min(feats[0], None),
                        P._fd_min(feats[0], np.zeros((0, 512), np.float32)),
                        P._fd_min(feats[0], banks[0][0])], np.float64)
    np.savez_compressed(os.path.join(OUT, "fd_min.npz"), feats=np.stack(feats),
                        bank_sizes=np.array([b.shape[0] for b in banks]),
                        banks=np.concatenate(banks, 0), fd=np.array(fds, np.float64), fd_edge=fd_edge)

    # ---- _stream_ref_bank_update action sequences ----
    seqs = {}
    for case, (cap, n) in enumerate([(4, 40), (64, 120), (8, 60)]):
        cfg = _Cfg(prescan_bank_max=cap, prescan_diversity_dedup_cos=0.968, prescan_replace_margin=0.010,
                   prescan_weights=(0.70, 0.25, 0.05))
        base = rng.standard_normal(512).astype(np.float32)
        vecs, quals, actions, idxs, banks_out = [], [], [], [], []
        lst, arr = [], None
        for i in range(n):
            mode = rng.integers(4)
            if mode == 0:
                v = base + rng.standard_normal(512).astype(np.float32) * 0.02   # near-duplicates
            elif mode == 1:
                v = base + rng.standard_normal(512).astype(np.float32) * 0.8
            elif mode == 2:
                v = rng.standard_normal(512).astype(np.float32)
            else:
                v = (np.zeros(512, np.float32) if rng.random() < 0.1 else base * rng.uniform(0.5, 2))
            q = float(rng.uniform(0, 1200))
            arr, act, idx = P()._stream_ref_bank_update(lst, arr, v, q, cfg)
            vecs.append(v)
            quals.append(q)
            actions.append(["skip", "added", "dup", "replaced"].index(act))
            idxs.append(-1 if idx is None else idx)
        seqs[f"case{case}_cap"] = np.array(cap)
        seqs[f"case{case}_vecs"] = np.stack(vecs)
        seqs[f"case{case}_quals"] = np.array(quals)
        seqs[f"case{case}_actions"] = np.array(actions)
        seqs[f"case{case}_idx"] = np.array(idxs)
        seqs[f"case{case}_final"] = np.asarray(arr, np.float32)
    np.savez_compressed(os.path.join(OUT, "bank_update.npz"), **seqs)

    # ---- _arcface_encode through a scripted linear session ----
    class Sess:
        # a fixed weight-free linear "network": 64 block sums of the NCHW input, scaled
        def run(self, names, feed):
            X = next(iter(feed.values()))
            n = X.shape[0]
            flat = X.reshape(n, -1)[:, : 64 * 588].reshape(n, 64, 588)
            return [(flat.sum(axis=2) * np.float32(0.01)).astype(np.float32)]

        def get_outputs(self):
            return [types.SimpleNamespace(name="out")]

    chips = rng.integers(0, 256, size=(5, 112, 112, 3), dtype=np.uint8)
    enc = {}
    for fast, esc in ((False, False), (True, False), (True, True)):
        obj = object.__new__(FE)
        obj._fast_prescan, obj._prescan_escalate = fast, esc
        obj._arc_fixed_batch = False
        obj.arc_sess = Sess()
        obj.arc_input = "in"
        f = obj._arcface_encode([c for c in chips])
        enc[f"feat_fast{int(fast)}_esc{int(esc)}"] = f
    pre = FE._arcface_preprocess(object.__new__(FE), chips[0])
    np.savez_compressed(os.path.join(OUT, "arcface_encode.npz"), chips=chips, pre0=pre, **enc)

    # ---- _canon_5pts / _iou / _nms_boxes / best_face ----
    pts_all, canon_ok, canon_out = [], [], []
    for t in range(200):
        base = FE._ARC_DST * rng.uniform(0.3, 3) + rng.uniform(-20, 20, 2)
        p = base + rng.normal(0, rng.choice([0.0, 1.0, 5.0, 20.0]), base.shape)
        p = p[rng.permutation(5)].astype(np.float32)
        if t % 17 == 0:
            p[rng.integers(5), rng.integers(2)] = np.nan
        c = FE._canon_5pts(p)
        pts_all.append(p)
        canon_ok.append(c is not None)
        canon_out.append(c if c is not None else np.zeros((5, 2), np.float32))
    boxes = rng.integers(0, 200, size=(300, 4))
    boxes[:, 2:] = boxes[:, :2] + rng.integers(-5, 80, size=(300, 2))
    ious = np.array([FE._iou(boxes[i], boxes[i + 1]) for i in range(299)])
    nms_in = [tuple(int(v) for v in b) for b in boxes[:60]]
    nms_out = np.array(FE._nms_boxes(nms_in, 0.5))
    faces = [{"bbox": np.array(b, np.int32), "quality": float(q)} for b, q in
             zip(boxes[:20], rng.choice([1.0, 2.0, 3.0], 20))]
    bf = FE.best_face(faces)
    bf_idx = [i for i, f in enumerate(faces) if f is bf][0]
    np.savez_compressed(os.path.join(OUT, "landmarks_boxes.npz"), pts=np.stack(pts_all), canon_ok=np.array(canon_ok),
                        canon=np.stack(canon_out), boxes=boxes, ious=ious, nms_out=nms_out,
                        bf_quality=np.array([f["quality"] for f in faces]), bf_idx=np.array(bf_idx),
                        arc_dst=FE._ARC_DST)

    # ---- utils + main helpers ----
    a = rng.standard_normal((50, 512)).astype(np.float32)
    b = rng.standard_normal((50, 512)).astype(np.float32)
    cd = np.array([U.cosine_distance(a[i], b[i]) for i in range(50)])
    l2 = np.stack([U.l2_normalize(a[i]) for i in range(50)])
    ebr_in, ebr_out = [], []
    for t in range(300):
        W, H = int(rng.integers(50, 2000)), int(rng.integers(50, 2000))
        x1, y1 = float(rng.uniform(-10, W)), float(rng.uniform(-10, H))
        x2, y2 = x1 + float(rng.uniform(0, W / 2)), y1 + float(rng.uniform(0, H / 2))
        rw, rh = [(2, 3), (16, 9), (1, 1), (4, 5)][t % 4]
        anchor = None if t % 3 else (float(rng.uniform(0, W)), float(rng.uniform(0, H)))
        hb = float(rng.uniform(-0.5, 0.5)) if t % 5 == 0 else 0.0
        r = U.expand_box_to_ratio(x1, y1, x2, y2, rw, rh, W, H, anchor=anchor, head_bias=hb)
        ebr_in.append([x1, y1, x2, y2, rw, rh, W, H, -1 if anchor is None else anchor[0],
                       -1 if anchor is None else anchor[1], hb])
        ebr_out.append(r)
    comb = []
    for fd_, rd_ in [(0.2, 0.5), (None, 0.3), (0.4, None), (None, None), (0.1, 0.1)]:
        for mode in ("min", "avg", "face_priority"):
            v = M.combine_scores(fd_, rd_, mode=mode)
            comb.append(np.nan if v is None else v)
    np.savez_compressed(os.path.join(OUT, "utils_main.npz"), a=a, b=b, cosdist=cd, l2=l2,
                        ebr_in=np.array(ebr_in), ebr_out=np.array(ebr_out), combine=np.array(comb, np.float64))
    # ---- post-match geometry (main.py:17-83, utils.py:152-197) ----
    rng2 = np.random.default_rng(20260516)
    esm_in, esm_out = [], []
    for t in range(400):
        W, H = int(rng2.integers(200, 3000)), int(rng2.integers(200, 2000))
        x1, y1 = int(rng2.integers(0, W - 20)), int(rng2.integers(0, H - 20))
        x2, y2 = int(rng2.integers(x1 + 10, W + 1)), int(rng2.integers(y1 + 10, H + 1))
        ratio = ["2:3", "16:9", "1:1", "4:5"][t % 4]
        fb = None
        if t % 3:
            fx1, fy1 = float(rng2.uniform(x1, x2)), float(rng2.uniform(y1, y2))
            fb = (fx1, fy1, fx1 + float(rng2.uniform(4, 400)), fy1 + float(rng2.uniform(4, 400)))
        r = M._enforce_scale_and_margins((x1, y1, x2, y2), ratio, W, H, fb)
        esm_in.append([x1, y1, x2, y2, t % 4, W, H] + (list(fb) if fb else [-1, -1, -1, -1]))
        esm_out.append(r)
    clip_in, clip_out = [], []
    for t in range(200):
        W, H = int(rng2.integers(50, 2000)), int(rng2.integers(50, 2000))
        b = [float(rng2.uniform(-300, W + 300)), float(rng2.uniform(-300, H + 300))]
        b += [b[0] + float(rng2.uniform(1, W)), b[1] + float(rng2.uniform(1, H))]
        clip_in.append(b + [W, H])
        clip_out.append(M._clip_to_frame(*b, W, H))
    borders, bb_out = [], []
    for t in range(24):
        H, W = int(rng2.integers(60, 400)), int(rng2.integers(60, 400))
        g = rng2.integers(30, 256, (H, W), dtype=np.uint8)
        top, bot, left, right = (int(rng2.integers(0, 40)) for _ in range(4))
        dark = int(rng2.integers(0, 12))
        g[:top] = dark; g[H - bot:] = dark; g[:, :left] = dark; g[:, W - right:] = dark
        img = np.repeat(g[..., None], 3, axis=2)
        thr = [10, 5, 20][t % 3]
        borders.append(img)
        bb_out.append(list(U.detect_black_borders(img, thr=thr)) + [thr])
    np.savez_compressed(os.path.join(OUT, "postmatch.npz"), esm_in=np.array(esm_in, np.float64),
                        esm_out=np.array(esm_out, np.int64), clip_in=np.array(clip_in, np.float64),
                        clip_out=np.array(clip_out, np.int64), bb_out=np.array(bb_out, np.int64),
                        **{f"border{i}": b for i, b in enumerate(borders)})
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
