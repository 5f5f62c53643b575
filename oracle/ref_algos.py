"""numpy restatements of the reference's host-side hot-path algorithms.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Each function names the
reference code it restates (paths relative to the xmarre/person_capture
snapshot). tests/test_oracle_golden.py pins them against vectors produced by
running the reference's own functions (tools/gen_golden.py).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

# person_capture/face_embedder.py:1279 (ArcFace 112x112 landmark template)
ARC_DST = np.array([[38.2946, 51.6963], [73.5318, 51.5014], [56.0252, 71.7366], [41.5493, 92.3655],
                    [70.7299, 92.2041]], dtype=np.float32)


# ---------------------------------------------------------------------------
# matching
# ---------------------------------------------------------------------------
def fd_min(feat, bank) -> float:
    """gui_app.py:660-674 Processor._fd_min: 1 - max cosine vs a unit-row bank."""
    if feat is None or bank is None:
        return 9.0
    v = np.asarray(feat, dtype=np.float32).reshape(-1)
    v = v / max(float(np.linalg.norm(v)), 1e-6)
    B = np.asarray(bank, dtype=np.float32)
    if B.ndim == 1:
        return 1.0 - float(np.dot(v, B))
    if B.size == 0:
        return 9.0
    s = B @ v
    return 9.0 if s.size == 0 else 1.0 - float(s.max())


def stream_ref_bank_update(bank_list: List[np.ndarray], bank_arr: Optional[np.ndarray], vec_new, quality: float,
                           cap: int = 64, dedup_cos: float = 0.968, rep_margin: float = 0.010,
                           weights=(0.70, 0.25, 0.05)):
    """gui_app.py:922-986 Processor._stream_ref_bank_update (config read from args).
    Returns (bank_arr, action, replaced_index); mutates bank_list like the reference."""
    if vec_new is None:
        return bank_arr, "skip", None
    wa, wd, wq = weights
    cap = max(1, int(cap))
    v = np.asarray(vec_new, dtype=np.float32).reshape(-1)
    nv = float(np.linalg.norm(v))
    if nv <= 1e-6:
        return bank_arr, "skip", None
    v = v / nv
    B = np.asarray(bank_arr if bank_arr is not None else bank_list, dtype=np.float32)
    if B.ndim == 1:
        B = B.reshape(1, -1)
    if B.size == 0:
        bank_list.append(v)
        return np.vstack(bank_list).astype(np.float32), "added", None
    sims = B @ v
    if sims.size > 0 and float(sims.max()) >= dedup_cos:
        return bank_arr, "dup", None
    anchor = B[0]
    ca = min(1.0, max(-1.0, float(np.dot(anchor, v))))
    fd_anchor = float(np.sqrt(max(0.0, 2.0 - 2.0 * ca)))
    nn_sim = float(sims.max()) if sims.size else 0.0
    q_term = float(min(max(quality or 0.0, 0.0), 1000.0) / 300.0)
    s_new = wa * (1.0 - fd_anchor) + wd * (1.0 - nn_sim) + wq * q_term
    if len(bank_list) < cap:
        bank_list.append(v)
        return np.vstack(bank_list).astype(np.float32), "added", None
    G = B @ B.T
    np.fill_diagonal(G, -1.0)
    nn_each = G.max(axis=1)
    ca_each = np.clip(B @ anchor, -1.0, 1.0)
    fa_each = np.sqrt(np.maximum(0.0, 2.0 - 2.0 * ca_each))
    s_bank = wa * (1.0 - fa_each) + wd * (1.0 - nn_each)
    worst = int(np.argmin(s_bank))
    if s_new > float(s_bank[worst]) + rep_margin:
        bank_list[worst] = v
        return np.vstack(bank_list).astype(np.float32), "replaced", worst
    return bank_arr, "skip", None


def l2_normalize(x, eps: float = 1e-10):
    """utils.py:108-110."""
    return x / (np.linalg.norm(x) + eps)


def cosine_distance(a, b) -> float:
    """utils.py:260-268."""
    va = np.asarray(list(a), dtype=np.float32).reshape(-1)
    vb = np.asarray(list(b), dtype=np.float32).reshape(-1)
    na = float(np.linalg.norm(va)) + 1e-9
    nb = float(np.linalg.norm(vb)) + 1e-9
    return 1.0 - float(np.dot(va / na, vb / nb))


def combine_scores(face_dist, reid_dist, mode: str = "min"):
    """main.py:127-144."""
    vals = [v for v in (face_dist, reid_dist) if v is not None]
    if not vals:
        return None
    if mode == "avg":
        return sum(vals) / len(vals)
    if mode == "face_priority":
        if face_dist is not None:
            return 0.7 * face_dist + 0.3 * (reid_dist if reid_dist is not None else 0.5)
        return reid_dist
    return min(vals)


# ---------------------------------------------------------------------------
# ArcFace pre/post
# ---------------------------------------------------------------------------
def arcface_preprocess(chip_bgr: np.ndarray) -> np.ndarray:
    """face_embedder.py:1281-1288 for an already-112x112 chip: RGB, /127.5 - 1, NCHW."""
    rgb = chip_bgr[..., ::-1]
    arr = rgb.astype(np.float32) / 127.5 - 1.0
    return np.transpose(arr, (2, 0, 1))[None, ...]


def arcface_postprocess(e: np.ndarray, e_flip: Optional[np.ndarray] = None) -> np.ndarray:
    """face_embedder.py:1383-1389: f = e (+ e_flip); f /= max(||f||, 1e-6)."""
    f = np.asarray(e, dtype=np.float32).copy()
    if e_flip is not None:
        f += np.asarray(e_flip, dtype=np.float32)
    n = np.linalg.norm(f, axis=1, keepdims=True).astype(np.float32, copy=False)
    np.maximum(n, 1e-6, out=n)
    f /= n
    return f.astype(np.float32, copy=False)


# ---------------------------------------------------------------------------
# landmarks / boxes
# ---------------------------------------------------------------------------
def canon_5pts(pts) -> Optional[np.ndarray]:
    """face_embedder.py:1431-1463 FaceEmbedder._canon_5pts."""
    if pts is None:
        return None
    pts = np.asarray(pts)
    if pts.shape != (5, 2):
        return None
    pts = pts.astype(np.float32)
    if not np.isfinite(pts).all():
        return None
    oy = np.argsort(pts[:, 1])
    eyes, nose, mouth = pts[oy[:2]], pts[oy[2]], pts[oy[3:]]
    le, re_ = eyes[np.argsort(eyes[:, 0])]
    lm, rm = mouth[np.argsort(mouth[:, 0])]
    if not (le[0] < re_[0] and lm[0] < rm[0]):
        return None
    if not (nose[1] > max(le[1], re_[1]) and nose[1] < min(lm[1], rm[1])):
        return None
    return np.stack([le, re_, nose, lm, rm], axis=0)


def iou(a, b) -> float:
    """face_embedder.py:2484-2494 FaceEmbedder._iou (no +1)."""
    iw = max(0, min(a[2], b[2]) - max(a[0], b[0]))
    ih = max(0, min(a[3], b[3]) - max(a[1], b[1]))
    inter = iw * ih
    aa = max(0, a[2] - a[0]) * max(0, a[3] - a[1])
    ab = max(0, b[2] - b[0]) * max(0, b[3] - b[1])
    d = aa + ab - inter
    return inter / d if d > 0 else 0.0


def nms_boxes(boxes, iou_thr: float = 0.5):
    """face_embedder.py:2496-2502 (area-descending greedy)."""
    kept = []
    for b in sorted(boxes, key=lambda t: (t[2] - t[0]) * (t[3] - t[1]), reverse=True):
        if all(iou(b, k) < iou_thr for k in kept):
            kept.append(b)
    return kept


def best_face(faces):
    """face_embedder.py:2504-2508."""
    if not faces:
        return None
    return max(faces, key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])))


def expand_box_to_ratio(x1, y1, x2, y2, ratio_w, ratio_h, frame_w, frame_h, anchor=None, head_bias=0.0):
    """utils.py:198-257."""
    cl = lambda v, lo, hi: max(lo, min(hi, v))
    x1, y1, x2, y2 = map(float, (x1, y1, x2, y2))
    bw, bh = max(1.0, x2 - x1), max(1.0, y2 - y1)
    target = float(ratio_w) / float(ratio_h)
    if anchor is not None:
        cx, cy = float(anchor[0]), float(anchor[1])
    else:
        cx, cy = x1 + bw * 0.5, y1 + bh * 0.5
    cy = cy - head_bias * bh
    if bw / bh < target:
        nw, nh = target * bh, bh
    else:
        nw, nh = bw, bw / target
    ax1, ay1, ax2, ay2 = cx - nw * 0.5, cy - nh * 0.5, cx + nw * 0.5, cy + nh * 0.5
    ax1, ay1 = cl(ax1, 0, frame_w - 1), cl(ay1, 0, frame_h - 1)
    ax2, ay2 = cl(ax2, 0, frame_w - 1), cl(ay2, 0, frame_h - 1)
    cw, ch = ax2 - ax1, ay2 - ay1
    if cw <= 1 or ch <= 1:
        return int(ax1), int(ay1), int(ax2), int(ay2)
    if abs(cw / ch - target) > 1e-4:
        if cw / ch < target:
            d = (ch - cw / target) * 0.5
            ay1 += d
            ay2 -= d
        else:
            d = (cw - ch * target) * 0.5
            ax1 += d
            ax2 -= d
        ax1, ay1 = cl(ax1, 0, frame_w - 1), cl(ay1, 0, frame_h - 1)
        ax2, ay2 = cl(ax2, 0, frame_w - 1), cl(ay2, 0, frame_h - 1)
    return int(round(ax1)), int(round(ay1)), int(round(ax2)), int(round(ay2))


# ---------------------------------------------------------------------------
# SCRFD decode + NMS  ([ext] insightface>=0.7.3 model_zoo/scrfd.py, called at face_embedder.py:2185)
# ---------------------------------------------------------------------------
def scrfd_letterbox_geometry(H: int, W: int, D: int) -> Tuple[int, int, float]:
    """SCRFD.detect sizing for input_size=(D, D)."""
    if float(H) / W > 1.0:
        nh = D
        nw = int(nh / (float(H) / W))
    else:
        nw = D
        nh = int(nw * (float(H) / W))
    return nw, nh, float(nh) / H


def scrfd_decode(head_outs: Sequence[np.ndarray], thresh: float, det_scale: float, strides=(8, 16, 32)):
    """head_outs[l]: [H][W][30] raw head tensor of stride l: cls logits(2) | bbox(8) | kps(20).
    SCRFD.forward + the first half of SCRFD.detect: sigmoid scores, keep >= thresh,
    distance2bbox / distance2kps of predictions*stride, divide by det_scale.
    Returns (pre_det [K,5] in concatenation order, kps [K,5,2])."""
    scores_l, boxes_l, kps_l = [], [], []
    for out, s in zip(head_outs, strides):
        Hh, Ww = out.shape[:2]
        flat = np.asarray(out, dtype=np.float32).reshape(Hh * Ww, -1)
        logit = flat[:, 0:2].reshape(-1)
        score = (1.0 / (1.0 + np.exp(-logit.astype(np.float64)))).astype(np.float32)  # f64 sigmoid, as the device
        bb = flat[:, 2:10].reshape(-1, 4) * np.float32(s)
        kp = flat[:, 10:30].reshape(-1, 10) * np.float32(s)
        ys, xs = np.mgrid[:Hh, :Ww]
        centers = (np.stack([xs, ys], axis=-1).astype(np.float32) * s).reshape(-1, 2)
        centers = np.repeat(centers, 2, axis=0)
        keep = np.where(score >= thresh)[0]
        x1 = centers[:, 0] - bb[:, 0]
        y1 = centers[:, 1] - bb[:, 1]
        x2 = centers[:, 0] + bb[:, 2]
        y2 = centers[:, 1] + bb[:, 3]
        boxes = np.stack([x1, y1, x2, y2], axis=-1)
        k = np.empty((kp.shape[0], 10), np.float32)
        k[:, 0::2] = centers[:, 0:1] + kp[:, 0::2]
        k[:, 1::2] = centers[:, 1:2] + kp[:, 1::2]
        scores_l.append(score[keep, None])
        boxes_l.append(boxes[keep])
        kps_l.append(k[keep].reshape(-1, 5, 2))
    scores = np.vstack(scores_l)
    boxes = np.vstack(boxes_l) / np.float32(det_scale)
    kps = np.vstack(kps_l) / np.float32(det_scale)
    pre = np.hstack((boxes, scores)).astype(np.float32, copy=False)
    return pre, kps.astype(np.float32, copy=False)


def scrfd_nms_keep(dets: np.ndarray, thresh: float = 0.4) -> List[int]:
    """SCRFD.nms: greedy, '+1' pixel areas, suppress ovr > thresh, float32 math."""
    x1, y1, x2, y2, sc = (dets[:, i] for i in range(5))
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    order = np.argsort(sc, kind="stable")[::-1]
    keep = []
    while order.size > 0:
        i = order[0]
        keep.append(int(i))
        rest = order[1:]
        w = np.maximum(np.float32(0.0), np.minimum(x2[i], x2[rest]) - np.maximum(x1[i], x1[rest]) + 1)
        h = np.maximum(np.float32(0.0), np.minimum(y2[i], y2[rest]) - np.maximum(y1[i], y1[rest]) + 1)
        inter = w * h
        ovr = inter / (areas[i] + areas[rest] - inter)
        order = rest[np.where(ovr <= np.float32(thresh))[0]]
    return keep


def scrfd_detect_post(head_outs, thresh: float, det_scale: float, nms_thresh: float = 0.4):
    """Second half of SCRFD.detect: order = argsort(score)[::-1] (stable), NMS, (det, kpss)."""
    pre, kps = scrfd_decode(head_outs, thresh, det_scale)
    order = np.argsort(pre[:, 4], kind="stable")[::-1]
    pre = pre[order]
    kps = kps[order]
    keep = scrfd_nms_keep(pre, nms_thresh)
    return pre[keep], kps[keep]


# ---------------------------------------------------------------------------
# YOLOv8 person detection: [ext] ultralytics 8.3.205 as called by PersonDetector.detect
# (detectors.py:271-296). Restated from its published algorithm (not vendored, no
# fixtures in the reference -> parity unpinned against ultralytics itself).
# ---------------------------------------------------------------------------
def yolo_letterbox(frame: np.ndarray, imgsz: int = 640, stride: int = 32) -> Tuple[np.ndarray, tuple]:
    """LetterBox(auto=True, center=True) + preprocess: returns the [Hp][Wp][3] f32 RGB/255
    canvas and the geometry (new_w, new_h, top, left, Hp, Wp)."""
    from oracle import cv_ops
    from person_capture_amd.models_yolo import letterbox_geometry   # sizing formulas only
    H, W = frame.shape[:2]
    g = letterbox_geometry(H, W, imgsz, stride)
    new_w, new_h, top, left, Hp, Wp = g
    if (W, H) != (new_w, new_h):
        x = (new_w * 3 // 16) * 16 if new_w * 3 >= 16 else 0
        while x < new_w * 3 - 8:
            x += 8
        img = cv_ops.resize_linear(frame, new_w, new_h, 1.0 / (float(new_w) / W), 1.0 / (float(new_h) / H), x)
    else:
        img = np.ascontiguousarray(frame)
    canvas = np.full((Hp, Wp, 3), 114, np.uint8)
    canvas[top:top + new_h, left:left + new_w] = img
    return canvas[..., ::-1].astype(np.float32) / np.float32(255.0), g


def yolo_postprocess(heads: Sequence[np.ndarray], conf: float, iou: float, max_det: int, Hp: int, Wp: int,
                     H0: int, W0: int, nk: int = 0):
    """Detect inference decode + ops.non_max_suppression(classes=[0]) + ops.scale_boxes for one
    image. heads: per stride [H][W][64+nc(+nk)] f32. Returns [k][5] (x1, y1, x2, y2, conf); with
    nk > 0 (Pose head, kpt ndim 3) also the keypoints [k][nk/3][3] of the kept boxes:
    Pose.kpts_decode (x = (raw * 2 + anchor - 0.5) * stride, sigmoid visibility), carried
    through the NMS, ops.scale_coords (unrounded pad, then /gain, clip) and Results'
    Keypoints masking (x, y = 0 where visibility < 0.5; [ext] ultralytics 8.3.205
    engine/results.py)."""
    f32 = np.float32
    cand = []
    aoff = 0
    for hd, s in zip(heads, (8, 16, 32)):
        h, w, _ = hd.shape
        flat = hd.reshape(h * w, -1).astype(f32)
        cls = flat[:, 64:flat.shape[1] - nk]
        j = np.argmax(cls, axis=1)
        best = cls[np.arange(h * w), j]
        score = (1.0 / (1.0 + np.exp(-best.astype(np.float64)))).astype(f32)   # f64, rounded (as the device)
        keep = np.nonzero((j == 0) & (score > f32(conf)))[0]
        for a in keep:
            d = []
            for k in range(4):
                b = flat[a, 16 * k:16 * k + 16]
                e = np.exp((b - b.max()).astype(np.float64)).astype(f32)
                ssum = f32(0.0)
                for v in e:
                    ssum = f32(ssum + v)
                dist = f32(0.0)
                for i in range(16):
                    dist = f32(dist + f32(e[i] / ssum) * f32(i))
                d.append(dist)
            y, x = divmod(int(a), w)
            ax, ay, sf = f32(x) + f32(0.5), f32(y) + f32(0.5), f32(s)
            x1, y1, x2, y2 = f32(ax - d[0]), f32(ay - d[1]), f32(ax + d[2]), f32(ay + d[3])
            cx, cy = f32(f32(f32(x1 + x2) / f32(2)) * sf), f32(f32(f32(y1 + y2) / f32(2)) * sf)
            bw, bh = f32(f32(x2 - x1) * sf), f32(f32(y2 - y1) * sf)
            hw_, hh_ = f32(bw / f32(2)), f32(bh / f32(2))
            kp = None
            if nk:
                raw = flat[a, flat.shape[1] - nk:]
                kp = np.zeros((nk // 3, 3), f32)
                for q in range(nk // 3):
                    kp[q, 0] = f32(f32(f32(raw[3 * q] * f32(2.0)) + f32(x)) * sf)
                    kp[q, 1] = f32(f32(f32(raw[3 * q + 1] * f32(2.0)) + f32(y)) * sf)
                    kp[q, 2] = f32(1.0 / (1.0 + np.exp(-float(raw[3 * q + 2]))))
            cand.append((f32(cx - hw_), f32(cy - hh_), f32(cx + hw_), f32(cy + hh_), score[a], aoff + int(a), kp))
        aoff += h * w
    cand.sort(key=lambda c: (-float(c[4]), c[5]))
    kept = []
    supp = [False] * len(cand)
    for i, ci in enumerate(cand):
        if supp[i]:
            continue
        kept.append(ci)
        if len(kept) >= max_det:
            break
        ai = f32(f32(ci[2] - ci[0]) * f32(ci[3] - ci[1]))
        for jx in range(i + 1, len(cand)):
            if supp[jx]:
                continue
            cj = cand[jx]
            ww = max(f32(min(ci[2], cj[2]) - max(ci[0], cj[0])), f32(0.0))
            hh = max(f32(min(ci[3], cj[3]) - max(ci[1], cj[1])), f32(0.0))
            inter = f32(ww * hh)
            aj = f32(f32(cj[2] - cj[0]) * f32(cj[3] - cj[1]))
            if f32(inter / f32(f32(ai + aj) - inter)) > f32(iou):
                supp[jx] = True
    from person_capture_amd.models_yolo import scale_geometry   # sizing formulas only
    gain, px, py = scale_geometry(Hp, Wp, H0, W0)
    g = f32(gain)
    out = np.zeros((len(kept), 5), f32)
    for r, c in enumerate(kept):
        out[r, 0] = min(max(f32(f32(c[0] - f32(px)) / g), f32(0)), f32(W0))
        out[r, 1] = min(max(f32(f32(c[1] - f32(py)) / g), f32(0)), f32(H0))
        out[r, 2] = min(max(f32(f32(c[2] - f32(px)) / g), f32(0)), f32(W0))
        out[r, 3] = min(max(f32(f32(c[3] - f32(py)) / g), f32(0)), f32(H0))
        out[r, 4] = c[4]
    if not nk:
        return out
    kx, ky = f32((Wp - W0 * gain) / 2), f32((Hp - H0 * gain) / 2)   # scale_coords: pad not rounded
    kpts = np.zeros((len(kept), nk // 3, 3), f32)
    for r, c in enumerate(kept):
        for q in range(nk // 3):
            x = min(max(f32(f32(c[6][q, 0] - kx) / g), f32(0)), f32(W0))
            y = min(max(f32(f32(c[6][q, 1] - ky) / g), f32(0)), f32(H0))
            v = c[6][q, 2]
            if v < f32(0.5):
                x = y = f32(0)
            kpts[r, q] = (x, y, v)
    return out, kpts
