"""CPU oracle of the whole per-frame identity path (test infrastructure only).

frame -> SCRFD letterbox (cv_ops.c) -> SCRFD fp32 forward (nets_torch) ->
decode + NMS (ref_algos) -> _accumulate / min-size / cross-rotation NMS
(face_embedder.py:2214-2443, 0-degree branch) -> crop -> _canon_5pts ->
estimateAffinePartial2D(LMEDS) restated below -> warpAffine (cv_ops.c) ->
quality (Laplacian variance) -> ArcFace fp32 forward with flip-TTA ->
L2 -> _fd_min against a bank.

Used (a) by the end-to-end parity test against the device FaceEmbedder and (b)
as bench.py's cpu_baseline ("port": the same algorithm on the host cores).
Frames on which the 0-degree pass finds no face would enter the TTA / edge-pad /
rotation fallbacks; this oracle reports them as NEEDS_FALLBACK instead.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import cv_ops
from . import nets_torch as nt
from . import ref_algos as ra

NEEDS_FALLBACK = "needs_fallback"


class CvRng:
    """cv::RNG multiply-with-carry (state * 4164903690 + carry), seeded with uint64(-1)."""

    def __init__(self, state: int = 0xFFFFFFFFFFFFFFFF):
        self.state = state & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        self.state = ((self.state & 0xFFFFFFFF) * 4164903690 + (self.state >> 32)) & 0xFFFFFFFFFFFFFFFF
        return self.state & 0xFFFFFFFF

    def uniform(self, a: int, b: int) -> int:
        return a if a == b else self.next() % (b - a) + a


def _similarity_2pt(f, t) -> np.ndarray:
    """AffinePartial2DEstimatorCallback::runKernel (2 points, closed form, double)."""
    x1, y1, x2, y2 = float(f[0][0]), float(f[0][1]), float(f[1][0]), float(f[1][1])
    X1, Y1, X2, Y2 = float(t[0][0]), float(t[0][1]), float(t[1][0]), float(t[1][1])
    with np.errstate(all="ignore"):   # IEEE semantics (a coincident pair gives inf/nan, as in C)
        d = float(np.float64(1.0) / np.float64((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2)))
    S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2))
    S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2))
    S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2))
    S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2))
    return np.array([S0, -S1, S2, S1, S0, S3], dtype=np.float64)


def _errors(src, dst, H) -> np.ndarray:
    h = H.astype(np.float32)
    f32 = np.float32
    out = np.empty(len(src), np.float32)
    with np.errstate(all="ignore"):
        for i in range(len(src)):
            fx, fy = f32(src[i][0]), f32(src[i][1])
            a = h[0] * fx + h[1] * fy + h[2] - f32(dst[i][0])
            b = h[3] * fx + h[4] * fy + h[5] - f32(dst[i][1])
            out[i] = a * a + b * b
    return out


def estimate_affine_partial_lmeds(src, dst) -> Optional[np.ndarray]:
    """cv2.estimateAffinePartial2D(src, dst, method=cv2.LMEDS) as used at face_embedder.py:1466:
    13 LMeDS iterations on random 2-point subsets, median residual, inlier set, then the
    least-squares similarity over the inliers (the fixed point of the LM refinement)."""
    src = np.asarray(src, np.float32)
    dst = np.asarray(dst, np.float32)
    n = len(src)
    if n < 2:
        return None
    if n == 2:
        return _similarity_2pt(src, dst).reshape(2, 3)
    niters = max(int(round(math.log(1 - 0.99) / math.log(1 - (1 - 0.45) ** 2))), 3)
    rng = CvRng()
    best, best_med = None, float("inf")
    for _ in range(niters):
        idx = []
        for i in range(2):
            while True:
                k = rng.uniform(0, n)
                if k not in idx:
                    break
            idx.append(k)
        H = _similarity_2pt(src[idx], dst[idx])
        err = _errors(src, dst, H)
        # OpenCV takes the median with nth_element over the residuals' int32 bit patterns
        med = float(np.sort(err.view(np.int32))[n // 2].view(np.float32))
        if med < best_med:
            best_med, best = med, H
    if best is None:
        return None
    if not best_med < float("inf"):
        return None
    sigma = max(2.5 * 1.4826 * (1 + 5.0 / (n - 2)) * math.sqrt(best_med), 0.001)
    err = _errors(src, dst, best)
    inl = [i for i in range(n) if err[i] <= np.float32(sigma * sigma)]
    if len(inl) < 2:
        return None
    p = src[inl].astype(np.float64)
    q = dst[inl].astype(np.float64)
    mx, my = p[:, 0].sum() / len(inl), p[:, 1].sum() / len(inl)
    nx, ny = q[:, 0].sum() / len(inl), q[:, 1].sum() / len(inl)
    sxx = sa = sb = 0.0
    for (px, py), (qx, qy) in zip(p, q):
        px, py, qx, qy = px - mx, py - my, qx - nx, qy - ny
        sxx += px * px + py * py
        sa += px * qx + py * qy
        sb += px * qy - py * qx
    if sxx <= 0:
        return best.reshape(2, 3)
    a, b = sa / sxx, sb / sxx
    return np.array([[a, -b, nx - (a * mx - b * my)], [b, a, ny - (b * mx + a * my)]], dtype=np.float64)


def align_chip(face_bgr: np.ndarray, canon5: np.ndarray) -> np.ndarray:
    """FaceEmbedder._align_by_5pts (face_embedder.py:1465-1473)."""
    M = estimate_affine_partial_lmeds(canon5, ra.ARC_DST)
    if M is None:
        M = estimate_affine_partial_lmeds(canon5[:3], ra.ARC_DST[:3])
    if M is None:
        raise NotImplementedError("resize fallback")
    return cv_ops.warp_affine(face_bgr, M.reshape(-1), 112, 112, border=2)


def detect_0deg(frame: np.ndarray, scrfd_params, variant: str, conf: float, D: int):
    H0, W0 = frame.shape[:2]
    nw, nh, ds = ra.scrfd_letterbox_geometry(H0, W0, D)
    sx, sy = 1.0 / (float(nw) / W0), 1.0 / (float(nh) / H0)
    simd_end = (nw * 3 // 16) * 16 if nw * 3 >= 16 else 0
    while simd_end < nw * 3 - 8:
        simd_end += 8
    blob = cv_ops.letterbox_blob(frame, D, nw, nh, sx, sy, simd_end)
    t = torch.from_numpy(np.ascontiguousarray(blob[None, ..., :3].transpose(0, 3, 1, 2)))
    heads = [h[0].numpy() for h in nt.scrfd_forward(scrfd_params, variant, t)]
    return ra.scrfd_detect_post(heads, conf, ds)


def extract_frame(frame: np.ndarray, scrfd_params, variant: str, arc_params, depth: int, conf: float = 0.5,
                  D: int = 640, bank: Optional[np.ndarray] = None, flip: bool = True):
    """One FaceEmbedder.extract(frame) of the SCRFD+ArcFace branch, 0-degree pass only."""
    H0, W0 = frame.shape[:2]
    det, kps = detect_0deg(frame, scrfd_params, variant, conf, D)
    dets = []
    for bb, kp in zip(det, kps):
        x1, y1, x2, y2 = [int(v) for v in bb[:4]]
        xa1, ya1 = max(0, min(W0 - 1, min(x1, x2))), max(0, min(H0 - 1, min(y1, y2)))
        xa2, ya2 = max(xa1 + 1, min(W0, max(x1, x2))), max(ya1 + 1, min(H0, max(y1, y2)))
        if xa2 - xa1 <= 2 or ya2 - ya1 <= 2:
            continue
        pts = np.asarray([[float(px) - xa1, float(py) - ya1] for (px, py) in np.asarray(kp, np.float32).reshape(-1, 2)],
                         np.float32)[:5]
        dets.append(((xa1, ya1, xa2, ya2), pts, float(bb[4])))
    dets = [d for d in dets if d[0][2] - d[0][0] >= 8 and d[0][3] - d[0][1] >= 8]
    if not dets:
        return NEEDS_FALLBACK
    dets.sort(key=lambda t: (t[2], (t[0][2] - t[0][0]) * (t[0][3] - t[0][1])), reverse=True)
    kept = []
    for d in dets:
        if all(ra.iou(d[0], k[0]) < 0.45 for k in kept):
            kept.append(d)
    chips, boxes, kps5 = [], [], []
    for (x1, y1, x2, y2), pts, _ in kept:
        face = frame[y1:y2, x1:x2]
        canon = ra.canon_5pts(pts)
        if canon is None:
            raise NotImplementedError("eye-roll fallback")
        chips.append(align_chip(face, canon))
        boxes.append((x1, y1, x2, y2))
        kps5.append(pts)
    chips = np.stack(chips)
    q = [cv_ops.face_quality(c) for c in chips]
    e = nt.iresnet_forward(arc_params, depth, nt.arcface_input_from_chips(chips)).numpy()
    ef = nt.iresnet_forward(arc_params, depth, nt.arcface_input_from_chips(chips[:, :, ::-1])).numpy() if flip else None
    feats = ra.arcface_postprocess(e, ef)
    out = []
    for i, b in enumerate(boxes):
        f = {"bbox": np.array(b, np.int32), "feat": feats[i], "quality": float(q[i]), "chip": chips[i],
             "kps5": kps5[i]}
        if bank is not None:
            f["fd"] = ra.fd_min(feats[i], bank)
        out.append(f)
    out.sort(key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])),
             reverse=True)
    return out
