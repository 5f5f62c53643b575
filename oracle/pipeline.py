"""CPU oracle of the whole per-frame identity path (test infrastructure only).

frame -> SCRFD letterbox (cv_ops.c) -> SCRFD fp32 forward (nets_torch) ->
decode + NMS (ref_algos) -> _accumulate / min-size / cross-rotation NMS
(face_embedder.py:2214-2443, 0-degree branch) -> crop -> _canon_5pts ->
estimateAffinePartial2D(LMEDS) restated below -> warpAffine (cv_ops.c) ->
quality (Laplacian variance) -> ArcFace fp32 forward with flip-TTA ->
L2 -> _fd_min against a bank.

Used (a) by the end-to-end parity test against the device FaceEmbedder and (b)
as bench.py's cpu_baseline ("port": the same algorithm on the host cores).
extract_frame is the 0-degree pass alone (frames on which it finds no face are reported
as NEEDS_FALLBACK); OracleFaceEmbedder below restates the whole branch: TTA scales,
edge replicate-pad, rotations with their gating state, eye-roll and resize fallbacks.
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
        dets.append(((xa1, ya1, xa2, ya2), pts, float(bb[4]), np.asarray(bb[:4], np.float64)))
    dets = [d for d in dets if d[0][2] - d[0][0] >= 8 and d[0][3] - d[0][1] >= 8]
    if not dets:
        return NEEDS_FALLBACK
    dets.sort(key=lambda t: (t[2], (t[0][2] - t[0][0]) * (t[0][3] - t[0][1])), reverse=True)
    kept = []
    for d in dets:
        if all(ra.iou(d[0], k[0]) < 0.45 for k in kept):
            kept.append(d)
    chips, boxes, kps5, boxes_f = [], [], [], []
    for (x1, y1, x2, y2), pts, _, bf in kept:
        face = frame[y1:y2, x1:x2]
        canon = ra.canon_5pts(pts)
        if canon is None:
            raise NotImplementedError("eye-roll fallback")
        chips.append(align_chip(face, canon))
        boxes.append((x1, y1, x2, y2))
        boxes_f.append(bf)
        kps5.append(pts)
    chips = np.stack(chips)
    q = [cv_ops.face_quality(c) for c in chips]
    e = nt.iresnet_forward(arc_params, depth, nt.arcface_input_from_chips(chips)).numpy()
    ef = nt.iresnet_forward(arc_params, depth, nt.arcface_input_from_chips(chips[:, :, ::-1])).numpy() if flip else None
    feats = ra.arcface_postprocess(e, ef)
    out = []
    for i, b in enumerate(boxes):
        # bbox_f: the detector's float box before the int() of _accumulate (face_embedder.py:2214-2239)
        f = {"bbox": np.array(b, np.int32), "feat": feats[i], "quality": float(q[i]), "chip": chips[i],
             "kps5": kps5[i], "bbox_f": boxes_f[i]}
        if bank is not None:
            f["fd"] = ra.fd_min(feats[i], bank)
        out.append(f)
    out.sort(key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])),
             reverse=True)
    return out


# ---------------------------------------------------------------------------
# The whole SCRFD branch with its fallbacks and per-instance state
# ---------------------------------------------------------------------------
def _round32(x: int) -> int:
    """face_embedder.py:86-87."""
    return ((int(x) + 31) // 32) * 32


def rotate(img: np.ndarray, deg: int) -> np.ndarray:
    """cv2.rotate (face_embedder.py:2165-2169): 90 = ROTATE_90_CLOCKWISE, 270 = COUNTERCLOCKWISE."""
    if deg == 90:
        return np.ascontiguousarray(np.rot90(img, -1))
    if deg == 180:
        return np.ascontiguousarray(img[::-1, ::-1])
    if deg == 270:
        return np.ascontiguousarray(np.rot90(img, 1))
    return img


def pad_replicate(img: np.ndarray, pad: int) -> np.ndarray:
    """cv2.copyMakeBorder(img, pad, pad, pad, pad, BORDER_REPLICATE)."""
    return np.pad(img, ((pad, pad), (pad, pad), (0, 0)), mode="edge")


def resize_for_arc(img: np.ndarray) -> np.ndarray:
    """cv2.resize(img, (112, 112), INTER_AREA if max(h, w) > 112 else INTER_LINEAR)
    (face_embedder.py:1579-1582, 2458-2460)."""
    h, w = img.shape[:2]
    return cv_ops.resize(img, (112, 112), interpolation=cv_ops.INTER_AREA if max(h, w) > 112 else cv_ops.INTER_LINEAR)


def align_by_5pts(bgr: np.ndarray, canon5: np.ndarray) -> np.ndarray:
    """FaceEmbedder._align_by_5pts (face_embedder.py:1465-1473) with its resize fallback."""
    M = estimate_affine_partial_lmeds(canon5, ra.ARC_DST)
    if M is None:
        M = estimate_affine_partial_lmeds(canon5[:3], ra.ARC_DST[:3])
    if M is None:
        return resize_for_arc(bgr)
    return cv_ops.warp_affine(bgr, M.reshape(-1), 112, 112, border=2)


def rotation_matrix_2d(cx: float, cy: float, angle_deg: float, scale: float) -> np.ndarray:
    """cv2.getRotationMatrix2D(center, angle, scale), double math (center as float32 Point2f)."""
    cx, cy = float(np.float32(cx)), float(np.float32(cy))
    a = angle_deg * (math.pi / 180.0)   # OpenCV: angle *= CV_PI/180
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                     [-beta, alpha, beta * cx + (1 - alpha) * cy]], dtype=np.float64)


def upright_by_eye_roll(bgr: np.ndarray, pts5, trace: Optional[list] = None) -> np.ndarray:
    """FaceEmbedder._upright_by_eye_roll (face_embedder.py:1571-1647); `trace` collects which
    exit was taken (resize / rotate+align / rotate+resize)."""
    trace = [] if trace is None else trace
    h, w = bgr.shape[:2]
    pts = np.asarray(pts5, dtype=np.float32)
    if pts.ndim != 2 or pts.shape[0] < 5 or pts.shape[1] < 2 or not np.isfinite(pts[:5, :2]).all():
        trace.append("roll_resize")
        return resize_for_arc(bgr)
    coords = pts[:5, :2].copy()
    coords[:, 0] = np.clip(coords[:, 0], 0.0, max(0, w - 1))
    coords[:, 1] = np.clip(coords[:, 1], 0.0, max(0, h - 1))
    vec = coords[1] - coords[0]
    if float(np.hypot(vec[0], vec[1])) < 1e-3:
        vec = coords[4] - coords[3]
        if float(np.hypot(vec[0], vec[1])) < 1e-3:
            trace.append("roll_resize")
        return resize_for_arc(bgr)
    angle = math.degrees(math.atan2(float(vec[1]), float(vec[0])))
    if angle < -90.0:
        angle += 180.0
    elif angle > 90.0:
        angle -= 180.0
    if abs(angle) < 8.0:
        trace.append("roll_resize")
        return resize_for_arc(bgr)
    if angle > 80.0:
        angle = 90.0
    elif angle < -80.0:
        angle = -90.0
    best_side = max(h, w)
    scale = 1.0 if best_side <= 256 else 256.0 / float(best_side)
    M = rotation_matrix_2d(w / 2.0, h / 2.0, -angle, scale)
    rotated = cv_ops.warp_affine(bgr, M.reshape(-1), w, h, border=2)
    pts_h = np.hstack([pts[:5, :2], np.ones((5, 1), dtype=np.float32)])
    pts_rot = (M @ pts_h.T).T.astype(np.float32)
    canon = ra.canon_5pts(pts_rot)
    if canon is not None:
        trace.append("roll_align")
        return align_by_5pts(rotated, canon.astype(np.float32))
    trace.append("roll_rot_resize")
    return resize_for_arc(rotated)


class OracleFaceEmbedder:
    """CPU restatement of FaceEmbedder's SCRFD branch with every fallback and the
    per-instance state that steers them (face_embedder.py:2095-2482): det-size policy
    (:2189-2208), 0-degree pass, TTA scales + edge replicate-pad probes (:2251-2315),
    min-size filter (:2317-2322), rotation gating (:2330-2360), rotated probe/heavy
    passes (:2362-2433), cross-rotation NMS (:2438-2443), crop/canon/align with the
    eye-roll and resize fallbacks (:2445-2460, 1465-1473, 1571-1647), quality, ArcFace
    flip-TTA (:1295) and _fd_min. `rot_phase` stands in for the reference's
    `id(self) & 7` term of the periodic rotation probe (pass the device instance's value).
    Attribute names and defaults are the reference's (:473-497)."""

    def __init__(self, scrfd_params, variant: str, arc_params, depth: int, conf: float = 0.5,
                 rot_phase: int = 0):
        self.p_s, self.variant, self.p_a, self.depth = scrfd_params, variant, arc_params, depth
        self.conf = float(conf)
        self.rot_phase = int(rot_phase)
        self.scrfd_tta_scales = (0.75, 0.60)
        self.scrfd_probe_conf_cap = 0.20
        self.scrfd_edge_pad_frac = 0.06
        self.scrfd_min_box_px = 8
        self._fast_prescan = False
        self._prescan_rr = 0
        self._prescan_rr_mode = "rr"
        self._prescan_escalate = False
        self._probe_conf = 0.03
        self._high_90 = 1536
        self._high_180 = 1280
        self._prescan_period = 3
        self._prescan_probe_imgsz = 384
        self._prescan_no_upscale_det = True
        self._heavy_cap = 2048
        self._frame_idx = 0
        self._no_face_streak = 0
        self._last_face_idx = -10 ** 9
        self._rot_cycle = 0
        self.rot_adaptive = True
        self.rot_every_n = 12
        self.rot_after_hit_frames = 8
        self.fast_no_face_imgsz = 512
        self.trace: List[str] = []      # branches taken by the last extract (tests assert coverage)

    def state(self) -> tuple:
        return (self._frame_idx, self._no_face_streak, self._last_face_idx, self._rot_cycle, self._prescan_rr)

    def detect(self, img: np.ndarray, D: int, conf: float):
        self.trace.append(f"detect{D}")
        return detect_0deg(img, self.p_s, self.variant, conf, D)

    def extract(self, bgr: np.ndarray, *, imgsz: Optional[int] = None, bank: Optional[np.ndarray] = None,
                keep_chips: bool = True):
        """FaceEmbedder.extract (face_embedder.py:1663-1669 -> 2095-2103 -> 2163-2482)."""
        if bgr is None or bgr.size == 0:
            return []
        self._frame_idx += 1
        self.trace = []
        H0, W0 = bgr.shape[:2]
        dyn = int(imgsz) if (imgsz is not None and imgsz > 0) else 640
        if self._no_face_streak >= 3:
            dyn = min(dyn, self.fast_no_face_imgsz)
        if self._fast_prescan:
            dyn = min(dyn, int(self._prescan_probe_imgsz))
            if self._prescan_no_upscale_det:
                dyn = min(dyn, max(320, (max(H0, W0) // 32) * 32))
        dyn = _round32(max(320, dyn))
        L = max(H0, W0)
        heavy_cap = max(int(self._heavy_cap), dyn)
        heavy90 = min(_round32(max(dyn, int(0.75 * L))), heavy_cap)
        heavy180 = min(_round32(max(dyn, int(0.67 * L))), heavy_cap)
        dets = []

        def mapxy(xr, yr, deg):
            if deg == 90:
                return yr, H0 - 1 - xr
            if deg == 180:
                return W0 - 1 - xr, H0 - 1 - yr
            if deg == 270:
                return W0 - 1 - yr, xr
            return xr, yr

        def accumulate(bb, kp, deg):
            x1, y1, x2, y2 = [int(v) for v in bb[:4]]
            x1o, y1o = mapxy(x1, y1, deg)
            x2o, y2o = mapxy(x2, y2, deg)
            xa1, ya1 = min(x1o, x2o), min(y1o, y2o)
            xa2, ya2 = max(x1o, x2o), max(y1o, y2o)
            xa1 = max(0, min(W0 - 1, xa1)); ya1 = max(0, min(H0 - 1, ya1))
            xa2 = max(xa1 + 1, min(W0, xa2)); ya2 = max(ya1 + 1, min(H0, ya2))
            if xa2 - xa1 <= 2 or ya2 - ya1 <= 2:
                return
            pts = None
            if kp is not None:
                m = []
                for (px, py) in np.asarray(kp, dtype=np.float32).reshape(-1, 2):
                    ox, oy = mapxy(float(px), float(py), deg)
                    m.append([float(ox - xa1), float(oy - ya1)])
                pts = np.asarray(m[:5], dtype=np.float32) if len(m) >= 5 else None
            dets.append(((xa1, ya1, xa2, ya2), pts, float(bb[4]) if len(bb) > 4 else 1.0))

        bboxes, kpss = self.detect(bgr, dyn, self.conf)
        for i, bb in enumerate(bboxes):
            accumulate(bb, None if kpss is None or i >= len(kpss) else kpss[i], 0)
        if not dets and not self._fast_prescan:
            tta = tuple(self.scrfd_tta_scales) + ((1.25,) if max(W0, H0) <= 1920 else ())
            probe_conf = min(float(self.conf), float(self.scrfd_probe_conf_cap))
            for s in tta:
                if s == 1.0:
                    continue
                self.trace.append(f"tta{s}")
                img_s = cv_ops.resize(bgr, None, fx=s, fy=s,
                                      interpolation=cv_ops.INTER_AREA if s < 1.0 else cv_ops.INTER_LINEAR)
                dyn_s = _round32(min(self._heavy_cap, max(320, int(dyn * s))))
                bb_s, kp_s = self.detect(img_s, dyn_s, probe_conf)
                if len(bb_s) == 0:
                    continue
                inv = 1.0 / s
                for i, bb in enumerate(bb_s):
                    kp = kp_s[i] if i < len(kp_s) else None
                    bb = np.asarray(bb).copy()
                    bb[:4] = np.asarray(bb[:4], dtype=np.float32) * inv
                    if kp is not None:
                        kp = np.asarray(kp, dtype=np.float32) * inv
                    accumulate(bb, kp, 0)
                if dets:
                    break
            if not dets:
                pad = int(round(min(64, float(self.scrfd_edge_pad_frac) * max(W0, H0))))
                if pad > 0:
                    self.trace.append("edgepad")
                    bb_p, kp_p = self.detect(pad_replicate(bgr, pad), dyn, probe_conf)
                    for i, bb in enumerate(bb_p):
                        kp = kp_p[i] if i < len(kp_p) else None
                        bb = np.asarray(bb).copy()
                        bb[:4] -= np.array([pad, pad, pad, pad], dtype=np.float32)
                        bb[0] = max(0.0, min(float(W0 - 1), float(bb[0])))
                        bb[1] = max(0.0, min(float(H0 - 1), float(bb[1])))
                        bb[2] = max(bb[0] + 1.0, min(float(W0), float(bb[2])))
                        bb[3] = max(bb[1] + 1.0, min(float(H0), float(bb[3])))
                        if kp is not None:
                            kp = np.asarray(kp, dtype=np.float32).copy()
                            kp[..., 0] = np.clip(kp[..., 0] - pad, 0, W0 - 1)
                            kp[..., 1] = np.clip(kp[..., 1] - pad, 0, H0 - 1)
                        accumulate(bb, kp, 0)
        min_px = int(self.scrfd_min_box_px)
        dets = [d for d in dets if d[0][2] - d[0][0] >= min_px and d[0][3] - d[0][1] >= min_px]
        if not dets:
            need_rot = False
            self._no_face_streak += 1
            if self.rot_adaptive:
                if (self._frame_idx - self._last_face_idx) <= self.rot_after_hit_frames:
                    need_rot = True
                elif ((self._frame_idx + self.rot_phase) % self.rot_every_n) == 0:
                    need_rot = True
            else:
                need_rot = True
        else:
            need_rot = False
            self._no_face_streak = 0
            self._last_face_idx = self._frame_idx
            self._rot_cycle = 0
        if self._fast_prescan:
            if dets:
                need_rot = False
            else:
                period = max(1, int(self._prescan_period))
                need_rot = need_rot or self._prescan_escalate or (((self._frame_idx + self._prescan_rr) % period) == 0)
        if self._fast_prescan and not dets and not need_rot:
            return []
        if not dets and need_rot:
            self._rot_cycle += 1
            if self._fast_prescan:
                rr = self._prescan_rr % 2
                if self._prescan_rr_mode == "rr":
                    rot_seq = ((90, 270)[rr],)
                    self._prescan_rr += 1
                else:
                    rot_seq = (90, 270)
            else:
                rot_seq = (90, 270, 180)
            for deg in rot_seq:
                self.trace.append(f"rot{deg}")
                rimg_probe = rotate(bgr, deg)
                probe_conf = max(0.02, float(self._probe_conf))
                probe_dyn = _round32(max(320, min(dyn, int(self._prescan_probe_imgsz))))
                probe_boxes, _ = self.detect(rimg_probe, probe_dyn, probe_conf)
                probe_hits = len(probe_boxes)
                do_heavy = probe_hits > 0 or (self._fast_prescan and self._prescan_escalate) or not self._fast_prescan
                if self._fast_prescan and probe_hits == 0:
                    continue
                pad = 24
                rimg = pad_replicate(rimg_probe, pad)
                if self._fast_prescan:
                    heavy = heavy180 if deg == 180 else heavy90
                    override = self._high_180 if deg == 180 else self._high_90
                    if override and override > 0:
                        heavy = max(heavy, _round32(int(override)))
                    heavy = min(heavy, int(self._heavy_cap))
                    det_sizes = [dyn] if not do_heavy else [heavy]
                else:
                    det_sizes = []
                    for base in (max(dyn, 1280), max(dyn, 1536)):
                        base = _round32(base)
                        if base not in det_sizes:
                            det_sizes.append(base)
                    det_sizes = det_sizes if do_heavy else [dyn]
                conf_deg = max(0.10, float(self.conf) * (0.8 if deg in (90, 270) else 0.6))
                rb = rk = None
                for det_size in det_sizes:
                    rb, rk = self.detect(rimg, det_size, conf_deg)
                    if len(rb) > 0:
                        break
                    rb = rk = None
                if rb is None or len(rb) == 0:
                    continue
                for i, bb in enumerate(rb):
                    kp = rk[i] if i < len(rk) else None
                    bb = np.asarray(bb).copy()
                    bb[:4] -= np.array([pad, pad, pad, pad], dtype=bb.dtype)
                    if kp is not None:
                        kp = np.asarray(kp).copy()
                        kp[..., 0] -= pad
                        kp[..., 1] -= pad
                    accumulate(bb, kp, deg)
                if dets:
                    break
        if not dets:
            return []
        dets = sorted(dets, key=lambda t: (t[2], (t[0][2] - t[0][0]) * (t[0][3] - t[0][1])), reverse=True)
        kept = []
        for d in dets:
            if all(ra.iou(d[0], k[0]) < 0.45 for k in kept):
                kept.append(d)
        faces, chips = [], []
        for (x1, y1, x2, y2), kps, _sc in kept:
            xi1 = max(0, min(W0 - 1, int(round(x1))))
            yi1 = max(0, min(H0 - 1, int(round(y1))))
            xi2 = max(xi1 + 1, min(W0, int(round(x2))))
            yi2 = max(yi1 + 1, min(H0, int(round(y2))))
            face = bgr[yi1:yi2, xi1:xi2]
            chip = None
            if kps is not None:
                pts = np.asarray(kps, dtype=np.float32)
                canon = ra.canon_5pts(pts)
                if canon is not None:
                    chip = align_by_5pts(face, canon)
                else:
                    self.trace.append("eyeroll")
                    chip = upright_by_eye_roll(face, pts, self.trace)
            if chip is None:
                self.trace.append("resize")
                chip = resize_for_arc(face)
            faces.append(((xi1, yi1, xi2, yi2), kps))
            chips.append(chip)
        chips = np.stack(chips)
        q = [cv_ops.face_quality(c) for c in chips]
        flip = (not self._fast_prescan) or self._prescan_escalate
        e = nt.iresnet_forward(self.p_a, self.depth, nt.arcface_input_from_chips(chips)).numpy()
        ef = nt.iresnet_forward(self.p_a, self.depth, nt.arcface_input_from_chips(chips[:, :, ::-1])).numpy() \
            if flip else None
        feats = ra.arcface_postprocess(e, ef)
        out = []
        for i, (b, kps) in enumerate(faces):
            f = {"bbox": np.array(b, np.int32), "feat": feats[i], "quality": float(q[i])}
            if keep_chips:
                f["chip"], f["kps5"] = chips[i], kps
            if bank is not None:
                f["fd"] = ra.fd_min(feats[i], bank)
            out.append(f)
        out.sort(key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])),
                 reverse=True)
        return out


def chip_for(face_bgr: np.ndarray, kps) -> np.ndarray:
    """The chip decision of face_embedder.py:2453-2460 for one face crop: canonical
    landmarks -> _align_by_5pts, else _upright_by_eye_roll; no landmarks -> resize."""
    if kps is not None:
        pts = np.asarray(kps, dtype=np.float32)
        canon = ra.canon_5pts(pts)
        return align_by_5pts(face_bgr, canon) if canon is not None else upright_by_eye_roll(face_bgr, pts)
    return resize_for_arc(face_bgr)
