"""Post-match geometry and scoring helpers of the reference's callers:
what main.py / gui_app.py run on an accepted person box before writing the crop.

  clip_to_frame, enforce_scale_and_margins   main.py:17-83 (gui_app.py:3076 is the same rule)
  calc_sharpness                             main.py:86-102: var(Laplacian CV_32F) / (mean^2 + 1e-6) of
                                             the gray crop, INTER_AREA-downscaled to <= 256 on the device
  detect_black_borders                       utils.py:152-197 (gui_app.py:3360 autocrop)
  combine_scores                             main.py:127-144
  index_row / INDEX_HEADER                   main.py:207-209, 344-346 (index.csv format)

BGR -> gray is OpenCV's fixed-point BT.601 (the same formula the device quality kernel uses).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np

from .utils import parse_ratio

INDEX_HEADER = ['frame', 'time_secs', 'score', 'face_dist', 'reid_dist', 'x1', 'y1', 'x2', 'y2', 'crop_path']


def gray_u8(bgr: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(BGR2GRAY) for u8: (B*1868 + G*9617 + R*4899 + 2^13) >> 14."""
    b = bgr[..., 0].astype(np.int32)
    g = bgr[..., 1].astype(np.int32)
    r = bgr[..., 2].astype(np.int32)
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def clip_to_frame(x1, y1, x2, y2, W, H):
    """main.py:17-32: shift the box back inside the frame, then round and clamp."""
    dx1 = -x1 if x1 < 0 else 0.0
    dx2 = W - x2 if x2 > W else 0.0
    dy1 = -y1 if y1 < 0 else 0.0
    dy2 = H - y2 if y2 > H else 0.0
    sx = dx1 if dx1 != 0.0 else (dx2 if dx2 != 0.0 else 0.0)
    sy = dy1 if dy1 != 0.0 else (dy2 if dy2 != 0.0 else 0.0)
    x1 += sx
    x2 += sx
    y1 += sy
    y2 += sy
    x1 = max(0, min(W - 1, int(round(x1))))
    x2 = max(x1 + 1, min(W, int(round(x2))))
    y1 = max(0, min(H - 1, int(round(y1))))
    y2 = max(y1 + 1, min(H, int(round(y2))))
    return x1, y1, x2, y2


def enforce_scale_and_margins(crop_xyxy, ratio_wh, frame_w, frame_h, face_box=None, face_max_frac=0.42,
                              side_margin_frac=0.30, min_h_frac=0.28, min_face_frac=0.18):
    """main.py:35-83: grow the crop so the face is at most face_max_frac of its height with side
    margins, and at least min_h_frac of the frame; shrink it when the face would be smaller than
    min_face_frac."""
    x1, y1, x2, y2 = map(int, crop_xyxy)
    cw, ch = float(x2 - x1), float(y2 - y1)
    try:
        rw, rh = parse_ratio(ratio_wh)
        asp = float(rw) / float(rh)
    except Exception:
        asp = cw / max(ch, 1e-6)
    min_required_h = max(ch, float(min_h_frac) * frame_h)
    max_allowed_h = float("inf")
    if face_box is not None:
        fx1, fy1, fx2, fy2 = face_box
        fw, fh = float(fx2 - fx1), float(fy2 - fy1)
        min_required_h = max(min_required_h, fh / max(face_max_frac, 1e-6),
                             (fw + 2.0 * side_margin_frac * fw) / max(asp, 1e-6))
        if min_face_frac > 0:
            max_allowed_h = min(max_allowed_h, fh / max(min_face_frac, 1e-6))
    if max_allowed_h < min_required_h:
        max_allowed_h = min_required_h
    if ch + 0.5 < min_required_h:
        new_h = min_required_h
    elif ch > max_allowed_h + 0.5:
        new_h = max_allowed_h
    else:
        return x1, y1, x2, y2
    need_w = new_h * asp
    cx = (x1 + x2) / 2.0
    cy = (y1 + y2) / 2.0
    return clip_to_frame(cx - need_w / 2.0, cy - new_h / 2.0, cx + need_w / 2.0, cy + new_h / 2.0, frame_w, frame_h)


def _laplacian_f32(g: np.ndarray) -> np.ndarray:
    """cv2.Laplacian(g, CV_32F) (ksize 1: [0 1 0; 1 -4 1; 0 1 0], BORDER_REFLECT_101): exact integers."""
    p = np.pad(g.astype(np.float32), 1, mode="reflect")
    return (p[1:-1, :-2] + p[1:-1, 2:] + p[:-2, 1:-1] + p[2:, 1:-1] - 4.0 * p[1:-1, 1:-1]).astype(np.float32)


def calc_sharpness(bgr: np.ndarray, ctx=None) -> float:
    """main.py:86-102. A crop larger than 256 px is INTER_AREA-downscaled on the device (ctx: a
    runtime.GpuContext; the gray image goes up as 3 equal channels, which cv2.resize treats
    channel by channel exactly as the single-channel call)."""
    if bgr is None or bgr.size == 0:
        return 0.0
    g = gray_u8(np.ascontiguousarray(bgr))
    h, w = g.shape[:2]
    if max(h, w) > 256:
        if ctx is None:
            raise RuntimeError("calc_sharpness: a crop above 256 px needs the device (pass ctx)")
        from .face_embedder import _DevImage, dev_resize   # cv2.resize dispatch on the device
        scale = 256.0 / float(max(h, w))
        dsize = (int(round(w * scale)), int(round(h * scale)))
        g3 = np.ascontiguousarray(np.repeat(g[..., None], 3, axis=2))
        buf = ctx.scratch("sharp_src", g3.nbytes)
        ctx.upload(g3, buf)
        small = dev_resize(ctx, _DevImage(buf.ptr, h, w, w * 3), "sharp_dst", dsize=dsize, area=True)
        g = ctx.download(small.ptr, (small.H, small.W, 3), np.uint8)[..., 0].copy()
    lap = _laplacian_f32(g)
    variance = float(np.var(lap))
    mean_intensity = float(np.mean(g))
    return variance / (mean_intensity * mean_intensity + 1e-6)


def detect_black_borders(bgr, thr=10, max_scan=None):
    """utils.py:152-197: constant dark borders -> content ROI (x1, y1, x2, y2). Row / column means of
    the gray image are integer sums (exact in float64, so any summation order gives the
    reference's values)."""
    if bgr is None or bgr.size == 0:
        return (0, 0, 0, 0)
    H, W = bgr.shape[:2]
    gray = gray_u8(np.ascontiguousarray(bgr))
    if max_scan is None:
        max_scan = max(64, min(H, W) // 8)
    rows = gray.astype(np.int64).sum(axis=1) / float(W)
    cols = gray.astype(np.int64).sum(axis=0) / float(H)

    def run(vals, idxs):
        n = 0
        for k in idxs:
            if vals[k] > thr:
                break
            n += 1
        return n
    top = run(rows, range(min(H, max_scan)))
    bottom = H - run(rows, range(H - 1, max(H - max_scan - 1, -1), -1))
    left = run(cols, range(min(W, max_scan)))
    right = W - run(cols, range(W - 1, max(W - max_scan - 1, -1), -1))
    clamp = lambda v, lo, hi: max(lo, min(hi, v))
    left = clamp(left, 0, right - 1)
    top = clamp(top, 0, bottom - 1)
    right = clamp(right, left + 1, W)
    bottom = clamp(bottom, top + 1, H)
    return int(left), int(top), int(right), int(bottom)


def combine_scores(face_dist, reid_dist, mode='min'):
    """main.py:127-144."""
    vals = []
    if face_dist is not None:
        vals.append(face_dist)
    if reid_dist is not None:
        vals.append(reid_dist)
    if not vals:
        return None
    if mode == 'min':
        return min(vals)
    if mode == 'avg':
        return sum(vals) / len(vals)
    if mode == 'face_priority':
        if face_dist is not None:
            return 0.7 * face_dist + 0.3 * (reid_dist if reid_dist is not None else 0.5)
        return reid_dist
    return min(vals)


def index_row(frame_idx: int, fps: float, score, fd, rd, box, crop_name: str) -> list:
    """One index.csv row as main.py:344-346 writes it."""
    t = frame_idx / fps
    return [frame_idx, f"{t:.3f}", f"{score:.4f}" if score is not None else "", f"{fd:.4f}" if fd is not None else "",
            f"{rd:.4f}" if rd is not None else "", box[0], box[1], box[2], box[3], crop_name]
