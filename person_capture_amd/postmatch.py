"""Post-match geometry and scoring helpers of the reference's callers:
what main.py / gui_app.py run on an accepted person box before writing the crop.

  clip_to_frame, enforce_scale_and_margins   main.py:17-83 (gui_app.py:3076 is the same rule)
  calc_sharpness                             main.py:86-102: var(Laplacian CV_32F) / (mean^2 + 1e-6) of
                                             the gray crop, INTER_AREA-downscaled to <= 256 on the device
  detect_black_borders                       utils.py:152-197 (gui_app.py:3360 autocrop)
  combine_scores                             main.py:127-144
  index_row / INDEX_HEADER                   main.py:207-209, 344-346 (index.csv format)
  debug_record / DebugLog                    gui_app.py:8013-8057, 4459-4470: the per-frame debug.jsonl line
  choose_best_ratio, head_proxy_box          gui_app.py:3147-3328, 1931-1962: the GUI's crop-ratio
                                             scorer (area, placement, face-fraction templates, head
                                             containment), SessionConfig defaults in CropScoreConfig

BGR -> gray is OpenCV's fixed-point BT.601 (the same formula the device quality kernel uses).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from .utils import expand_box_to_ratio, parse_ratio

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


@dataclass
class CropScoreConfig:
    """The SessionConfig fields the crop-ratio scorer reads, with their defaults
    (gui_app.py:431-492)."""
    crop_face_side_margin_frac: float = 0.30
    crop_top_headroom_max_frac: float = 0.15
    tight_face_relax_thresh: float = 0.48
    tight_face_relax_scale: float = 0.5
    crop_bottom_min_face_heights: float = 1.5
    crop_center_weight: float = 0.8
    face_anchor_down_frac: float = 1.1
    area_gamma: float = 0.60
    crop_penalty_weight: float = 3.0
    area_face_scale_weight: float = 0.70
    face_target_close_min_frac: float = 0.10
    face_target_upper: float = 0.20
    w_upper: float = 1.00
    face_target_cowboy: float = 0.08
    w_cowboy: float = 0.70
    face_target_body: float = 0.03
    w_body: float = 0.50
    face_target_close: float = 0.38
    w_close: float = 1.10
    face_target_tolerance: float = 0.04
    lambda_facefrac: float = 2.0
    square_pull_face_min: float = 0.16
    square_pull_weight: float = 1.10
    wide_face_min_frame_frac: float = 0.12
    wide_face_aspect_limit: float = 1.05
    wide_face_aspect_penalty_weight: float = 10.0
    crop_head_side_pad_frac: float = 0.88
    crop_head_top_pad_frac: float = 0.95
    crop_head_bottom_pad_frac: float = 0.30


def head_proxy_box(face_box, frame_w, frame_h, cfg: CropScoreConfig):
    """gui_app.py:1931-1962: the face box padded to protect hair/forehead/chin (None if degenerate)."""
    if face_box is None:
        return None
    try:
        fx1, fy1, fx2, fy2 = [float(v) for v in face_box]
    except (TypeError, ValueError):
        return None
    fw, fh = max(1.0, fx2 - fx1), max(1.0, fy2 - fy1)
    side = max(0.0, float(cfg.crop_head_side_pad_frac)) * fw
    hx1, hy1 = max(0.0, fx1 - side), max(0.0, fy1 - max(0.0, float(cfg.crop_head_top_pad_frac)) * fh)
    hx2 = min(float(frame_w), fx2 + side)
    hy2 = min(float(frame_h), fy2 + max(0.0, float(cfg.crop_head_bottom_pad_frac)) * fh)
    if hx2 <= hx1 + 1.0 or hy2 <= hy1 + 1.0:
        return None
    return hx1, hy1, hx2, hy2


def _placement_penalty(crop, face, cfg: CropScoreConfig) -> float:
    """Side-margin deficit + excess headroom + missing torso + face off-centre (gui_app.py:3163-3191)."""
    if face is None:
        return 0.0
    cx1, cy1, cx2, cy2 = crop
    fx1, fy1, fx2, fy2 = face
    cw, ch = max(1.0, cx2 - cx1), max(1.0, cy2 - cy1)
    fw, fh = max(1.0, fx2 - fx1), max(1.0, fy2 - fy1)
    left, right = max(0.0, fx1 - cx1), max(0.0, cx2 - fx2)
    top, bottom = max(0.0, fy1 - cy1), max(0.0, cy2 - fy2)
    side_def = max(0.0, float(cfg.crop_face_side_margin_frac) * fw - min(left, right)) / fw
    head_def = max(0.0, top / ch - float(cfg.crop_top_headroom_max_frac))
    relax = float(cfg.tight_face_relax_scale) if (fh / ch) >= float(cfg.tight_face_relax_thresh) else 1.0
    bottom_def = max(0.0, float(cfg.crop_bottom_min_face_heights) * fh * relax - bottom) / fh
    center_def = math.hypot((0.5 * (fx1 + fx2) - 0.5 * (cx1 + cx2)) / cw, (0.5 * (fy1 + fy2) - 0.5 * (cy1 + cy2)) / ch)
    return side_def + head_def + bottom_def + float(cfg.crop_center_weight) * center_def


def _huber(x: float, delta: float) -> float:
    ax = abs(x)
    return 0.5 * ax * ax if ax <= delta else delta * (ax - 0.5 * delta)


def _containment_deficit(crop, protect, margin_px: float = 0.0) -> float:
    """How far (in protect-box widths/heights) the crop cuts into the protected box (gui_app.py:3197-3207)."""
    if protect is None:
        return 0.0
    cx1, cy1, cx2, cy2 = crop
    px1, py1, px2, py2 = protect
    m = max(0.0, float(margin_px))
    dx = max(0.0, (cx1 + m) - px1) + max(0.0, px2 - (cx2 - m))
    dy = max(0.0, (cy1 + m) - py1) + max(0.0, py2 - (cy2 - m))
    return dx / max(1.0, px2 - px1) + dy / max(1.0, py2 - py1)


def _ratio_score(det_box, rw, rh, frame_w, frame_h, anchor, face_box, head_box, cfg: CropScoreConfig):
    """Score of one candidate ratio (lower wins) -> (score, expanded box, template loss)."""
    x1, y1, x2, y2 = det_box
    hb = 0.0
    if face_box is not None:   # push the framing down by ~face_anchor_down_frac face heights
        hb = -float(cfg.face_anchor_down_frac) * (max(1.0, face_box[3] - face_box[1]) / max(1.0, y2 - y1))
    box = expand_box_to_ratio(x1, y1, x2, y2, rw, rh, frame_w, frame_h, anchor=anchor, head_bias=hb)
    ex1, ey1, ex2, ey2 = box
    area = max(1, (ex2 - ex1) * (ey2 - ey1))
    area_term = pow(float(area) / float(max(1, (x2 - x1) * (y2 - y1))), float(cfg.area_gamma))
    total = area_term + float(cfg.crop_penalty_weight) * _placement_penalty(box, face_box, cfg)
    if head_box is not None:   # graded, very large: no candidate may cut the visible head
        total += 1.0e6 * _containment_deficit(box, head_box, margin_px=1.0)
    tmpl = 0.0
    if face_box is not None:
        fx1, fy1, fx2, fy2 = face_box
        fw, fh = max(1.0, fx2 - fx1), max(1.0, fy2 - fy1)
        face_frac = max(1.0, (fx2 - fx1) * (fy2 - fy1)) / max(1.0, float(area))
        if min(max(0.0, fx1 - ex1), max(0.0, ex2 - fx2)) < float(cfg.crop_face_side_margin_frac) * fw:
            total += 1e9   # hard side guard: this ratio would cut the face
        face_scale = max(fw / max(1.0, frame_w), fh / max(1.0, frame_h))
        total += (max(0.30, 1.0 - float(cfg.area_face_scale_weight) * face_scale) - 1.0) * area_term
        targets = [(cfg.face_target_upper, cfg.w_upper), (cfg.face_target_cowboy, cfg.w_cowboy),
                   (cfg.face_target_body, cfg.w_body)]
        if face_scale >= float(cfg.face_target_close_min_frac):
            targets.append((cfg.face_target_close, cfg.w_close))
        delta = float(cfg.face_target_tolerance)
        tmpl = min(float(w) * _huber(face_frac - float(t), delta) for t, w in targets)
        total += float(cfg.lambda_facefrac) * tmpl
        asp = float(rw) / float(rh)
        if fh / max(1.0, frame_h) > float(cfg.square_pull_face_min):
            total += float(cfg.square_pull_weight) * (fh / float(frame_h) - float(cfg.square_pull_face_min)) * \
                abs(asp - 1.0)
        wide_min = max(1e-6, float(cfg.wide_face_min_frame_frac))
        wide_limit = max(1.0, float(cfg.wide_face_aspect_limit))
        if face_scale >= wide_min and asp > wide_limit:
            total += float(cfg.wide_face_aspect_penalty_weight) * min(4.0, face_scale / wide_min) * (asp - wide_limit)
    return total, box, tmpl


def choose_best_ratio(det_box, ratios: Sequence[str], frame_w, frame_h, anchor=None, face_box=None,
                      cfg: Optional[CropScoreConfig] = None):
    """Processor._choose_best_ratio (gui_app.py:3147-3328): expand det_box to every candidate
    'W:H' ratio and keep the lowest score (first wins ties); unparsable ratios are skipped.
    Returns (int box, ratio string or None, template loss of the winner)."""
    cfg = cfg or CropScoreConfig()
    head_box = head_proxy_box(face_box, frame_w, frame_h, cfg)
    best, best_ratio, best_score, best_tmpl = None, None, 1e9, 0.0
    for rs in ratios:
        try:
            rw, rh = parse_ratio(rs)
        except (ValueError, AttributeError, TypeError):
            continue
        total, box, tmpl = _ratio_score(det_box, rw, rh, frame_w, frame_h, anchor, face_box, head_box, cfg)
        if total < best_score:
            best_score, best_ratio, best_tmpl = total, rs, tmpl
            best = tuple(int(round(v)) for v in box)
    if best is None:   # nothing scored below 1e9: the first ratio unbiased, else the detection itself
        try:
            rw, rh = parse_ratio(str(ratios[0]))
            box = expand_box_to_ratio(*det_box, rw, rh, frame_w, frame_h, anchor=anchor, head_bias=0.0)
            return tuple(int(round(v)) for v in box), str(ratios[0]), 0.0
        except Exception:
            return tuple(int(round(v)) for v in det_box), None, 0.0
    return best, best_ratio, best_tmpl


# (SessionConfig field, type) of the debug.jsonl "cfg" block in the reference's order (gui_app.py:8024-8044)
DEBUG_CFG_FIELDS = (
    ("face_det_conf", float), ("face_det_pad", float), ("face_thresh", float), ("reid_thresh", float),
    ("face_quality_min", float), ("face_visible_uses_quality", bool), ("prefer_face_when_available", bool),
    ("require_face_if_visible", bool), ("match_mode", str), ("allow_faceless_when_locked", bool),
    ("faceless_reid_thresh", float), ("faceless_iou_min", float), ("faceless_persist_frames", int),
    ("faceless_min_area_frac", float), ("faceless_max_area_frac", float), ("faceless_center_max_frac", float),
    ("faceless_min_motion_frac", float), ("learn_bank_runtime", bool), ("drop_reid_if_any_face_match", bool),
)


def debug_record(frame: int, persons: int, faces_detected: int, faces_pass_quality: int, any_face_detected: bool,
                 any_face_visible: bool, min_fd_all, best_face_dist, cfg, candidates) -> dict:
    """One per-frame debug.jsonl object (gui_app.py:8013-8057). `cfg`: SessionConfig-like object or
    mapping holding DEBUG_CFG_FIELDS; `candidates`: dicts with fd, rd (None allowed), sharp, box[, reasons]."""
    get = (lambda k: cfg[k]) if isinstance(cfg, dict) else (lambda k: getattr(cfg, k))
    opt = lambda v: float(v) if v is not None else None
    return {
        "frame": frame, "persons": int(persons), "faces_detected": int(faces_detected),
        "faces_pass_quality": int(faces_pass_quality), "any_face_detected": bool(any_face_detected),
        "any_face_visible": bool(any_face_visible), "min_fd_all": opt(min_fd_all), "best_face_dist": opt(best_face_dist),
        "cfg": {k: t(get(k)) for k, t in DEBUG_CFG_FIELDS},
        "candidates": [{"fd": opt(c["fd"]), "rd": opt(c["rd"]), "sharp": float(c["sharp"]),
                        "box": [int(v) for v in c["box"]], "reasons": c.get("reasons", [])} for c in candidates],
    }


class DebugLog:
    """<dbg_dir>/debug.jsonl: one JSON object per line, flushed per frame (gui_app.py:4459-4470)."""

    def __init__(self, dbg_dir: str):
        import os
        os.makedirs(dbg_dir, exist_ok=True)
        self.f = open(os.path.join(dbg_dir, "debug.jsonl"), "w", encoding="utf-8")

    def write(self, obj: dict) -> None:
        import json
        json.dump(obj, self.f, ensure_ascii=False)
        self.f.write("\n")
        self.f.flush()

    def close(self) -> None:
        self.f.close()
