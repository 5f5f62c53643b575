"""Hot-path helpers with the reference's semantics (person_capture/utils.py):
vector normalisation / cosine distance used by the match step, and the crop
geometry the callers apply to accepted boxes."""
from __future__ import annotations

import os
from typing import Iterable

import numpy as np


def parse_ratio(s: str):
    """utils.py:101-103 — 'W:H' -> (float W, float H)."""
    w, h = s.split(":")
    return float(w), float(h)


def ensure_dir(p) -> None:
    os.makedirs(p, exist_ok=True)


def l2_normalize(x, eps: float = 1e-10):
    """utils.py:108-110: x / (||x|| + eps)."""
    return x / (np.linalg.norm(x) + eps)


def cosine_distance(a: Iterable[float], b: Iterable[float]) -> float:
    """utils.py:260-268: 1 - dot(a/(|a|+1e-9), b/(|b|+1e-9)) in float32."""
    va = np.asarray(list(a), dtype=np.float32).reshape(-1)
    vb = np.asarray(list(b), dtype=np.float32).reshape(-1)
    na = float(np.linalg.norm(va)) + 1e-9
    nb = float(np.linalg.norm(vb)) + 1e-9
    return 1.0 - float(np.dot(va / na, vb / nb))


def crop_img(frame, box):
    x1, y1, x2, y2 = [int(v) for v in box]
    return frame[y1:y2, x1:x2]


def _clamp(v, lo, hi):
    return max(lo, min(hi, v))


def expand_box_to_ratio(x1, y1, x2, y2, ratio_w, ratio_h, frame_w, frame_h, anchor=None, head_bias=0.0):
    """utils.py:198-257: the smallest box of exactly ratio_w:ratio_h around the input box
    (optionally re-centred on `anchor` and shifted by head_bias * box height), clamped into
    the frame and shrunk symmetrically if clamping broke the ratio."""
    x1, y1, x2, y2 = (float(v) for v in (x1, y1, x2, y2))
    bw = max(1.0, x2 - x1)
    bh = max(1.0, y2 - y1)
    target = float(ratio_w) / float(ratio_h)
    cx, cy = (float(anchor[0]), float(anchor[1])) if anchor is not None else (x1 + bw * 0.5, y1 + bh * 0.5)
    cy -= head_bias * bh
    new_w, new_h = (target * bh, bh) if bw / bh < target else (bw, bw / target)
    l, t = _clamp(cx - new_w * 0.5, 0, frame_w - 1), _clamp(cy - new_h * 0.5, 0, frame_h - 1)
    r, b = _clamp(cx + new_w * 0.5, 0, frame_w - 1), _clamp(cy + new_h * 0.5, 0, frame_h - 1)
    cw, ch = r - l, b - t
    if cw <= 1 or ch <= 1:
        return int(l), int(t), int(r), int(b)
    cur = cw / ch
    if abs(cur - target) > 1e-4:
        if cur < target:
            dy = (ch - cw / target) * 0.5
            t += dy
            b -= dy
        else:
            dx = (cw - ch * target) * 0.5
            l += dx
            r -= dx
        l, t = _clamp(l, 0, frame_w - 1), _clamp(t, 0, frame_h - 1)
        r, b = _clamp(r, 0, frame_w - 1), _clamp(b, 0, frame_h - 1)
    return int(round(l)), int(round(t)), int(round(r)), int(round(b))
