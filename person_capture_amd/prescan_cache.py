"""Pre-scan result cache of the GUI (Processor._prescan_cache_meta / _load_prescan_cache /
_save_prescan_cache, gui_app.py:709-735, 780-920): the spans and grown reference bank of a
pre-scan, keyed by the video's and reference images' file identities, fps, frame count and
every setting that can change the pre-scan's output. Same key (sha256 of the sorted-key
compact JSON of the meta), same .npz layout (meta / spans / ref_face_feat / has_ref), so a
cache written by either implementation is read by the other.

Settings a caller does not pass take SessionConfig's defaults (gui_app.py:431-594)."""
from __future__ import annotations

import hashlib
import json
import os
from pathlib import Path
from typing import Iterable, List, Mapping, Optional, Tuple

import numpy as np

# (key, SessionConfig default) in the reference's order (gui_app.py:790-825)
PRESCAN_KEY_DEFAULTS: Tuple[Tuple[str, object], ...] = (
    ("prescan_stride", 24), ("prescan_max_width", 416), ("prescan_decode_max_w", 384),
    ("prescan_face_conf", 0.5), ("prescan_fd_enter", 0.45), ("prescan_fd_add", 0.22),
    ("prescan_fd_exit", 0.52), ("prescan_add_cooldown_samples", 5), ("prescan_rot_probe_period", 3),
    ("prescan_probe_imgsz", 512), ("prescan_no_upscale_det", True), ("prescan_probe_conf", 0.03),
    ("prescan_heavy_90", 1536), ("prescan_heavy_180", 1280), ("prescan_min_segment_sec", 1.0),
    ("prescan_pad_sec", 1.5), ("prescan_bridge_gap_sec", 1.0), ("prescan_exit_cooldown_sec", 0.50),
    ("prescan_boundary_refine_sec", 0.75), ("prescan_refine_stride_min", 3), ("prescan_trim_pad", True),
    ("prescan_skip_trailing_refine", True), ("prescan_refine_budget_sec", 1.5), ("prescan_bank_max", 64),
    ("prescan_diversity_dedup_cos", 0.968), ("prescan_replace_margin", 0.010), ("prescan_fd9_skip", True),
    ("prescan_fd9_grace", 1), ("prescan_fd9_probe_period", 2), ("prescan_weights", (0.70, 0.25, 0.05)),
    ("face_model", "scrfd_10g_bnkps"), ("clip_face_backbone", "ViT-L-14"),
    ("clip_face_pretrained", "laion2b_s32b_b82k"), ("use_arcface", True),
)
CACHE_VERSION = 1


def file_identity(path) -> dict:
    """Processor._cache_file_identity (gui_app.py:709-725): absolute path + size + mtime_ns."""
    p = str(path or "").strip()
    if not p:
        return {"path": "", "missing": True}
    try:
        ap = os.path.abspath(p)
    except (TypeError, ValueError):
        ap = p
    try:
        st = os.stat(ap)
    except OSError:
        return {"path": ap, "missing": True}
    return {"path": ap, "size": int(st.st_size or 0), "mtime_ns": int(st.st_mtime_ns)}


def _jsonable(v):
    """Processor._jsonable_cfg_value (gui_app.py:727-735): tuples -> lists, numpy scalars -> python."""
    if isinstance(v, (tuple, list)):
        return [_jsonable(x) for x in v]
    if isinstance(v, (np.floating, np.integer)):
        return v.item()
    return v


def cache_meta(settings: Mapping[str, object], video, refs, fps: float, total_frames: int) -> dict:
    """The cache meta and its key (gui_app.py:787-841). `settings`: any SessionConfig-like mapping
    or object attributes; `refs`: the ';'-joined reference string or a list of paths."""
    get = (lambda k, d: settings.get(k, d)) if isinstance(settings, Mapping) else \
        (lambda k, d: getattr(settings, k, d))
    if isinstance(refs, str):
        refs = [r.strip() for r in refs.split(";") if r.strip()]
    meta = {
        "version": CACHE_VERSION,
        "video": file_identity(video),
        "refs": [file_identity(r) for r in (refs or [])],
        "fps": round(float(fps or 0.0), 6),
        "total_frames": int(total_frames or 0),
        "settings": {k: _jsonable(get(k, d)) for k, d in PRESCAN_KEY_DEFAULTS},
    }
    meta["key"] = hashlib.sha256(json.dumps(meta, sort_keys=True, separators=(",", ":")).encode("utf-8")).hexdigest()
    return meta


def cache_root(cache_dir: str = "prescan_cache", base: Optional[Path] = None) -> Path:
    """gui_app.py:780-785: relative cache dirs live under the application root (`base`)."""
    root = Path(str(cache_dir or "prescan_cache").strip() or "prescan_cache")
    if not root.is_absolute():
        root = Path(base or os.getcwd()) / root
    return root


def cache_path(root: Path, meta: dict) -> Path:
    return Path(root) / f"{meta.get('key') or ''}.npz"


def load(root: Path, meta: dict, mode: str = "auto") -> Tuple[bool, List[Tuple[int, int]], Optional[np.ndarray]]:
    """gui_app.py:847-882: (hit, spans, ref bank) — a miss on another key/version, an absent
    file, a mode other than auto/reuse or an unreadable file (never unpickled)."""
    if str(mode or "auto").lower() not in ("auto", "reuse"):
        return False, [], None
    path = cache_path(root, meta)
    if not path.is_file():
        return False, [], None
    try:
        with np.load(str(path), allow_pickle=False) as data:
            stored = json.loads(str(data["meta"].item()))
            if stored.get("key") != meta.get("key") or stored.get("version") != meta.get("version"):
                return False, [], None
            arr = np.asarray(data["spans"], dtype=np.int64).reshape(-1, 2)
            spans = [(int(s), int(e)) for s, e in arr.tolist() if int(e) >= int(s)]
            has_ref = bool(int(np.asarray(data["has_ref"] if "has_ref" in data.files else [0]).reshape(-1)[0]))
            feat = None
            if has_ref and "ref_face_feat" in data.files:
                f = np.asarray(data["ref_face_feat"], dtype=np.float32)
                if f.size > 0:
                    feat = f.reshape(f.shape[0], -1) if f.ndim >= 2 else f.reshape(1, -1)
            return True, spans, feat
    except Exception:   # any damaged file is a miss, as gui_app.py:880 treats it
        return False, [], None


def save(root: Path, meta: dict, spans: Iterable[Tuple[int, int]], ref_face_feat: Optional[np.ndarray],
         mode: str = "auto") -> Optional[Path]:
    """gui_app.py:884-920: written to <key>.npz.tmp, then renamed over the cache file."""
    if str(mode or "auto").lower() not in ("auto", "refresh", "reuse"):
        return None
    path = cache_path(root, meta)
    path.parent.mkdir(parents=True, exist_ok=True)
    spans_arr = np.asarray(list(spans or []), dtype=np.int64).reshape(-1, 2)
    if ref_face_feat is None:
        feat, has_ref = np.zeros((0, 0), np.float32), np.array([0], np.uint8)
    else:
        feat = np.asarray(ref_face_feat, dtype=np.float32)
        feat = feat.reshape(1, -1) if feat.ndim == 1 else feat
        has_ref = np.array([1], np.uint8)
    tmp = path.with_suffix(path.suffix + ".tmp")
    with open(tmp, "wb") as f:
        np.savez_compressed(f, meta=np.array(json.dumps(meta, sort_keys=True), dtype=np.str_), spans=spans_arr,
                            ref_face_feat=feat, has_ref=has_ref)
    os.replace(tmp, path)
    return path
