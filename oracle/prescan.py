"""CPU oracle of Processor._prescan's sampling loop (test infrastructure only).

Sequential restatement of gui_app.py:1140-1668 (minus the GUI command queue, decoder
seeking, previews and the edge-refinement re-scan) over oracle/pipeline.OracleFaceEmbedder:
per sample the escalation hint from the span state, the fd9 skip gate, the INTER_AREA
downscale to prescan_max_width (cv_ops.resize), extract, _fd_min per face against the live
bank, _stream_ref_bank_update (ref_algos) with the add cooldown and the quality gate, the
enter/exit hysteresis with pad / min length / merge, the end-of-video close and the gap
bridging. `cfg` is any object with the SessionConfig prescan_* fields.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from . import cv_ops
from . import ref_algos as ra


def prescan(face, cfg, fps: float, total_frames: int, frame_at, ref_feat=None):
    """face: an OracleFaceEmbedder. Returns (spans, bank, records) with records
    [(idx, extracted, best, n_faces, action, active)] per sample."""
    if ref_feat is None:
        bank_list: List[np.ndarray] = []
    else:
        arr = np.asarray(ref_feat, dtype=np.float32)
        if arr.ndim == 1:
            arr = arr.reshape(1, -1)
        arr = arr / np.maximum(np.linalg.norm(arr, axis=1, keepdims=True), 1e-6)
        bank_list = [row.copy() for row in arr]
    bank = np.vstack(bank_list).astype(np.float32) if bank_list else None
    stride = max(1, int(cfg.prescan_stride))
    pad = int(round(cfg.prescan_pad_sec * fps))
    min_len = int(round(cfg.prescan_min_segment_sec * fps))
    Wmax = int(cfg.prescan_max_width)
    enter, exit_ = float(cfg.prescan_fd_enter), float(cfg.prescan_fd_exit)
    fd_add = float(cfg.prescan_fd_add)
    face.conf = min(0.95, max(0.01, float(cfg.prescan_face_conf)))
    face._probe_conf = float(cfg.prescan_probe_conf)
    face._prescan_period = int(cfg.prescan_rot_probe_period)
    face._prescan_probe_imgsz = int(cfg.prescan_probe_imgsz)
    face._prescan_no_upscale_det = bool(cfg.prescan_no_upscale_det)
    face._high_90, face._high_180 = int(cfg.prescan_heavy_90), int(cfg.prescan_heavy_180)
    face.rot_adaptive = False            # configure_rotation_strategy(adaptive=False)
    face._rot_cycle = 0
    face._fast_prescan, face._prescan_rr_mode, face._prescan_rr = True, "rr", 0
    face._prescan_escalate = False
    cooldown = int(cfg.prescan_add_cooldown_samples)
    last_add = -10 ** 9
    spans: List[Tuple[int, int]] = []
    active, start, neg_run, fd9_streak, processed = False, 0, 0, 0, 0
    records = []
    for idx in range(0, total_frames, stride):
        sample_idx = processed
        processed += 1
        face._prescan_rr_mode = "full" if active else "rr"
        face._prescan_escalate = bool(active)
        best = 9.0
        skip = False
        if (not active) and cfg.prescan_fd9_skip:
            grace = max(0, int(cfg.prescan_fd9_grace))
            period = max(1, int(cfg.prescan_fd9_probe_period))
            if fd9_streak >= grace and (fd9_streak % period) != 0:
                skip = True
        action = ""
        n = 0
        if not skip:
            frame = frame_at(idx)
            h, w = frame.shape[:2]
            if w > Wmax:
                nh = int(round(h * (Wmax / float(w))))
                frame = cv_ops.resize(frame, (Wmax, nh), interpolation=cv_ops.INTER_AREA)
            faces = face.extract(frame)
            n = len(faces)
            for f in faces:
                fd = ra.fd_min(f["feat"], bank)
                best = min(best, fd)
                if fd <= fd_add and (sample_idx - last_add) >= cooldown and f.get("quality", 1e9) >= cfg.face_quality_min:
                    bank, action, _ = ra.stream_ref_bank_update(bank_list, bank, f["feat"], float(f["quality"]),
                                                                cap=int(cfg.prescan_bank_max),
                                                                dedup_cos=float(cfg.prescan_diversity_dedup_cos),
                                                                rep_margin=float(cfg.prescan_replace_margin),
                                                                weights=tuple(cfg.prescan_weights))
                    if action in ("added", "replaced"):
                        last_add = sample_idx
        fd9_streak = fd9_streak + 1 if best >= 8.99 else 0
        if best <= enter:
            if not active:
                active, fd9_streak, start = True, 0, idx
            neg_run = 0
        elif active:
            neg_run += 1
            exit_cool = int(round(max(0.0, float(cfg.prescan_exit_cooldown_sec)) * fps))
            if neg_run * stride >= exit_cool or best >= exit_:
                s, e = max(0, start - pad), min(total_frames - 1, idx + pad)
                if e - s + 1 >= min_len:
                    if spans and s <= spans[-1][1] + 1:
                        spans[-1] = (spans[-1][0], max(spans[-1][1], e))
                    else:
                        spans.append((s, e))
                active, neg_run, fd9_streak = False, 0, 0
        records.append((idx, not skip, float(best), n, action, active))
    if active:
        s, e = max(0, start - pad), total_frames - 1
        if e - s + 1 >= min_len:
            if spans and s <= spans[-1][1] + 1:
                spans[-1] = (spans[-1][0], max(spans[-1][1], e))
            else:
                spans.append((s, e))
    if spans and cfg.prescan_bridge_gap_sec > 0:
        gap = int(round(cfg.prescan_bridge_gap_sec * fps))
        bridged = []
        cs, ce = spans[0]
        for s, e in spans[1:]:
            if s - ce <= gap:
                ce = max(ce, e)
            else:
                bridged.append((cs, ce))
                cs, ce = s, e
        bridged.append((cs, ce))
        spans = bridged
    return spans, bank, records
