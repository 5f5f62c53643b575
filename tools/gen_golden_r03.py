#!/usr/bin/env python3
"""Golden vectors for the round-3 post-match rows, made by running the reference's OWN
Processor methods (xmarre/person_capture at /root/reference, read-only), taken from
gui_app.py by AST (PySide6 is absent) together with the SessionConfig dataclass:

  _choose_best_ratio (+ _face_head_proxy_box)      gui_app.py:3147-3328, 1931-1962
  _prescan_cache_meta / _save_prescan_cache        gui_app.py:709-735, 787-920

Writes data only: tests/golden/choose_ratio.npz, tests/golden/prescan_cache_keys.json and
tests/golden/prescan_cache_ref.npz (a cache file written by the reference's saver).
Run: python tools/gen_golden_r03.py  (in the container that has /root/reference)
"""
from __future__ import annotations

import ast
import dataclasses
import hashlib
import json
import math
import os
import shutil
import sys
import tempfile
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _extract():
    src = open(os.path.join(REF, "person_capture", "gui_app.py"), encoding="utf-8").read()
    tree = ast.parse(src)
    want = {"_choose_best_ratio", "_face_head_proxy_box", "_prescan_cache_meta", "_cache_file_identity",
            "_jsonable_cfg_value", "_prescan_cache_root", "_prescan_cache_path", "_save_prescan_cache",
            "_load_prescan_cache", "_clip_to_frame"}
    body, cfg_cls = [], None
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == "Processor":
            body = [it for it in node.body if isinstance(it, ast.FunctionDef) and it.name in want]
        if isinstance(node, ast.ClassDef) and node.name == "SessionConfig":
            cfg_cls = node
    proc = ast.ClassDef(name="Processor", bases=[], keywords=[], body=body, decorator_list=[])
    mod = ast.Module(body=[cfg_cls, proc], type_ignores=[])
    ast.fix_missing_locations(mod)
    sys.path.insert(0, REF)
    from gen_golden import _stub_cv2
    _stub_cv2()
    import person_capture.utils as U
    ns = {"np": np, "json": json, "math": math, "os": os, "hashlib": hashlib, "Path": Path, "List": List,
          "Optional": Optional, "Tuple": Tuple, "dataclass": dataclasses.dataclass, "field": dataclasses.field,
          "parse_ratio": U.parse_ratio, "expand_box_to_ratio": U.expand_box_to_ratio,
          "_REPO_ROOT": Path(REF)}
    for k in ("Dict", "Any", "Sequence", "Iterable", "Union", "Callable"):
        ns[k] = getattr(__import__("typing"), k)
    exec(compile(mod, "<gui_app subset>", "exec"), ns)
    return ns["Processor"], ns["SessionConfig"]


def main():
    P, SessionConfig = _extract()
    cfg = SessionConfig()
    proc = P()
    proc.cfg = cfg
    proc._abort = False
    proc._status = lambda *a, **k: None
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20260517)

    # ---- _choose_best_ratio ----
    ratio_sets = [["2:3", "1:1", "3:2"], ["9:16", "4:5", "1:1", "16:9"], ["3:2"], ["bad", "2:3"], ["x:y"]]
    frames = [(1920, 1080), (3840, 2160), (640, 480)]
    rows = []
    for case in range(400):
        fw, fh = frames[case % 3]
        w = float(rng.uniform(20, fw * 0.6))
        h = float(rng.uniform(20, fh * 0.9))
        x1 = float(rng.uniform(-0.05 * fw, fw - w * 0.5))
        y1 = float(rng.uniform(-0.05 * fh, fh - h * 0.5))
        det = (int(x1), int(y1), int(x1 + w), int(y1 + h))
        face = None
        if case % 4 != 0:
            s = float(rng.uniform(0.08, 0.7)) * min(w, h)
            fx1 = x1 + float(rng.uniform(0, max(1.0, w - s)))
            fy1 = y1 + float(rng.uniform(0, max(1.0, h * 0.5)))
            face = (fx1, fy1, fx1 + s, fy1 + s * float(rng.uniform(1.0, 1.35)))
        anchor = None if case % 3 else (x1 + w * float(rng.uniform(0.3, 0.7)), y1 + h * float(rng.uniform(0.2, 0.6)))
        rs = ratio_sets[case % len(ratio_sets)]
        box, ratio, tl = proc._choose_best_ratio(det, rs, fw, fh, anchor=anchor, face_box=face)
        rows.append((case % len(ratio_sets), fw, fh, det, anchor, face, box, -1 if ratio is None else rs.index(ratio),
                     float(tl)))
    np.savez_compressed(
        os.path.join(OUT, "choose_ratio.npz"),
        ratio_sets=np.array(json.dumps(ratio_sets)),
        set_idx=np.array([r[0] for r in rows]), frame=np.array([(r[1], r[2]) for r in rows]),
        det=np.array([r[3] for r in rows], np.float64),
        anchor=np.array([r[4] if r[4] is not None else (np.nan, np.nan) for r in rows], np.float64),
        face=np.array([r[5] if r[5] is not None else (np.nan,) * 4 for r in rows], np.float64),
        box=np.array([r[6] for r in rows], np.int64), ratio_idx=np.array([r[7] for r in rows]),
        tmpl_loss=np.array([r[8] for r in rows], np.float64))

    # ---- pre-scan cache key over setting changes ----
    keys = []
    variants = [{}, {"prescan_stride": 12}, {"prescan_weights": (0.6, 0.3, 0.1)}, {"prescan_fd_enter": 0.4},
                {"face_model": "scrfd_2.5g_bnkps"}, {"use_arcface": False}, {"prescan_fd9_skip": False},
                {"prescan_weights": (np.float32(0.7), 0.25, 0.05)}]
    for i, v in enumerate(variants):
        c = SessionConfig()
        for k, val in v.items():
            setattr(c, k, val)
        c.video = "/nonexistent/clip_%d.mp4" % i
        c.ref = "/nonexistent/a.jpg; /nonexistent/b.png" if i % 2 else ""
        for fps, total in ((30.0, 9000), (29.97002997, 1234)):
            meta = proc._prescan_cache_meta(c, fps, total)
            keys.append({"settings": {k: (list(map(float, val)) if isinstance(val, tuple) else
                                          (val.item() if isinstance(val, np.generic) else val))
                                      for k, val in v.items()},
                         "video": c.video, "ref": c.ref, "fps": fps, "total_frames": total, "meta": meta})
    json.dump(keys, open(os.path.join(OUT, "prescan_cache_keys.json"), "w"), indent=0, sort_keys=True)

    # ---- a cache file written by the reference's saver ----
    tmp = tempfile.mkdtemp()
    try:
        c = SessionConfig()
        c.video = "/nonexistent/clip.mp4"
        c.ref = ""
        c.prescan_cache_dir = tmp
        spans = [(10, 250), (400, 401), (900, 1700)]
        bank = rng.standard_normal((5, 512)).astype(np.float32)
        bank /= np.linalg.norm(bank, axis=1, keepdims=True)
        proc._save_prescan_cache(c, 30.0, 3000, spans, bank)
        meta = proc._prescan_cache_meta(c, 30.0, 3000)
        shutil.copy(os.path.join(tmp, meta["key"] + ".npz"), os.path.join(OUT, "prescan_cache_ref.npz"))
        json.dump({"key": meta["key"], "spans": spans, "video": c.video, "fps": 30.0, "total_frames": 3000},
                  open(os.path.join(OUT, "prescan_cache_ref.json"), "w"))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    # ---- debug.jsonl record layout (key order of the dict literal at gui_app.py:8015-8055) ----
    tree = ast.parse(open(os.path.join(REF, "person_capture", "gui_app.py"), encoding="utf-8").read())
    lay = None
    for node in ast.walk(tree):
        if isinstance(node, ast.Dict) and any(isinstance(k, ast.Constant) and k.value == "faces_pass_quality"
                                              for k in node.keys):
            keys = [k.value for k in node.keys]
            cfg_d = node.values[keys.index("cfg")]
            cand = node.values[keys.index("candidates")].elt
            lay = {"top_keys": keys, "cfg_keys": [k.value for k in cfg_d.keys],
                   "candidate_keys": [k.value for k in cand.keys]}
    lay["cfg_defaults"] = {k: getattr(cfg, k) for k in lay["cfg_keys"]}
    json.dump(lay, open(os.path.join(OUT, "debug_record_layout.json"), "w"), indent=0)
    print("wrote choose_ratio.npz, prescan_cache_keys.json, prescan_cache_ref.npz, debug_record_layout.json")


if __name__ == "__main__":
    main()
