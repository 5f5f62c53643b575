"""Crop-ratio chooser and pre-scan cache against goldens made by running the reference's own
Processor methods (tools/gen_golden_r03.py: gui_app.py _choose_best_ratio 3147-3328 with
_face_head_proxy_box 1931-1962; _prescan_cache_meta / _save_prescan_cache 787-920).
CPU only."""
import json
import os

import numpy as np

from person_capture_amd import prescan_cache as pc
from person_capture_amd.postmatch import CropScoreConfig, choose_best_ratio

G = os.path.join(os.path.dirname(__file__), "golden")


def test_choose_best_ratio_matches_reference():
    d = np.load(os.path.join(G, "choose_ratio.npz"), allow_pickle=False)
    sets = json.loads(str(d["ratio_sets"]))
    for i in range(len(d["set_idx"])):
        rs = sets[int(d["set_idx"][i])]
        fw, fh = (int(v) for v in d["frame"][i])
        det = tuple(int(v) for v in d["det"][i])
        anchor = None if np.isnan(d["anchor"][i][0]) else tuple(float(v) for v in d["anchor"][i])
        face = None if np.isnan(d["face"][i][0]) else tuple(float(v) for v in d["face"][i])
        box, ratio, tl = choose_best_ratio(det, rs, fw, fh, anchor=anchor, face_box=face, cfg=CropScoreConfig())
        assert tuple(box) == tuple(int(v) for v in d["box"][i]), i
        assert (-1 if ratio is None else rs.index(ratio)) == int(d["ratio_idx"][i]), i
        assert tl == float(d["tmpl_loss"][i]), i


def test_prescan_cache_keys_match_reference():
    for case in json.load(open(os.path.join(G, "prescan_cache_keys.json"))):
        settings = {k: tuple(v) if isinstance(v, list) else v for k, v in case["settings"].items()}
        meta = pc.cache_meta(settings, case["video"], case["ref"], case["fps"], case["total_frames"])
        assert meta == case["meta"]


def test_prescan_cache_reads_reference_file_and_round_trips(tmp_path):
    info = json.load(open(os.path.join(G, "prescan_cache_ref.json")))
    meta = pc.cache_meta({}, info["video"], "", info["fps"], info["total_frames"])
    assert meta["key"] == info["key"]
    root = tmp_path / "cache"
    root.mkdir()
    ref_file = os.path.join(G, "prescan_cache_ref.npz")
    (root / f"{meta['key']}.npz").write_bytes(open(ref_file, "rb").read())
    hit, spans, bank = pc.load(root, meta)
    assert hit and spans == [tuple(s) for s in info["spans"]] and bank.shape == (5, 512)
    # our writer produces the same arrays; a different key or mode misses
    out = pc.save(tmp_path / "mine", meta, spans, bank)
    with np.load(out, allow_pickle=False) as a, np.load(ref_file, allow_pickle=False) as b:
        assert sorted(a.files) == sorted(b.files)
        for k in a.files:
            assert np.array_equal(a[k], b[k]), k
    other = pc.cache_meta({"prescan_stride": 12}, info["video"], "", info["fps"], info["total_frames"])
    assert pc.load(root, other) == (False, [], None)
    assert pc.load(root, meta, mode="refresh") == (False, [], None)
    assert pc.save(tmp_path / "off", meta, spans, None, mode="off") is None
    # no reference bank: has_ref 0 -> None back
    pc.save(tmp_path / "nb", meta, spans, None)
    assert pc.load(tmp_path / "nb", meta) == (True, spans, None)


def test_run_cached_hit_skips_the_loop(tmp_path):
    from person_capture_amd.prescan import PrescanConfig, run_cached

    class Runner:
        cfg, fps, total, calls = PrescanConfig(), 30.0, 600, 0

        def run(self, frame_at):
            self.calls += 1
            return [(0, 99)], np.eye(2, 512, dtype=np.float32)

    r = Runner()
    a = run_cached(r, None, "/nonexistent/v.mp4", "", cache_dir=str(tmp_path))
    b = run_cached(r, None, "/nonexistent/v.mp4", "", cache_dir=str(tmp_path))
    assert r.calls == 1 and a[2] is False and b[2] is True
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
    r.cfg = PrescanConfig(prescan_stride=12)   # another key: a miss
    assert run_cached(r, None, "/nonexistent/v.mp4", "", cache_dir=str(tmp_path))[2] is False and r.calls == 2


def test_cache_damaged_file_is_a_miss_and_save_failure_keeps_result(tmp_path):
    """gui_app.py:880/919 catch every exception: a truncated .npz is a miss, and a cache
    directory that cannot be written still returns the freshly computed result."""
    from person_capture_amd.prescan import PrescanConfig, run_cached

    meta = pc.cache_meta({}, "/nonexistent/v.mp4", "", 30.0, 600)
    root = tmp_path / "c"
    out = pc.save(root, meta, [(0, 9)], np.eye(2, 512, dtype=np.float32))
    data = open(out, "rb").read()
    for cut in (0, 10, len(data) // 2):
        open(out, "wb").write(data[:cut])
        assert pc.load(root, meta) == (False, [], None)

    class Runner:
        cfg, fps, total, calls = PrescanConfig(), 30.0, 600, 0

        def run(self, frame_at):
            self.calls += 1
            return [(0, 99)], np.eye(2, 512, dtype=np.float32)

    blocker = tmp_path / "file_not_dir"
    blocker.write_text("x")   # the cache "directory" is a file: mkdir / open fail
    r = Runner()
    spans, bank, hit = run_cached(r, None, "/nonexistent/v.mp4", "", cache_dir=str(blocker / "sub"))
    assert not hit and spans == [(0, 99)] and bank.shape == (2, 512) and r.calls == 1
    assert "Error" in r.cache_error


def test_cache_key_follows_the_face_backend(tmp_path):
    """The key records the detector that ran (face_model is a key field, gui_app.py:821)."""
    from person_capture_amd.prescan import PrescanConfig, _runner_settings

    class Face:
        detector_backend, scrfd_variant, use_arcface = "scrfd", "10g", True

    class Runner:
        cfg, fps, total, face = PrescanConfig(), 30.0, 600, Face()

    keys = set()
    for backend, variant, path in (("scrfd", "10g", ""), ("scrfd", "2.5g", ""), ("yolo", "10g", "yolov8l-face")):
        r = Runner()
        r.face = Face()
        r.face.detector_backend, r.face.scrfd_variant, r.face._scrfd_model_path = backend, variant, path
        s = _runner_settings(r)
        keys.add(pc.cache_meta(s, "/nonexistent/v.mp4", "", 30.0, 600)["key"])
    assert len(keys) == 3
    r = Runner()
    assert _runner_settings(r)["face_model"] == "scrfd_10g_bnkps"
    # the default SCRFD-10G runner keys like the reference's SessionConfig defaults
    assert pc.cache_meta(_runner_settings(r), "/x.mp4", "", 30.0, 600)["key"] == \
        pc.cache_meta(PrescanConfig(), "/x.mp4", "", 30.0, 600)["key"]


def test_debug_record_layout_matches_reference(tmp_path):
    from person_capture_amd.postmatch import DEBUG_CFG_FIELDS, DebugLog, debug_record
    lay = json.load(open(os.path.join(G, "debug_record_layout.json")))
    assert [k for k, _ in DEBUG_CFG_FIELDS] == lay["cfg_keys"]
    cands = [{"fd": 0.31, "rd": None, "sharp": 12.5, "box": (1.0, 2, 3, 4.0)},
             {"fd": None, "rd": 0.2, "sharp": 3, "box": [5, 6, 7, 8], "reasons": ["faceless"]}]
    rec = debug_record(7, 2, 3, 1, True, False, None, 0.31, lay["cfg_defaults"], cands)
    assert list(rec) == lay["top_keys"] and list(rec["cfg"]) == lay["cfg_keys"]
    assert rec["cfg"] == lay["cfg_defaults"]
    assert all(list(c) == lay["candidate_keys"] for c in rec["candidates"])
    log = DebugLog(str(tmp_path))
    log.write(rec)
    log.write(rec)
    log.close()
    lines = open(tmp_path / "debug.jsonl", encoding="utf-8").read().splitlines()
    assert len(lines) == 2 and json.loads(lines[0]) == json.loads(json.dumps(rec))
