"""Parity of the SCRFD fallback branches and the chip fallbacks against the full CPU
restatement oracle/pipeline.OracleFaceEmbedder (face_embedder.py:2163-2482, 1465-1473,
1571-1647), f32 parity mode, frame sequences through one extract_batch call each.

The synthetic (untrained) detector scores every anchor near sigmoid(-1.4), so with its
stock head the TTA probes (conf 0.2) fire on thousands of anchors. The sequences below
shift the score-head bias by DELTA (the same params on both sides) so that, on small
flat / noise-patch / noise-band frames, the 0-degree pass finds nothing and each
fallback is reached and hits a few faces: TTA 0.75, 0.6, 1.25, edge replicate-pad,
rotations 90/270/180 with probe + heavy 1280/1536 passes, the no-face streak
(det size 512 after 3 empty frames, which also makes the batch path's speculative
det size wrong and re-runs those frames synchronously), the after-hit window and the
periodic rotation gate (rot_phase = the device instance's id(self) & 7), the fast
pre-scan round-robin rotations with the heavy _high_90 / _high_180 sizes and the
single-forward embed, the eye-roll re-alignment and the resize fallback.
Which branches each sequence reached is read from the oracle's trace and asserted,
so a sequence that silently stopped exercising a branch fails.

Per frame: the same faces with identical int boxes; a face whose chip is byte-identical
to the oracle's has its embedding within 1e-4 (north_star) and quality within 1e-9 rel;
a face whose landmarks differ in the last f32 bits is checked through the chain (the
oracle's chip decision on the device landmarks gives the device chip byte for byte,
the oracle embedding of that chip matches within 1e-4). The per-instance policy state
(_frame_idx, _no_face_streak, _last_face_idx, _rot_cycle, _prescan_rr) ends identical.
"""
import numpy as np
import pytest

from oracle import cv_ops
from oracle import nets_torch as nt
from oracle import pipeline as op
from oracle import ref_algos as ra
from person_capture_amd import face_embedder as fe_mod

pytestmark = pytest.mark.gpu

TOL = 1e-4
DELTA = -1.4
H, W = 240, 320


def _gray(v=128, h=H, w=W):
    return np.full((h, w, 3), v, np.uint8)


def _noise(seed, h=H, w=W):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def _patch(sz, seed):
    rng = np.random.default_rng(seed)
    f = _gray()
    y, x = rng.integers(0, H - sz), rng.integers(0, W - sz)
    f[y:y + sz, x:x + sz] = rng.integers(0, 256, (sz, sz, 3), dtype=np.uint8)
    return f


def _corner(sz, seed):
    f = _gray()
    f[0:sz, W - sz:W] = np.random.default_rng(seed).integers(0, 256, (sz, sz, 3), dtype=np.uint8)
    return f


def _band(trial):
    rng = np.random.default_rng(100 + trial)
    f = np.full((H, W, 3), int(rng.integers(40, 220)), np.uint8)
    b = int(rng.integers(4, 40))
    side = int(rng.integers(0, 4))
    bd = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if side == 0:
        f[:b] = bd[:b]
    elif side == 1:
        f[-b:] = bd[-b:]
    elif side == 2:
        f[:, :b] = bd[:, :b]
    else:
        f[:, -b:] = bd[:, -b:]
    return f


def fallback_sequence():
    """Frames (240x320) and the branches the oracle reaches on them at DELTA."""
    return [_noise(0), _gray(), _patch(64, 3), _patch(48, 6), _band(2), _corner(48, 7), _gray(), _gray(90),
            _gray(200), _gray(60), _band(8), _gray(), _gray(30), _gray(), _gray(), _gray(), _gray(), _gray(70),
            _gray(150), _gray(), _gray(110)]


def prescan_sequence():
    """Pre-scan sized frames (4K -> 416 wide, gui_app.py:1505-1507)."""
    return [_noise(20, 234, 416), _gray(128, 234, 416), _gray(90, 234, 416), _gray(200, 234, 416),
            _noise(21, 234, 416)[::2, ::2].repeat(2, 0).repeat(2, 1), _gray(60, 234, 416), _gray(30, 234, 416),
            _gray(170, 234, 416)]


# Landmark layouts (detector order: eye, eye, nose, mouth, mouth; units of 1.5 strides) that
# _canon_5pts rejects. It sorts by y, so with SCRFD's free-form landmarks only exact ties
# make it fail; a zero kps weight makes every anchor emit the layout exactly, ties included.
KPS_LAYOUTS = {
    # nose level with the eyes, eye line horizontal: eye-roll angle 0 < 8 deg -> resize
    "tie_level": [[-0.8, -0.6], [0.8, -0.6], [0.0, -0.6], [-0.6, 1.0], [0.6, 1.0]],
    # both eyes on one vertical line: eye-roll by 90 deg; the rotated points still tie -> resize
    "tie_vertical": [[0.0, -1.0], [0.0, -0.5], [0.5, 0.2], [-0.5, 0.8], [0.5, 1.0]],
    # eye line at ~30 deg with the nose level with one eye: eye-roll by 30 deg
    "tie_tilted": [[-0.5, -0.8], [0.5, -0.22], [0.1, -0.22], [-0.4, 0.9], [0.6, 1.1]],
    # all five points on the anchor centre: no eye or mouth line -> resize
    "zero": [[0.0, 0.0]] * 5,
}


def shifted_params(p, delta=DELTA, kps_layout=None):
    p = dict(p)
    for s in (8, 16, 32):
        if delta:
            p[f"bbox_head.{s}.cls.bias"] = p[f"bbox_head.{s}.cls.bias"] + np.float32(delta)
        if kps_layout is not None:
            kb = p[f"bbox_head.{s}.kps.bias"]
            A = kb.size // 10
            p[f"bbox_head.{s}.kps.bias"] = np.tile(np.asarray(KPS_LAYOUTS[kps_layout], np.float32).reshape(-1) * 1.5, A)
            p[f"bbox_head.{s}.kps.weight"] = np.zeros_like(p[f"bbox_head.{s}.kps.weight"])
    return p


def _device_embedder(monkeypatch, params_fn, conf=0.5):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PRECISION", "f32")
    monkeypatch.setenv("PERSON_CAPTURE_AMD_ARCFACE", "iresnet50")
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PIPE_CHUNK", "4")   # several pipelined detection chunks
    fe = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_2.5g_bnkps", conf=conf)
    fe._scrfd_params = params_fn(fe._scrfd_params)
    fe._scrfd_engines.clear()
    fe.scrfd = fe._engine(640)
    fe.debug_chips = True
    return fe


def _state(o):
    return (o._frame_idx, o._no_face_streak, o._last_face_idx, o._rot_cycle, o._prescan_rr)


def _embed(o, chip, flip):
    e = nt.iresnet_forward(o.p_a, o.depth, nt.arcface_input_from_chips(chip[None])).numpy()
    ef = nt.iresnet_forward(o.p_a, o.depth, nt.arcface_input_from_chips(chip[None, :, ::-1])).numpy() if flip else None
    return ra.arcface_postprocess(e, ef)[0]


def _compare(frames, got, oracle, ref, flip=True):
    n_exact = n_chained = 0
    for fi, (frame, g, r) in enumerate(zip(frames, got, ref)):
        assert len(g) == len(r), f"frame {fi}: {len(g)} faces vs oracle {len(r)}"
        gs = sorted(g, key=lambda f: tuple(f["bbox"]))
        rs = sorted(r, key=lambda f: tuple(f["bbox"]))
        for a, b in zip(gs, rs):
            assert np.array_equal(a["bbox"], b["bbox"]), (fi, a["bbox"], b["bbox"])
            if np.array_equal(a["chip"], b["chip"]):
                assert np.abs(a["feat"] - b["feat"]).max() < TOL, fi
                assert abs(a["quality"] - b["quality"]) <= 1e-9 * max(1.0, b["quality"])
                n_exact += 1
            else:
                assert (a["kps5"] is None) == (b["kps5"] is None)
                assert np.abs(a["kps5"] - b["kps5"]).max() < 1e-3, fi
                x1, y1, x2, y2 = a["bbox"]
                chip = op.chip_for(frame[y1:y2, x1:x2], a["kps5"])
                assert np.array_equal(chip, a["chip"]), fi
                assert abs(cv_ops.face_quality(chip) - a["quality"]) <= 1e-9 * max(1.0, a["quality"])
                assert np.abs(_embed(oracle, chip, flip) - a["feat"]).max() < TOL, fi
                n_chained += 1
        # the device output order is the reference's (quality, area) descending sort
        keys = [(f["quality"], int((f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1]))) for f in g]
        assert keys == sorted(keys, reverse=True)
    return n_exact, n_chained


def _run(fe, oracle, frames):
    got = fe.extract_batch(frames)
    ref, traces = [], set()
    for f in frames:
        ref.append(oracle.extract(f))
        traces.update(t for t in oracle.trace if not t.startswith("detect"))
        traces.update(f"size{t[6:]}" for t in oracle.trace if t.startswith("detect"))
    return got, ref, traces


def test_scrfd_fallback_branches(gpu_ctx, monkeypatch):
    fe = _device_embedder(monkeypatch, shifted_params)
    fe.rot_every_n = 3
    fe.rot_after_hit_frames = 6
    o = op.OracleFaceEmbedder(fe._scrfd_params, "2.5g", fe._arc_params, 50, conf=0.5, rot_phase=id(fe) & 7)
    o.rot_every_n, o.rot_after_hit_frames = 3, 6
    frames = fallback_sequence()
    got, ref, traces = _run(fe, o, frames)
    print("branches:", sorted(traces), "fallback detections prefetched/inline:", fe.fb_stats, fe.fb_kind_stats)
    assert fe.fb_stats[0] > 0   # the batched speculative prefetch served some of them
    assert fe.fb_kind_stats["rot"][0] > 0   # normal-mode rotation passes too (gate simulated per chunk)
    for b in ("tta0.75", "tta0.6", "tta1.25", "edgepad", "rot90", "rot270", "rot180", "eyeroll",
              "size512", "size1280", "size1536"):
        assert b in traces, b
    ne, nc = _compare(frames, got, o, ref)
    assert ne + nc >= 10
    assert _state(fe) == _state(o)


def test_prescan_fast_branches(gpu_ctx, monkeypatch):
    """set_prescan_fast(True) (gui_app.py:1114-1135): det size capped to the probe size and
    the source, round-robin 90/270 rotations every _prescan_period frames, heavy passes at
    the _high_90 override (1536), one ArcFace forward per face (no flip)."""
    fe = _device_embedder(monkeypatch, shifted_params)
    fe.set_prescan_fast(True)
    o = op.OracleFaceEmbedder(fe._scrfd_params, "2.5g", fe._arc_params, 50, conf=0.5, rot_phase=id(fe) & 7)
    o._fast_prescan = True
    frames = prescan_sequence()
    fe.configure_rotation_strategy(adaptive=False)   # as Processor._prescan does (gui_app.py:1188)
    o.rot_adaptive = False
    got, ref, traces = _run(fe, o, frames)
    print("branches:", sorted(traces), "fallback detections prefetched/inline:", fe.fb_stats)
    assert fe.fb_stats[0] > 0
    for b in ("rot90", "rot270", "size384", "size1536"):
        assert b in traces, b
    assert "tta0.75" not in traces and "edgepad" not in traces
    ne, nc = _compare(frames, got, o, ref, flip=False)
    assert ne + nc >= 3
    assert _state(fe) == _state(o)


@pytest.mark.parametrize("layout,exit_", [("tie_level", "roll_resize"), ("tie_vertical", "roll_rot_resize"),
                                          ("tie_tilted", "roll_align"), ("zero", "roll_resize")])
def test_chip_fallbacks(gpu_ctx, monkeypatch, layout, exit_):
    """Landmark layouts that _canon_5pts rejects (KPS_LAYOUTS): the eye-roll re-alignment
    (face_embedder.py:1571-1647: rotate the crop about its centre by the eye-line angle,
    re-canonicalise the rotated landmarks, LMEDS + warp) and its INTER_AREA / INTER_LINEAR
    resize exits (:1579-1618, 2458-2460)."""
    fe = _device_embedder(monkeypatch, lambda p: shifted_params(p, 0.0, kps_layout=layout))
    o = op.OracleFaceEmbedder(fe._scrfd_params, "2.5g", fe._arc_params, 50, conf=0.5, rot_phase=id(fe) & 7)
    frames = [_noise(30 + i) for i in range(3)]
    got, ref, traces = _run(fe, o, frames)
    print(layout, "branches:", sorted(traces))
    assert "eyeroll" in traces and exit_ in traces
    ne, nc = _compare(frames, got, o, ref)
    assert ne + nc >= 3
