"""BASELINE C5 composed: the pre-scan path on its configured networks and sizes, f32 (the
parity mode), against the CPU oracle chained the same way.

4K frames (3840x2160) resident in HBM -> PrescanRunner (Processor._prescan's sampling loop,
gui_app.py:1101-1668; batched speculative chunks of 8 samples) -> INTER_AREA downscale to
416 wide on the device -> fast pre-scan SCRFD-10G -> ArcFace IResNet-100 (one forward per
face, two while a span is active: escalation) -> fd against a 1024-row bank (one row planted
from scene A's faces, 1023 random unit rows), bank growth (replace-worst: the bank is over
prescan_bank_max) and span hysteresis.
Oracle: oracle/prescan.prescan over oracle/pipeline.OracleFaceEmbedder (SCRFD-10G + r100 in
torch fp32 on the host) on the same frames. Spans, per-sample decisions, the grown bank and
the embedder's policy state must agree; 16 samples (stride 2 over 32 frames) keep the CPU
oracle within about a minute on the GPU box's host share."""
import numpy as np
import pytest

from oracle import cv_ops
from oracle import pipeline as op
from oracle import prescan as oprescan
from oracle import ref_algos as ra
from person_capture_amd import face_embedder as fe_mod
from person_capture_amd.prescan import PrescanConfig, PrescanRunner

pytestmark = pytest.mark.gpu
H, W, N, FPS = 2160, 3840, 32, 4.0
BANK_ROWS = 1024


def _scene(i):
    """0 blank, 1 scene A, 2 scene B: blank 0-3, A 4-13, blank 14-17, B 18-23, A 24-31."""
    if 4 <= i < 14 or i >= 24:
        return 1
    return 2 if 18 <= i < 24 else 0


def _scene_img(seed):
    s = np.random.default_rng(seed).integers(0, 256, (234, 416, 3)).astype(np.float32)
    s = np.clip(128 + 0.3 * (s - 128), 0, 255).astype(np.uint8)
    return cv_ops.resize(s, (W, H), interpolation=0)


@pytest.mark.timeout(600)
def test_c5_prescan_4k_r100_bank1024(gpu_ctx, monkeypatch):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PRECISION", "f32")
    monkeypatch.delenv("PERSON_CAPTURE_AMD_ARCFACE", raising=False)   # IResNet-100, the default
    # scenes: 416x234 noise at 0.3 contrast, nearest-upscaled to 4K, whose INTER_AREA downscale
    # the synthetic SCRFD-10G finds 7 / 8 faces in at 0 degrees (full-resolution 4K noise averages
    # to a flat 416-wide image with no faces; full contrast gives >100, too many for the CPU oracle)
    scenes = [np.full((H, W, 3), 120, np.uint8), _scene_img(1), _scene_img(2)]
    fe = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5)
    assert fe._arc_depth == 100 and fe.scrfd_variant == "10g"
    cfg = PrescanConfig(prescan_stride=2, prescan_add_cooldown_samples=2)
    # planted bank: an oracle embedding of scene A's first face (downscaled as the pre-scan does),
    # the synthetic embedder's common component partly removed, then 1023 random unit rows
    o0 = op.OracleFaceEmbedder(fe._scrfd_params, "10g", fe._arc_params, 100, conf=0.5)
    o0._fast_prescan, o0._prescan_probe_imgsz = True, cfg.prescan_probe_imgsz
    small = lambda fr: cv_ops.resize(fr, (416, 234), interpolation=3)
    fa = [f["feat"] for f in o0.extract(small(scenes[1]))]
    fb = [f["feat"] for f in o0.extract(small(scenes[2]))]
    assert fa and fb
    mean = np.mean(fa + fb, axis=0)
    rnd = np.random.default_rng(9).standard_normal((BANK_ROWS - 1, 512)).astype(np.float32)
    rows = [(fa[0] - 0.5 * mean) / np.linalg.norm(fa[0] - 0.5 * mean)] + list(rnd / np.linalg.norm(rnd, axis=1,
                                                                                               keepdims=True))
    bank = np.stack(rows).astype(np.float32)
    da = [ra.fd_min(v, bank) for v in fa]
    db = [ra.fd_min(v, bank) for v in fb]
    lo, hi = min(da), min(db)
    assert lo < hi
    cfg.prescan_fd_enter = (lo + hi) / 2
    cfg.prescan_fd_exit = hi + 1e-3
    cfg.prescan_fd_add = cfg.prescan_fd_enter
    cfg.face_quality_min = 0.0
    # oracle
    o = op.OracleFaceEmbedder(fe._scrfd_params, "10g", fe._arc_params, 100, conf=0.5, rot_phase=id(fe) & 7)
    o_spans, o_bank, o_rec = oprescan.prescan(o, cfg, FPS, N, lambda i: scenes[_scene(i)], ref_feat=bank)
    # device: the three distinct 4K frames resident in HBM
    fsz = scenes[0].nbytes
    d = fe._ctx.alloc(3 * fsz)
    for k, s in enumerate(scenes):
        fe._ctx.upload(s, d, offset=k * fsz)
    at = lambda i: fe_mod._DevImage(d.ptr + _scene(i) * fsz, H, W, W * 3)
    r = PrescanRunner(fe, cfg, FPS, N, ref_feat=bank, batch=8)
    spans, dbank = r.run(at)
    print("oracle spans", o_spans, "device spans", spans, "chunks", r.chunks, "cuts", r.cuts,
          "bank", None if dbank is None else dbank.shape, "faces", sum(x.n_faces for x in r.records), flush=True)
    assert spans == o_spans and len(spans) >= 1
    assert len(r.records) == len(o_rec)
    for a, b in zip(r.records, o_rec):
        assert (a.idx, a.extracted, a.n_faces, a.bank_action, a.active) == (b[0], b[1], b[3], b[4], b[5]), (a, b)
        assert (a.best == b[2] == 9.0) or abs(a.best - b[2]) < 1e-4, (a, b)
    # the bank is over prescan_bank_max (64): growth replaces its worst-scored rows (random ones)
    assert sum(1 for x in o_rec if x[4] == "replaced") > 0 and any(x[5] for x in o_rec)
    assert dbank.shape == o_bank.shape == (BANK_ROWS, 512)
    assert np.abs(dbank - o_bank).max() < 1e-3
    assert fe.policy_state() == (o._frame_idx, o._no_face_streak, o._last_face_idx, o._rot_cycle, o._prescan_rr)
