"""Pre-scan driver (Processor._prescan's sampling loop, gui_app.py:1101-1668) on the device
against the CPU oracle oracle/prescan.py over oracle/pipeline.OracleFaceEmbedder, f32:
a synthetic 60-frame 1280x720 clip at stride 2 (blank stretches -> fd9 skip gating and
rotation probes; two scenes of the planted identity -> span entry, bank growth, exit
cooldown; another scene in between), INTER_AREA downscale to 416 on the device, fast
pre-scan SCRFD, one ArcFace forward per face (two while a span is active: escalation).
The batched speculative driver (chunks of 8 samples, cut and rolled back at every regime
change) must give the oracle's spans, bank, per-sample decisions and the FaceEmbedder's
final policy state; the same driver at batch 1 (the reference's own one-sample order) must
agree with it exactly."""
import numpy as np
import pytest

from oracle import pipeline as op
from oracle import prescan as oprescan
from oracle import ref_algos as ra
from person_capture_amd import face_embedder as fe_mod
from person_capture_amd.prescan import PrescanConfig, PrescanRunner

pytestmark = pytest.mark.gpu
H, W, N, FPS = 720, 1280, 60, 4.0


def _clip():
    A = np.random.default_rng(100).integers(0, 256, (H, W, 3), dtype=np.uint8)
    B = np.random.default_rng(200).integers(0, 256, (H, W, 3), dtype=np.uint8)
    blank = np.full((H, W, 3), 120, np.uint8)
    frames = []
    for i in range(N):
        frames.append(A if 10 <= i < 30 or 50 <= i < N else (B if 40 <= i < 50 else blank))
    return np.stack(frames)


def test_prescan_driver_matches_oracle(gpu_ctx, monkeypatch):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PRECISION", "f32")
    monkeypatch.setenv("PERSON_CAPTURE_AMD_ARCFACE", "iresnet50")
    clip = _clip()
    fe = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_2.5g_bnkps", conf=0.5)
    cfg = PrescanConfig(prescan_stride=2, prescan_add_cooldown_samples=2)
    # planted bank: the oracle embeddings of scene A's faces (downscaled as the pre-scan does), with the
    # synthetic embedder's common component partly removed so that scene B does not match
    o0 = op.OracleFaceEmbedder(fe._scrfd_params, "2.5g", fe._arc_params, 50, conf=0.5)
    o0._fast_prescan, o0._prescan_probe_imgsz = True, cfg.prescan_probe_imgsz
    small = lambda fr: __import__("oracle.cv_ops", fromlist=["x"]).resize(fr, (416, 234), interpolation=3)
    fa = [f["feat"] for f in o0.extract(small(clip[10]))]
    fb = [f["feat"] for f in o0.extract(small(clip[40]))]
    assert fa and fb
    mean = np.mean(fa + fb, axis=0)
    bank = np.stack([(v - 0.5 * mean) / np.linalg.norm(v - 0.5 * mean) for v in fa[:1]]).astype(np.float32)
    da = [ra.fd_min(v, bank) for v in fa]
    db = [ra.fd_min(v, bank) for v in fb]
    # thresholds between the two scenes (the defaults assume a trained embedder)
    lo, hi = min(da), min(db)
    assert lo < hi
    cfg.prescan_fd_enter = (lo + hi) / 2
    cfg.prescan_fd_exit = hi + 1e-3
    cfg.prescan_fd_add = cfg.prescan_fd_enter
    cfg.face_quality_min = 0.0
    # oracle
    o = op.OracleFaceEmbedder(fe._scrfd_params, "2.5g", fe._arc_params, 50, conf=0.5, rot_phase=id(fe) & 7)
    o_spans, o_bank, o_rec = oprescan.prescan(o, cfg, FPS, N, lambda i: clip[i], ref_feat=bank)
    # device: frames resident in HBM
    d = fe._ctx.alloc(clip.nbytes)
    fe._ctx.upload(clip, d)
    fsz = clip[0].nbytes
    at = lambda i: fe_mod._DevImage(d.ptr + i * fsz, H, W, W * 3)
    r = PrescanRunner(fe, cfg, FPS, N, ref_feat=bank, batch=8)
    spans, dbank = r.run(at)
    print("oracle spans", o_spans, "device spans", spans, "chunks", r.chunks, "cuts", r.cuts,
          "bank", None if dbank is None else dbank.shape)
    assert spans == o_spans and len(spans) >= 1
    assert len(r.records) == len(o_rec)
    for a, b in zip(r.records, o_rec):
        assert (a.idx, a.extracted, a.n_faces, a.bank_action, a.active) == (b[0], b[1], b[3], b[4], b[5]), (a, b)
        assert (a.best == b[2] == 9.0) or abs(a.best - b[2]) < 1e-4, (a, b)
    assert sum(1 for x in o_rec if not x[1]) > 0 and sum(1 for x in o_rec if x[4] == "added") > 0
    # bank rows are end-to-end features (independent nets, and a landmark a few f32 bits apart moves
    # a few chip pixels); the bit-exact chained feature checks are test_gpu_fallbacks / bench_config
    assert dbank.shape == o_bank.shape and np.abs(dbank - o_bank).max() < 1e-3
    assert fe.policy_state() == (o._frame_idx, o._no_face_streak, o._last_face_idx, o._rot_cycle, o._prescan_rr)
    assert r.cuts > 0
    # the same driver one sample per extract (the reference's order) agrees exactly
    fe2 = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_2.5g_bnkps", conf=0.5)
    r1 = PrescanRunner(fe2, cfg, FPS, N, ref_feat=bank, batch=1)
    spans1, bank1 = r1.run(at)
    assert spans1 == spans and np.array_equal(bank1, dbank)
    assert [(x.idx, x.extracted, x.best, x.n_faces, x.bank_action) for x in r1.records] == \
        [(x.idx, x.extracted, x.best, x.n_faces, x.bank_action) for x in r.records]
