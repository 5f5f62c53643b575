"""Sharded pre-scan of one clip (person_capture_amd/prescan_shard.py) on the GPU: the C5
scenes of tests/test_gpu_c5_composed.py (4K frames resident in HBM, INTER_AREA to 416, fast
pre-scan SCRFD-10G + IResNet-100, 1024-row bank with a planted row, replace-worst growth,
spans), f32 parity mode, cut into 2 and 3 contiguous shards. Each shard runs on its own
FaceEmbedder (its own policy state; the ranks of one node run one after another in this
process), rank 0 merges with re-extraction of speculation misses. Spans, per-sample records,
the grown bank and the embedder's final policy state must equal the sequential CPU oracle
(oracle/prescan.py over oracle/pipeline.OracleFaceEmbedder)."""
import numpy as np
import pytest

from oracle import pipeline as op
from oracle import prescan as oprescan
from oracle import ref_algos as ra
from person_capture_amd import face_embedder as fe_mod
from person_capture_amd.prescan import PrescanConfig, PrescanRunner
from person_capture_amd.prescan_shard import merge
from person_capture_amd.shard import shard_bounds
from test_gpu_c5_composed import BANK_ROWS, FPS, H, N, W, _scene, _scene_img
from oracle import cv_ops

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_sharded_prescan_equals_oracle(gpu_ctx, monkeypatch):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PRECISION", "f32")
    monkeypatch.delenv("PERSON_CAPTURE_AMD_ARCFACE", raising=False)
    scenes = [np.full((H, W, 3), 120, np.uint8), _scene_img(1), _scene_img(2)]
    fe = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5)   # weights; oracle phase
    cfg = PrescanConfig(prescan_stride=2, prescan_add_cooldown_samples=2)
    o0 = op.OracleFaceEmbedder(fe._scrfd_params, "10g", fe._arc_params, 100, conf=0.5)
    o0._fast_prescan, o0._prescan_probe_imgsz = True, cfg.prescan_probe_imgsz
    small = lambda fr: cv_ops.resize(fr, (416, 234), interpolation=3)
    fa = [f["feat"] for f in o0.extract(small(scenes[1]))]
    fb = [f["feat"] for f in o0.extract(small(scenes[2]))]
    mean = np.mean(fa + fb, axis=0)
    rnd = np.random.default_rng(9).standard_normal((BANK_ROWS - 1, 512)).astype(np.float32)
    rows = [(fa[0] - 0.5 * mean) / np.linalg.norm(fa[0] - 0.5 * mean)] + list(rnd / np.linalg.norm(rnd, axis=1,
                                                                                               keepdims=True))
    bank = np.stack(rows).astype(np.float32)
    lo, hi = min(ra.fd_min(v, bank) for v in fa), min(ra.fd_min(v, bank) for v in fb)
    cfg.prescan_fd_enter = (lo + hi) / 2
    cfg.prescan_fd_exit = hi + 1e-3
    cfg.prescan_fd_add = cfg.prescan_fd_enter
    cfg.face_quality_min = 0.0
    o = op.OracleFaceEmbedder(fe._scrfd_params, "10g", fe._arc_params, 100, conf=0.5, rot_phase=id(fe) & 7)
    o_spans, o_bank, o_rec = oprescan.prescan(o, cfg, FPS, N, lambda i: scenes[_scene(i)], ref_feat=bank)
    o_state = (o._frame_idx, o._no_face_streak, o._last_face_idx, o._rot_cycle, o._prescan_rr)

    fsz = scenes[0].nbytes
    d = fe._ctx.alloc(3 * fsz)
    for k, s in enumerate(scenes):
        fe._ctx.upload(s, d, offset=k * fsz)
    at = lambda i: fe_mod._DevImage(d.ptr + _scene(i) * fsz, H, W, W * 3)
    for world in (2, 3):
        fresh = [fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps", conf=0.5) for _ in range(world)]
        runners = []
        for rank in range(world):
            r = PrescanRunner(fresh[rank], cfg, FPS, N, ref_feat=bank, batch=4)
            r.run(at, positions=shard_bounds(len(r.samples()), rank, world), speculate=True)
            runners.append(r)
        spans, dbank, recs, stats = merge(runners[0], at, [x for r in runners for x in r.spec],
                                          runners[0].initial_state)
        print(f"world {world}: spans {spans} (oracle {o_spans}), reused {stats.reused}, "
              f"re-extracted {stats.reextracted}, skipped {stats.skipped}", flush=True)
        assert spans == o_spans and len(spans) >= 1
        assert len(recs) == len(o_rec)
        for a, b in zip(recs, o_rec):
            assert (a.idx, a.extracted, a.n_faces, a.bank_action, a.active) == (b[0], b[1], b[3], b[4], b[5]), (a, b)
            assert (a.best == b[2] == 9.0) or abs(a.best - b[2]) < 1e-4, (a, b)
        assert dbank.shape == o_bank.shape and np.abs(dbank - o_bank).max() < 1e-3
        assert fresh[0].policy_state() == o_state
        assert stats.reused > 0
