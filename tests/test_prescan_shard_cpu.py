"""Sharded pre-scan merge protocol on the CPU (person_capture_amd/prescan_shard.py).

A host stand-in for the FaceEmbedder follows the SCRFD pre-scan policy's state machine
(face_embedder.py _scrfd_policy with rot_adaptive off: every empty sample probes rotations,
"rr" mode one of (90, 270) by the round-robin counter, "full" mode both; streak / last-face /
rotation-cycle / round-robin updates) over synthetic scenes: faces at 0 degrees, none, or
a face only a 90-degree probe finds (so the round-robin phase decides the result and shard
speculation can miss). Its embeddings depend on the regime (escalation = flip-TTA). The
sharded run - speculation per shard, gather, rank-0 replay with re-extraction of misses -
must give the sequential loop's spans, per-sample records, bank and final policy state: in
process for 1-7 shards, and over gloo worlds of 2 and 8 processes (the 8-GPU C5 layout). A miss
is served by a batched speculative chunk on rank 0 from the true state, whose records serve the
samples after it as well.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from person_capture_amd.face_embedder import FaceEmbedder
from person_capture_amd.prescan import PrescanConfig, PrescanRunner
from person_capture_amd.prescan_shard import merge, run_sharded

DIM = 16


class FakeIm:
    def __init__(self, scene, H=234, W=416):
        self.ptr, self.H, self.W, self.scene = 1, H, W, scene


def _feat(scene, k, active):
    """Identity A in scenes 1, 3, 4, identity B in scene 2; per-face noise (cos ~0.92 within
    an identity: bank growth adds rather than dedups)."""
    ident = np.random.default_rng(2 if scene == 2 else 1).standard_normal(DIM).astype(np.float32)
    v = ident + 0.3 * np.linalg.norm(ident) / np.sqrt(DIM) * \
        np.random.default_rng(1000 * scene + k).standard_normal(DIM).astype(np.float32)
    if active:   # escalated: the flip-TTA embedding differs slightly
        v = v + 0.05 * np.random.default_rng(77 + scene).standard_normal(DIM).astype(np.float32)
    return v / np.linalg.norm(v)


class FakeFace:
    """The pre-scan policy state machine of FaceEmbedder._scrfd_policy over synthetic scenes:
    scene 0 empty, 1..3 faces at 0 degrees, 4 a face only a 90-degree probe finds."""
    prescan_policy_key = FaceEmbedder.prescan_policy_key
    policy_transfer = staticmethod(FaceEmbedder.policy_transfer)
    _dyn_for = FaceEmbedder._dyn_for

    def __init__(self):
        self._frame_idx, self._no_face_streak, self._last_face_idx, self._rot_cycle, self._prescan_rr = \
            0, 0, -10 ** 9, 0, 0
        self._fast_prescan, self._prescan_rr_mode, self._prescan_escalate = False, "rr", False
        self.rot_adaptive, self.fast_no_face_imgsz = True, 512
        self.state_trace = None
        self.calls = 0

    def configure_rotation_strategy(self, adaptive=None, **_):
        if adaptive is not None:
            self.rot_adaptive = bool(adaptive)
        self._rot_cycle = 0

    def set_prescan_fast(self, enable, mode="rr"):
        self._fast_prescan, self._prescan_rr_mode = bool(enable), str(mode)
        if enable:
            self._prescan_rr = 0

    def set_prescan_hint(self, escalate=False):
        self._prescan_escalate = bool(escalate)

    def policy_state(self):
        return (self._frame_idx, self._no_face_streak, self._last_face_idx, self._rot_cycle, self._prescan_rr)

    def set_policy_state(self, s):
        self._frame_idx, self._no_face_streak, self._last_face_idx, self._rot_cycle, self._prescan_rr = s

    def extract_batch(self, frames, dev_frames=None, **_):
        out = []
        for i, im in enumerate(dev_frames):
            self.calls += 1
            active = self._prescan_escalate
            faces = []
            if 1 <= im.scene <= 3:
                faces = [{"bbox": np.array([0, 0, 9, 9]), "feat": _feat(im.scene, k, active), "quality": 100.0}
                         for k in range(im.scene % 2 + 1)]
                self._no_face_streak, self._last_face_idx, self._rot_cycle = 0, self._frame_idx, 0
            else:
                self._no_face_streak += 1
                self._rot_cycle += 1
                if self._prescan_rr_mode == "rr":
                    seq = ((90, 270)[self._prescan_rr % 2],)
                    self._prescan_rr += 1
                else:
                    seq = (90, 270)
                if im.scene == 4 and 90 in seq:
                    faces = [{"bbox": np.array([1, 1, 9, 9]), "feat": _feat(4, 0, active), "quality": 100.0}]
            self._frame_idx += 1
            if self.state_trace is not None:
                self.state_trace.append((i, self.policy_state()))
            out.append(faces)
        return out


# scene per sample: runs of faces of two identities, empty stretches, 90-degree-only faces
SCENES = ([0] * 5 + [1] * 6 + [0] * 4 + [4] * 5 + [2] * 7 + [0] * 6 + [3] * 4 + [4, 0] * 4 + [1] * 5 + [0] * 9)
FPS, STRIDE = 2.0, 2


def _cfg():
    c = PrescanConfig(prescan_stride=STRIDE, prescan_add_cooldown_samples=2, prescan_bank_max=6,
                      prescan_pad_sec=1.0, prescan_min_segment_sec=1.0, prescan_bridge_gap_sec=1.0)
    c.face_quality_min = 0.0
    bank = np.stack([_feat(1, 0, False)])
    c.prescan_fd_enter = c.prescan_fd_add = 0.3
    c.prescan_fd_exit = 0.6
    return c, bank


TOTAL = len(SCENES) * STRIDE
frame_at = lambda idx: FakeIm(SCENES[idx // STRIDE])


def _sequential():
    cfg, bank = _cfg()
    face = FakeFace()
    r = PrescanRunner(face, cfg, FPS, TOTAL, ref_feat=bank, batch=1)
    spans, b = r.run(frame_at)
    return spans, b, [vars(x) for x in r.records], face.policy_state()


def _sharded_in_process(world, batch):
    """The ranks run one after another in this process; gather = the list of their records."""
    cfg, bank = _cfg()
    specs, runners = [], []
    from person_capture_amd.shard import shard_bounds
    for rank in range(world):
        face = FakeFace()
        r = PrescanRunner(face, cfg, FPS, TOTAL, ref_feat=bank, batch=batch)
        r.run(frame_at, positions=shard_bounds(len(r.samples()), rank, world), speculate=True)
        specs.append(list(r.spec))
        runners.append(r)
    spans, b, recs, stats = merge(runners[0], frame_at, [x for s in specs for x in s], runners[0].initial_state)
    return spans, b, [vars(x) for x in recs], runners[0].face.policy_state(), stats


def _same(a, b):
    sa, ba, ra, pa = a[:4]
    sb, bb, rb, pb = b[:4]
    assert sa == sb and len(sa) >= 2
    assert ra == rb
    assert pa == pb
    assert ba.shape == bb.shape and np.array_equal(ba, bb)


def test_sequential_reference_exercises_the_policy():
    spans, bank, recs, pol = _sequential()
    acts = {r["bank_action"] for r in recs}
    assert "added" in acts or "replaced" in acts
    assert any(r["active"] for r in recs) and any(not r["extracted"] for r in recs)


@pytest.mark.parametrize("world,batch", [(1, 4), (2, 4), (3, 1), (4, 8), (5, 2), (7, 3)])
def test_sharded_merge_equals_sequential(world, batch):
    seq = _sequential()
    got = _sharded_in_process(world, batch)
    _same(got, seq)
    stats = got[4]
    assert stats.samples == len(SCENES) and stats.reused > 0
    if world == 1:
        assert stats.reextracted == 0


def test_speculation_misses_are_reextracted():
    """Shards that start inside an open span (or at another round-robin phase) speculate
    in the wrong regime: those samples are extracted again on rank 0, and the result is
    still the sequential one."""
    seq = _sequential()
    total = 0
    for world in (3, 4, 5, 7):
        got = _sharded_in_process(world, 2)
        _same(got, seq)
        total += got[4].reextracted
    assert total > 0


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, bank = _cfg()
        out = run_sharded(FakeFace(), cfg, FPS, TOTAL, frame_at, ref_feat=bank, batch=4, rank=rank, world=world)
        if rank == 0:
            spans, b, recs, stats = out
            q.put((spans, b, [vars(x) for x in recs], stats.reused, stats.reextracted, stats.per_rank_spec))
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_prescan_gloo(world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_worker, args=(world, port, q), nprocs=world, join=True)
    spans, b, recs, reused, reex, per_rank = q.get(timeout=120)
    seq = _sequential()
    assert spans == seq[0] and recs == seq[2] and np.array_equal(b, seq[1])
    assert len(per_rank) == world and all(n > 0 for n in per_rank) and reused > 0


def test_misses_run_as_batched_chunks():
    """Every miss starts one rank-0 chunk, and a chunk's later records serve later samples: at 7
    shards of batch 4 the rank-0 chunks extract more samples than there were miss events, and the
    merge's extract_batch calls number the chunks, not the re-extracted samples."""
    cfg, bank = _cfg()
    from person_capture_amd.shard import shard_bounds
    specs, runners = [], []
    for rank in range(7):
        r = PrescanRunner(FakeFace(), cfg, FPS, TOTAL, ref_feat=bank, batch=4)
        r.run(frame_at, positions=shard_bounds(len(r.samples()), rank, 7), speculate=True)
        specs.append(list(r.spec))
        runners.append(r)
    r0 = runners[0]
    chunks_before = r0.chunks
    spans, b, recs, st = merge(r0, frame_at, [x for sp in specs for x in sp], r0.initial_state)
    _same((spans, b, [vars(x) for x in recs], r0.face.policy_state()), _sequential())
    assert st.misses > 0 and st.rechunks == st.misses == r0.chunks - chunks_before
    assert st.reextracted >= st.from_rechunks >= st.misses
    assert st.reused + st.from_rechunks + st.skipped == st.samples and st.merge_s > 0
