"""Sharded pre-scan of ONE clip over N GPUs with the single-stream result.

Processor._prescan (gui_app.py:1101-1668) is a sequential loop: whether sample k+1 is
extracted (the fd9 gate), which detector regime it runs under (a span open: escalation and
the full rotation mode) and what the bank holds (_stream_ref_bank_update) depend on every
earlier sample. The extraction itself - detections and embeddings of one sample - depends
only on the regime and on a small part of the FaceEmbedder's policy state
(FaceEmbedder.prescan_policy_key), not on the bank. So:

  1. every rank runs the pre-scan loop over its contiguous run of sample positions as if the
     clip started there (PrescanRunner.run(positions=..., speculate=True): batched on its
     GPU, with its own loop state), recording each extracted sample with the regime and
     policy state it ran under (SpecRecord);
  2. the records are gathered on rank 0 (host objects over gloo; no device collective);
  3. rank 0 replays the loop in sample order with the true state - fd9 gate, fd against the
     live bank, bank growth, span hysteresis, close and bridge (PrescanRunner's own host
     logic) - taking a sample's speculative result when its policy key equals the true one
     (the true policy state then advances by FaceEmbedder.policy_transfer) and extracting it
     again on its own GPU under the true state when it does not (the sample was skipped by
     the shard's gate, or ran in the other regime, or from another round-robin phase).

The result - spans, per-sample records, grown bank and the embedder's final policy state -
is the single-stream loop's (tests/test_gpu_prescan_shard.py against oracle/prescan.py).
Speculation misses cost one re-extraction each on rank 0; they occur near shard starts and
regime changes.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .prescan import PrescanRunner, SampleRecord, SpecRecord, _host_faces, _LoopState
from .shard import shard_bounds


@dataclass
class MergeStats:
    samples: int = 0
    skipped: int = 0
    reused: int = 0        # speculative results taken
    reextracted: int = 0   # extracted again on rank 0 under the true state
    per_rank_spec: List[int] = field(default_factory=list)


def sample_dims(runner: PrescanRunner, im) -> Tuple[int, int]:
    """(H, W) of a sample after the pre-scan downscale (gui_app.py:1505-1507)."""
    if hasattr(im, "ptr"):
        H, W = int(im.H), int(im.W)
    else:
        H, W = int(im.shape[0]), int(im.shape[1])
    Wmax = int(runner.cfg.prescan_max_width)
    if W > Wmax:
        return int(round(H * (Wmax / float(W)))), Wmax
    return H, W


def merge(runner: PrescanRunner, frame_at: Callable[[int], object], spec: Sequence[SpecRecord],
          initial_state: tuple):
    """Rank 0: the single-stream loop over all samples, reusing speculative results whose
    policy key matches. `runner` is rank 0's PrescanRunner (its FaceEmbedder re-extracts
    misses). Returns (spans, bank, records, MergeStats)."""
    f = runner.face
    runner.setup_face()
    samples = runner.samples()
    by_pos = {r.pos: r for r in spec}
    st = _LoopState(runner.ref_feat)
    pol = tuple(initial_state)
    stats = MergeStats(samples=len(samples))
    records: List[SampleRecord] = []
    for j, idx in enumerate(samples):
        skip, _ = runner._gate(st)
        faces: list = []
        if skip:
            stats.skipped += 1
        else:
            r = by_pos.get(j)
            hit = False
            if r is not None and r.active == st.active:
                H, W = sample_dims(runner, frame_at(idx))
                hit = f.prescan_policy_key(r.state_in, r.active, H, W) == f.prescan_policy_key(pol, st.active, H, W)
            if hit:
                faces = r.faces
                pol = f.policy_transfer(r.state_in, r.state_out, pol)
                stats.reused += 1
            else:
                got, pol = runner.extract_one(frame_at, j, st.active, pol)
                faces = _host_faces(got)
                stats.reextracted += 1
        rec = runner._finish_sample(st, idx, st.processed, faces, not skip)
        st.processed += 1
        records.append(rec)
    spans = runner.close(st)
    f.set_policy_state(pol)
    f.set_prescan_fast(False)
    f.set_prescan_hint(escalate=False)
    runner.final_state = st
    return spans, st.bank, records, stats


def run_sharded(face, cfg, fps: float, total_frames: int, frame_at: Callable[[int], object], ref_feat=None,
                batch: int = 32, rank: Optional[int] = None, world: Optional[int] = None, gather=None):
    """One clip's pre-scan over `world` ranks (one FaceEmbedder per rank / GPU). Every rank
    calls this; rank 0 returns (spans, bank, records, MergeStats), the others None.
    gather(obj) -> list of every rank's obj on rank 0 (None elsewhere); default: the
    torch.distributed host group (gloo) when world > 1."""
    rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else int(world)
    runner = PrescanRunner(face, cfg, fps, total_frames, ref_feat=ref_feat, batch=batch)
    pos = shard_bounds(len(runner.samples()), rank, world)
    runner.run(frame_at, positions=pos, speculate=True)
    spec = list(runner.spec or [])
    if world == 1:
        parts = [spec]
    elif gather is not None:
        parts = gather(spec)
    else:
        import torch.distributed as dist
        parts = [None] * world if rank == 0 else None
        dist.gather_object(spec, parts, dst=0)
    if rank != 0:
        return None
    allspec = [r for p in parts for r in p]
    out = merge(runner, frame_at, allspec, runner.initial_state)
    out[3].per_rank_spec = [len(p) for p in parts]
    return out
