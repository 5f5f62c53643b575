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
A speculation miss costs one batched speculative chunk on rank 0 (from the missed sample under
the true state); misses occur near shard starts and regime changes.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .prescan import PrescanRunner, SampleRecord, SpecRecord, _host_faces, _LoopState
from .shard import shard_bounds


@dataclass
class MergeStats:
    samples: int = 0
    skipped: int = 0
    reused: int = 0        # speculative results of the ranks taken
    misses: int = 0        # samples whose policy key or regime matched no rank's record
    rechunks: int = 0      # speculative chunks rank 0 ran for them (one extract_batch each)
    reextracted: int = 0   # samples extracted on rank 0 in those chunks
    from_rechunks: int = 0  # samples taken from rank 0's own chunks
    merge_s: float = 0.0   # wall time of the merge on rank 0 (the serial part of a sharded clip)
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


def _pick(f, cands: Sequence[SpecRecord], active: bool, pol: tuple) -> Optional[SpecRecord]:
    """The first candidate record of a sample that ran in the true regime with the true policy key
    (its dims were recorded by the rank that extracted it: no frame is fetched for the check)."""
    for r in cands:
        if r.active == active:
            H, W = r.dims
            if f.prescan_policy_key(r.state_in, r.active, H, W) == f.prescan_policy_key(pol, active, H, W):
                return r
    return None


def merge(runner: PrescanRunner, frame_at: Callable[[int], object], spec: Sequence[SpecRecord],
          initial_state: tuple):
    """Rank 0: the single-stream loop over all samples, reusing speculative results whose
    policy key matches. A sample no rank's record serves (a miss: near shard starts and regime
    changes, or a whole shard speculated at the other round-robin parity) starts a speculative
    chunk on rank 0 from that sample under the TRUE regime and policy state - one batched
    extract_batch of up to `batch` samples (PrescanRunner.spec_chunk), whose records then serve the
    following samples too - instead of one extraction per missed sample. `runner` is rank 0's
    PrescanRunner. Returns (spans, bank, records, MergeStats)."""
    t0 = time.perf_counter()
    f = runner.face
    runner.setup_face()
    samples = runner.samples()
    cands: Dict[int, List[SpecRecord]] = {}
    for r in spec:
        cands.setdefault(r.pos, []).append(r)
    st = _LoopState(runner.ref_feat)
    pol = tuple(initial_state)
    stats = MergeStats(samples=len(samples))
    records: List[SampleRecord] = []
    own = set()   # ids of the records rank 0 extracted in its own chunks
    for j, idx in enumerate(samples):
        skip, _ = runner._gate(st)
        faces: list = []
        if skip:
            stats.skipped += 1
        else:
            r = _pick(f, cands.get(j, ()), st.active, pol)
            if r is None:
                stats.misses += 1
                f.set_policy_state(pol)
                plan, active0, state0, by_pos, state_after, dims = runner.spec_chunk(frame_at, st, j, len(samples))
                stats.rechunks += 1
                last, fresh = state0, []
                for jj, sk in plan:
                    if not sk:
                        fresh.append(SpecRecord(jj, active0, last, state_after[jj], _host_faces(by_pos[jj]), dims[jj]))
                        last = state_after[jj]
                stats.reextracted += len(fresh)
                for x in fresh:
                    own.add(id(x))
                    cands.setdefault(x.pos, []).insert(0, x)
                r = _pick(f, cands.get(j, ()), st.active, pol)
                if r is None:   # the chunk ran sample j from exactly this regime and state
                    raise RuntimeError(f"pre-scan merge: sample {j} unmatched after re-extraction")
            faces = r.faces
            pol = f.policy_transfer(r.state_in, r.state_out, pol)
            if id(r) in own:
                stats.from_rechunks += 1
            else:
                stats.reused += 1
        rec = runner._finish_sample(st, idx, st.processed, faces, not skip)
        st.processed += 1
        records.append(rec)
    spans = runner.close(st)
    f.set_policy_state(pol)
    f.set_prescan_fast(False)
    f.set_prescan_hint(escalate=False)
    runner.final_state = st
    stats.merge_s = time.perf_counter() - t0
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
