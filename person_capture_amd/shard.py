"""Frame-shard runner: one process per GPU, frames dealt round-robin by index, no
device collective (SURVEY.md §8e — detect/align/embed/match has no cross-frame
reduction). Results come back to rank 0 in frame order over a host (gloo) gather.

Launch with `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...`;
each rank binds `cuda:LOCAL_RANK` and builds its own FaceEmbedder (context, stream,
weights). Sequential policy state of the reference (the adaptive rotation gate's
no-face streak, pre-scan bank growth, lock-ROI) is per instance: callers that need
single-stream semantics replay match.stream_ref_bank_update / span hysteresis on
rank 0 over the gathered, frame-ordered results.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence


def shard_indices(n: int, rank: int, world: int) -> List[int]:
    """Frame i goes to rank i mod world."""
    return list(range(rank, n, world))


def merge_in_order(n: int, world: int, per_rank: Sequence[Sequence]) -> list:
    """Inverse of shard_indices: per_rank[r][k] is the result of frame r + k*world."""
    out = [None] * n
    for r, res in enumerate(per_rank):
        for k, v in enumerate(res):
            out[r + k * world] = v
    return out


class FrameShardRunner:
    """Runs `extract_fn(frames_of_this_rank) -> list of per-frame results` on every rank
    and gathers the per-frame results on rank 0 in global frame order."""

    def __init__(self, extract_fn: Callable[[list], list], rank: Optional[int] = None,
                 world: Optional[int] = None):
        self.extract_fn = extract_fn
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world

    def process(self, frames: Sequence) -> Optional[list]:
        n = len(frames)
        mine = shard_indices(n, self.rank, self.world)
        res = self.extract_fn([frames[i] for i in mine]) if mine else []
        if self.world == 1:
            return list(res)
        import torch.distributed as dist
        gathered = [None] * self.world if self.rank == 0 else None
        dist.gather_object(list(res), gathered, dst=0)
        if self.rank != 0:
            return None
        return merge_in_order(n, self.world, gathered)


def face_runner(device_index: Optional[int] = None, **face_kwargs) -> FrameShardRunner:
    """A FrameShardRunner over a FaceEmbedder on this rank's GPU."""
    from .face_embedder import FaceEmbedder
    local = int(os.environ.get("LOCAL_RANK", "0")) if device_index is None else device_index
    face_kwargs.setdefault("yolo_model", "scrfd_10g_bnkps")
    fe = FaceEmbedder(ctx=f"cuda:{local}", **face_kwargs)
    return FrameShardRunner(lambda fr: fe.extract_batch(fr))
