"""Frame-shard runner: one process per GPU, each rank takes one contiguous run of
frames, no device collective (SURVEY.md §8e — detect/align/embed/match has no
cross-frame reduction). Results come back to rank 0 in frame order over a host
(gloo) gather.

Contiguous runs (not round-robin) so that the per-instance sequential state of the
reference's FaceEmbedder — the no-face streak that shrinks the det size
(face_embedder.py:2190-2204), the adaptive rotation gate over _frame_idx /
_last_face_idx (:2330-2347) — sees the same consecutive frames inside a run as a
single stream does; only the first frames of each run start from a fresh state.

Launch with `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...`
(or `bench.py --gpus N`, which spawns the ranks itself); each rank binds
`cuda:LOCAL_RANK` and builds its own FaceEmbedder (context, stream, weights).
The pre-scan loop of one clip is sequential (fd9 gate, bank growth, span hysteresis):
prescan_shard.run_sharded shards its sample positions the same way, gathers each rank's
speculative per-sample results (with the regime and policy state they ran under) on rank 0,
and replays the loop there in sample order, extracting again the samples whose speculative
state was wrong - the single-stream spans and bank (tests/test_prescan_shard_cpu.py,
tests/test_gpu_prescan_shard.py).
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence


def shard_bounds(n: int, rank: int, world: int) -> range:
    """Rank r gets frames [r*n//world, (r+1)*n//world): contiguous, sizes differ by <= 1."""
    return range(rank * n // world, (rank + 1) * n // world)


def shard_indices(n: int, rank: int, world: int) -> List[int]:
    return list(shard_bounds(n, rank, world))


def merge_in_order(n: int, world: int, per_rank: Sequence[Sequence]) -> list:
    """Inverse of shard_indices: rank results concatenated in rank order."""
    out: list = []
    for r, res in enumerate(per_rank):
        if len(res) != len(shard_bounds(n, r, world)):
            raise ValueError(f"rank {r} returned {len(res)} results for {len(shard_bounds(n, r, world))} frames")
        out.extend(res)
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


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_local_ranks(cmd: Sequence[str], world: int, env: Optional[dict] = None, timeout: Optional[float] = None,
                      poll_s: float = 0.2, grace_s: float = 5.0) -> int:
    """Start `world` rank processes of `cmd` on this node with the torch.distributed.run
    environment (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1,
    MASTER_PORT). The caller must not have touched the GPU: the ranks are fresh
    processes (no exec of the caller).

    Fail fast like torchrun: the children are polled together, and the first rank that
    exits non-zero (or the whole job running past `timeout` seconds) terminates its
    siblings (SIGTERM, then SIGKILL after `grace_s`) instead of leaving them blocked in
    the rendezvous or a barrier. Returns that rank's exit code (124 on timeout), else 0."""
    import subprocess
    import time
    port = _free_port()
    base = dict(os.environ if env is None else env)
    base.setdefault("PC_DIST_TIMEOUT_S", str(int(timeout)) if timeout else "300")
    procs = []
    for r in range(world):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(list(cmd), env=e))
    t0 = time.monotonic()
    failed = 0
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc is not None and rc != 0]
        if bad:
            failed = bad[0]
            break
        if all(rc == 0 for rc in rcs):
            return 0
        if timeout is not None and time.monotonic() - t0 > timeout:
            failed = 124
            break
        time.sleep(poll_s)
    # a rank failed (or the job timed out): take the others down
    for p in procs:
        if p.poll() is None:
            p.terminate()
    t1 = time.monotonic()
    while any(p.poll() is None for p in procs) and time.monotonic() - t1 < grace_s:
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait()
    return failed


def dist_timeout():
    """Rendezvous / collective timeout of the host process group (gloo): a rank whose
    peer died returns an error in seconds instead of gloo's 30-minute default."""
    import datetime
    return datetime.timedelta(seconds=float(os.environ.get("PC_DIST_TIMEOUT_S", "300")))


def device_for_rank(local_rank: int) -> int:
    """cuda:LOCAL_RANK, folded onto the visible devices when ranks outnumber them (a
    rehearsal of N ranks on a smaller box shares GPUs; the driver's N-GPU node does not)."""
    import torch
    n = torch.cuda.device_count()   # counts devices without initialising HIP
    return local_rank % n if n > 0 else local_rank


def face_runner(device_index: Optional[int] = None, **face_kwargs) -> FrameShardRunner:
    """A FrameShardRunner over a FaceEmbedder on this rank's GPU."""
    from .face_embedder import FaceEmbedder
    local = int(os.environ.get("LOCAL_RANK", "0")) if device_index is None else device_index
    face_kwargs.setdefault("yolo_model", "scrfd_10g_bnkps")
    fe = FaceEmbedder(ctx=f"cuda:{local}", **face_kwargs)
    return FrameShardRunner(lambda fr: fe.extract_batch(fr))
