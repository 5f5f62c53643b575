"""Multi-process (gloo, world_size 2, CPU) coverage of the frame-shard runner:
contiguous assignment and frame-ordered gather on rank 0; the bench's
max-over-ranks timing reduction; and the rank launcher bench.py --gpus N uses."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from person_capture_amd.shard import FrameShardRunner, merge_in_order, shard_indices


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = [f"frame{i}" for i in range(n)]
    seen = []

    def extract(fr):
        seen.extend(fr)
        return [{"frame": f, "rank": rank} for f in fr]

    out = FrameShardRunner(extract).process(frames)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, seen, out, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [0, 1, 7, 8])
def test_frame_shard_gloo_world2(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, seen, out, mx = q.get(timeout=120)
        res[r] = (seen, out, mx)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    h = n // 2
    assert res[0][0] == [f"frame{i}" for i in range(0, h)]
    assert res[1][0] == [f"frame{i}" for i in range(h, n)]
    assert res[1][1] is None
    assert [d["frame"] for d in res[0][1]] == [f"frame{i}" for i in range(n)]
    assert all(d["rank"] == (0 if i < h else 1) for i, d in enumerate(res[0][1]))
    assert res[0][2] == res[1][2] == 2.0


def test_shard_helpers():
    for n in range(0, 20):
        for w in (1, 2, 3, 8):
            parts = [shard_indices(n, r, w) for r in range(w)]
            assert [i for p in parts for i in p] == list(range(n))   # contiguous, in rank order
            assert max(map(len, parts)) - min(map(len, parts)) <= 1
            assert merge_in_order(n, w, parts) == list(range(n))


def test_bench_launcher_world2():
    """bench.py --gpus 2 (no torch.distributed.run) spawns two rank processes with the
    launcher environment; they init gloo, split the frames contiguously and rank 0 prints
    ONE JSON line with n_gpus 2 and the frames of both ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                        "--batch", "5"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["frames"] == 2 * 5 * 3 and out["local_rank"] == 0


def test_bench_launcher_fails_fast():
    """One of two ranks exits 1 before the rendezvous: the launcher takes the other rank
    (blocked in init_process_group) down and returns non-zero within seconds, instead of
    hanging until gloo's timeout."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1",
                        "--batch", "2", "--fail-rank", "1"], capture_output=True, text=True, timeout=120, env=env)
    dt = time.monotonic() - t
    assert r.returncode != 0
    assert dt < 60, dt


def test_spawn_timeout_kills_ranks():
    import sys
    import time
    from person_capture_amd.shard import spawn_local_ranks
    t = time.monotonic()
    rc = spawn_local_ranks([sys.executable, "-c", "import time; time.sleep(600)"], 2, timeout=2.0, grace_s=2.0)
    assert rc == 124 and time.monotonic() - t < 30


def test_bench_dry_run_c5_world2():
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--workload",
                        "c5", "--steps", "2", "--batch", "3"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2
