"""Small-batch conv plans (pc_api.cpp plan_conv, small=true): tiles chosen for a few images,
and long-K convs split over K on the generic kernel with the partials finished by
splitk_finish (bias per channel / border class, PReLU, residual, act order). The same rows
run as a small batch and inside a large batch (max-batch plans) must agree within the f16
tolerance (split-K sums in another order, so not bit for bit), and split-K must have run.
Split-K is opt-in (PC_SMALL_SPLITK=1); without it the small plans keep the K order, and a
frame's results do not depend on its batch (test_gpu_face_embedder)."""
import os

import numpy as np
import pytest

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import Net

pytestmark = pytest.mark.gpu


def _run(ctx, net, x, N):
    d = ctx.upload(x[:N])
    net.profile(True)
    net.run(d.ptr, N)
    recs = net.profile_ops()
    net.profile(False)
    out = net.read_output(0, N)
    d.free()
    return out, recs


@pytest.mark.parametrize("depth", [100, 50])
def test_arcface_small_batch_split_k_matches_large_batch(gpu_ctx, monkeypatch, depth):
    monkeypatch.setenv("PC_SMALL_SPLITK", "1")   # opt-in: results then depend on the batch size
    P = models.compile_iresnet(models.synth_iresnet(depth, seed=4), depth)
    net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=64)   # small plans for <= 16 images
    try:
        _check_arcface(gpu_ctx, net)
    finally:
        net.close()


def _check_arcface(gpu_ctx, net):
    rng = np.random.default_rng(9)
    x = np.zeros((40, 112, 112, 4), np.float16)
    x[..., :3] = rng.uniform(-1, 1, (40, 112, 112, 3))
    small, recs = _run(gpu_ctx, net, x, 12)
    large, _ = _run(gpu_ctx, net, x, 40)
    codes = [int(r[4]) for r in recs]
    assert codes.count(-1) >= 20, f"too few split-K generic launches in the small-batch run: {codes.count(-1)}"
    ref = large[:12]
    err = np.abs(small - ref).max() / max(1.0, np.abs(ref).max())
    assert err < 1e-2, err
    e1 = small.reshape(12, -1)
    e2 = ref.reshape(12, -1)
    cos = (e1 * e2).sum(1) / np.linalg.norm(e1, axis=1) / np.linalg.norm(e2, axis=1)
    assert cos.min() > 0.9999, cos.min()


def test_scrfd_single_frame_matches_batch(gpu_ctx, monkeypatch):
    monkeypatch.setenv("PC_SMALL_SPLITK", "1")
    P = models.compile_scrfd(models.synth_scrfd("2.5g", seed=2), "2.5g", 320)
    net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=24)
    try:
        _check_scrfd(gpu_ctx, net)
    finally:
        net.close()


def _check_scrfd(gpu_ctx, net):
    rng = np.random.default_rng(3)
    x = np.zeros((20, 320, 320, 4), np.float16)
    x[..., :3] = rng.uniform(-1, 1, (20, 320, 320, 3))
    for k in range(3):
        d = gpu_ctx.upload(x[:1])
        net.run(d.ptr, 1)
        one = net.read_output(k, 1)
        d2 = gpu_ctx.upload(x)
        net.run(d2.ptr, 20)
        many = net.read_output(k, 20)[:1]
        err = np.abs(one - many).max() / max(1.0, np.abs(many).max())
        assert err < 3e-2, (k, err)
        d.free()
        d2.free()
