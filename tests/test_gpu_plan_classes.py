"""Small-batch plan classes (pc_api.cpp plan_conv / plan_class): a run of a few images takes
the tiles planned for its batch class (1 / 4 / 16 / 32 / 64 images, up to a quarter of
max_batch) - including the deep-ring small conv_fast tiles 15-19 that only those plans use.
Tile shape, ring depth and K-row width do not change any output's K order, so the same rows must come out
bit for bit as inside a large batch (the max-batch plans): extract() and extract_batch() are
bit-identical by contract (test_gpu_face_embedder). The f16x3 split program too: its fused split
tiles walk K in channel groups of 64 (every tap of a group, then the next group), an order that
64- and 128-byte K rows share, so its classes pick their row widths freely - and do."""
import numpy as np
import pytest

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import Net

pytestmark = pytest.mark.gpu


def _run(ctx, net, x, N, outs, forms=None):
    d = ctx.upload(np.ascontiguousarray(x[:N]))
    net.profile(True)
    net.run(d.ptr, N)
    recs = net.profile_ops()
    codes = [int(r[4]) for r in recs]
    if forms is not None:   # op -> (kernel code, conv_fast form bits)
        forms.update({int(r[0]): (int(r[4]), int(r[5])) for r in recs})
    net.profile(False)
    res = [net.read_output(k, N).copy() for k in range(outs)]
    d.free()
    return res, codes


def _images(n, side, seed):
    x = np.zeros((n, side, side, 4), np.float16)
    x[..., :3] = np.random.default_rng(seed).uniform(-1, 1, (n, side, side, 3))
    return x


@pytest.mark.parametrize("depth,mode", [(100, "f16"), (50, "f16"), (100, "f16x3"), (100, "f16c8")])
def test_arcface_small_batches_bit_identical_to_large_batch(gpu_ctx, depth, mode):
    """f16x3 / f16c8 too: their plans keep one K-row width per conv, so the f16 and
    block-scaled e4m3 MFMAs accumulate in the same order in every plan class."""
    P = models.compile_iresnet(models.synth_iresnet(depth, seed=4), depth, split=mode == "f16x3", c8=mode == "f16c8")
    net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=512)
    try:
        x = _images(200, 112, 9)
        if P.input_centered:
            x *= 127.5
        if mode == "f16c8":
            d = gpu_ctx.upload(x)
            net.calibrate(d.ptr, 200)
            d.free()
        large_forms, rows_differ = {}, 0
        (large,), _ = _run(gpu_ctx, net, x, 200, 1, large_forms)
        ran_small = ran_hxs = 0
        for N in (1, 2, 5, 12, 30, 64):
            small_forms = {}
            (small,), codes = _run(gpu_ctx, net, x, N, 1, small_forms)
            # conv_fast small-batch tiles (C8: 615..), conv_hxi's small-batch forms (f16x3: 506-508)
            ran_small += sum(1 for c in codes if 115 <= c % 500 < 120 or 506 <= c <= 508)
            ran_hxs += sum(1 for c in codes if 506 <= c <= 508)
            # fused split tiles of one conv at different K-row widths in the two classes (the
            # channel-group K order makes them accumulate alike)
            rows_differ += sum(1 for op, (c, f) in small_forms.items() if 100 <= c < 200 and f & 1 and
                               op in large_forms and large_forms[op][1] & 1 and (f ^ large_forms[op][1]) & 4)
            assert small.dtype == large.dtype
            assert np.array_equal(small.view(np.uint8), large[:N].view(np.uint8)), \
                (N, float(np.abs(small.astype(np.float64) - large[:N]).max()))
        assert ran_small >= 100, ran_small
        if mode == "f16x3":
            assert rows_differ > 0
            assert ran_hxs == 5 * 86, ran_hxs   # (N = 1 .. 30: 58 + 24 + 4 layers each; 64 rows: the tiles)
    finally:
        net.close()


@pytest.mark.parametrize("split", [False, True])
def test_scrfd_single_frame_bit_identical_to_batch(gpu_ctx, split):
    P = models.compile_scrfd(models.synth_scrfd("10g", seed=2), "10g", 320, split=split)
    net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=64)   # f16x3: a split program on an f16 net
    try:
        x = _images(40, 320, 3)
        nout = len(P.outputs)
        large, lcodes = _run(gpu_ctx, net, x, 40, nout)
        if split:   # the halo-staged kernels run the large batch's 64- / 96-channel layers (round 6: in
            # the fused tiles' accumulation order), the small classes the fused tiles - same bits
            assert 500 in lcodes and 501 in lcodes, lcodes
        for N in (1, 3, 16):
            small, codes = _run(gpu_ctx, net, x, N, nout)
            assert any(115 <= c < 120 for c in codes), codes
            if split and N == 1:
                assert 500 not in codes and 501 not in codes, codes
                assert 504 in codes, codes   # conv_hxg's small-batch form on the 80x80 / 40x40 x96 layers
            for k in range(nout):
                assert np.array_equal(small[k].view(np.uint8), large[k][:N].view(np.uint8)), (N, k)
    finally:
        net.close()


def test_graph_replay_of_a_full_arcface_quantum(gpu_ctx):
    """FaceEmbedder replays captured HIP graphs for ArcFace runs up to 4 x PERSON_CAPTURE_AMD_GRAPH_BATCH
    rows (default 512: a whole C3 quantum of 256 rows): the capture and its replays give the eager run's
    bits, and a profiled run executes eagerly (its per-op events are the point)."""
    P = models.compile_iresnet(models.synth_iresnet(100, seed=12), 100, split=True)
    net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=256)
    try:
        x = _images(256, 112, 13) * 127.5
        d = gpu_ctx.upload(x)
        net.run(d.ptr, 256)
        eager = net.read_output(0, 256).copy()
        net.set_graph(True, max_batch=512)
        outs = []
        for _ in range(2):   # capture, then replay
            net.run(d.ptr, 256)
            outs.append(net.read_output(0, 256).copy())
        net.profile(True)
        net.run(d.ptr, 256)
        nrec = len(net.profile_ops())
        net.profile(False)
        d.free()
        for o in outs:
            assert np.array_equal(o.view(np.uint8), eager.view(np.uint8))
        assert nrec >= 90, nrec   # (one record per op of the run)
    finally:
        net.close()
