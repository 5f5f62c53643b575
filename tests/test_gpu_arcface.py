"""ArcFace IResNet embed on the GPU (pc_arcface_embed) vs the fp32 CPU oracle.

Oracle: oracle/nets_torch.iresnet_forward on the unfolded params, fed the
reference preprocessing (face_embedder.py:1281-1288), combined with the
reference's flip-TTA sum and L2 normalisation (face_embedder.py:1383-1389,
restated in oracle/ref_algos.arcface_postprocess, pinned by golden vectors).
Tolerances: f32 path (PC_PREC_F32), the f16x3 split path (PC_PREC_F16X3, the default of FaceEmbedder,
DESIGN.md §3.7) and the opt-in f16c8 path (PC_PREC_F16C8) max-abs 1e-4 on unit embeddings and on cosine distances
(north_star); plain f16 (the reference's TRT fp16 precision) max-abs 1e-2 on embeddings,
5e-3 on cosine distances — measured error is reported in the assertion messages."""
import numpy as np
import pytest

from oracle import nets_torch as nt
from oracle import ref_algos as ra
from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F16C8, PC_PREC_F16X3, PC_PREC_F32
from person_capture_amd.engines import ArcFaceEngine, BankMatcher

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def r100():
    return models.synth_iresnet(100, seed=0)


def _oracle_embed(p, chips, flip=True):
    e = nt.iresnet_forward(p, 100, nt.arcface_input_from_chips(chips)).numpy()
    ef = nt.iresnet_forward(p, 100, nt.arcface_input_from_chips(chips[:, :, ::-1])).numpy() if flip else None
    return ra.arcface_postprocess(e, ef)


@pytest.mark.parametrize("prec,tol_e,tol_fd", [(PC_PREC_F32, 1e-4, 1e-4), (PC_PREC_F16X3, 1e-4, 1e-4),
                                              (PC_PREC_F16C8, 1e-4, 1e-4), (PC_PREC_F16, 1e-2, 5e-3)])
def test_arcface_embed_parity(gpu_ctx, r100, prec, tol_e, tol_fd):
    rng = np.random.default_rng(11)
    chips = rng.integers(0, 256, size=(6, 112, 112, 3), dtype=np.uint8)
    eng = ArcFaceEngine(gpu_ctx, r100, 100, precision=prec, max_batch=16)
    got = eng.embed(chips, flip=True)
    ref = _oracle_embed(r100, chips, flip=True)
    assert got.shape == ref.shape == (6, 512)
    err = np.abs(got - ref).max()
    assert err < tol_e, f"embedding max-abs err {err}"
    # cosine distances against a bank drawn from the oracle's own embeddings
    bank = ref[::-1].copy()
    fd_ref = np.array([ra.fd_min(v, bank) for v in ref], np.float32)
    fd_gpu, _ = BankMatcher(gpu_ctx).match(got, bank)
    dfd = np.abs(fd_gpu - fd_ref).max()
    assert dfd < tol_fd, f"cosine distance max-abs err {dfd}"


def test_arcface_no_flip_and_graph(gpu_ctx, r100):
    rng = np.random.default_rng(12)
    chips = rng.integers(0, 256, size=(3, 112, 112, 3), dtype=np.uint8)
    eng = ArcFaceEngine(gpu_ctx, r100, 100, precision=PC_PREC_F32, max_batch=4, graph=True)
    a = eng.embed(chips, flip=False)
    b = eng.embed(chips, flip=False)   # graph replay
    ref = _oracle_embed(r100, chips, flip=False)
    assert np.abs(a - ref).max() < 1e-4
    assert np.array_equal(a, b)


def test_arcface_f16x3_program_and_prep(gpu_ctx, r100):
    """The f16x3 program: a centred input (x - 127.5 exact in f16, the 1/127.5 in the split stem
    weights), split-K FC over the split 7x7x512 map; no resident chains (they are f16 only). The
    centred preprocessing itself is exact: pc_arcface_prep(PC_PREC_F16X3) == chip - 127.5."""
    import ctypes as C
    from person_capture_amd._lib import check
    eng = ArcFaceEngine(gpu_ctx, r100, 100, precision=PC_PREC_F16X3, max_batch=8)
    assert eng.program.split and eng.program.input_centered
    assert eng.net.chain_info()[0] == 0
    rng = np.random.default_rng(13)
    chips = rng.integers(0, 256, size=(2, 112, 112, 3), dtype=np.uint8)
    d = gpu_ctx.upload(chips)
    out = gpu_ctx.alloc(4 * 112 * 112 * 4 * 2)
    check(gpu_ctx.lib.pc_arcface_prep(gpu_ctx.handle, PC_PREC_F16X3, C.c_void_p(d.ptr), 2, 112, 1,
                                      C.c_void_p(out.ptr)), gpu_ctx.handle, "arcface_prep")
    got = gpu_ctx.download(out.ptr, (4, 112, 112, 4), np.float16).astype(np.float32)
    want = chips[..., ::-1].astype(np.float32) - 127.5
    assert np.array_equal(got[:2, ..., :3], want) and np.array_equal(got[2:, ..., :3], want[:, :, ::-1])
    assert not got[..., 3].any()


def test_arcface_f16c8_program(gpu_ctx, r100):
    """The f16c8 program: every trunk activation f16c8 but the FC's input (plain split), calibrated
    e4m3 scales (finite maxima for every conv output), every conv reading f16c8 on conv_fast's C8
    tiles (profile code 600 + tile) and no resident chains; 12 chips within 1e-4 of the oracle
    with and without graph replay."""
    eng = ArcFaceEngine(gpu_ctx, r100, 100, precision=PC_PREC_F16C8, max_batch=24, graph=True)
    P = eng.program
    assert P.input_centered and P.c8 and eng.net.chain_info()[0] == 0
    c8_convs = [i for i, w in enumerate(P.ops) if w[0] == 1 and P.tc8[w[3]]]
    assert len(c8_convs) == len([w for w in P.ops if w[0] == 1]) - 1   # all but the FC
    assert eng.absmax is not None and all(eng.absmax[t] > 0 for t in range(len(P.tc8)) if P.tc8[t])
    rng = np.random.default_rng(14)
    chips = rng.integers(0, 256, size=(12, 112, 112, 3), dtype=np.uint8)
    eng.net.set_graph(False)
    eng.net.profile(True)
    a = eng.embed(chips, flip=True)
    codes = {int(r[0]): int(r[4]) for r in eng.net.profile_ops()}
    eng.net.profile(False)
    assert all(600 <= codes[i] < 700 for i in c8_convs), codes
    eng.net.set_graph(True)
    b = eng.embed(chips, flip=True)
    c = eng.embed(chips, flip=True)
    ref = _oracle_embed(r100, chips, flip=True)
    err = float(np.abs(a - ref).max())
    print(f"f16c8 IResNet-100: max |de| {err:.2e}")
    assert err < 1e-4 and np.array_equal(b, c) and float(np.abs(b - ref).max()) < 1e-4


def test_arcface_f16x3_wg_form_bit_identical(gpu_ctx, monkeypatch):
    """The 256x224 fused split tile's WG form (weight fragments from global memory into registers,
    only the split pixel rows staged: pc_conv_fast.hip WG, pc_api.cpp pack_wfrag) runs the b256
    14x14x256 layers and gives the staged form's bits (PC_SX_WG=0): same K order, same passes."""
    from person_capture_amd.runtime import Net
    monkeypatch.setenv("PC_CONV_HXI", "0")   # (the 14x14x256 layers on the tiles, not conv_hxi)
    P = models.compile_iresnet(models.synth_iresnet(100, seed=4), 100, split=True)
    x = np.zeros((256, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(5).uniform(-127.5, 127.5, (256, 112, 112, 3))
    d = gpu_ctx.upload(x)
    outs, forms = [], []
    try:
        for wg in ("1", "0"):
            monkeypatch.setenv("PC_SX_WG", wg)
            net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=256)
            try:
                net.profile(True)
                net.run(d.ptr, 256)
                forms.append([(int(r[4]), int(r[5])) for r in net.profile_ops()])
                net.profile(False)
                outs.append(net.read_output(0, 256).copy())
            finally:
                net.close()
    finally:
        d.free()
    wg_launches = sum(1 for c, f in forms[0] if c == 113 and f & 3 == 3)
    assert wg_launches >= 50, forms[0]
    assert not any(f & 2 for c, f in forms[1] if 100 <= c < 200)
    assert sum(1 for c, f in forms[1] if c == 113 and f & 3 == 1) == wg_launches
    assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8))


def test_arcface_f16x3_wg_layouts_bit_identical(gpu_ctx, monkeypatch):
    """The WG tiles' wave layouts: 8x1 waves of 32x224 on the 256x224 tile and 4x2
    of 32x128 on 128x256 (default) against the 4x2 / 2x4 layouts of the cfg table (PC_WG_LAYOUT=0).
    Every accumulator takes the same MFMAs in the same order, so the outputs are bit-identical;
    the batch of 256 runs the 14x14x256 layers on 256x224 and the 28x28x128 layers on 128x256."""
    from person_capture_amd.runtime import Net
    monkeypatch.setenv("PC_CONV_HXI", "0")   # (the 14x14x256 layers on the 256x224 tile, not conv_hxi)
    P = models.compile_iresnet(models.synth_iresnet(100, seed=6), 100, split=True)
    x = np.zeros((256, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(7).uniform(-127.5, 127.5, (256, 112, 112, 3))
    d = gpu_ctx.upload(x)
    net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=256)
    outs = []
    try:
        net.profile(True)
        for lay in ("1", "0", "1"):
            monkeypatch.setenv("PC_WG_LAYOUT", lay)
            net.run(d.ptr, 256)
            outs.append(net.read_output(0, 256).copy())
        codes = {(int(r[4]), int(r[5])) for r in net.profile_ops()}
        net.profile(False)
    finally:
        net.close()
        d.free()
    assert (113, 3) in codes and (101, 3) in codes, codes
    assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8))
    assert np.array_equal(outs[0].view(np.uint8), outs[2].view(np.uint8))


@pytest.mark.parametrize("batch", [256, 300])
def test_arcface_f16x3_hxi_bit_identical(gpu_ctx, monkeypatch, batch):
    """conv_hxi (pc_conv_hxi.hip: a workgroup per 14x14 image / per 7 rows of a 28x28 image, the padded
    halo staged per group of 64 input channels) runs the 58 14x14x256 and 24 28x28x128
    layers of a large batch (profile codes 502 / 503; PC_CONV_HXI=19: those and the 4 7x7x512 ones, code
    505, at pitch 9 - fragments that span two rows) and gives the fused tiles'
    bits (PC_CONV_HXI=0): same K order (64-channel groups, taps, 32-channel blocks), same MFMA order per
    k-step, conv_epilogue_lds's arithmetic (with and without residual). The 28x28 form runs at two
    workgroups per CU with one halo stage (default) or one per CU with two (PC_HXI28_OCC=1): same bits."""
    from person_capture_amd.runtime import Net
    P = models.compile_iresnet(models.synth_iresnet(100, seed=8), 100, split=True)
    x = np.zeros((batch, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(9).uniform(-127.5, 127.5, (batch, 112, 112, 3))
    d = gpu_ctx.upload(x)
    outs, codes = [], []
    try:
        for hxi, env in (("19", {}), ("0", {}), ("19", {"PC_HXI28_OCC": "1"})):
            monkeypatch.setenv("PC_CONV_HXI", hxi)
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=batch)
            try:
                net.profile(True)
                net.run(d.ptr, batch)
                codes.append([int(r[4]) for r in net.profile_ops()])
                net.profile(False)
                outs.append(net.read_output(0, batch).copy())
            finally:
                net.close()
    finally:
        d.free()
    assert sum(1 for c in codes[0] if c == 502) == 58 and sum(1 for c in codes[0] if c == 503) == 24, codes[0]
    assert sum(1 for c in codes[0] if c == 505) == 4, codes[0]
    assert not {502, 503, 505} & set(codes[1])
    assert codes[2] == codes[0]
    assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8))
    assert np.array_equal(outs[0].view(np.uint8), outs[2].view(np.uint8))


@pytest.mark.parametrize("batch", [1, 12, 30])
def test_arcface_f16x3_hxi_small_bit_identical(gpu_ctx, monkeypatch, batch):
    """conv_hxi's small-batch forms (PC_CONV_HXI bit 5; codes 506 / 507 / 508: 32 output channels of 7 rows
    per workgroup, 16 workgroups per image) run the 14x14x256 / 28x28x128 / 7x7x512 layers of the plans for
    <= 32 images - a per-frame extract()'s rows - and give the fused tiles' bits (PC_CONV_HXI=0)."""
    from person_capture_amd.runtime import Net
    P = models.compile_iresnet(models.synth_iresnet(100, seed=12), 100, split=True)
    x = np.zeros((batch, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(13).uniform(-127.5, 127.5, (batch, 112, 112, 3))
    d = gpu_ctx.upload(x)
    outs, codes = [], []
    try:
        for hxi in ("59", "0"):
            monkeypatch.setenv("PC_CONV_HXI", hxi)
            net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=512)
            try:
                net.profile(True)
                net.run(d.ptr, batch)
                codes.append([int(r[4]) for r in net.profile_ops()])
                net.profile(False)
                outs.append(net.read_output(0, batch).copy())
            finally:
                net.close()
    finally:
        d.free()
    assert [sum(1 for c in codes[0] if c == k) for k in (506, 507, 508)] == [58, 24, 4], codes[0]
    assert not {502, 503, 505, 506, 507, 508} & set(codes[1])
    assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8))


def test_arcface_f16_hxi_bit_identical(gpu_ctx, monkeypatch):
    """The plain f16 form of conv_hxi (BASELINE C2's fp16 net: the halo holds every input channel, K walks
    taps then 32-channel blocks - the plain tiles' and the resident chain's order) on the 14x14x256 and
    28x28x128 layers (PC_CONV_HXI bits 2 / 3, chains off) gives the default plan's bits (resident chains
    on the 14x14 stage, conv_fast tiles on 28x28)."""
    from person_capture_amd.runtime import Net
    P = models.compile_iresnet(models.synth_iresnet(100, seed=10), 100, split=False)
    x = np.zeros((256, 112, 112, 4), np.float16)
    x[..., :3] = np.random.default_rng(11).uniform(-1, 1, (256, 112, 112, 3))
    d = gpu_ctx.upload(x)
    outs, codes = [], []
    try:
        for env in ({"PC_CONV_HXI": "12", "PC_CHAIN_MIN": "100000"}, {"PC_CONV_HXI": "0"}):
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=256)
            try:
                net.profile(True)
                net.run(d.ptr, 256)
                codes.append([int(r[4]) for r in net.profile_ops()])
                net.profile(False)
                outs.append(net.read_output(0, 256).copy())
            finally:
                net.close()
            monkeypatch.delenv("PC_CHAIN_MIN", raising=False)
    finally:
        d.free()
    assert sum(1 for c in codes[0] if c == 502) == 58 and sum(1 for c in codes[0] if c == 503) == 24, codes[0]
    assert 300 in codes[1] and 502 not in codes[1]   # (300: a resident chain launch)
    assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8))
