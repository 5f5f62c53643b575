"""ArcFace IResNet embed on the GPU (pc_arcface_embed) vs the fp32 CPU oracle.

Oracle: oracle/nets_torch.iresnet_forward on the unfolded params, fed the
reference preprocessing (face_embedder.py:1281-1288), combined with the
reference's flip-TTA sum and L2 normalisation (face_embedder.py:1383-1389,
restated in oracle/ref_algos.arcface_postprocess, pinned by golden vectors).
Tolerances: f32 path (PC_PREC_F32) max-abs 1e-4 on unit embeddings and on
cosine distances (north_star); f16 path (the throughput configuration, like the
reference's TRT fp16 engines) max-abs 1e-2 on embeddings, 5e-3 on cosine
distances — measured error is reported in the assertion messages."""
import numpy as np
import pytest

from oracle import nets_torch as nt
from oracle import ref_algos as ra
from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F32
from person_capture_amd.engines import ArcFaceEngine, BankMatcher

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def r100():
    return models.synth_iresnet(100, seed=0)


def _oracle_embed(p, chips, flip=True):
    e = nt.iresnet_forward(p, 100, nt.arcface_input_from_chips(chips)).numpy()
    ef = nt.iresnet_forward(p, 100, nt.arcface_input_from_chips(chips[:, :, ::-1])).numpy() if flip else None
    return ra.arcface_postprocess(e, ef)


@pytest.mark.parametrize("prec,tol_e,tol_fd", [(PC_PREC_F32, 1e-4, 1e-4), (PC_PREC_F16, 1e-2, 5e-3)])
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
