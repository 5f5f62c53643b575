"""CPU check of the inference-time algebra in person_capture_amd/models.py: the
compiled programs (BN folded, pre-BN border tables, avg-down as 2x2/s2,
PAFPN fusions, FC as split-K 7x7 conv) run through a torch interpreter of the
device semantics must match the literal fp32 oracle nets."""
import numpy as np
import pytest
import torch

from oracle import nets_torch as nt
from person_capture_amd import models
from program_emulator import run_program


@pytest.fixture(scope="module")
def r18():
    return models.synth_iresnet(18, seed=1)


def test_iresnet_program_matches_oracle(r18):
    rng = np.random.default_rng(0)
    chips = rng.integers(0, 256, (2, 112, 112, 3), dtype=np.uint8)
    ref = nt.iresnet_forward(r18, 18, nt.arcface_input_from_chips(chips)).numpy()
    P = models.compile_iresnet(r18, 18)
    x = np.zeros((2, 112, 112, 4), np.float32)
    x[..., :3] = chips[..., ::-1].astype(np.float32) / 127.5 - 1.0
    (e,) = run_program(P, x)
    got = e[:, :512, 0, 0].numpy()
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-4


@pytest.mark.parametrize("variant", ["2.5g", "10g"])
def test_scrfd_program_matches_oracle(variant):
    p = models.synth_scrfd(variant, seed=2)
    D = 160 if variant == "10g" else 192
    rng = np.random.default_rng(1)
    x = np.zeros((1, D, D, 4), np.float32)
    x[..., :3] = (rng.integers(0, 256, (1, D, D, 3)).astype(np.float32) - 127.5) / 128.0
    ref = nt.scrfd_forward(p, variant, torch.from_numpy(np.ascontiguousarray(x[..., :3].transpose(0, 3, 1, 2))))
    P = models.compile_scrfd(p, variant, D)
    outs = run_program(P, x)
    for o, r in zip(outs, ref):
        got = o.permute(0, 2, 3, 1)[..., :30].numpy()
        r = r.numpy()
        assert np.abs(got - r).max() / max(1.0, np.abs(r).max()) < 1e-4


def test_program_serialization_and_buffer_reuse(r18):
    P = models.compile_iresnet(r18, 18)
    blob = P.serialize()
    w = np.frombuffer(blob[:32], dtype="<i4")
    assert w[0] == 0x544E4350 and w[1] == 1
    phys, mapping = P._assign_buffers()
    assert len(phys) < len(P.vbufs) / 4          # liveness reuse
    # no op may write a buffer it also reads
    for op in P.ops:
        ins, out = P._op_io(op)
        ob = mapping[P.tensors[out][0]]
        for t in ins:
            if P.tensors[t][0] >= 0:
                assert mapping[P.tensors[t][0]] != ob
    assert 4e9 < P.flops_per_image < 8e9           # IResNet-18 at 112x112


@pytest.mark.parametrize("variant", ["2.5g", "10g"])
def test_scrfd_split_program_is_f32_class(variant):
    """f16x3 detector: with every activation stored as f16 hi + lo and the
    weights expanded to [W_hi, W_hi, W_lo] per tap, the emulated device semantics (f16
    rounding of both halves and of the weight halves) stay at f32-class error against the
    fp32 oracle - what the f16 form (1e-2-class) cannot."""
    p = models.synth_scrfd(variant, seed=2)
    D = 160 if variant == "10g" else 192
    rng = np.random.default_rng(1)
    x = np.zeros((1, D, D, 4), np.float32)
    x[..., :3] = (rng.integers(0, 256, (1, D, D, 3)).astype(np.float32) - 127.5) / 128.0
    ref = nt.scrfd_forward(p, variant, torch.from_numpy(np.ascontiguousarray(x[..., :3].transpose(0, 3, 1, 2))))
    P = models.compile_scrfd(p, variant, D, split=True)
    assert sum(P.tsplit) > 0 and all(P.tensors[t][6] == 0 for t in range(len(P.tensors)) if P.tsplit[t])
    words = np.frombuffer(P.serialize(), dtype="<i4")
    nbuf, nten = words[2], words[3]
    trec = words[8 + 4 * nbuf: 8 + 4 * nbuf + 8 * nten].reshape(nten, 8)
    assert list(trec[:, 7]) == P.tsplit
    outs = run_program(P, x)
    worst = 0.0
    for o, r in zip(outs, ref):
        got = o.permute(0, 2, 3, 1)[..., :30].numpy()
        r = r.numpy()
        worst = max(worst, np.abs(got - r).max() / max(1.0, np.abs(r).max()))
    # (the plain program in fp32 emulation, i.e. only the folding algebra, is at ~3e-6 here)
    assert worst < 1e-5, worst
