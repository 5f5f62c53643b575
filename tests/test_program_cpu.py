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


@pytest.mark.parametrize("mode", ["split", "c8"])
def test_iresnet_f32_class_program_flags(r18, mode):
    """The f16x3 / f16c8 IResNet programs: centred input (split-word bit 1 of the
    input tensor), 1/127.5 folded into the stem weights, every trunk activation split - f16c8
    (bit 2) in the c8 form except the FC's input, which stays [hi | lo] for split-K - and the
    split weight columns [W_hi, W_hi, W_lo] that reproduce the f32 weights to f32 precision."""
    P = models.compile_iresnet(r18, 18, split=mode == "split", c8=mode == "c8")
    assert P.input_centered and P.split and P.c8 == (mode == "c8")
    fc = P.ops[-1]
    assert fc[24] > 1 and not P.tc8[fc[3]] and P.tsplit[fc[3]]
    convs = [w for w in P.ops if w[0] == 1]
    assert all(P.tsplit[w[3]] for w in convs)
    if mode == "c8":
        assert all(P.tc8[w[3]] for w in convs[:-1])
    plain = models.compile_iresnet(r18, 18)
    st, st0 = P.ops[0], plain.ops[0]
    assert np.allclose(P.arrays[st[7]] * 127.5, plain.arrays[st0[7]], rtol=1e-6, atol=1e-9)
    # serialized split words: input bit 1, f16c8 bit 2
    blob = P.serialize()
    head = np.frombuffer(blob[:32], dtype="<i4")
    nbuf, nten = head[2], head[3]
    words = np.frombuffer(blob[32 + nbuf * 16: 32 + nbuf * 16 + nten * 32], dtype="<i4").reshape(nten, 8)
    assert words[P.input, 7] & 2
    assert all(bool(words[t, 7] & 4) == bool(P.tc8[t]) for t in range(nten))
    # split weight columns sum back to the plain program's weights (f32 products of f16 halves)
    w1 = convs[0]   # layer1.0.conv1: one 3x3 segment
    a, b = P.arrays[w1[13]].reshape(w1[14], -1), plain.arrays[plain.ops[1][13]].reshape(w1[14], -1)
    cp = P.dims(w1[3])[2]
    taps = a.reshape(w1[14], 9, 3, cp)
    assert np.allclose(taps[:, :, 0] + taps[:, :, 2], b.reshape(w1[14], 9, cp), rtol=0, atol=1e-7)
