"""f16x3 SCRFD (the default detector precision) on the GPU.

Every activation of the split program is an f16 pair [hi | lo] and every conv walks K as
[hi, lo, hi] against [W_hi, W_hi, W_lo]: the net must be f32-class against the fp32 oracle
(oracle/nets_torch.scrfd_forward) on every conv kernel family that can run it - the split
2-D block kernel (conv_t2d SPLIT), the statically scheduled kernel (conv_fast SPLIT
epilogue; fused split tiles - hi and lo pixel rows with both weight halves per K tile - or the
virtual [hi, lo, hi] K) and the generic implicit GEMM (conv_igemm, run-time split flags) - with the split
stem (W_hi + W_lo K steps) and the split max pool. The t2d and conv_fast paths accumulate K
in the same order, so the whole net is bit-identical between them. At the detection level
the f16x3 boxes and landmarks are the f32 path's (the property the headline's identical
accept decisions rest on, bench.py parity).
"""
import numpy as np
import pytest
import torch

from oracle import cv_ops
from oracle import nets_torch as nt
from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16X3, PC_PREC_F32
from person_capture_amd.engines import ScrfdEngine, make_letterbox_desc

pytestmark = pytest.mark.gpu

# f32-class bound on the head tensors (relative to max(1, |ref|)): the f32 device mode is held
# to 1e-4 in tests/test_gpu_scrfd.py; the split form measures ~1e-5 (printed)
TOL_X3 = 1e-4


@pytest.fixture(scope="module")
def s10g():
    return models.synth_scrfd("10g", seed=0)


def _frame(seed, H=360, W=640):
    return np.random.default_rng(seed).integers(0, 256, size=(H, W, 3), dtype=np.uint8)


def _heads_vs_oracle(ctx, p, variant, D, frames, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    eng = ScrfdEngine(ctx, p, variant, D=D, precision=PC_PREC_F16X3, max_batch=len(frames))
    devs = [ctx.upload(f) for f in frames]
    eng.detect_frames([(d.ptr, f.shape[0], f.shape[1], f.strides[0]) for d, f in zip(devs, frames)], thresh=0.5)
    outs = [eng.net.read_output(lvl, len(frames)) for lvl in range(3)]
    worst = 0.0
    for i, f in enumerate(frames):
        desc, _ = make_letterbox_desc(0, f.shape[0], f.shape[1], f.strides[0], D)
        blob = cv_ops.letterbox_blob(f, D, desc.new_w, desc.new_h, desc.scale_x, desc.scale_y, desc.simd_end)
        x = torch.from_numpy(np.ascontiguousarray(blob[None, ..., :3].transpose(0, 3, 1, 2)))
        ref = [t[0].numpy() for t in nt.scrfd_forward(p, variant, x)]
        for lvl in range(3):
            got = outs[lvl][i, ..., :30]
            worst = max(worst, float(np.abs(got - ref[lvl]).max() / max(1.0, np.abs(ref[lvl]).max())))
    for k in env:
        monkeypatch.delenv(k)
    return worst, outs, eng


KERNEL_MODES = {
    "default": {},                                             # split t2d (32-ch trunk), halo-staged 64-ch, fused tiles
    "virtual": {"PC_SPLIT_FUSED": "0"},                        # conv_fast walking the virtual [hi, lo, hi] K
    "t2d64": {"PC_T2D_SPLIT64": "1"},                          # + the opt-in 64-channel split t2d
    "fast": {"PC_CONV_T2D": "0"},                              # conv_fast everywhere it runs
    "igemm": {"PC_CONV_T2D": "0", "PC_CONV_FAST": "0"},        # the generic kernel
    "nohx": {"PC_CONV_HX": "0"},                               # 64/96-ch layers on conv_fast's fused tiles
    "nohxg": {"PC_CONV_HXG": "0"},                             # 96-ch layers on conv_fast's fused tiles
}


@pytest.mark.parametrize("mode", list(KERNEL_MODES))
def test_split_net_parity_f32_class(gpu_ctx, s10g, mode, monkeypatch):
    worst, _, _ = _heads_vs_oracle(gpu_ctx, s10g, "10g", 320, [_frame(1), _frame(2)], KERNEL_MODES[mode],
                                   monkeypatch)
    print(f"f16x3 SCRFD-10G D=320 [{mode}]: head rel err {worst:.2e}")
    assert worst < TOL_X3, worst


def test_split_net_parity_2_5g(gpu_ctx, monkeypatch):
    p = models.synth_scrfd("2.5g", seed=0)
    worst, _, _ = _heads_vs_oracle(gpu_ctx, p, "2.5g", 320, [_frame(3)], {}, monkeypatch)
    print(f"f16x3 SCRFD-2.5G D=320: head rel err {worst:.2e}")
    assert worst < TOL_X3, worst


def test_split_t2d_close_to_conv_fast(gpu_ctx, s10g, monkeypatch):
    """The split t2d kernel sums the three products per 32-channel chunk (W_hi*hi, W_lo*hi,
    W_hi*lo), the implicit-GEMM kernels per [hi, lo, hi] block: the same values to f32 class
    (relative 1e-5 on the heads), not bitwise."""
    frames = [_frame(4), _frame(5)]
    _, a, _ = _heads_vs_oracle(gpu_ctx, s10g, "10g", 320, frames, {}, monkeypatch)
    _, b, _ = _heads_vs_oracle(gpu_ctx, s10g, "10g", 320, frames, {"PC_CONV_T2D": "0"}, monkeypatch)
    for x, y in zip(a, b):
        assert np.abs(x - y).max() / max(1.0, np.abs(y).max()) < 1e-5


def test_split_t2d_ran(gpu_ctx, s10g):
    """The planner sends the 32-channel split trunk convs to the split t2d kernel (64 channels:
    opt-in PC_T2D_SPLIT64, measured slower than conv_fast)."""
    eng = ScrfdEngine(gpu_ctx, s10g, "10g", D=320, precision=PC_PREC_F16X3, max_batch=1)
    f = _frame(6)
    d = gpu_ctx.upload(f)
    eng.net.profile(True)
    eng.detect_frames([(d.ptr, f.shape[0], f.shape[1], f.strides[0])], thresh=0.5)
    codes = [int(r[4]) for r in eng.net.profile_ops()]
    eng.net.profile(False)
    assert sum(1 for c in codes if 200 <= c < 300) == 2, codes   # stem.3 (32->32), stem.6 (32->64)


@pytest.mark.parametrize("seed", [20, 21])
def test_split_detections_match_f32(gpu_ctx, s10g, seed):
    """1080p frame at D=640: the f16x3 detector's boxes and landmarks are the f32 path's
    (same count; boxes within 1e-3 px, landmarks within 1e-3 px), ignoring candidates whose
    score lies within 1e-4 of the threshold."""
    D, thresh = 640, 0.5
    f = _frame(seed, 1080, 1920)
    d = gpu_ctx.upload(f)
    src = [(d.ptr, f.shape[0], f.shape[1], f.strides[0])]
    (a_det, a_kps), = ScrfdEngine(gpu_ctx, s10g, "10g", D=D, precision=PC_PREC_F16X3, max_batch=1).detect_frames(
        src, thresh=thresh)
    (b_det, b_kps), = ScrfdEngine(gpu_ctx, s10g, "10g", D=D, precision=PC_PREC_F32, max_batch=1).detect_frames(
        src, thresh=thresh)
    ka = np.abs(a_det[:, 4] - thresh) > 1e-4
    kb = np.abs(b_det[:, 4] - thresh) > 1e-4
    assert ka.sum() == kb.sum() and ka.sum() > 0
    db = np.abs(a_det[ka] - b_det[kb]).max()
    dk = np.abs(a_kps[ka] - b_kps[kb]).max()
    print(f"f16x3 vs f32 detections: {int(ka.sum())} faces, max |dbox| {db:.2e} px, max |dkps| {dk:.2e} px")
    assert db < 1e-3 and dk < 1e-3


@pytest.mark.parametrize("hx", ["default", "off"])
def test_split_hx_ran(gpu_ctx, s10g, hx, monkeypatch):
    """The planner sends the f16x3 64 -> 64 channel 3x3 layers of a C3 detection chunk (32 frames) to
    the halo-staged kernel (profile code 500): at D=640 the 160x160, 80x80 and 40x40 ones (40 is not a
    multiple of its 16-pixel blocks: partial blocks), and never under PC_CONV_HX=0. (A single frame's
    grids are too small for it: its plan keeps the fused tiles, bit-identically - test_gpu_plan_classes.)"""
    if hx == "off":
        monkeypatch.setenv("PC_CONV_HX", "0")
    eng = ScrfdEngine(gpu_ctx, s10g, "10g", D=640, precision=PC_PREC_F16X3, max_batch=32)
    f = _frame(7)
    d = gpu_ctx.upload(f)
    eng.net.profile(True)
    eng.detect_frames([(d.ptr, f.shape[0], f.shape[1], f.strides[0])] * 32, thresh=0.5)
    recs = eng.net.profile_ops()
    eng.net.profile(False)
    hx_ops = [int(r[0]) for r in recs if int(r[4]) == 500]
    if hx == "off":
        assert not hx_ops
        return
    sizes = {eng.program.tensors[eng.program.ops[o][1]][1] for o in hx_ops}
    assert {160, 80, 40} <= sizes, sorted(sizes)


def test_split_net_parity_d640_hxg(gpu_ctx, s10g, monkeypatch):
    """D=640: the 96-channel trunk at 80x80 / 40x40 / 20x20 runs on conv_hxg (the 16x20 blocks cover
    80 exactly; 40 and 20 leave partial blocks) - f32 class against the oracle on the heads."""
    worst, _, eng = _heads_vs_oracle(gpu_ctx, s10g, "10g", 640, [_frame(8, 720, 1280)], {}, monkeypatch)
    print(f"f16x3 SCRFD-10G D=640 (conv_hxg on the 96-channel trunk): head rel err {worst:.2e}")
    assert worst < TOL_X3, worst


@pytest.mark.parametrize("hxg", ["default", "off"])
def test_split_hxg_ran(gpu_ctx, s10g, hxg, monkeypatch):
    """The planner sends the f16x3 96 -> 96 channel 3x3 layers of a C3 detection chunk (32 frames) to
    conv_hxg (profile code 501) where its grid fills the CUs - the 80x80 and 40x40 maps of D=640 - and
    never under PC_CONV_HXG=0 (conv_hx64 keeps the 64-channel ones); a single frame keeps the fused
    tiles on all of them."""
    if hxg == "off":
        monkeypatch.setenv("PC_CONV_HXG", "0")
    eng = ScrfdEngine(gpu_ctx, s10g, "10g", D=640, precision=PC_PREC_F16X3, max_batch=32)
    f = _frame(9)
    d = gpu_ctx.upload(f)
    eng.net.profile(True)
    eng.detect_frames([(d.ptr, f.shape[0], f.shape[1], f.strides[0])] * 32, thresh=0.5)
    recs = eng.net.profile_ops()
    eng.net.profile(False)
    codes = [int(r[4]) for r in recs]
    assert 500 in codes
    hxg_ops = [int(r[0]) for r in recs if int(r[4]) == 501]
    if hxg == "off":
        assert not hxg_ops
        return
    sizes = {eng.program.tensors[eng.program.ops[o][1]][1] for o in hxg_ops}
    assert {80, 40} <= sizes, sorted(sizes)
    eng.net.profile(True)
    eng.detect_frames([(d.ptr, f.shape[0], f.shape[1], f.strides[0])], thresh=0.5)
    assert not any(int(r[4]) in (500, 501) for r in eng.net.profile_ops())   # one frame: the fused tiles
    eng.net.profile(False)
