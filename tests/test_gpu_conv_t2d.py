"""Parity of the 2-D block conv kernel (pc_conv_t2d.hip: 3x3 stride-1 convs over 32/64
channels, weights in registers, persistent workgroups over 16-pixel-wide blocks).

* against the statically scheduled implicit-GEMM kernel (pc_conv_fast.hip) on the same
  f16 inputs: EQUAL values - both accumulate K in the same order (tap-major, 32-channel
  MFMA steps), so the only difference allowed is the sign of an exact zero;
* against a torch fp32 restatement of the op (2e-2 relative, the f16 conv tolerance of
  tests/test_gpu_conv.py).
Shapes cover ragged blocks (W and H not multiples of the block), images of the batch
sharing a block column, every epilogue mode the planner sends here (channel / border-class
bias, none / ReLU / PReLU, same-pixel residual before or after the activation, output
channels < npad) and the SCRFD / IResNet trunk shapes; SiLU and f32 outputs stay on the
implicit-GEMM kernels (test_t2d_planner_declines)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from person_capture_amd import program as pg
from person_capture_amd._lib import PC_PREC_F16

pytestmark = pytest.mark.gpu


def _nchw(a):
    return torch.from_numpy(np.ascontiguousarray(np.transpose(a, (0, 3, 1, 2))).astype(np.float32))


def _build(case, rng):
    N, H, W, cin, cout, act, bmode, res, after, out_f32 = case
    cp, npad = pg.cpad(cin), pg.cpad(cout)
    P = pg.Program()
    x = P.input_tensor(H, W, cp)
    y = P.act(H, W, npad, is_f32=out_f32)
    w = rng.standard_normal((cout, cin, 3, 3)) * np.sqrt(2.0 / (cin * 9))
    wp = pg.pack_conv_weights([w], [cp], npad)
    bias = rng.standard_normal((9, npad)) * 0.5 if bmode == pg.BIAS_BORDER9 else \
        pg.pad_vec(rng.standard_normal(cout) * 0.1, npad)
    slope = pg.pad_vec(rng.uniform(0.1, 0.3, cout), npad)
    kw = {}
    r = None
    if res:
        # the residual is the input itself (IResNet / SCRFD basic block: cin == cout)
        assert cp == npad
        r = x
        kw = dict(res=x, res_mode=pg.RES_SAME, act_after_res=after)
    P.conv(y, [(x, 3, 3, 1, 1, cin)], wp, cout, bias=bias, bias_mode=bmode, slope=slope, act=act, **kw)
    P.outputs = [y]
    xin = np.zeros((N, H, W, cp), np.float32)
    xin[..., :cin] = rng.standard_normal((N, H, W, cin))
    xin = xin.astype(np.float16).astype(np.float32)
    return P, xin, wp.astype(np.float16).astype(np.float32), bias, slope, r is not None


def _run(gpu_ctx, monkeypatch, P, xin, N, mode):
    from person_capture_amd.runtime import Net
    monkeypatch.setenv("PC_CONV_T2D", mode)
    monkeypatch.setenv("PC_T2D_128", "1")   # the opt-in 128-channel shape is tested too
    net = Net(gpu_ctx, P.serialize(), precision=PC_PREC_F16, max_batch=N)
    d = gpu_ctx.upload(xin.astype(np.float16))
    net.run(d.ptr, N)
    out = net.read_output(0, N)
    # profile code 200 + v: the 2-D block kernel, variant v (pc_conv_t2d.hip kT2d); folded to 200
    kinds = {200 if 200 <= int(r[4]) < 300 else int(r[4]) for r in _profile_kinds(net, d, N)}
    return out, kinds


def _profile_kinds(net, d, N):
    net.profile(True)
    net.run(d.ptr, N)
    recs = net.profile_ops()
    net.profile(False)
    return recs


CASES = [
    # N, H, W, cin, cout, act, bias_mode, residual, act_after_res, out_f32
    (3, 16, 16, 64, 64, pg.ACT_PRELU, pg.BIAS_BORDER9, 0, 0, 0),      # IResNet conv1 (folded pre-BN)
    (2, 40, 56, 64, 64, pg.ACT_NONE, pg.BIAS_CHANNEL, 1, 0, 0),       # ragged W, residual after act
    (2, 28, 20, 64, 64, pg.ACT_RELU, pg.BIAS_CHANNEL, 1, 1, 0),       # act(acc + b + res)
    (3, 37, 33, 32, 32, pg.ACT_RELU, pg.BIAS_CHANNEL, 0, 0, 0),       # npad 32: 32-row blocks, ragged
    (2, 32, 48, 32, 64, pg.ACT_PRELU, pg.BIAS_CHANNEL, 0, 0, 0),
    (2, 18, 30, 64, 56, pg.ACT_RELU, pg.BIAS_CHANNEL, 0, 0, 0),       # cout < npad
    (2, 20, 17, 32, 28, pg.ACT_PRELU, pg.BIAS_BORDER9, 0, 0, 0),
    (4, 80, 80, 64, 64, pg.ACT_RELU, pg.BIAS_CHANNEL, 1, 1, 0),       # SCRFD stage shape
    (2, 160, 160, 32, 32, pg.ACT_RELU, pg.BIAS_CHANNEL, 0, 0, 0),     # SCRFD stem shape (half size)
    (8, 56, 56, 64, 64, pg.ACT_NONE, pg.BIAS_CHANNEL, 1, 0, 0),       # IResNet stage 1
    # wide shapes (one wave per SIMD, 216 / 288 weight registers)
    (2, 80, 80, 96, 96, pg.ACT_RELU, pg.BIAS_CHANNEL, 1, 1, 0),       # SCRFD-10G 80x80x96 block conv2
    (3, 23, 37, 96, 80, pg.ACT_RELU, pg.BIAS_CHANNEL, 0, 0, 0),       # ragged, cout < npad 96
    (2, 40, 40, 64, 96, pg.ACT_RELU, pg.BIAS_CHANNEL, 0, 0, 0),       # 64 -> 96
    (3, 28, 28, 128, 128, pg.ACT_PRELU, pg.BIAS_BORDER9, 0, 0, 0),    # IResNet 28x28x128 conv1
    (4, 28, 28, 128, 128, pg.ACT_NONE, pg.BIAS_CHANNEL, 1, 0, 0),     # IResNet 28x28x128 conv2 + residual
    (2, 13, 50, 128, 120, pg.ACT_RELU, pg.BIAS_CHANNEL, 0, 0, 0),     # ragged, cout < npad 128
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:5])) + f"-a{c[5]}b{c[6]}r{c[7]}{c[8]}f{c[9]}")
def test_t2d_vs_fast_and_torch(gpu_ctx, monkeypatch, case):
    N, H, W, cin, cout, act, bmode, res, after, out_f32 = case
    rng = np.random.default_rng(sum(case) * 7919 % 65536)
    P, xin, wq, bias, slope, has_res = _build(case, rng)
    got, kinds = _run(gpu_ctx, monkeypatch, P, xin, N, "2")
    assert kinds == {200}, f"planner did not put the conv on the 2-D block kernel: {kinds}"
    ref_fast, kinds_f = _run(gpu_ctx, monkeypatch, P, xin, N, "0")
    assert 200 not in kinds_f
    assert got.shape == ref_fast.shape
    assert np.array_equal(got, ref_fast), \
        f"t2d != fast kernel: {np.count_nonzero(got != ref_fast)} elements, max {np.abs(got - ref_fast).max()}"
    # torch fp32 restatement
    cp, npad = pg.cpad(cin), pg.cpad(cout)
    wt = torch.from_numpy(np.ascontiguousarray(wq.reshape(npad, 3, 3, cp).transpose(0, 3, 1, 2))).float()
    ref = F.conv2d(_nchw(xin), wt, padding=1)
    if bmode == pg.BIAS_BORDER9:
        b9 = torch.from_numpy(bias.reshape(3, 3, npad)).float()
        rh = torch.where(torch.arange(H) - 1 < 0, 0, torch.where(torch.arange(H) + 1 >= H, 2, 1))
        rw = torch.where(torch.arange(W) - 1 < 0, 0, torch.where(torch.arange(W) + 1 >= W, 2, 1))
        ref = ref + b9[rh[:, None], rw[None, :]].permute(2, 0, 1)[None]
    else:
        ref = ref + torch.from_numpy(bias).float().view(1, -1, 1, 1)

    def act_f(v):
        if act == pg.ACT_RELU:
            return F.relu(v)
        if act == pg.ACT_PRELU:
            return torch.where(v > 0, v, v * torch.from_numpy(slope).float().view(1, -1, 1, 1))
        if act == pg.ACT_SILU:
            return F.silu(v)
        return v
    X = _nchw(xin)
    if has_res and after:
        ref = act_f(ref + X)
    elif has_res:
        ref = act_f(ref) + X
    else:
        ref = act_f(ref)
    ref = ref[:, :cout].permute(0, 2, 3, 1).numpy()
    err = np.abs(got[..., :cout] - ref).max() / max(1.0, np.abs(ref).max())
    assert err < 2e-2, f"max rel err {err}"
    assert np.all(got[..., cout:] == 0), "channel padding must be zero"


def test_t2d_auto_plan_covers_trunks(gpu_ctx):
    """The default planner puts the SCRFD-10G 320/160/80 stride-1 3x3 convs over 32/64
    channels and IResNet's 112/56 stage-1 convs (conv1 of block 1, both convs of blocks 2-3) on the 2-D
    block kernel in f16."""
    from person_capture_amd import models
    from person_capture_amd.runtime import Net
    for P, B, want in ((models.compile_scrfd(models.synth_scrfd("10g", seed=0, calibrate=False), "10g", 640), 2, 9),
                       (models.compile_iresnet(models.synth_iresnet(100, seed=0, calibrate=False), 100), 4, 5)):
        net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=B)
        H, W, C = P.dims(P.input)
        d = gpu_ctx.upload(np.zeros((B, H, W, C), np.float16))
        recs = _profile_kinds(net, d, B)
        n_t2d = sum(1 for r in recs if 200 <= int(r[4]) < 300)
        del net, d
        assert n_t2d >= want, n_t2d


@pytest.mark.parametrize("act,out_f32", [(pg.ACT_SILU, 0), (pg.ACT_RELU, 1)])
def test_t2d_planner_declines(gpu_ctx, monkeypatch, act, out_f32):
    """Smooth activations and f32 outputs are not run on the 2-D block kernel, even forced."""
    case = (2, 16, 16, 32, 32, act, pg.BIAS_CHANNEL, 0, 0, out_f32)
    P, xin, *_ = _build(case, np.random.default_rng(5))
    _, kinds = _run(gpu_ctx, monkeypatch, P, xin, 2, "2")
    assert 200 not in kinds
