"""Kernel-level parity of the implicit-GEMM conv engine (pc_conv.hip) against a
plain torch fp32 restatement of each op's semantics (segments, border-class
bias, activations, residual modes, split-K, stem, max-pool)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from person_capture_amd import program as pg
from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F32

pytestmark = pytest.mark.gpu


def _nchw(x_nhwc):
    return torch.from_numpy(np.ascontiguousarray(np.transpose(x_nhwc, (0, 3, 1, 2))).astype(np.float32))


def _unpack(wp, segs_shapes):
    """[npad][ktot] -> list of [npad][cin_pad][kh][kw]"""
    out, k0 = [], 0
    for (cp, kh, kw) in segs_shapes:
        n = kh * kw * cp
        w = wp[:, k0:k0 + n].reshape(wp.shape[0], kh, kw, cp).transpose(0, 3, 1, 2)
        out.append(torch.from_numpy(np.ascontiguousarray(w)).float())
        k0 += n
    return out


def _act(y, act, slope):
    if act == pg.ACT_RELU:
        return F.relu(y)
    if act == pg.ACT_PRELU:
        return torch.where(y > 0, y, y * torch.from_numpy(slope).float().view(1, -1, 1, 1))
    if act == pg.ACT_SILU:
        return F.silu(y)
    return y


def _run(gpu_ctx, P, x_nhwc, prec, batch):
    from person_capture_amd.runtime import Net
    net = Net(gpu_ctx, P.serialize(), precision=prec, max_batch=batch)
    dt = np.float32 if prec == PC_PREC_F32 else np.float16
    d = gpu_ctx.upload(x_nhwc.astype(dt))
    net.run(d.ptr, batch)
    return [net.read_output(i, batch) for i in range(len(P.outputs))], net


CASES = [
    # H, cin, cout, k, stride, act, bias_mode, out_f32
    (14, 64, 128, 3, 1, pg.ACT_RELU, pg.BIAS_CHANNEL, 0),
    (14, 64, 64, 3, 2, pg.ACT_PRELU, pg.BIAS_CHANNEL, 0),
    (15, 32, 96, 3, 2, pg.ACT_PRELU, pg.BIAS_CHANNEL, 0),
    (20, 96, 224, 1, 1, pg.ACT_NONE, pg.BIAS_CHANNEL, 0),
    (12, 64, 30, 3, 1, pg.ACT_NONE, pg.BIAS_CHANNEL, 1),
    (28, 128, 256, 3, 1, pg.ACT_SILU, pg.BIAS_CHANNEL, 0),
    (16, 64, 64, 3, 1, pg.ACT_PRELU, pg.BIAS_BORDER9, 0),
]


ALL_CFGS = ([None] + [f"{c}{r}" for c in range(14) for r in ("", ":64")] + [f"h{k}" for k in range(5)]
            + [f"f{k}{r}" for k in range(15) for r in ("", ":64")])


def _set_cfg(monkeypatch, cfg):
    """cfg = "<tile id>[:64]": PC_CONV_CFG forces the tile where its channel tile divides
    npad (otherwise the planner's choice runs) and turns the halo kernel off; ":64" forces
    64-byte K-tiles. cfg = "h<k>" forces halo tile k where it applies, "f<k>[:64]" the
    static-schedule tile k (where its channel tile divides npad)."""
    if cfg is None:
        return
    if cfg.startswith("h"):   # halo kernel tile k (pc_conv_halo.hip), stride-1 "same" convs only
        monkeypatch.setenv("PC_CONV_HALO", str(int(cfg[1:]) + 1))
        return
    c, _, rowb = cfg.partition(":")
    if c.startswith("f"):     # static-schedule kernel tile k (pc_conv_fast.hip)
        monkeypatch.setenv("PC_CONV_FAST", str(int(c[1:]) + 1))
        if rowb:
            monkeypatch.setenv("PC_CONV_ROWB", rowb)
        return
    monkeypatch.setenv("PC_CONV_CFG", c)
    if rowb:
        monkeypatch.setenv("PC_CONV_ROWB", rowb)


@pytest.mark.parametrize("cfg", ALL_CFGS)
@pytest.mark.parametrize("prec", [PC_PREC_F32, PC_PREC_F16])
@pytest.mark.parametrize("case", CASES)
def test_single_conv(gpu_ctx, monkeypatch, prec, case, cfg):
    """Every tile configuration of pc_conv.hip at both K-tile widths."""
    _set_cfg(monkeypatch, cfg)
    H, cin, cout, k, s, act, bmode, out_f32 = case
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    N = 3
    cp, npad = pg.cpad(cin), pg.cpad(cout)
    pad = k // 2
    Ho = (H + 2 * pad - k) // s + 1
    P = pg.Program()
    x = P.input_tensor(H, H, cp)
    y = P.act(Ho, Ho, npad, is_f32=out_f32)
    w = rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (cin * k * k))
    wp = pg.pack_conv_weights([w], [cp], npad)
    if bmode == pg.BIAS_BORDER9:
        bias = rng.standard_normal((9, npad)) * 0.5
    else:
        bias = pg.pad_vec(rng.standard_normal(cout) * 0.1, npad)
    slope = pg.pad_vec(rng.uniform(0.1, 0.3, cout), npad)
    P.conv(y, [(x, k, k, s, pad, cin)], wp, cout, bias=bias, bias_mode=bmode, slope=slope, act=act)
    P.outputs = [y]
    xin = np.zeros((N, H, H, cp), np.float32)
    xin[..., :cin] = rng.standard_normal((N, H, H, cin))
    if prec == PC_PREC_F16:
        xin = xin.astype(np.float16).astype(np.float32)
        wp = wp.astype(np.float16).astype(np.float32)
    (got,), _ = _run(gpu_ctx, P, xin, prec, N)
    ref = F.conv2d(_nchw(xin), _unpack(wp, [(cp, k, k)])[0], stride=s, padding=pad)
    if bmode == pg.BIAS_BORDER9:
        b9 = torch.from_numpy(bias.reshape(3, 3, npad)).float()
        ih0 = torch.arange(Ho) * s - pad
        rc = torch.where(ih0 < 0, 0, torch.where(ih0 + k - 1 >= H, 2, 1))
        bmap = b9[rc[:, None], rc[None, :]]          # [Ho][Wo][npad]
        ref = ref + bmap.permute(2, 0, 1)[None]
    else:
        ref = ref + torch.from_numpy(bias).float().view(1, -1, 1, 1)
    ref = _act(ref, act, slope)[:, :cout].permute(0, 2, 3, 1).numpy()
    tol = 2e-4 if prec == PC_PREC_F32 else 2e-2
    err = np.abs(got[..., :cout] - ref).max() / max(1.0, np.abs(ref).max())
    assert err < tol, f"max rel err {err}"
    assert np.all(got[..., cout:] == 0), "channel padding must be zero"


@pytest.mark.parametrize("cfg", ALL_CFGS)
@pytest.mark.parametrize("prec", [PC_PREC_F32, PC_PREC_F16])
def test_two_segments_residual_upsample_splitk(gpu_ctx, monkeypatch, prec, cfg):
    _set_cfg(monkeypatch, cfg)
    """op1: conv3x3/s2 on x -> r (14x14); op2: conv3x3 on r + 1x1/s2 on x (2 segments), + up2(q) residual;
    op3: 7x7 valid split-K conv on op2 -> f32; op4: 1x1 conv with same-pixel residual, act after res."""
    rng = np.random.default_rng(7)
    N, H, C = 2, 28, 64
    P = pg.Program()
    x = P.input_tensor(H, H, C)
    r = P.act(14, 14, 128)
    q = P.act(7, 7, 128)
    o2 = P.act(14, 14, 128)
    o3 = P.act(4, 4, 512, is_f32=1)
    o4 = P.act(14, 14, 128)
    W = lambda co, ci, k: rng.standard_normal((co, ci, k, k)) * np.sqrt(2.0 / (ci * k * k))
    w1 = W(128, 64, 3); b1 = rng.standard_normal(128) * 0.1
    wq = W(128, 64, 3); bq = rng.standard_normal(128) * 0.1
    w2a = W(128, 128, 3); w2b = W(128, 64, 1); b2 = rng.standard_normal(128) * 0.1
    w3 = W(512, 128, 7) * 0.3; b3 = rng.standard_normal(512) * 0.1
    w4 = W(128, 128, 1); b4 = rng.standard_normal(128) * 0.1
    wp1 = pg.pack_conv_weights([w1], [64], 128)
    wpq = pg.pack_conv_weights([wq], [64], 128)
    wp2 = pg.pack_conv_weights([w2a, w2b], [128, 64], 128)
    wp3 = pg.pack_conv_weights([w3], [128], 512)
    wp4 = pg.pack_conv_weights([w4], [128], 128)
    P.conv(r, [(x, 3, 3, 2, 1, 64)], wp1, 128, bias=b1, act=pg.ACT_RELU)
    P.conv(q, [(x, 3, 3, 4, 1, 64)], wpq, 128, bias=bq, act=pg.ACT_NONE)
    P.conv(o2, [(r, 3, 3, 1, 1, 128), (x, 1, 1, 2, 0, 64)], wp2, 128, bias=b2, act=pg.ACT_RELU,
           res=q, res_mode=pg.RES_UP2, act_after_res=0)
    P.conv(o3, [(o2, 7, 7, 2, 0, 128)], wp3, 512, bias=b3, splitk=8)
    P.conv(o4, [(o2, 1, 1, 1, 0, 128)], wp4, 128, bias=b4, act=pg.ACT_RELU, res=r, res_mode=pg.RES_SAME,
           act_after_res=1)
    P.outputs = [o2, o3, o4]
    xin = rng.standard_normal((N, H, H, C)).astype(np.float32)
    q16 = (lambda a: a.astype(np.float16).astype(np.float32)) if prec == PC_PREC_F16 else (lambda a: a)
    xin = q16(xin)
    (g2, g3, g4), _ = _run(gpu_ctx, P, xin, prec, N)
    t = lambda a: torch.from_numpy(np.asarray(a)).float()
    X = _nchw(xin)
    U = lambda wp, shapes: _unpack(q16(wp), shapes)
    R = F.relu(F.conv2d(X, U(wp1, [(64, 3, 3)])[0], stride=2, padding=1) + t(b1).view(1, -1, 1, 1))
    Q = F.conv2d(X, U(wpq, [(64, 3, 3)])[0], stride=4, padding=1) + t(bq).view(1, -1, 1, 1)
    if prec == PC_PREC_F16:
        R, Q = t(q16(R.numpy())), t(q16(Q.numpy()))
    wa, wb = U(wp2, [(128, 3, 3), (64, 1, 1)])
    O2 = F.relu(F.conv2d(R, wa, padding=1) + F.conv2d(X, wb, stride=2) + t(b2).view(1, -1, 1, 1))
    O2 = O2 + F.interpolate(Q, size=(14, 14), mode="nearest")
    if prec == PC_PREC_F16:
        O2 = t(q16(O2.numpy()))
    O3 = F.conv2d(O2, U(wp3, [(128, 7, 7)])[0], stride=2) + t(b3).view(1, -1, 1, 1)
    O4 = F.relu(F.conv2d(O2, U(wp4, [(128, 1, 1)])[0]) + t(b4).view(1, -1, 1, 1) + R)
    tol = 2e-4 if prec == PC_PREC_F32 else 2e-2
    for got, ref in ((g2, O2), (g3, O3), (g4, O4)):
        ref = ref.permute(0, 2, 3, 1).numpy()
        err = np.abs(got - ref).max() / max(1.0, np.abs(ref).max())
        assert err < tol, err


@pytest.mark.parametrize("prec", [PC_PREC_F32, PC_PREC_F16])
def test_stem_and_maxpool(gpu_ctx, prec):
    rng = np.random.default_rng(3)
    N, H = 2, 33
    P = pg.Program()
    x = P.input_tensor(H, H, 4)
    y = P.act(17, 17, 64)
    z = P.act(9, 9, 64)
    w = rng.standard_normal((28, 3, 3, 4)) * 0.3
    w[..., 3] = 0
    b = rng.standard_normal(28) * 0.1
    P.stem(y, x, w, b, stride=2, pad=1, act=pg.ACT_RELU)
    P.maxpool(z, y, 3, 2, 1)
    P.outputs = [y, z]
    xin = np.zeros((N, H, H, 4), np.float32)
    xin[..., :3] = rng.standard_normal((N, H, H, 3))
    if prec == PC_PREC_F16:
        xin = xin.astype(np.float16).astype(np.float32)
    (gy, gz), _ = _run(gpu_ctx, P, xin, prec, N)
    X = _nchw(xin)
    Wt = torch.from_numpy(np.transpose(w, (0, 3, 1, 2)).copy()).float()
    Y = F.relu(F.conv2d(X, Wt, stride=2, padding=1) + torch.from_numpy(b).float().view(1, -1, 1, 1))
    if prec == PC_PREC_F16:
        Y = torch.from_numpy(Y.numpy().astype(np.float16).astype(np.float32))
    Z = F.max_pool2d(Y, 3, 2, 1)
    tol = 2e-5 if prec == PC_PREC_F32 else 2e-2
    assert np.abs(gy[..., :28] - Y.permute(0, 2, 3, 1).numpy()).max() < tol
    assert np.all(gy[..., 28:] == 0)
    assert np.abs(gz[..., :28] - Z.permute(0, 2, 3, 1).numpy()).max() < tol
    # the pool itself is exact: max over the device's own stem output (both precisions;
    # f16 runs the 8-channel vector pool)
    Zs = F.max_pool2d(torch.from_numpy(gy).permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).numpy()
    assert np.array_equal(gz, Zs)
