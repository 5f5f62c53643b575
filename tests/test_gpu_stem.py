"""Parity of the fused network stem (pc_stem.hip: 3x3 conv over a 3-channel NHWC4 input,
gathered straight into one MFMA K step) in f16:

* equal to the im2col + 1x1 implicit-GEMM path (PC_STEM_UNFUSED=1) - same K positions,
  same MFMA; only the sign of an exact zero may differ;
* within 2e-2 of a torch fp32 restatement.
Shapes: SCRFD's stem (stride 2, 28 channels padded to 32, ReLU), IResNet's (stride 1,
64 channels, PReLU), odd sizes (partial 16-pixel groups, image borders) and an output
wider than the filter count (zeroed channel padding)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from person_capture_amd import program as pg
from person_capture_amd._lib import PC_PREC_F16

pytestmark = pytest.mark.gpu

CASES = [
    # N, H, W, cout, out channels, stride, act
    (2, 64, 48, 28, 32, 2, pg.ACT_RELU),
    (3, 33, 35, 64, 64, 1, pg.ACT_PRELU),
    (2, 17, 9, 28, 64, 2, pg.ACT_RELU),
    (1, 40, 40, 32, 32, 1, pg.ACT_NONE),
]


def _run(gpu_ctx, monkeypatch, P, xin, N, unfused):
    from person_capture_amd.runtime import Net
    if unfused:
        monkeypatch.setenv("PC_STEM_UNFUSED", "1")
    else:
        monkeypatch.delenv("PC_STEM_UNFUSED", raising=False)
    net = Net(gpu_ctx, P.serialize(), precision=PC_PREC_F16, max_batch=N)
    d = gpu_ctx.upload(xin.astype(np.float16))
    net.run(d.ptr, N)
    out = net.read_output(0, N)
    net.close()
    return out


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_fused_stem(gpu_ctx, monkeypatch, case):
    N, H, W, cout, cy, s, act = case
    rng = np.random.default_rng(H * 131 + W)
    Ho, Wo = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
    P = pg.Program()
    x = P.input_tensor(H, W, 4)
    y = P.act(Ho, Wo, cy)
    w = rng.standard_normal((cout, 3, 3, 4)) * 0.3
    w[..., 3] = 0
    b = rng.standard_normal(cout) * 0.1
    slope = rng.uniform(0.1, 0.3, cout)
    P.stem(y, x, w, b, stride=s, pad=1, act=act, slope=slope if act == pg.ACT_PRELU else None)
    P.outputs = [y]
    xin = np.zeros((N, H, W, 4), np.float32)
    xin[..., :3] = rng.standard_normal((N, H, W, 3))
    xin = xin.astype(np.float16).astype(np.float32)
    got = _run(gpu_ctx, monkeypatch, P, xin, N, False)
    ref2 = _run(gpu_ctx, monkeypatch, P, xin, N, True)
    assert np.array_equal(got, ref2), f"fused != im2col path: {np.count_nonzero(got != ref2)} elements"
    X = torch.from_numpy(np.ascontiguousarray(np.transpose(xin, (0, 3, 1, 2))))
    Wt = torch.from_numpy(np.ascontiguousarray(np.transpose(w, (0, 3, 1, 2)))).float()
    Wt = Wt.half().float()
    Y = F.conv2d(X, Wt, stride=s, padding=1) + torch.from_numpy(b).float().view(1, -1, 1, 1)
    if act == pg.ACT_RELU:
        Y = F.relu(Y)
    elif act == pg.ACT_PRELU:
        Y = torch.where(Y > 0, Y, Y * torch.from_numpy(slope).float().view(1, -1, 1, 1))
    ref = Y.permute(0, 2, 3, 1).numpy()
    err = np.abs(got[..., :cout] - ref).max() / max(1.0, np.abs(ref).max())
    assert err < 2e-2, err
    assert np.all(got[..., cout:] == 0)
