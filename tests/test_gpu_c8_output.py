"""f16c8 outputs written by a conv whose inputs are not f16c8: the planner restricts such
convs to conv_fast's fused tiles with the LDS epilogue (the only one that writes the e4m3 region,
pc_api.cpp plan_conv). A 96-channel output would otherwise land on a 96-wide tile whose per-fragment
epilogue writes f16 lo values into the f8 bytes. The hi half of the f16c8 output must equal the hi
half of the same conv in the plain f16x3 program bit for bit (same K order, same epilogue
arithmetic), and its lo8 bytes must decode to the f16x3 lo half within e4m3 precision."""
import numpy as np
import pytest

from person_capture_amd import program as pg
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import Net

pytestmark = pytest.mark.gpu

H = W = 16
CIN, CMID, COUT = 32, 64, 96


def _program(c8: bool, seed: int = 3) -> pg.Program:
    rng = np.random.default_rng(seed)
    P = pg.Program(split=True, c8=c8)
    xin = P.input_tensor(H, W, CIN)
    x = P.act(H, W, CMID)
    P.plain_split(x)   # a plain f16x3 input for the second conv
    y = P.act(H, W, COUT)
    w1 = rng.standard_normal((CMID, CIN, 3, 3)) * 0.1
    P.conv(x, [(xin, 3, 3, 1, 1, CIN)], pg.pack_conv_weights([w1], [CIN], CMID), CMID,
           bias=pg.pad_vec(rng.standard_normal(CMID) * 0.1, CMID), act=pg.ACT_RELU)
    w2 = rng.standard_normal((COUT, CMID, 3, 3)) * 0.05
    P.conv(y, [(x, 3, 3, 1, 1, CMID)], pg.pack_conv_weights([w2], [CMID], COUT), COUT,
           bias=pg.pad_vec(rng.standard_normal(COUT) * 0.1, COUT))
    P.outputs.append(y)
    return P


def test_c8_output_from_plain_split_input(gpu_ctx):
    x = np.random.default_rng(4).uniform(-1, 1, (2, H, W, CIN)).astype(np.float16)
    d = gpu_ctx.upload(x)
    res = {}
    try:
        for c8 in (False, True):
            P = _program(c8)
            assert P.tc8[P.outputs[0]] == int(c8)
            net = Net(gpu_ctx, P.serialize(), PC_PREC_F16, max_batch=2)
            try:
                net.profile(True)
                net.run(d.ptr, 2)
                codes = {int(r[0]): int(r[4]) for r in net.profile_ops()}
                net.profile(False)
                ptr, (h, w, cc, cs, is_f32) = net.output(0)
                res[c8] = (gpu_ctx.download(ptr, (2, h, w, cs), np.float16).copy(), codes)
            finally:
                net.close()
    finally:
        d.free()
    (plain, _), (c8o, codes) = res[False], res[True]
    # the second conv ran a fused conv_fast tile whose channel width has the LDS epilogue (32-wide here)
    assert 100 <= codes[1] < 200 and codes[1] - 100 in (7, 12, 18), codes
    assert np.array_equal(plain[..., :COUT].view(np.uint16), c8o[..., :COUT].view(np.uint16))
