"""Resident block chain (pc_conv_chain.hip) vs the same IResNet run one conv launch at
a time. The chain keeps conv_fast's K order and epilogue arithmetic, so the network
output must be bit-identical (tolerance 0) with the chain on and off, at batch sizes
below, at and above one round of 256 workgroups. The f16 IResNet itself is checked
against the fp32 oracle in test_gpu_arcface.py / test_gpu_bench_config.py."""
import os

import numpy as np
import pytest

from person_capture_amd import models
from person_capture_amd._lib import PC_PREC_F16
from person_capture_amd.runtime import Net

pytestmark = pytest.mark.gpu

CHAIN_CODE = 300   # pc_net_profile_ops kernel code of a chain launch


def _net(ctx, P, max_batch, chain):
    old = {k: os.environ.get(k) for k in ("PC_CHAIN", "PC_CHAIN_MIN")}
    try:
        if chain:
            os.environ.pop("PC_CHAIN", None)
            os.environ["PC_CHAIN_MIN"] = "1"
        else:
            os.environ["PC_CHAIN"] = "0"
        return Net(ctx, P.serialize(), PC_PREC_F16, max_batch=max_batch)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _run(ctx, net, x, N):
    d = ctx.upload(x)
    net.profile(True)
    net.run(d.ptr, N)
    codes = [int(r[4]) for r in net.profile_ops()]
    net.profile(False)
    out = net.read_output(0, N)
    d.free()
    return out, codes


@pytest.mark.parametrize("depth,batches", [(100, (3, 64, 256, 300)), (50, (17,))])
def test_chain_equals_per_conv_launches(gpu_ctx, depth, batches):
    p = models.synth_iresnet(depth, seed=3)
    P = models.compile_iresnet(p, depth)
    mb = max(batches)
    on = _net(gpu_ctx, P, mb, True)
    off = _net(gpu_ctx, P, mb, False)
    rng = np.random.default_rng(5)
    for N in batches:
        x = np.zeros((N, 112, 112, 4), np.float16)
        x[..., :3] = rng.uniform(-1.0, 1.0, (N, 112, 112, 3))
        a, ca = _run(gpu_ctx, on, x, N)
        b, cb = _run(gpu_ctx, off, x, N)
        assert CHAIN_CODE in ca, "chain kernel not used"
        assert CHAIN_CODE not in cb
        assert np.isfinite(a).all()
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"N={N}: {len(bad)} differing outputs, max |d| {np.abs(a - b).max()}"
    on.close()
    off.close()


def test_teardown_after_failed_assertion():
    """r04n: after this file's chain test failed, the pytest process dumped core at exit - the
    failed test's nets (never closed) were garbage-collected after the session fixture had closed
    their context, and pc_net_destroy ran on the destroyed context. Contexts now close their nets
    first and close themselves at interpreter exit. A child process leaves a net alive past its
    context's close and another alive at exit after an exception: it must exit with the
    exception's status, not a signal."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from person_capture_amd import models\n"
        "from person_capture_amd.runtime import GpuContext, Net\n"
        "from person_capture_amd._lib import PC_PREC_F16\n"
        "import numpy as np\n"
        "P = models.compile_iresnet(models.synth_iresnet(18, seed=1, calibrate=False), 18).serialize()\n"
        "c1 = GpuContext(0); a = Net(c1, P, PC_PREC_F16, max_batch=2)\n"
        "d = c1.upload(np.zeros((2, 112, 112, 4), np.float16)); a.run(d.ptr, 2); c1.sync()\n"
        "c1.close()\n"
        "del a\n"
        "c2 = GpuContext(0); b = Net(c2, P, PC_PREC_F16, max_batch=2)\n"
        "assert False, 'a failed test leaves its net and context alive'\n" % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])
    assert "AssertionError" in r.stderr
