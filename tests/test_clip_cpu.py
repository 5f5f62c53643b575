"""CPU checks of the ReID (OpenCLIP ViT) build: the compiled tower (patch matrix 1x1 conv,
class/positional table in ln_pre, fused bias/GELU/residual 1x1 convs, attention op,
class-token projection by a stride-T conv) through the device-semantics emulator vs the
literal oracle forward; the host Pillow-coefficient restatement vs Pillow itself."""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import nets_torch as nt
from person_capture_amd import models_clip as mc
from program_emulator import run_program


def test_clip_program_matches_oracle():
    p = mc.synth_clip_vit("ViT-tiny-14", seed=1)
    rng = np.random.default_rng(2)
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in ((300, 180), (224, 224))]
    xs = [nt.clip_preprocess_pil(im) for im in imgs]
    ref = nt.clip_vit_forward(p, "ViT-tiny-14", torch.stack(xs)).numpy()
    P = mc.compile_clip_vit(p, "ViT-tiny-14")
    x = np.concatenate([nt.clip_patch_matrix(t)[:, None] for t in xs], axis=0)   # [N][1][257][608]
    (o,) = run_program(P, x)
    got = o[:, :, 0, 0].numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-4


def test_clip_flops_vit_l14():
    # ~162 GFLOP per crop; weights are not synthesised here (1.2 GB)
    c = mc.clip_cfg("ViT-L-14")
    w, L, T = c["width"], c["layers"], 257
    per_layer = 2 * T * w * 3 * w + 4 * T * T * w + 2 * T * w * w + 4 * T * w * c["mlp"]
    total = 2 * 256 * 588 * w + L * per_layer + 2 * w * c["out"]
    assert 150e9 < total < 175e9
    with pytest.raises(RuntimeError):
        mc.clip_cfg("RN50")


def _pil_coeffs_ref(in_size, out_size):
    """Pillow Resample.c precompute_coeffs + normalize_coeffs_8bpc (python restatement)."""
    import math
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support = 2.0 * fs
    ksize = int(math.ceil(support)) * 2 + 1

    def f(x):
        a = -0.5
        x = abs(x)
        if x < 1.0:
            return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
        if x < 2.0:
            return (((x - 5) * x + 8) * x - 4) * a
        return 0.0
    bounds, kk = [], []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [f((x + xmin - center + 0.5) / fs) for x in range(xmax)]
        ww = sum(k)
        k = [v / ww for v in k] + [0.0] * (ksize - xmax)
        kk.append([int(-0.5 + v * (1 << 22)) if v < 0 else int(0.5 + v * (1 << 22)) for v in k])
        bounds.append((xmin, xmax))
    return ksize, np.array(bounds, np.int32), np.array(kk, np.int32)


@pytest.mark.parametrize("n_in,n_out", [(100, 224), (1080, 224), (224, 224), (37, 224), (640, 395)])
def test_pil_coeffs_host_restatement(n_in, n_out):
    from person_capture_amd import _lib
    lib = _lib.load()
    bounds = np.zeros((n_out, 2), np.int32)
    kk = np.zeros((n_out * 64,), np.int32)
    k = lib.pc_pil_bicubic_coeffs(n_in, n_out, 0, n_out, bounds.ctypes.data_as(C.POINTER(C.c_int32)),
                                  kk.ctypes.data_as(C.POINTER(C.c_int32)), 64)
    ks, rb, rk = _pil_coeffs_ref(n_in, n_out)
    assert k == ks
    assert np.array_equal(bounds, rb)
    assert np.array_equal(kk[:n_out * k].reshape(n_out, k), rk)


def _pil_resample_emul(rgb, rw, rh):
    """Two-pass fixed-point resample with the host tables (what pc_clip.hip computes)."""
    from person_capture_amd import _lib
    lib = _lib.load()
    h, w = rgb.shape[:2]

    def tab(n_in, n_out):
        b = np.zeros((n_out, 2), np.int32)
        kk = np.zeros((n_out * 64,), np.int32)
        k = lib.pc_pil_bicubic_coeffs(n_in, n_out, 0, n_out, b.ctypes.data_as(C.POINTER(C.c_int32)),
                                      kk.ctypes.data_as(C.POINTER(C.c_int32)), 64)
        return b, kk[:n_out * k].reshape(n_out, k)
    hb, hk = tab(w, rw)
    vb, vk = tab(h, rh)
    tmp = np.zeros((h, rw, 3), np.int64)
    for x in range(rw):
        xmin, xn = hb[x]
        s = (1 << 21) + (rgb[:, xmin:xmin + xn, :].astype(np.int64) * hk[x, :xn][None, :, None]).sum(1)
        tmp[:, x] = np.clip(s >> 22, 0, 255)
    out = np.zeros((rh, rw, 3), np.uint8)
    for y in range(rh):
        ymin, yn = vb[y]
        s = (1 << 21) + (tmp[ymin:ymin + yn].astype(np.int64) * vk[y, :yn][:, None, None]).sum(0)
        out[y] = np.clip(s >> 22, 0, 255)
    return out


@pytest.mark.parametrize("h,w", [(300, 180), (97, 61), (500, 240)])
def test_pil_bicubic_bit_exact(h, w):
    """The device algorithm (host tables + integer two-pass) equals Pillow's resize."""
    from PIL import Image
    from person_capture_amd import _lib
    lib = _lib.load()
    rgb = np.random.default_rng(h * w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    g = (C.c_int32 * 4)()
    lib.pc_clip_geometry(h, w, 224, g)
    rw, rh = g[0], g[1]
    ref = np.array(Image.fromarray(rgb).resize((rw, rh), Image.BICUBIC))
    assert np.array_equal(_pil_resample_emul(rgb, rw, rh), ref)
