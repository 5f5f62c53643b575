"""ReID body embedding on the GPU (OpenCLIP ViT image tower) vs the CPU oracle.

* preprocessing: the device Pillow-bicubic/centre-crop/normalise kernel writes the
  patch matrix bit-exactly equal to the reference's own stack run here (Pillow
  Image.resize(BICUBIC) + crop + ToTensor/Normalize arithmetic) — pinned to Pillow.
* tower (f32, ViT-L/14 at reduced depth): unit embeddings within 1e-4 of
  oracle/nets_torch.clip_vit_forward + F.normalize.
* full ViT-L/14 f16 (the throughput mode): cosine >= 0.99 vs the f32 oracle.
* ReIDEmbedder.extract contract (skips None / empty crops, unit float32 rows).
"""
import numpy as np
import pytest
import torch

from oracle import nets_torch as nt
from person_capture_amd import models_clip as mc
from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F32, CropDesc, check
from person_capture_amd.reid_embedder import ClipEngine, ReIDEmbedder, clip_weights

pytestmark = pytest.mark.gpu

CROPS = [(300, 180), (97, 61), (224, 224), (1080, 400), (150, 700)]


def _crop(seed, h, w):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_clip_prep_bit_exact_vs_pillow(gpu_ctx):
    crops = [_crop(i, h, w) for i, (h, w) in enumerate(CROPS)]
    bufs = [gpu_ctx.upload(c) for c in crops]
    arr = (CropDesc * len(crops))()
    for i, (c, b) in enumerate(zip(crops, bufs)):
        arr[i].d_src, arr[i].H, arr[i].W, arr[i].row_stride = b.ptr, c.shape[0], c.shape[1], c.strides[0]
    out = gpu_ctx.alloc(len(crops) * 257 * 608 * 4)
    check(gpu_ctx.lib.pc_clip_prep(gpu_ctx.handle, PC_PREC_F32, arr, len(crops), out.ptr), gpu_ctx.handle, "clip_prep")
    got = gpu_ctx.download(out.ptr, (len(crops), 257, 608), np.float32)
    for i, c in enumerate(crops):
        ref = nt.clip_patch_matrix(nt.clip_preprocess_pil(c))[0]
        assert np.array_equal(got[i], ref), i


def _ref_embed(p, name, crops):
    x = torch.stack([nt.clip_preprocess_pil(c) for c in crops])
    e = nt.clip_vit_forward(p, name, x)
    return torch.nn.functional.normalize(e, dim=1).numpy()


def test_clip_tower_f32_parity(gpu_ctx):
    name = "ViT-L-14-d2"
    p = clip_weights(name, 0)
    eng = ClipEngine(gpu_ctx, p, name, precision=PC_PREC_F32, max_batch=4)
    crops = [_crop(10 + i, h, w) for i, (h, w) in enumerate(CROPS[:4])]
    bufs = [gpu_ctx.upload(c) for c in crops]
    d = gpu_ctx.alloc(len(crops) * 768 * 4)
    eng.embed_device([(b.ptr, c.shape[0], c.shape[1], c.strides[0]) for b, c in zip(bufs, crops)], d.ptr)
    got = gpu_ctx.download(d.ptr, (len(crops), 768), np.float32)
    ref = _ref_embed(p, name, crops)
    assert np.abs(got - ref).max() < 1e-4
    assert np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-5)


def test_reid_embedder_vit_l14_f16(gpu_ctx, monkeypatch):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_REID_PRECISION", "f16")
    reid = ReIDEmbedder(device="cuda:0")
    assert reid.device == "cuda" and reid.dim == 768
    crops = [_crop(20 + i, h, w) for i, (h, w) in enumerate(CROPS[:2])]
    out = reid.extract([crops[0], None, np.zeros((0, 5, 3), np.uint8), crops[1]])
    assert len(out) == 2 and all(f.dtype == np.float32 and f.shape == (768,) for f in out)
    ref = _ref_embed(clip_weights("ViT-L-14", 0), "ViT-L-14", crops)
    for a, b in zip(out, ref):
        assert abs(np.linalg.norm(a) - 1.0) < 1e-4
        assert float(np.dot(a, b)) > 0.99
    assert reid.extract([]) == [] and reid.extract([None]) == []
    sl = _crop(5, 400, 400)[50:350, 100:260]   # non-contiguous slice
    assert len(reid.extract([sl])) == 1
