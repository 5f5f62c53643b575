"""CPU-side checks of the boundary and host logic (no GPU compute):
the C-ABI library loads and exports every function include/pcgpu.h declares; the
native host geometry (LMEDS similarity, affine inversion) agrees bit-for-bit with
the oracle restatements; INTER_AREA tables match the C oracle; letterbox geometry
matches insightface's; constructor error behaviour mirrors the reference."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle import cv_ops
from oracle import pipeline as op
from oracle import ref_algos as ra
from person_capture_amd import _lib, engines, imageops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "pcgpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(pc_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    # every binding in the ctypes table is declared in the header
    for n in _lib.SIGNATURES:
        assert n in names, n
    assert lib.pc_abi_version() == 1


def test_ctx_create_without_gpu_fails_cleanly():
    lib = _lib.load()
    h = C.c_void_p()
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a device is present")
    assert lib.pc_ctx_create(0, C.byref(h)) != 0


def test_lmeds_native_matches_oracle():
    rng = np.random.default_rng(1)
    for t in range(200):
        base = ra.ARC_DST * rng.uniform(0.5, 3) + rng.uniform(-50, 50, 2)
        noise = rng.choice([0.0, 0.3, 2.0, 15.0])
        src = (base + rng.normal(0, noise, base.shape)).astype(np.float32)
        if t % 25 == 0:
            src[3] = src[0]   # degenerate pair
        Mo = op.estimate_affine_partial_lmeds(src, ra.ARC_DST)
        Mp, ok = imageops.estimate_affine_partial(src[None], ra.ARC_DST)
        assert (Mo is not None) == bool(ok[0])
        if Mo is not None:
            assert np.array_equal(Mo, Mp[0])
        M3o = op.estimate_affine_partial_lmeds(src[:3], ra.ARC_DST[:3])
        M3p, ok3 = imageops.estimate_affine_partial(src[None, :3], ra.ARC_DST[:3])
        if M3o is not None:
            assert np.array_equal(M3o, M3p[0])


def test_invert_affine_matches_oracle():
    rng = np.random.default_rng(2)
    for _ in range(50):
        M = rng.standard_normal(6)
        assert np.array_equal(imageops.invert_affine(M), cv_ops.invert_affine(M))


@pytest.mark.parametrize("s,d", [(3840, 416), (2160, 234), (1920, 640), (500, 112), (113, 112), (1000, 333)])
def test_area_tables_match_c(s, d):
    tab, start = imageops.area_tables(s, d)
    si, di, al = cv_ops.area_tab(s, d, float(s) / d)
    assert len(tab) == len(si)
    assert [t.si for t in tab] == si.tolist()
    assert [t.di for t in tab] == di.tolist()
    assert np.array_equal(np.array([t.alpha for t in tab], np.float32), al)
    assert start[0] == 0 and start[d] == len(tab)


@pytest.mark.parametrize("HW,D", [((1080, 1920), 640), ((480, 300), 320), ((2160, 3840), 384), ((97, 61), 320)])
def test_letterbox_geometry(HW, D):
    assert engines.letterbox_geometry(HW[0], HW[1], D) == ra.scrfd_letterbox_geometry(HW[0], HW[1], D)


def test_simd_end():
    assert engines.opencv_vresize_simd_end(1920) == 1920
    assert engines.opencv_vresize_simd_end(600) == 592
    assert engines.opencv_vresize_simd_end(12) == 8    # one 8-lane step (x=0 < 12-8), scalar tail 8..11
    assert engines.opencv_vresize_simd_end(8) == 0


def test_ctor_errors_mirror_reference():
    from person_capture_amd import face_embedder as fe_mod
    with pytest.raises(RuntimeError):
        fe_mod.FaceEmbedder(ctx="cpu", yolo_model="scrfd_10g_bnkps")
    with pytest.raises(RuntimeError):
        fe_mod.FaceEmbedder(ctx="cuda", yolo_model="yolov8l-face.pt")
    with pytest.raises(RuntimeError):
        fe_mod.FaceEmbedder(ctx="cuda", yolo_model="scrfd_10g_bnkps", use_arcface=False)


def test_person_reid_ctor_errors_mirror_reference():
    """No CPU path on this build: device='cpu' raises RuntimeError at construction, like the
    reference does when its backend is unavailable (detectors.py:28-31, reid_embedder.py:24-27);
    an OpenCLIP tower this build does not have is refused the same way."""
    from person_capture_amd.detectors import PersonDetector
    from person_capture_amd.models_clip import clip_cfg
    from person_capture_amd.reid_embedder import ReIDEmbedder
    with pytest.raises(RuntimeError):
        PersonDetector("yolov8n.pt", device="cpu")
    with pytest.raises(RuntimeError):
        ReIDEmbedder(device="cpu")
    with pytest.raises(RuntimeError):
        clip_cfg("RN50x64")


def test_library_has_no_undefined_internal_symbols():
    """Every kernel stub and internal function the library references is defined in it
    (a template kernel whose host-side instantiation silently failed leaves an undefined
    __device_stub__ symbol that only shows up as a dlopen error on the GPU box)."""
    import shutil
    import subprocess
    from person_capture_amd._lib import LIB_PATH
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not available")
    out = subprocess.run([nm, "-D", "--undefined-only", str(LIB_PATH)], capture_output=True, text=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "_ZN2pc" in ln]
    assert not bad, bad
