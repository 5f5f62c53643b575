"""Byte-exact parity of the image kernels (pc_image.hip) against the C
restatement of OpenCV's u8 arithmetic (oracle/cv_ops.c). Bit-exact is the bar:
these are integer/fixed-point computations."""
import ctypes as C

import numpy as np
import pytest

from oracle import cv_ops
from person_capture_amd._lib import PC_PREC_F32, AreaTab, WarpDesc, check
from person_capture_amd.engines import make_letterbox_desc

pytestmark = pytest.mark.gpu


def _frame(rng, H, W):
    return rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)


@pytest.mark.parametrize("HW,D", [((1080, 1920), 640), ((360, 640), 640), ((234, 416), 384), ((480, 300), 320),
                                  ((1080, 1920), 1408), ((97, 61), 320)])
def test_letterbox_blob_bit_exact(gpu_ctx, HW, D):
    rng = np.random.default_rng(HW[0] * 7 + D)
    H, W = HW
    img = _frame(rng, H, W)
    d_img = gpu_ctx.upload(img)
    desc, det_scale = make_letterbox_desc(d_img.ptr, H, W, img.strides[0], D)
    out = gpu_ctx.alloc(D * D * 4 * 4)
    arr = (type(desc) * 1)(desc)
    check(gpu_ctx.lib.pc_letterbox(gpu_ctx.handle, PC_PREC_F32, arr, 1, D, C.c_void_p(out.ptr)), gpu_ctx.handle)
    got = gpu_ctx.download(out.ptr, (D, D, 4), np.float32)
    ref = cv_ops.letterbox_blob(img, D, desc.new_w, desc.new_h, desc.scale_x, desc.scale_y, desc.simd_end)
    assert np.array_equal(got, ref)


def _warp_desc(d_src, row_stride, w, h, iM, d_dst, ow, oh, border=2):
    d = WarpDesc()
    d.d_src = d_src
    d.row_stride, d.w, d.h = row_stride, w, h
    for i in range(6):
        d.M[i] = float(iM[i])
    d.d_dst = d_dst
    d.out_w, d.out_h, d.border = ow, oh, border
    return d


def test_warp_affine_bit_exact(gpu_ctx):
    rng = np.random.default_rng(5)
    frame = _frame(rng, 300, 400)
    d_frame = gpu_ctx.upload(frame)
    crops = [(10, 20, 120, 140), (0, 0, 60, 50), (300, 200, 100, 100), (37, 91, 13, 17), (5, 5, 1, 1)]
    mats = []
    for (x0, y0, w, h) in crops:
        ang = rng.uniform(-0.6, 0.6)
        sc = rng.uniform(0.5, 2.5)
        M = np.array([[sc * np.cos(ang), -sc * np.sin(ang), rng.uniform(-30, 30)],
                      [sc * np.sin(ang), sc * np.cos(ang), rng.uniform(-30, 30)]])
        mats.append(M)
    n = len(crops)
    d_out = gpu_ctx.alloc(n * 112 * 112 * 3)
    descs = []
    for i, ((x0, y0, w, h), M) in enumerate(zip(crops, mats)):
        iM = cv_ops.invert_affine(M.reshape(-1))
        border = 2 if i % 2 == 0 else 4
        descs.append(_warp_desc(d_frame.ptr + y0 * frame.strides[0] + x0 * 3, frame.strides[0], w, h, iM,
                                d_out.ptr + i * 112 * 112 * 3, 112, 112, border))
    arr = (WarpDesc * n)(*descs)
    check(gpu_ctx.lib.pc_warp_affine(gpu_ctx.handle, arr, n), gpu_ctx.handle)
    got = gpu_ctx.download(d_out.ptr, (n, 112, 112, 3), np.uint8)
    for i, ((x0, y0, w, h), M) in enumerate(zip(crops, mats)):
        crop = frame[y0:y0 + h, x0:x0 + w]
        ref = cv_ops.warp_affine(crop, M.reshape(-1), 112, 112, border=2 if i % 2 == 0 else 4)
        assert np.array_equal(got[i], ref), f"crop {i}"


def test_face_quality(gpu_ctx):
    rng = np.random.default_rng(9)
    chips = rng.integers(0, 256, size=(7, 112, 112, 3), dtype=np.uint8)
    chips[3] = 128          # flat chip -> variance 0
    chips[4, :, :56] = 0    # step edge
    d = gpu_ctx.upload(chips)
    out = gpu_ctx.alloc(7 * 8)
    check(gpu_ctx.lib.pc_face_quality(gpu_ctx.handle, C.c_void_p(d.ptr), 7, 112, C.c_void_p(out.ptr)),
          gpu_ctx.handle)
    got = gpu_ctx.download(out.ptr, (7,), np.float64)
    ref = np.array([cv_ops.face_quality(c) for c in chips])
    assert np.allclose(got, ref, rtol=1e-12, atol=1e-9)
    assert got[3] == 0.0


@pytest.mark.parametrize("side", [5, 37, 128])
def test_face_quality_other_sides(gpu_ctx, side):
    """Chip sizes whose bytes are not whole 16-byte words (the byte-load path) and the largest side."""
    rng = np.random.default_rng(side)
    chips = rng.integers(0, 256, size=(3, side, side, 3), dtype=np.uint8)
    d = gpu_ctx.upload(chips)
    out = gpu_ctx.alloc(3 * 8)
    check(gpu_ctx.lib.pc_face_quality(gpu_ctx.handle, C.c_void_p(d.ptr), 3, side, C.c_void_p(out.ptr)),
          gpu_ctx.handle)
    got = gpu_ctx.download(out.ptr, (3,), np.float64)
    ref = np.array([cv_ops.face_quality(c) for c in chips])
    assert np.allclose(got, ref, rtol=1e-12, atol=1e-9)


def test_arcface_prep_and_flip(gpu_ctx):
    rng = np.random.default_rng(10)
    chips = rng.integers(0, 256, size=(3, 112, 112, 3), dtype=np.uint8)
    d = gpu_ctx.upload(chips)
    out = gpu_ctx.alloc(6 * 112 * 112 * 4 * 4)
    check(gpu_ctx.lib.pc_arcface_prep(gpu_ctx.handle, PC_PREC_F32, C.c_void_p(d.ptr), 3, 112, 1, C.c_void_p(out.ptr)),
          gpu_ctx.handle)
    got = gpu_ctx.download(out.ptr, (6, 112, 112, 4), np.float32)
    ref = chips[..., ::-1].astype(np.float32) / 127.5 - 1.0    # face_embedder.py:1282-1286
    assert np.array_equal(got[:3, ..., :3], ref)
    assert np.array_equal(got[3:, ..., :3], ref[:, :, ::-1])   # cv2.flip(b, 1) copy
    assert np.all(got[..., 3] == 0)


@pytest.mark.parametrize("deg,pad", [(0, 24), (90, 0), (180, 24), (270, 24), (90, 7)])
def test_rotate_pad(gpu_ctx, deg, pad):
    rng = np.random.default_rng(deg + pad)
    img = _frame(rng, 37, 53)
    d = gpu_ctx.upload(img)
    rot = {0: img, 90: np.rot90(img, -1), 180: np.rot90(img, 2), 270: np.rot90(img, 1)}[deg]
    ref = np.pad(rot, ((pad, pad), (pad, pad), (0, 0)), mode="edge")
    out = gpu_ctx.alloc(ref.nbytes)
    check(gpu_ctx.lib.pc_rotate_pad(gpu_ctx.handle, C.c_void_p(d.ptr), 37, 53, img.strides[0], deg, pad,
                                    C.c_void_p(out.ptr)), gpu_ctx.handle)
    got = gpu_ctx.download(out.ptr, ref.shape, np.uint8)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("HW,OW", [((2160, 3840), 416), ((1080, 1920), 416), ((500, 333), 112)])
def test_resize_area_bit_exact(gpu_ctx, HW, OW):
    from person_capture_amd.imageops import area_tables
    rng = np.random.default_rng(OW)
    H, W = HW
    OH = int(round(H * OW / W))
    img = _frame(rng, H, W)
    d = gpu_ctx.upload(img)
    (xt, xs), (yt, ys) = area_tables(W, OW), area_tables(H, OH)
    out = gpu_ctx.alloc(OH * OW * 3)
    check(gpu_ctx.lib.pc_resize_area(gpu_ctx.handle, C.c_void_p(d.ptr), img.strides[0], xt, xs, len(xt), yt, ys,
                                     len(yt), C.c_void_p(out.ptr), OH, OW), gpu_ctx.handle)
    got = gpu_ctx.download(out.ptr, (OH, OW, 3), np.uint8)
    ref = cv_ops.resize_area(img, OW, OH)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("offset", [0, 3])
def test_resize_area_batch_bit_exact(gpu_ctx, offset):
    """pc_resize_area_batch (the pre-scan chunk's downscale in one launch, face_embedder.dev_resize_batch):
    16-byte aligned frames take the row-staged kernel (resize_area_rows_u8), a view 3 bytes into its
    buffer the per-pixel one; every frame equals the oracle's INTER_AREA."""
    from person_capture_amd.face_embedder import _DevImage, dev_resize_batch
    rng = np.random.default_rng(40 + offset)
    H, W, OW = 2160, 3840, 416
    OH = int(round(H * OW / W))
    frames = [_frame(rng, H, W) for _ in range(3)]
    bufs = [gpu_ctx.alloc(f.nbytes + 64) for f in frames]
    ims = []
    for f, b in zip(frames, bufs):
        host = np.zeros(f.nbytes + 64, np.uint8)
        host[offset:offset + f.nbytes] = f.reshape(-1)
        gpu_ctx.upload(host, b)
        ims.append(_DevImage(b.ptr + offset, H, W, W * 3))
    outs = dev_resize_batch(gpu_ctx, ims, [f"t_area_batch{i}" for i in range(3)], (OW, OH))
    for f, o in zip(frames, outs):
        assert (o.H, o.W) == (OH, OW)
        got = gpu_ctx.download(o.ptr, (OH, OW, 3), np.uint8)
        assert np.array_equal(got, cv_ops.resize_area(f, OW, OH))


# (H, W, dsize, fx, area): chip resize fallbacks (face_embedder.py:2458-2460, 1579-1582) with
# mixed axes (one down, one up -> area-mode linear), exact 2x/3x (resizeAreaFast), same size
# (copy), pure up/down; TTA rescales by fx (:2264); the pre-scan downscale (gui_app.py:1505-1507)
_RESIZE_CASES = [
    (130, 100, (112, 112), 0, True), (100, 130, (112, 112), 0, True), (224, 224, (112, 112), 0, True),
    (336, 224, (112, 112), 0, True), (336, 336, (112, 112), 0, True), (112, 200, (112, 112), 0, True),
    (60, 50, (112, 112), 0, False), (113, 90, (112, 112), 0, True), (112, 112, (112, 112), 0, True),
    (720, 1280, None, 0.75, True), (720, 1280, None, 0.6, True), (480, 640, None, 1.25, False),
    (360, 640, None, 0.5, False), (2160, 3840, (416, 234), 0, True), (150, 77, (112, 112), 0, False),
]


@pytest.mark.parametrize("H,W,dsize,fx,area", _RESIZE_CASES)
def test_cv_resize_dispatch_bit_exact(gpu_ctx, H, W, dsize, fx, area):
    """Every cv2.resize the path makes, through the same OpenCV 4.9 dispatch (copy / area fast /
    area / linear with area-mode coefficients) as oracle/cv_ops.resize: bit-exact."""
    from person_capture_amd.face_embedder import FaceEmbedder, _DevImage
    fe = FaceEmbedder.__new__(FaceEmbedder)
    fe._ctx = gpu_ctx
    rng = np.random.default_rng(H * 7 + W)
    big = _frame(rng, H + 3, W + 5)
    img = big[1:H + 1, 2:W + 2]                       # a non-contiguous crop, as the callers pass
    d = gpu_ctx.upload(big)
    src = _DevImage(d.ptr + 1 * big.strides[0] + 2 * 3, H, W, big.strides[0])
    out = fe._dev_resize(src, "t_resize", dsize=dsize, fx=fx, fy=fx, area=area)
    got = gpu_ctx.download(out.ptr, (out.H, out.W, 3), np.uint8)
    ref = cv_ops.resize(img, dsize, fx, fx, cv_ops.INTER_AREA if area else cv_ops.INTER_LINEAR)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
