"""ctypes wrapper of oracle/cv_ops.c (test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_SO = _HERE / "_build" / "libcvops.so"
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not _SO.is_file() or _SO.stat().st_mtime < (_HERE / "cv_ops.c").stat().st_mtime:
            build()
        _lib = C.CDLL(str(_SO))
        P, I, D = C.c_void_p, C.c_int, C.c_double
        _lib.cv_resize_linear_u8.argtypes = [P, I, I, I, P, I, I, D, D, I]
        _lib.cv_letterbox_blob.argtypes = [P, I, I, I, I, I, I, D, D, I, P]
        _lib.cv_invert_affine.argtypes = [P, P]
        _lib.cv_warp_affine_u8.argtypes = [P, I, I, I, P, P, I, I, I]
        _lib.cv_area_tab.argtypes = [I, I, D, P, P, P]
        _lib.cv_area_tab.restype = I
        _lib.cv_resize_area_u8.argtypes = [P, I, I, I, P, I, I]
        _lib.cv_resize_area2_u8.argtypes = [P, I, I, I, P, I, I, D, D]
        _lib.cv_resize_area_fast_u8.argtypes = [P, I, I, I, P, I, I]
        _lib.cv_resize_linear2_u8.argtypes = [P, I, I, I, P, I, I, D, D, D, D, I, I]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def resize_linear(img: np.ndarray, new_w: int, new_h: int, scale_x: float, scale_y: float, simd_end: int):
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    out = np.empty((new_h, new_w, 3), np.uint8)
    lib().cv_resize_linear_u8(_p(img), H, W, img.strides[0], _p(out), new_w, new_h, scale_x, scale_y, simd_end)
    return out


def letterbox_blob(img: np.ndarray, D: int, new_w: int, new_h: int, scale_x: float, scale_y: float, simd_end: int):
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    out = np.empty((D, D, 4), np.float32)
    lib().cv_letterbox_blob(_p(img), H, W, img.strides[0], D, new_w, new_h, scale_x, scale_y, simd_end, _p(out))
    return out


def invert_affine(M) -> np.ndarray:
    M = np.ascontiguousarray(np.asarray(M, np.float64).reshape(6))
    out = np.empty(6, np.float64)
    lib().cv_invert_affine(_p(M), _p(out))
    return out


def warp_affine(crop: np.ndarray, M_fwd, out_w: int, out_h: int, border: int = 2) -> np.ndarray:
    """cv2.warpAffine(crop, M_fwd, (out_w, out_h), INTER_LINEAR, border) with M_fwd src->dst."""
    crop = np.ascontiguousarray(crop, np.uint8)
    h, w = crop.shape[:2]
    iM = invert_affine(M_fwd)
    out = np.empty((out_h, out_w, 3), np.uint8)
    lib().cv_warp_affine_u8(_p(crop), crop.strides[0], w, h, _p(iM), _p(out), out_w, out_h, border)
    return out


def area_tab(ssize: int, dsize: int, scale: float):
    si = np.empty(ssize * 2 + 2, np.int32)
    di = np.empty(ssize * 2 + 2, np.int32)
    al = np.empty(ssize * 2 + 2, np.float32)
    k = lib().cv_area_tab(ssize, dsize, scale, _p(si), _p(di), _p(al))
    return si[:k], di[:k], al[:k]


def resize_area(img: np.ndarray, OW: int, OH: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    out = np.empty((OH, OW, 3), np.uint8)
    lib().cv_resize_area_u8(_p(img), H, W, img.strides[0], _p(out), OH, OW)
    return out


def gray_u8(bgr: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(BGR2GRAY) u8: (B*1868 + G*9617 + R*4899 + 2^13) >> 14."""
    b = bgr[..., 0].astype(np.int32)
    g = bgr[..., 1].astype(np.int32)
    r = bgr[..., 2].astype(np.int32)
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def face_quality(chip_bgr: np.ndarray) -> float:
    """face_embedder.py:1274-1276: var(Laplacian(gray, CV_64F)) with ksize=1, BORDER_REFLECT_101."""
    g = gray_u8(chip_bgr).astype(np.float64)
    p = np.pad(g, 1, mode="reflect")     # numpy 'reflect' == OpenCV BORDER_REFLECT_101
    lap = p[1:-1, :-2] + p[1:-1, 2:] + p[:-2, 1:-1] + p[2:, 1:-1] - 4.0 * g
    return float(lap.var())


INTER_LINEAR = 1
INTER_AREA = 3
_DBL_EPSILON = 2.220446049250313e-16


def simd_end(width_bytes: int) -> int:
    """Byte index where OpenCV's 128-bit vertical linear pass stops (16-byte, then 8-byte steps)."""
    x = (width_bytes // 16) * 16 if width_bytes >= 16 else 0
    while x < width_bytes - 8:
        x += 8
    return x


def resize(img: np.ndarray, dsize=None, fx: float = 0.0, fy: float = 0.0,
           interpolation: int = INTER_LINEAR) -> np.ndarray:
    """cv2.resize for u8 BGR with OpenCV 4.9's dispatch (imgproc/src/resize.cpp, cv::resize and
    hal::resize): dsize from fx/fy by cvRound, copy when the size is unchanged, scale = 1/inv_scale,
    INTER_LINEAR at exactly 2x2 down -> area fast, INTER_AREA with both axes downscaling -> the area
    paths (integer ratio: resizeAreaFast; else the generic tables), INTER_AREA otherwise -> the
    linear kernel with area-mode coefficients."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    if dsize is None or tuple(dsize) == (0, 0):
        inv_x, inv_y = float(fx), float(fy)
        new_w, new_h = int(round(W * inv_x)), int(round(H * inv_y))
    else:
        new_w, new_h = int(dsize[0]), int(dsize[1])
        inv_x, inv_y = float(new_w) / W, float(new_h) / H
    if (new_w, new_h) == (W, H):
        return img.copy()
    sx, sy = 1.0 / inv_x, 1.0 / inv_y
    isx, isy = int(round(sx)), int(round(sy))
    fast = abs(sx - isx) < _DBL_EPSILON and abs(sy - isy) < _DBL_EPSILON
    if interpolation == INTER_LINEAR and fast and isx == 2 and isy == 2:
        interpolation = INTER_AREA
    out = np.empty((new_h, new_w, 3), np.uint8)
    if interpolation == INTER_AREA and sx >= 1 and sy >= 1:
        if fast:
            lib().cv_resize_area_fast_u8(_p(img), img.strides[0], isx, isy, _p(out), new_h, new_w)
        else:
            lib().cv_resize_area2_u8(_p(img), H, W, img.strides[0], _p(out), new_h, new_w, sx, sy)
        return out
    lib().cv_resize_linear2_u8(_p(img), H, W, img.strides[0], _p(out), new_w, new_h, sx, sy, inv_x, inv_y,
                               1 if interpolation == INTER_AREA else 0, simd_end(new_w * 3))
    return out
