"""Host-side geometry for the device image kernels: INTER_AREA coefficient
tables, 5-point canonicalisation and similarity estimation (native, in
libpcgpu's pc_host.cpp), warp descriptors."""
from __future__ import annotations

import ctypes as C
import functools
import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import AreaTab, WarpDesc

# face_embedder.py:1279 — ArcFace 112x112 5-point template
ARC_DST = np.array([[38.2946, 51.6963], [73.5318, 51.5014], [56.0252, 71.7366], [41.5493, 92.3655],
                    [70.7299, 92.2041]], dtype=np.float32)
BORDER_REFLECT = 2
BORDER_REFLECT_101 = 4


def border_constant(value: int) -> int:
    """cv2.BORDER_CONSTANT with a gray borderValue (value, value, value) in the warp descriptor."""
    return (int(value) & 0xFF) << 8


_DBL_EPSILON = 2.220446049250313e-16


def resize_plan(H: int, W: int, dsize: Optional[Tuple[int, int]] = None, fx: float = 0.0, fy: float = 0.0,
                area: bool = False) -> dict:
    """Which cv2.resize kernel OpenCV 4.9 runs for a u8 image (imgproc/src/resize.cpp: cv::resize
    then hal::resize) and its exact parameters:
      'copy'       dsize == source size
      'area_fast'  INTER_AREA (or INTER_LINEAR at exactly 2x2 down) at integer ratios (isx, isy)
      'area'       INTER_AREA, both axes downscale, generic tables at (scale_x, scale_y)
      'linear'     bilinear fixed point; area_mode when INTER_AREA was asked but an axis upscales
    dsize = (new_w, new_h) sets inv_scale = new/old; else new = cvRound(old * f), inv_scale = f.
    scale = 1 / inv_scale (not old/new: they can differ in the last bit)."""
    if dsize is None or tuple(dsize) == (0, 0):
        inv_x, inv_y = float(fx), float(fy)
        new_w, new_h = int(round(W * inv_x)), int(round(H * inv_y))
    else:
        new_w, new_h = int(dsize[0]), int(dsize[1])
        inv_x, inv_y = float(new_w) / W, float(new_h) / H
    p = {"new_w": new_w, "new_h": new_h, "inv_x": inv_x, "inv_y": inv_y}
    if (new_w, new_h) == (W, H):
        p["kind"] = "copy"
        return p
    sx, sy = 1.0 / inv_x, 1.0 / inv_y
    isx, isy = int(round(sx)), int(round(sy))
    fast = abs(sx - isx) < _DBL_EPSILON and abs(sy - isy) < _DBL_EPSILON
    p.update(scale_x=sx, scale_y=sy, isx=isx, isy=isy, area_mode=0)
    if not area and fast and isx == 2 and isy == 2:
        area = True
    if area and sx >= 1 and sy >= 1:
        p["kind"] = "area_fast" if fast else "area"
    else:
        p["kind"] = "linear"
        p["area_mode"] = 1 if area else 0
    return p


def area_tables(ssize: int, dsize: int, scale: float = None):
    """cv::computeResizeAreaTab (cn = 1) as ctypes arrays + per-destination start offsets.
    scale defaults to 1/(dsize/ssize) as hal::resize computes it (explicit dsize); cv2.resize(fx=s) uses 1/s.
    Cached per (ssize, dsize, scale): the pre-scan resizes every frame with one geometry."""
    scale = 1.0 / (float(dsize) / ssize) if scale is None else float(scale)
    return _area_tables(int(ssize), int(dsize), scale)


@functools.lru_cache(maxsize=256)
def _area_tables(ssize: int, dsize: int, scale: float):
    si: List[int] = []
    di: List[int] = []
    al: List[float] = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            si.append(sx1 - 1); di.append(dx); al.append((sx1 - fsx1) / cell)
        for sx in range(sx1, sx2):
            si.append(sx); di.append(dx); al.append(1.0 / cell)
        if fsx2 - sx2 > 1e-3:
            si.append(sx2); di.append(dx); al.append(min(min(fsx2 - sx2, 1.0), cell) / cell)
    n = len(si)
    tab = (AreaTab * n)()
    alf = np.asarray(al, dtype=np.float64).astype(np.float32)
    for k in range(n):
        tab[k].si, tab[k].di, tab[k].alpha = si[k], di[k], float(alf[k])
    start = np.searchsorted(np.asarray(di), np.arange(dsize + 1), side="left").astype(np.int32)
    starts = (C.c_int32 * (dsize + 1))(*start.tolist())
    return tab, starts


def canon_5pts(pts) -> Optional[np.ndarray]:
    """FaceEmbedder._canon_5pts (face_embedder.py:1431-1463): order 5 landmarks as
    [left eye, right eye, nose, left mouth, right mouth] or reject."""
    if pts is None:
        return None
    a = np.asarray(pts)
    if a.shape != (5, 2):
        return None
    a = a.astype(np.float32)
    if not np.isfinite(a).all():
        return None
    by_y = np.argsort(a[:, 1])
    eyes = a[by_y[:2]]
    nose = a[by_y[2]]
    mouth = a[by_y[3:]]
    le, ri = eyes[np.argsort(eyes[:, 0])]
    lm, rm = mouth[np.argsort(mouth[:, 0])]
    if not (le[0] < ri[0] and lm[0] < rm[0]):
        return None
    if not (max(le[1], ri[1]) < nose[1] < min(lm[1], rm[1])):
        return None
    return np.stack([le, ri, nose, lm, rm], axis=0)


def canon_5pts_batch(pts: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """canon_5pts over a stack [m][5][2] -> (ordered [m][5][2] float32, valid [m]).
    Stable sorts on 5 keys equal numpy's default (insertion sort below 16 elements),
    so every valid row is exactly canon_5pts of that row."""
    a = np.asarray(pts, dtype=np.float32).reshape(-1, 5, 2)
    m = a.shape[0]
    if m == 0:
        return a.copy(), np.zeros((0,), bool)
    finite = np.isfinite(a).all(axis=(1, 2))
    a = np.where(finite[:, None, None], a, np.float32(0))
    r = np.arange(m)[:, None]
    by_y = np.argsort(a[:, :, 1], axis=1, kind="stable")
    s = a[r, by_y]                                   # rows sorted by y
    eyes, nose, mouth = s[:, :2], s[:, 2], s[:, 3:]
    eyes = eyes[r, np.argsort(eyes[:, :, 0], axis=1, kind="stable")]
    mouth = mouth[r, np.argsort(mouth[:, :, 0], axis=1, kind="stable")]
    le, ri, lm, rm = eyes[:, 0], eyes[:, 1], mouth[:, 0], mouth[:, 1]
    ok = finite & (le[:, 0] < ri[:, 0]) & (lm[:, 0] < rm[:, 0])
    ok &= (np.maximum(le[:, 1], ri[:, 1]) < nose[:, 1]) & (nose[:, 1] < np.minimum(lm[:, 1], rm[:, 1]))
    return np.stack([le, ri, nose, lm, rm], axis=1), ok


# pc_warp_desc (include/pcgpu.h) as a numpy record, for building descriptor arrays in bulk
WARP_DESC_DTYPE = np.dtype({"names": ["d_src", "row_stride", "w", "h", "M", "d_dst", "out_w", "out_h", "border"],
                            "formats": [np.uint64, np.int32, np.int32, np.int32, (np.float64, 6), np.uint64,
                                        np.int32, np.int32, np.int32],
                            "offsets": [0, 8, 12, 16, 24, 72, 80, 84, 88], "itemsize": 96})


def invert_affine_batch(M: np.ndarray) -> np.ndarray:
    """pc_invert_affine (cv2.invertAffineTransform) over [n][6], same operation order."""
    M = np.asarray(M, np.float64).reshape(-1, 6)
    D = M[:, 0] * M[:, 4] - M[:, 1] * M[:, 3]
    nz = D != 0
    D = np.where(nz, 1.0 / np.where(nz, D, 1.0), 0.0)
    A11, A22, A12, A21 = M[:, 4] * D, M[:, 0] * D, -M[:, 1] * D, -M[:, 3] * D
    out = np.empty_like(M)
    out[:, 0], out[:, 1], out[:, 2] = A11, A12, -A11 * M[:, 2] - A12 * M[:, 5]
    out[:, 3], out[:, 4], out[:, 5] = A21, A22, -A21 * M[:, 2] - A22 * M[:, 5]
    return out


def warp_descs(d_src, row_stride, w, h, M_fwd, d_dst, out_w: int = 112, out_h: int = 112,
               border: int = BORDER_REFLECT) -> np.ndarray:
    """warp_desc over arrays (one descriptor per row of M_fwd [n][6])."""
    M_fwd = np.asarray(M_fwd, np.float64).reshape(-1, 6)
    d = np.zeros(M_fwd.shape[0], WARP_DESC_DTYPE)
    d["d_src"] = np.asarray(d_src, np.uint64)
    d["row_stride"], d["w"], d["h"] = row_stride, w, h
    d["M"] = invert_affine_batch(M_fwd)
    d["d_dst"] = np.asarray(d_dst, np.uint64)
    d["out_w"], d["out_h"], d["border"] = out_w, out_h, border
    return d


def estimate_affine_partial(src_sets: np.ndarray, dst: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Batched cv2.estimateAffinePartial2D(src, dst, method=LMEDS) (native).
    src_sets [n][k][2] float32, dst [k][2] -> (M [n][2][3] float64, ok [n] bool)."""
    lib = _lib.load()
    src = np.ascontiguousarray(src_sets, dtype=np.float32)
    d = np.ascontiguousarray(dst, dtype=np.float32)
    n, k = src.shape[0], src.shape[1]
    M = np.zeros((n, 6), np.float64)
    ok = np.zeros((n,), np.int32)
    if n:
        rc = lib.pc_estimate_affine_partial(src.ctypes.data_as(C.c_void_p), d.ctypes.data_as(C.c_void_p), k, n,
                                            M.ctypes.data_as(C.c_void_p), ok.ctypes.data_as(C.c_void_p))
        if rc != 0:
            raise RuntimeError(f"pc_estimate_affine_partial failed ({rc})")
    return M.reshape(n, 2, 3), ok.astype(bool)


def invert_affine(M) -> np.ndarray:
    lib = _lib.load()
    m = np.ascontiguousarray(np.asarray(M, np.float64).reshape(6))
    out = np.zeros(6, np.float64)
    lib.pc_invert_affine(m.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
    return out


def align_matrices(canon_sets: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """FaceEmbedder._align_by_5pts matrix selection (face_embedder.py:1466-1468):
    LMEDS on 5 points, else on the first 3; ok=False means the resize fallback."""
    M5, ok5 = estimate_affine_partial(canon_sets, ARC_DST)
    if ok5.all() or canon_sets.shape[0] == 0:
        return M5, ok5
    bad = np.where(~ok5)[0]
    M3, ok3 = estimate_affine_partial(canon_sets[bad, :3], ARC_DST[:3])
    M5[bad] = M3
    ok5[bad] = ok3
    return M5, ok5


def warp_desc(d_src: int, row_stride: int, w: int, h: int, M_fwd, d_dst: int, out_w: int = 112, out_h: int = 112,
              border: int = BORDER_REFLECT) -> WarpDesc:
    iM = invert_affine(M_fwd)
    d = WarpDesc()
    d.d_src = int(d_src)
    d.row_stride, d.w, d.h = int(row_stride), int(w), int(h)
    for i in range(6):
        d.M[i] = float(iM[i])
    d.d_dst = int(d_dst)
    d.out_w, d.out_h, d.border = int(out_w), int(out_h), int(border)
    return d
