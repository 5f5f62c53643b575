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


def area_tables(ssize: int, dsize: int, scale: float = None):
    """cv::computeResizeAreaTab (cn = 1) as ctypes arrays + per-destination start offsets.
    scale defaults to ssize/dsize (explicit dsize); cv2.resize(fx=s) uses 1/s.
    Cached per (ssize, dsize, scale): the pre-scan resizes every frame with one geometry."""
    scale = float(ssize) / dsize if scale is None else float(scale)
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
