"""ctypes binding of libpcgpu.so (the C ABI in include/pcgpu.h).

Loaded the way the reference loads its native preview DLL
(person_capture/hdr_preview.py:19-102): explicit argtypes/restype, opaque
context pointers. There is no fallback: if the library is missing or fails to
load, every GPU entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# PC_LIB_PATH: an alternative build of the same library (interleaved A/B runs of two
# builds on one box, tools/gpu_run.sh "ab"), so the in-tree library is never swapped
LIB_PATH = Path(os.environ.get("PC_LIB_PATH") or Path(__file__).resolve().parent / "lib" / "libpcgpu.so")

PC_OK = 0
PC_PREC_F16 = 0
PC_PREC_F32 = 1
# host-side mode (not a pc_net_create precision): an f16 net running the f16x3 split program
# (models.compile_scrfd(split=True)) - f32-class detections on f16 MFMA
PC_PREC_F16X3 = 2
# host-side mode: an f16 net running the f16c8 program (models.compile_iresnet(c8=True), DESIGN.md
# §3.7) - f16 hi with e4m3 lo / hi bytes, x_hi*W_hi on f16 MFMA + the corrections on block-scaled e4m3
PC_PREC_F16C8 = 3


def net_precision(mode: int) -> int:
    """The pc_net_create precision of a host precision mode."""
    return PC_PREC_F16 if mode in (PC_PREC_F16X3, PC_PREC_F16C8) else mode

_lib = None


class LetterboxDesc(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("H", C.c_int32), ("W", C.c_int32), ("row_stride", C.c_int32),
                ("new_w", C.c_int32), ("new_h", C.c_int32), ("scale_x", C.c_double), ("scale_y", C.c_double),
                ("simd_end", C.c_int32), ("pad_", C.c_int32)]


class WarpDesc(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("row_stride", C.c_int32), ("w", C.c_int32), ("h", C.c_int32),
                ("pad0_", C.c_int32), ("M", C.c_double * 6), ("d_dst", C.c_void_p), ("out_w", C.c_int32),
                ("out_h", C.c_int32), ("border", C.c_int32), ("pad1_", C.c_int32)]


class ResizeDesc(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("H", C.c_int32), ("W", C.c_int32), ("row_stride", C.c_int32),
                ("new_w", C.c_int32), ("new_h", C.c_int32), ("scale_x", C.c_double), ("scale_y", C.c_double),
                ("simd_end", C.c_int32), ("area_mode", C.c_int32), ("d_dst", C.c_void_p),
                ("inv_x", C.c_double), ("inv_y", C.c_double)]


class AreaTab(C.Structure):
    _fields_ = [("si", C.c_int32), ("di", C.c_int32), ("alpha", C.c_float)]


class YoloLetterboxDesc(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("H", C.c_int32), ("W", C.c_int32), ("row_stride", C.c_int32),
                ("new_w", C.c_int32), ("new_h", C.c_int32), ("top", C.c_int32), ("left", C.c_int32),
                ("scale_x", C.c_double), ("scale_y", C.c_double), ("simd_end", C.c_int32), ("identity", C.c_int32)]


class YoloScale(C.Structure):
    _fields_ = [("gain", C.c_float), ("pad_x", C.c_float), ("pad_y", C.c_float), ("W0", C.c_float),
                ("H0", C.c_float)]


class CropDesc(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("H", C.c_int32), ("W", C.c_int32), ("row_stride", C.c_int32),
                ("pad_", C.c_int32)]


assert C.sizeof(YoloLetterboxDesc) == 64 and C.sizeof(YoloScale) == 20 and C.sizeof(CropDesc) == 24
assert C.sizeof(ResizeDesc) == 80 and C.sizeof(LetterboxDesc) == 56 and C.sizeof(WarpDesc) == 96 and C.sizeof(AreaTab) == 12

_P = C.c_void_p
_I = C.c_int
_SZ = C.c_size_t
_F = C.c_float

SIGNATURES = {
    "pc_abi_version": ([], _I),
    "pc_ctx_create": ([_I, C.POINTER(_P)], _I),
    "pc_ctx_destroy": ([_P], _I),
    "pc_last_error": ([_P], C.c_char_p),
    "pc_ctx_set_stream": ([_P, _P], _I),
    "pc_ctx_stream": ([_P], _P),
    "pc_ctx_set_priority": ([_P, _I], _I),
    "pc_ctx_sync": ([_P], _I),
    "pc_device_alloc": ([_P, _SZ, C.POINTER(_P)], _I),
    "pc_device_free": ([_P, _P], _I),
    "pc_copy_h2d": ([_P, _P, _P, _SZ], _I),
    "pc_copy_d2h": ([_P, _P, _P, _SZ], _I),
    "pc_copy_d2d": ([_P, _P, _P, _SZ], _I),
    "pc_memset": ([_P, _P, _I, _SZ], _I),
    "pc_copy_2d": ([_P, _P, _SZ, _P, _SZ, _SZ, _SZ], _I),
    "pc_host_alloc": ([_P, _SZ, C.POINTER(_P)], _I),
    "pc_host_free": ([_P, _P], _I),
    "pc_fence_create": ([_P, C.POINTER(_P)], _I),
    "pc_fence_record": ([_P, _P], _I),
    "pc_fence_wait": ([_P, _P], _I),
    "pc_fence_destroy": ([_P, _P], _I),
    "pc_net_create": ([_P, _P, _SZ, _I, _I, C.POINTER(_P)], _I),
    "pc_net_destroy": ([_P], _I),
    "pc_net_run": ([_P, _P, _I], _I),
    "pc_net_input_dims": ([_P, C.POINTER(C.c_int32)], _I),
    "pc_net_output": ([_P, _I, C.POINTER(_P), C.POINTER(C.c_int32)], _I),
    "pc_net_num_outputs": ([_P], _I),
    "pc_net_stats": ([_P, C.POINTER(C.c_double), C.POINTER(C.c_int32)], _I),
    "pc_ctx_wait_fence": ([_P, _P], _I),
    "pc_frame_stage": ([_P, _P, _P, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int], _I),
    "pc_net_chain_info": ([_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)], _I),
    "pc_net_set_chain_min_batch": ([_P, C.c_int32], _I),
    "pc_net_set_graph": ([_P, _I], _I),
    "pc_net_set_graph_max_batch": ([_P, C.c_int32], _I),
    "pc_net_profile": ([_P, _I], _I),
    "pc_net_calibrate": ([_P, _P, _I, _I, C.POINTER(C.c_float)], _I),
    "pc_net_profile_read": ([_P, C.POINTER(C.c_double)], _I),
    "pc_net_profile_ops": ([_P, C.POINTER(C.c_double), _I], _I),
    "pc_letterbox": ([_P, _I, C.POINTER(LetterboxDesc), _I, _I, _P], _I),
    "pc_warp_affine": ([_P, C.POINTER(WarpDesc), _I], _I),
    "pc_resize_linear": ([_P, C.POINTER(ResizeDesc), _I], _I),
    "pc_face_quality": ([_P, _P, _I, _I, _P], _I),
    "pc_arcface_prep": ([_P, _I, _P, _I, _I, _I, _P], _I),
    "pc_rotate_pad": ([_P, _P, _I, _I, _I, _I, _I, _P], _I),
    "pc_resize_area_fast": ([_P, _P, _I, _I, _I, _P, _I, _I], _I),
    "pc_resize_area": ([_P, _P, _I, C.POINTER(AreaTab), C.POINTER(C.c_int32), _I, C.POINTER(AreaTab),
                        C.POINTER(C.c_int32), _I, _P, _I, _I], _I),
    "pc_resize_area_batch": ([_P, _P, _P, _I, _I, C.POINTER(AreaTab), C.POINTER(C.c_int32), _I, C.POINTER(AreaTab),
                              C.POINTER(C.c_int32), _I, _I, _I], _I),
    "pc_scrfd_detect": ([_P, C.POINTER(LetterboxDesc), _I, _I, _F, _F, C.POINTER(_F), _I, _P, _P, _P, _P], _I),
    "pc_embed_finalize": ([_P, _P, _I, _I, _I, _I, _P], _I),
    "pc_arcface_embed": ([_P, _P, _I, _I, _P], _I),
    "pc_bank_match": ([_P, _P, _I, _P, _I, _I, _P, _P], _I),
    "pc_estimate_affine_partial": ([_P, _P, _I, _I, _P, _P], _I),
    "pc_invert_affine": ([_P, _P], _I),
    "pc_yolo_letterbox": ([_P, _I, C.POINTER(YoloLetterboxDesc), _I, _I, _I, _P], _I),
    "pc_yolo_detect": ([_P, C.POINTER(YoloLetterboxDesc), _I, _I, _I, _F, _F, C.POINTER(YoloScale), _I, _P, _P,
                        _P], _I),
    "pc_yolo_pose_detect": ([_P, C.POINTER(YoloLetterboxDesc), _I, _I, _I, _F, _F, C.POINTER(YoloScale), _P, _I,
                             _I, _P, _P, _P, _P], _I),
    "pc_clip_prep": ([_P, _I, C.POINTER(CropDesc), _I, _P], _I),
    "pc_clip_embed": ([_P, C.POINTER(CropDesc), _I, _P], _I),
    "pc_l2_normalize": ([_P, _P, _I, _I, _I, _F, _P], _I),
    "pc_pil_bicubic_coeffs": ([_I, _I, _I, _I, C.POINTER(C.c_int32), C.POINTER(C.c_int32), _I], _I),
    "pc_clip_geometry": ([_I, _I, _I, C.POINTER(C.c_int32)], _I),
}


def load(path: os.PathLike = LIB_PATH) -> C.CDLL:
    """Load libpcgpu.so (raises if absent: the GPU path has no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    p = Path(path)
    if not p.is_file():
        raise RuntimeError(f"pcgpu native library not built: {p} (run __graft_entry__.build() or make -C "
                           f"person_capture_amd/csrc)")
    try:
        # the torch-ROCm HIP runtime (same soname) must be the one this library binds to
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(str(p))
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.pc_abi_version() != 1:
        raise RuntimeError("pcgpu ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int, ctx=None, what: str = "") -> None:
    if rc != PC_OK:
        msg = ""
        if ctx is not None and _lib is not None:
            m = _lib.pc_last_error(ctx)
            msg = m.decode() if m else ""
        raise RuntimeError(f"pcgpu {what} failed (status {rc}): {msg}")
