"""PersonDetector — drop-in for person_capture/detectors.py on the MI355X.

Same class name, constructor keywords (model_name='yolov8n.pt', device='cuda',
progress=None), ``device`` attribute and ``detect(frame, conf=0.35)`` contract as the
reference (detectors.py:12-82, 271-296): a list of ``{"xyxy": [x1, y1, x2, y2],
"conf": float, "cls": 0}`` for class person only, ``[]`` on any failure. The reference
calls ultralytics ``predict(conf, iou=0.45, classes=[0], max_det=40, imgsz=640)`` with
rect letterboxing; here the whole predict runs on the device through one C-ABI call
(pc_yolo_detect): letterbox kernel -> YOLOv8 MFMA conv program -> DFL decode ->
class-0 NMS -> scale_boxes, with only the kept boxes copied back.

Weights: ``yolov8{n,s,m,l,x}.pt`` are fetched from the ultralytics hub by the
reference (detectors.py:209-229); none exist offline, so seeded weights of the same
architecture are synthesised (models_yolo.synth_yolov8).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import models_yolo
from ._lib import PC_PREC_F16, PC_PREC_F32, YoloLetterboxDesc, YoloScale, check
from .engines import opencv_vresize_simd_end
from .runtime import GpuContext, Net

_WEIGHTS: Dict[Tuple[str, int], dict] = {}


def _precision() -> int:
    v = os.getenv("PERSON_CAPTURE_AMD_PRECISION", "f16").strip().lower()
    return PC_PREC_F32 if v in ("f32", "fp32", "float32") else PC_PREC_F16


def _device_index(device: str) -> int:
    s = str(device)
    if not s.startswith("cuda"):
        raise RuntimeError("PersonDetector on this build runs on the MI355X HIP device only (device='cuda' or "
                           "'cuda:N'); there is no CPU detection path.")
    return int(s.split(":", 1)[1]) if ":" in s and s.split(":", 1)[1].isdigit() else 0


def yolo_weights(scale: str, seed: int = 0) -> dict:
    key = (scale, seed)
    if key not in _WEIGHTS:
        _WEIGHTS[key] = models_yolo.synth_yolov8(scale, seed=seed)
    return _WEIGHTS[key]


class YoloEngine:
    """YOLOv8 at one letterbox canvas size (Hp x Wp), up to max_batch frames per call."""

    def __init__(self, ctx: GpuContext, params: dict, scale: str, Hp: int, Wp: int, precision: int = PC_PREC_F16,
                 max_batch: int = 16, max_det: int = 40):
        self.ctx, self.Hp, self.Wp, self.max_batch, self.max_det = ctx, Hp, Wp, max_batch, max_det
        self.program = models_yolo.compile_yolov8(params, scale, Hp, Wp)
        self.net = Net(ctx, self.program.serialize(), precision=precision, max_batch=max_batch)

    @property
    def flops_per_image(self) -> float:
        return self.net.flops_per_image

    def detect_device(self, frames: Sequence[Tuple[int, int, int, int]], conf: float, iou: float = 0.45):
        """frames: (device ptr, H, W, row_stride) BGR u8 sharing this canvas. Enqueues the
        detection and returns the (dets, count) device buffers."""
        n = len(frames)
        descs = (YoloLetterboxDesc * n)()
        scales = (YoloScale * n)()
        for i, (ptr, H, W, rs) in enumerate(frames):
            new_w, new_h, top, left, Hp, Wp = models_yolo.letterbox_geometry(H, W)
            if (Hp, Wp) != (self.Hp, self.Wp):
                raise ValueError("frame does not letterbox to this engine's canvas")
            d = descs[i]
            d.d_src, d.H, d.W, d.row_stride = int(ptr), H, W, rs
            d.new_w, d.new_h, d.top, d.left = new_w, new_h, top, left
            d.scale_x, d.scale_y = 1.0 / (float(new_w) / W), 1.0 / (float(new_h) / H)
            d.simd_end = opencv_vresize_simd_end(new_w * 3)
            d.identity = 1 if (new_w, new_h) == (W, H) else 0
            gain, px, py = models_yolo.scale_geometry(Hp, Wp, H, W)
            scales[i].gain, scales[i].pad_x, scales[i].pad_y = gain, float(px), float(py)
            scales[i].W0, scales[i].H0 = float(W), float(H)
        dd = self.ctx.scratch(f"yolo_dets{self.Hp}x{self.Wp}", n * self.max_det * 5 * 4)
        dc = self.ctx.scratch(f"yolo_cnt{self.Hp}x{self.Wp}", n * 4)
        dn = self.ctx.scratch(f"yolo_ncand{self.Hp}x{self.Wp}", n * 4)
        check(self.ctx.lib.pc_yolo_detect(self.net.handle, descs, n, self.Hp, self.Wp, C.c_float(conf),
                                          C.c_float(iou), scales, self.max_det, C.c_void_p(dd.ptr),
                                          C.c_void_p(dc.ptr), C.c_void_p(dn.ptr)), self.ctx.handle, "yolo_detect")
        return dd, dc, dn

    def read(self, bufs, n: int) -> List[np.ndarray]:
        dd, dc, _ = bufs
        cnt = self.ctx.download(dc.ptr, (n,), np.int32)
        dets = self.ctx.download(dd.ptr, (n, self.max_det, 5), np.float32)
        return [dets[i, :min(int(cnt[i]), self.max_det)].copy() for i in range(n)]


class PersonDetector:
    def __init__(self, model_name='yolov8n.pt', device='cuda', progress=None):
        self._device_index = _device_index(device)
        self.device = 'cuda'
        self.progress = progress
        self.model_name = model_name
        self.scale = models_yolo.yolo_scale_of(model_name)
        self.precision = _precision()
        from .face_embedder import get_context
        self._ctx = get_context(self._device_index)
        seed = int(os.getenv("PERSON_CAPTURE_AMD_SEED", "0"))
        if callable(progress):
            progress(f"pcgpu: synthetic weights for yolov8{self.scale} (no checkpoint offline)")
        self._params = yolo_weights(self.scale, seed)
        self._engines: Dict[Tuple[int, int], YoloEngine] = {}
        self._max_batch = int(os.getenv("PERSON_CAPTURE_AMD_YOLO_BATCH", "16"))
        self._engine_tag = f"pcgpu-yolov8{self.scale}"

    def _engine(self, Hp: int, Wp: int) -> YoloEngine:
        e = self._engines.get((Hp, Wp))
        if e is None:
            e = YoloEngine(self._ctx, self._params, self.scale, Hp, Wp, self.precision, self._max_batch)
            self._engines[(Hp, Wp)] = e
        return e

    @staticmethod
    def _to_dicts(dets: np.ndarray) -> List[dict]:
        return [{"xyxy": [float(v) for v in d[:4]], "conf": float(d[4]), "cls": 0} for d in dets]

    def detect_batch(self, frames: Sequence[np.ndarray], conf: float = 0.35, iou: float = 0.45) -> List[List[dict]]:
        """Batched detect(): frames grouped by letterbox canvas, one device call per group."""
        out: List[List[dict]] = [[] for _ in frames]
        groups: Dict[Tuple[int, int], List[int]] = {}
        for i, f in enumerate(frames):
            if f is None or getattr(f, "size", 0) == 0:
                continue
            H, W = f.shape[:2]
            g = models_yolo.letterbox_geometry(H, W)
            groups.setdefault((g[4], g[5]), []).append(i)
        for (Hp, Wp), idx in groups.items():
            eng = self._engine(Hp, Wp)
            for s in range(0, len(idx), eng.max_batch):
                part = idx[s:s + eng.max_batch]
                bufs, devs = [], []
                for i in part:
                    f = np.ascontiguousarray(frames[i], dtype=np.uint8)
                    d = self._ctx.scratch(f"yolo_frame{len(devs)}", f.nbytes)
                    self._ctx.upload(f, d)
                    devs.append((d.ptr, f.shape[0], f.shape[1], f.strides[0]))
                res = eng.read(eng.detect_device(devs, conf, iou), len(part))
                for i, r in zip(part, res):
                    out[i] = self._to_dicts(r)
        return out

    def detect_device(self, d_frames: Sequence[Tuple[int, int, int, int]], conf: float = 0.35,
                      iou: float = 0.45) -> List[np.ndarray]:
        """Frames already in HBM: (ptr, H, W, row_stride) -> per frame [k][5] arrays."""
        out: List[Optional[np.ndarray]] = [None] * len(d_frames)
        groups: Dict[Tuple[int, int], List[int]] = {}
        for i, (_, H, W, _) in enumerate(d_frames):
            g = models_yolo.letterbox_geometry(H, W)
            groups.setdefault((g[4], g[5]), []).append(i)
        for (Hp, Wp), idx in groups.items():
            eng = self._engine(Hp, Wp)
            for s in range(0, len(idx), eng.max_batch):
                part = idx[s:s + eng.max_batch]
                res = eng.read(eng.detect_device([d_frames[i] for i in part], conf, iou), len(part))
                for i, r in zip(part, res):
                    out[i] = r
        return out

    def detect(self, frame, conf=0.35):
        """Return list of dicts for class=person only (detectors.py:271-296)."""
        try:
            if frame is None or frame.size == 0:
                return []
            return self.detect_batch([frame], conf=float(conf))[0]
        except Exception:
            return []
