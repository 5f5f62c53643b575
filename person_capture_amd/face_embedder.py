"""FaceEmbedder — drop-in for person_capture/face_embedder.py (SCRFD + ArcFace branch).

Same module/class name, constructor keywords, mutable attributes, methods and
return values as the reference class (face_embedder.py:376-2508); the numeric
work runs on the MI355X through the pcgpu C ABI:

  reference (per frame)                          here
  ---------------------------------------------  ------------------------------------------
  cv2.resize + blobFromImage (CPU)               pc_letterbox (device, byte-exact restatement)
  ORT/TensorRT SCRFD session.run, H2D/D2H        pc_net_run on the SCRFD program (MFMA convs)
  numpy anchor decode + greedy NMS               pc_scrfd_detect decode + NMS kernels
  cv2.rotate / copyMakeBorder / resize (TTA)     pc_rotate_pad / pc_resize_linear / pc_resize_area
  cv2.estimateAffinePartial2D (CPU)              pc_estimate_affine_partial (native host code)
  cv2.warpAffine 112x112 (CPU)                   pc_warp_affine (device, all faces in one launch)
  cvtColor + Laplacian().var() (CPU)             pc_face_quality (device)
  2N batch-1 TRT ArcFace runs + PCIe trips       pc_arcface_embed: one batched IResNet run, flip-sum + L2 fused

The detector policy (det-size selection, TTA / edge-pad / rotation fallbacks,
adaptive rotation gating, cross-rotation NMS, landmark canonicalisation,
sorting) stays on the host and follows _extract_with_scrfd_raw
(face_embedder.py:2163-2482) step by step.

Weights: scrfd_*_bnkps.onnx and arcface_r100.onnx (glintr100 / w600k_r50) are looked up
where the reference's _ensure_file looks (plus PERSON_CAPTURE_AMD_MODELS) and mapped by
onnx_models.py; when they are absent (the reference would download them; there is no
network here) seeded synthetic weights of the same architectures stand in
(person_capture_amd/models.py) and `weights_source` says so.

The YOLOv8-face backend (the reference default, Y8F_DEFAULT) runs too: face_yolo.py
(YOLOv8 Pose program on the device, the branch policy of face_embedder.py:1671-2093 on the
host, 0-degree predicts batched across frames in extract_batch). The OpenCLIP face-embedding
backend (use_arcface=False) is not on this build's hot path and raises RuntimeError at
construction, as the reference does for unavailable backends. Host frames reach the device
through the native pinned staging ring (pc_frame_stage) on a copy stream.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import imageops, models, onnx_models
from ._lib import PC_PREC_F16, PC_PREC_F16C8, PC_PREC_F16X3, PC_PREC_F32, ResizeDesc, WarpDesc, check
from .engines import ArcFaceEngine, ScrfdEngine, opencv_vresize_simd_end
from .face_yolo import YoloFaceBranch
from .runtime import GpuContext

Y8F_DEFAULT = "yolov8l-face.pt"   # reference default (face_embedder.py:33)
_ARC_SIDE = 112

_CTX_CACHE: Dict[int, GpuContext] = {}
_WEIGHT_CACHE: Dict[Tuple[str, int], models.Params] = {}


class _IBox(tuple):
    """An integer face box (x1, y1, x2, y2) that keeps the detector's float box it was truncated
    from (`f`, reported with the debug chips: parity reports locate one-pixel box differences
    between precisions at the int() of _accumulate, face_embedder.py:2214-2239)."""

    def __new__(cls, box, f=None):
        t = super().__new__(cls, box)
        t.f = None if f is None else np.asarray(f, np.float64).copy()
        return t

    def __reduce__(self):
        return (_IBox, (tuple(self), self.f))


def _round32(x: int) -> int:
    return ((int(x) + 31) // 32) * 32


def _device_index(ctx: str) -> int:
    s = str(ctx)
    if not s.startswith("cuda"):
        raise RuntimeError("SCRFD requires a CUDA device (use device='cuda' or 'cuda:N'); on this build "
                           "'cuda' addresses the MI355X HIP device.")
    if ":" in s:
        try:
            return int(s.split(":", 1)[1])
        except ValueError:
            return 0
    return 0


def get_context(device_index: int, role: str = "") -> GpuContext:
    """The shared context (stream) of a device; role "embed" is a second one, on which the
    face embedder runs chips -> ArcFace -> bank match beside the detections of the main one."""
    key = (device_index, role) if role else device_index
    c = _CTX_CACHE.get(key)
    if c is None:
        c = GpuContext(device_index)
        prio = os.getenv("PERSON_CAPTURE_AMD_EMBED_PRIORITY", "") if role == "embed" else ""
        if prio:   # HIP stream priority of the embed stream (lower = higher), e.g. -1
            c.set_priority(int(prio))
        _CTX_CACHE[key] = c
    return c


_PREC_WORDS = {"f32": PC_PREC_F32, "fp32": PC_PREC_F32, "float32": PC_PREC_F32,
               "f16": PC_PREC_F16, "fp16": PC_PREC_F16, "float16": PC_PREC_F16, "half": PC_PREC_F16,
               "f16x3": PC_PREC_F16X3, "x3": PC_PREC_F16X3, "split": PC_PREC_F16X3,
               "f16c8": PC_PREC_F16C8, "c8": PC_PREC_F16C8}


def _prec_word(var: str, allowed: Tuple[int, ...]) -> Optional[int]:
    """The precision named by environment variable `var` (None when unset); an unknown word or a form
    this net does not run raises instead of silently running plain f16."""
    v = os.getenv(var, "").strip().lower()
    if not v:
        return None
    p = _PREC_WORDS.get(v)
    if p is None or p not in allowed:
        names = sorted(k for k, q in _PREC_WORDS.items() if q in allowed)
        raise ValueError(f"{var}={v!r}: expected one of {names}")
    return p


def _precision(var: str = "PERSON_CAPTURE_AMD_PRECISION") -> int:
    """The run mode: f16 (the timed mode; each net then takes its own default form) or f32 (parity)."""
    p = _prec_word(var, (PC_PREC_F16, PC_PREC_F32))
    if p is None and var != "PERSON_CAPTURE_AMD_PRECISION":
        p = _prec_word("PERSON_CAPTURE_AMD_PRECISION", (PC_PREC_F16, PC_PREC_F32))
    return PC_PREC_F16 if p is None else p


def _det_precision() -> int:
    """SCRFD precision. Default f16x3 (split hi/lo activations and weights on the f16 MFMA
    path): its boxes, landmarks and therefore chips and accept decisions are
    the f32 path's, where plain f16 moved sub-pixel landmarks enough to flip decisions on
    noise frames (bench.py parity). PERSON_CAPTURE_AMD_DET_PRECISION=f16 / f32 select the
    others; with PERSON_CAPTURE_AMD_PRECISION=f32 (the parity mode) the detector is f32 too."""
    p = _prec_word("PERSON_CAPTURE_AMD_DET_PRECISION", (PC_PREC_F32, PC_PREC_F16X3, PC_PREC_F16))
    if p is None:
        return PC_PREC_F32 if _precision() == PC_PREC_F32 else PC_PREC_F16X3
    return p


def _arc_precision() -> int:
    """ArcFace precision. Default f16x3: the split IResNet program (every activation
    and weight f16 hi + f16 lo, 3 f16 MFMAs per product, exact centred input) - embeddings within
    2.7e-6 and cosine distances within 1e-4 of the fp32 path, where plain f16 (the reference's
    TensorRT precision, face_embedder.py:445) moved fd by up to 2.2e-4 on identical chips. f16c8 (e4m3
    lo / hi bytes, the corrections on the block-scaled e4m3 MFMA: half the MFMA issues, 1.5e-5) ran
    no faster on the same staging-bound tiles (r05d: C2 22.5 vs 22.3 ms) and is opt-in.
    PERSON_CAPTURE_AMD_ARC_PRECISION=f16x3 / f16c8 / f16 / f32 select (anything else raises); with
    PERSON_CAPTURE_AMD_PRECISION=f32 (the parity mode) ArcFace is f32 too."""
    p = _prec_word("PERSON_CAPTURE_AMD_ARC_PRECISION", (PC_PREC_F32, PC_PREC_F16X3, PC_PREC_F16C8, PC_PREC_F16))
    if p is None:
        return PC_PREC_F32 if _precision() == PC_PREC_F32 else PC_PREC_F16X3
    return p


def synthetic_weights(kind: str, seed: int = 0) -> models.Params:
    key = (kind, seed)
    p = _WEIGHT_CACHE.get(key)
    if p is None:
        if kind.startswith("scrfd_"):
            p = models.synth_scrfd(kind.split("_", 1)[1], seed=seed)
        elif kind.startswith("iresnet"):
            p = models.synth_iresnet(int(kind[len("iresnet"):]), seed=seed)
        else:
            raise KeyError(kind)
        _WEIGHT_CACHE[key] = p
    return p


class _DevImage:
    """A BGR u8 image resident on the device (owned buffer or a view)."""

    __slots__ = ("ptr", "H", "W", "stride", "_buf")

    def __init__(self, ptr: int, H: int, W: int, stride: int, buf=None):
        self.ptr, self.H, self.W, self.stride, self._buf = int(ptr), int(H), int(W), int(stride), buf


def cv_resize_into(ctx: GpuContext, img: _DevImage, p: dict, d_dst: int) -> None:
    """Run the cv2.resize kernel imageops.resize_plan chose, writing new_h x new_w x 3 contiguous at d_dst."""
    lib, h = ctx.lib, ctx.handle
    nw, nh = p["new_w"], p["new_h"]
    kind = p["kind"]
    if kind == "copy":
        check(lib.pc_copy_2d(h, C.c_void_p(d_dst), nw * 3, C.c_void_p(img.ptr), img.stride, nw * 3, nh), h, "copy_2d")
    elif kind == "area_fast":
        check(lib.pc_resize_area_fast(h, img.ptr, img.stride, p["isx"], p["isy"], d_dst, nh, nw), h,
              "resize_area_fast")
    elif kind == "area":
        (xt, xs), (yt, ys) = imageops.area_tables(img.W, nw, p["scale_x"]), imageops.area_tables(img.H, nh, p["scale_y"])
        check(lib.pc_resize_area(h, img.ptr, img.stride, xt, xs, len(xt), yt, ys, len(yt), d_dst, nh, nw), h,
              "resize_area")
    else:
        d = ResizeDesc()
        d.d_src, d.H, d.W, d.row_stride = img.ptr, img.H, img.W, img.stride
        d.new_w, d.new_h, d.scale_x, d.scale_y = nw, nh, p["scale_x"], p["scale_y"]
        d.inv_x, d.inv_y, d.area_mode = p["inv_x"], p["inv_y"], p["area_mode"]
        d.simd_end = opencv_vresize_simd_end(nw * 3)
        d.d_dst = d_dst
        check(lib.pc_resize_linear(h, (ResizeDesc * 1)(d), 1), h, "resize_linear")


def dev_resize(ctx: GpuContext, img: _DevImage, key: str, dsize: Optional[Tuple[int, int]] = None, fx: float = 0.0,
               fy: float = 0.0, area: bool = False) -> _DevImage:
    """cv2.resize(img, dsize or None, fx, fy, INTER_AREA if area else INTER_LINEAR) on the device, into
    the context's scratch buffer `key`."""
    p = imageops.resize_plan(img.H, img.W, dsize, fx, fy, area)
    buf = ctx.scratch(key, p["new_w"] * p["new_h"] * 3)
    cv_resize_into(ctx, img, p, buf.ptr)
    return _DevImage(buf.ptr, p["new_h"], p["new_w"], p["new_w"] * 3, buf)


def dev_resize_batch(ctx: GpuContext, imgs: Sequence[_DevImage], keys: Sequence[str], dsize: Tuple[int, int],
                     area: bool = True) -> List[_DevImage]:
    """dev_resize of several images to one dsize: the frames that share a source geometry and take the
    generic INTER_AREA path go through one pc_resize_area_batch launch (the pre-scan's speculative
    chunk, gui_app.py:1505-1507 per sample); anything else one dev_resize each. Same bytes."""
    out: List[Optional[_DevImage]] = [None] * len(imgs)
    groups: Dict[Tuple[int, int, int], List[int]] = {}
    for i, im in enumerate(imgs):
        p = imageops.resize_plan(im.H, im.W, dsize, 0.0, 0.0, area)
        if p["kind"] == "area":
            groups.setdefault((im.H, im.W, im.stride), []).append(i)
        else:
            out[i] = dev_resize(ctx, im, keys[i], dsize, area=area)
    for (H, W, stride), idx in groups.items():
        p = imageops.resize_plan(H, W, dsize, 0.0, 0.0, area)
        nw, nh = p["new_w"], p["new_h"]
        (xt, xs), (yt, ys) = imageops.area_tables(W, nw, p["scale_x"]), imageops.area_tables(H, nh, p["scale_y"])
        bufs = [ctx.scratch(keys[i], nw * nh * 3) for i in idx]
        srcs = (C.c_void_p * len(idx))(*[imgs[i].ptr for i in idx])
        dsts = (C.c_void_p * len(idx))(*[b.ptr for b in bufs])
        check(ctx.lib.pc_resize_area_batch(ctx.handle, srcs, dsts, len(idx), stride, xt, xs, len(xt), yt, ys, len(yt),
                                           nh, nw), ctx.handle, "resize_area_batch")
        for i, b in zip(idx, bufs):
            out[i] = _DevImage(b.ptr, nh, nw, nw * 3, b)
    return out


class FaceEmbedder(YoloFaceBranch):
    """Face detection (SCRFD, or the YOLOv8-face default) + ArcFace identity embedding on the MI355X.
    Returns list of dicts: {'bbox': np.int32[x1,y1,x2,y2], 'feat': np.float32[D], 'quality': float}."""

    def __init__(self, ctx: str = 'cuda', yolo_model: str = Y8F_DEFAULT, conf: float = 0.30,
                 use_arcface: bool = True,
                 clip_model_name: str = 'ViT-L-14',
                 clip_pretrained: str = 'laion2b_s32b_b82k',
                 progress=None, trt_lib_dir: Optional[str] = None):
        self.progress = progress
        self.trt_lib_dir = trt_lib_dir
        self.conf = float(conf)
        model = yolo_model if isinstance(yolo_model, str) else ""
        override = os.getenv("PERSON_CAPTURE_AMD_FACE_MODEL", "").strip()
        if not model.lower().startswith("scrfd") and override:
            model = override
        if not use_arcface:
            raise RuntimeError("OpenCLIP face embeddings are not part of this MI355X build; use_arcface=True.")
        # backend choice as the reference (face_embedder.py:383-420, 500-520): names starting with
        # "scrfd" select SCRFD, anything else is a YOLOv8-face checkpoint name
        self.detector_backend = "scrfd" if os.path.basename(model).lower().startswith("scrfd") else "yolo"
        base = os.path.basename(model).lower().replace(".onnx", "").replace("_trt", "")
        self.scrfd_variant = "2.5g" if "2.5g" in base else "10g"
        self._scrfd_model_path = model
        self._device_index = _device_index(ctx)
        self.device = 'cuda'
        self.use_arcface = True
        self.backend = 'arcface'
        self.det = None
        self.insight_app = None
        self.precision = _precision()
        # detector precision (default: the embedder's): SCRFD f32 + ArcFace f16 gives the f32
        # chips (the f16 landmarks move noise-frame chips, bench.py f16_parity attribution)
        self.det_precision = _det_precision()
        self.arc_precision = _arc_precision()
        self._ctx = get_context(self._device_index)
        self._scrfd_ctx_id = self._device_index
        seed = int(os.getenv("PERSON_CAPTURE_AMD_SEED", "0"))
        arc_kind = os.getenv("PERSON_CAPTURE_AMD_ARCFACE", "iresnet100")
        # model files resolved as the reference does (face_embedder.py:598-606, 729-734): the SCRFD
        # file named by yolo_model (+ ".onnx"), then arcface_r100.onnx (glintr100 / w600k_r50 as
        # the zip fallback names them); weights mapped by onnx_models. Without the files (there is
        # no download here) seeded synthetic weights of the same architectures stand in, unless
        # PERSON_CAPTURE_AMD_REQUIRE_WEIGHTS=1.
        self.weights_source: Dict[str, str] = {}
        scrfd_file = model if model.lower().endswith(".onnx") else model + ".onnx"
        scrfd_path = onnx_models.find_model_file(scrfd_file) if self.detector_backend == "scrfd" else None
        arc_path = next((p for p in map(onnx_models.find_model_file,
                                        (onnx_models.ARCFACE_ONNX,) + onnx_models.ARCFACE_ALT) if p), None)
        if os.getenv("PERSON_CAPTURE_AMD_REQUIRE_WEIGHTS", "0") == "1" and not (
                (scrfd_path or self.detector_backend != "scrfd") and arc_path):
            raise RuntimeError(f"model files not found: {scrfd_file if not scrfd_path else ''} "
                               f"{onnx_models.ARCFACE_ONNX if not arc_path else ''}".strip())
        try:
            if self.detector_backend == "yolo":
                self._init_yolo_face(model or Y8F_DEFAULT, seed)
                self._scrfd_params = None
            elif scrfd_path:
                self._scrfd_params, self.scrfd_variant = onnx_models.load_scrfd(scrfd_path)
                self.weights_source["scrfd"] = scrfd_path
            else:
                self._scrfd_params = synthetic_weights(f"scrfd_{self.scrfd_variant}", seed)
                self.weights_source["scrfd"] = f"synthetic:scrfd_{self.scrfd_variant}:seed{seed}"
            if arc_path:
                self._arc_params, self._arc_depth, _ = onnx_models.load_arcface(arc_path)
                self.weights_source["arcface"] = arc_path
            else:
                self._arc_params = synthetic_weights(arc_kind, seed)
                self._arc_depth = int(arc_kind[len("iresnet"):])
                self.weights_source["arcface"] = f"synthetic:{arc_kind}:seed{seed}"
        except (ValueError, KeyError, OSError) as e:
            raise RuntimeError(f"failed to load face models: {e}") from e
        if callable(progress):
            progress("pcgpu: weights " + " ".join(f"{k}={v}" for k, v in self.weights_source.items()))
        self._det_batch = int(os.getenv("PERSON_CAPTURE_AMD_DET_BATCH", "8"))
        # ArcFace rows per net run (flip-TTA: half as many faces). 512 = 256 faces, so the embed quantum
        # below (146 faces = 292 rows, one round of the 256x224 tiles) fits one run; with 256 rows the
        # quantum was capped at 128 faces outside bench.py, which always set 512
        self._arc_batch = int(os.getenv("PERSON_CAPTURE_AMD_ARC_BATCH", "512"))
        # frames per detection chunk of extract_batch: the host policy of chunk c runs
        # while the device works on chunk c+1 (0 = one chunk, no overlap)
        self._pipe_chunk = int(os.getenv("PERSON_CAPTURE_AMD_PIPE_CHUNK", "32"))
        self._pipe_ahead = int(os.getenv("PERSON_CAPTURE_AMD_PIPE_AHEAD", "2"))
        # at the end of every detection chunk's policy (but the last), launch the faces
        # collected so far as ArcFace batches of whole quanta: the device then never waits
        # for the host to fill a full batch. The quantum is the face count whose flip-TTA
        # images fill one round of the dominant 14x14x256 conv over the CUs: one image per
        # workgroup on conv_hxi (f16x3, pc_conv_hxi.hip) = 256 rows = 128 faces (round 5's
        # 256x224 tiles: 256 CUs x 224 px / 196 px per image / 2 images per face = 146); partial
        # rounds cost a whole round of that layer. 0 = full batches only. (Resident block chains
        # change the round: see below. f16 beside the detection stream: 128 faces too - C3 r04:
        # 1578 / 1596 frames/s against 1561 / 1562 / 1567 with 146, profiles/r04sw_c3_pipeline_sweep.txt.)
        self._embed_quantum = int(os.getenv("PERSON_CAPTURE_AMD_EMBED_QUANTUM", "128"))
        # batched speculative fallback passes (TTA / edge pad / pre-scan rotations) per chunk
        self._fb_prefetch = os.getenv("PERSON_CAPTURE_AMD_FALLBACK_PREFETCH", "1") != "0"
        # host phase timers of extract_batch (diagnostics; bench.py prints them)
        self.host_times: Optional[Dict[str, float]] = {} if os.getenv("PERSON_CAPTURE_AMD_HOST_TIMING") else None
        self._scrfd_engines: Dict[int, ScrfdEngine] = {}
        # SCRFD backend: the embed side (warp/resize chips, quality, ArcFace, bank match,
        # readbacks) runs on a second stream, so a chunk's ArcFace batches execute beside the
        # detection chunks queued ahead of it instead of behind them (the small late SCRFD
        # layers and every launch's last partial round leave CUs idle). Its only inputs from
        # the detection stream are the frames, which are on the device before the host has
        # the detections that name the faces (the host waited on their fence).
        # PERSON_CAPTURE_AMD_EMBED_STREAM=0: one stream.
        two = self.detector_backend == "scrfd" and os.getenv("PERSON_CAPTURE_AMD_EMBED_STREAM", "1") != "0"
        self._ectx = get_context(self._device_index, "embed") if two else self._ctx
        if two and "PERSON_CAPTURE_AMD_EMBED_QUANTUM" not in os.environ:
            # (f16: 128 faces, r04. f16x3: the 14x14x256 layers run one image per workgroup on
            # conv_hxi (pc_conv_hxi.hip), so a round is 256 rows = 128 faces - C3 r06 962 vs 876 frames/s
            # with the 146 of round 5's 256x224 tiles, profiles/r06e_*)
            self._embed_quantum = 128
        # host frames (extract / extract_batch without dev_frames) reach the device through the
        # native pinned staging ring on a copy stream of their own (pc_frame_stage)
        self._h2d = get_context(self._device_index, "h2d")
        self._stage_threads = int(os.getenv("PERSON_CAPTURE_AMD_STAGE_THREADS", "8"))
        self._arc = ArcFaceEngine(self._ectx, self._arc_params, self._arc_depth, precision=self.arc_precision,
                                  max_batch=self._arc_batch)
        # HIP graphs for net runs (unchanged callers' per-frame extract(): a SCRFD pass of one frame and
        # an ArcFace pass of its faces are ~60 and ~100 small launches each; a C3 ArcFace quantum ~120):
        # SCRFD runs of at most this many images and ArcFace runs of 4x as many rows replay a captured
        # graph (bit-identical, the same launches). 128 (round 6; was 8): C3 1014 -> 1030 frames/s, C4 /
        # C5 unchanged (profiles/r06aj_graph_batch_ab.txt). PERSON_CAPTURE_AMD_GRAPH_BATCH=0 launches eagerly
        self._graph_batch = int(os.getenv("PERSON_CAPTURE_AMD_GRAPH_BATCH", "128"))
        if self._graph_batch > 0:
            self._arc.net.set_graph(True, max_batch=4 * self._graph_batch)
        self._arc_feat_dim = self._arc.dim
        self._arc_fixed_batch = False
        # resident block chains (one image per CU through the 14x14x256 stage) need whole CUs:
        # beside the detection stream they lose to the per-conv kernels (measured C3 r03: 1705
        # vs 1925 frames/s), so they run only when ArcFace has the device to itself. A chain
        # round is one image per CU: 128 flip-TTA faces on 256 CUs.
        if two and os.getenv("PERSON_CAPTURE_AMD_CHAIN", "auto") == "auto":
            self._arc.net.set_chain_min_batch(0)
        nch, min_b, per_round = self._arc.net.chain_info()
        if nch > 0 and min_b < (1 << 30) and "PERSON_CAPTURE_AMD_EMBED_QUANTUM" not in os.environ:
            self._embed_quantum = max(1, per_round // 2)
        # --- SCRFD probe controls (face_embedder.py:473-476) ---
        self.scrfd_tta_scales = (0.75, 0.60)
        self.scrfd_probe_conf_cap = 0.20
        self.scrfd_edge_pad_frac = 0.06
        self.scrfd_min_box_px = 8
        # --- pre-scan controls (:477-487) ---
        self._fast_prescan = False
        self._prescan_rr = 0
        self._prescan_rr_mode = "rr"
        self._prescan_escalate = False
        self._probe_conf = 0.03
        self._high_90 = 1536
        self._high_180 = 1280
        self._prescan_period = 3
        self._prescan_probe_imgsz = 384
        self._prescan_no_upscale_det = True
        self._heavy_cap = 2048
        # --- adaptive rotation controls (:489-497) ---
        self._frame_idx = 0
        self._no_face_streak = 0
        self._last_face_idx = -10 ** 9
        self._rot_cycle = 0
        self.rot_adaptive = True
        self.rot_every_n = 12
        self.rot_after_hit_frames = 8
        self.fast_no_face_imgsz = 512
        self._scrfd_fixed_shape = (640, 640)
        # when a list, extract_batch appends (frame index, policy_state()) after each frame's
        # detector policy (the speculative pre-scan driver rolls back with it)
        self.state_trace: Optional[list] = None
        self._fb_cache: Dict[tuple, tuple] = {}
        self.fb_stats = [0, 0]   # fallback detections served by the batched prefetch / run one by one
        self.fb_kind_stats: Dict[str, List[int]] = {}   # the same per view kind ("tta", "pad", "rot")
        # 0-degree passes served by the speculative batch / re-run because the state changed the det size
        self.spec_stats = [0, 0]
        if self.detector_backend == "scrfd":
            self.scrfd = self._engine(640)
            if callable(progress):
                progress(f"SCRFD(pcgpu) ready on cuda:{self._device_index} det=(640, 640)")
        else:
            self.scrfd = None
            self.det = f"pcgpu-yolov8{self.yolo_scale}-face"
            self.backend = "arcface"
            if callable(progress):
                progress(f"YOLOv8-face(pcgpu) ready on cuda:{self._device_index}")

    # ------------------------------------------------------------------ knobs
    def set_prescan_fast(self, enable: bool, *, mode: str = "rr") -> None:
        """face_embedder.py:1224-1231."""
        self._fast_prescan = bool(enable)
        self._prescan_rr_mode = str(mode)
        if enable:
            self._prescan_rr = 0

    def set_prescan_hint(self, *, escalate: bool = False) -> None:
        """face_embedder.py:1233-1236."""
        self._prescan_escalate = bool(escalate)

    def configure_rotation_strategy(self, *, adaptive: Optional[bool] = None, every_n: Optional[int] = None,
                                    after_hit_frames: Optional[int] = None,
                                    fast_no_face_imgsz: Optional[int] = None) -> None:
        """face_embedder.py:1238-1272."""
        if adaptive is not None:
            self.rot_adaptive = bool(adaptive)
        if every_n is not None:
            try:
                self.rot_every_n = max(1, int(every_n))
            except Exception:
                pass
        if after_hit_frames is not None:
            try:
                self.rot_after_hit_frames = max(0, int(after_hit_frames))
            except Exception:
                pass
        if fast_no_face_imgsz is not None:
            try:
                self.fast_no_face_imgsz = max(0, int(fast_no_face_imgsz))
            except Exception:
                pass
        self._rot_cycle = 0

    # ------------------------------------------------------------------ engines
    def _engine(self, D: int) -> ScrfdEngine:
        e = self._scrfd_engines.get(D)
        if e is None:
            # heavy fallback sizes (up to 2048) run on single frames: keep their activation
            # buffers at the footprint of a det_batch x 640 engine
            mb = max(1, min(self._det_batch, self._det_batch * 640 * 640 // (D * D)))
            e = ScrfdEngine(self._ctx, self._scrfd_params, self.scrfd_variant, D=D, precision=self.det_precision,
                            max_batch=mb, max_det=1024)
            if self._graph_batch > 0:   # per-frame / fallback runs: one graph launch per net run
                e.net.set_graph(True, max_batch=self._graph_batch)
            self._scrfd_engines[D] = e
        return e

    def _upload(self, bgr: np.ndarray, key: str = "frame") -> _DevImage:
        a = np.asarray(bgr)
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError("expected an HxWx3 BGR uint8 image")
        buf = self._ctx.scratch(key, a.shape[0] * a.shape[1] * 3)
        self._h2d.stage_frame(a, buf.ptr, self._stage_threads)
        self._ctx.wait_fence(self._h2d.fence("h2d_up"))
        return _DevImage(buf.ptr, a.shape[0], a.shape[1], a.shape[1] * 3, buf)

    def _detect_batch(self, imgs: Sequence[_DevImage], dyn: int, conf: float):
        eng = self._engine(int(dyn))
        return eng.detect_frames([(im.ptr, im.H, im.W, im.stride) for im in imgs], thresh=float(conf))

    # ------------------------------------------------------------------ batched fallback passes
    def _fb_detect(self, im: _DevImage, view: tuple, dyn: int, conf: float, make):
        """One fallback detection of `view` of frame `im` (("tta", s), ("pad", p), ("rot", deg, pad))
        at det size dyn and threshold conf: from the speculative batch prefetch when it ran with
        exactly these parameters, else now (make() builds the view image on the device)."""
        key = (im.ptr, im.H, im.W, im.stride) + tuple(view) + (int(dyn), float(conf))
        hit = self._fb_cache.pop(key, None)
        per = self.fb_kind_stats.setdefault(view[0], [0, 0])
        if hit is not None:
            self.fb_stats[0] += 1
            per[0] += 1
            return hit
        self.fb_stats[1] += 1
        per[1] += 1
        return self._detect_once(make(), dyn, conf)

    def _fb_run(self, jobs: list) -> None:
        """jobs: (key, view image, det size, conf): batched per (size, conf), results into the cache."""
        groups: Dict[Tuple[int, float], list] = {}
        for key, img, D, cf in jobs:
            groups.setdefault((D, cf), []).append((key, img))
        for (D, cf), lst in groups.items():
            res = self._engine(D).detect_frames([(g.ptr, g.H, g.W, g.stride) for _, g in lst], thresh=cf)
            for (key, _), r in zip(lst, res):
                self._fb_cache[key] = r

    def _prefetch_rotations_normal(self, idx: List[int], imgs, spec_dyn: list, still_empty: set, scratch_img) -> None:
        """Normal-mode rotation passes (face_embedder.py:2330-2433) of the chunk's frames that stay
        empty after TTA and edge pad: the gate is simulated over the chunk (frame counter, last
        face index; rotations assumed to find nothing), then stage by stage over the frames still
        empty — per degree 90 / 270 / 180 the probe and the heavy passes at 1280 / 1536, a frame
        leaving the plan at its first hit, as the policy does."""
        fi, last = self._frame_idx, self._last_face_idx
        plan = []
        for i in idx:
            if imgs[i] is None or spec_dyn[i] is None:
                continue
            fi += 1
            if i not in still_empty:
                last = fi   # faces at 0 degrees or in the TTA / pad passes
                continue
            if self.rot_adaptive:
                need = (fi - last) <= self.rot_after_hit_frames or ((fi + (id(self) & 7)) % self.rot_every_n) == 0
            else:
                need = True
            if need:
                plan.append(i)
        if not plan:
            return
        probe_conf = max(0.02, float(getattr(self, "_probe_conf", 0.02)))
        pad = 24
        pending = list(plan)
        for deg in (90, 270, 180):
            if not pending:
                break
            conf_deg = max(0.10, float(self.conf) * (0.8 if deg in (90, 270) else 0.6))
            jobs = []
            for i in pending:
                im = imgs[i]
                probe_dyn = _round32(max(320, min(spec_dyn[i], int(getattr(self, "_prescan_probe_imgsz", 384)))))
                img_r = scratch_img("rot", i, lambda k: self._dev_rotate_pad(im, deg, 0, key=k))
                jobs.append(((im.ptr, im.H, im.W, im.stride, "rot", deg, 0, probe_dyn, float(probe_conf)), img_r,
                             probe_dyn, probe_conf))
            self._fb_run(jobs)
            heavy_img = {i: scratch_img("rot", i, lambda k, im=imgs[i]: self._dev_rotate_pad(im, deg, pad, key=k))
                         for i in pending}
            left = list(pending)
            for stage in range(2):
                jobs = []
                for i in left:
                    im, dyn = imgs[i], spec_dyn[i]
                    sizes = []
                    for base in (max(dyn, 1280), max(dyn, 1536)):
                        if _round32(base) not in sizes:
                            sizes.append(_round32(base))
                    if stage < len(sizes):
                        jobs.append(((im.ptr, im.H, im.W, im.stride, "rot", deg, pad, sizes[stage], float(conf_deg)),
                                     heavy_img[i], sizes[stage], conf_deg))
                self._fb_run(jobs)
                hit = {j[0][:4] for j in jobs if len(self._fb_cache.get(j[0], ((),))[0])}
                left = [i for i in left if (imgs[i].ptr, imgs[i].H, imgs[i].W, imgs[i].stride) not in hit]
            # a hit at this degree ends the frame's rotation passes (dets found -> break)
            pending = left

    def _empty_at_0(self, im: _DevImage, first) -> bool:
        bb, kp = first
        min_px = int(getattr(self, "scrfd_min_box_px", 8))
        d = self._accumulate0(np.asarray(bb), np.asarray(kp, np.float32), im.W, im.H) if len(bb) else []
        return not any(x[0][2] - x[0][0] >= min_px and x[0][3] - x[0][1] >= min_px for x in d)

    def _prefetch_fallbacks(self, idx: List[int], imgs: Sequence[Optional[_DevImage]], spec: list,
                            spec_dyn: list) -> None:
        """Speculative batched fallback passes for the frames of a chunk whose 0-degree pass (at the
        predicted det size) found nothing, in the order _scrfd_policy would run them: TTA scales then
        the edge pad (stage by stage over the frames still empty), or in fast pre-scan with fixed
        rotation gating the round-robin rotation probe and, where it hits, the heavy pass. Results
        are cached under their exact parameters; the sequential policy walk consumes them (a frame
        whose state-dependent parameters came out differently simply misses and detects then)."""
        empty = [i for i in idx if imgs[i] is not None and spec[i] is not None and spec_dyn[i] is not None
                 and self._empty_at_0(imgs[i], spec[i])]
        if not empty:
            return
        ks = 0

        def scratch_img(kind, i, build):
            nonlocal ks
            ks += 1
            return build(f"fb_{kind}{ks}")

        if not self._fast_prescan:
            probe_conf = min(float(self.conf), float(self.scrfd_probe_conf_cap))
            pending = list(empty)
            for s in tuple(self.scrfd_tta_scales) + (1.25,):
                jobs = []
                for i in pending:
                    im = imgs[i]
                    if s == 1.25 and max(im.W, im.H) > 1920:
                        continue
                    dyn_s = _round32(min(self._heavy_cap, max(320, int(spec_dyn[i] * s))))
                    img_s = scratch_img("tta", i, lambda k: self._dev_resize(im, k, fx=s, fy=s, area=s < 1.0))
                    key = (im.ptr, im.H, im.W, im.stride, "tta", s, dyn_s, float(probe_conf))
                    jobs.append((key, img_s, dyn_s, probe_conf))
                self._fb_run(jobs)
                pending = [i for i in pending if not any(len(self._fb_cache.get(j[0], ((),))[0]) for j in jobs
                                                         if j[0][:4] == (imgs[i].ptr, imgs[i].H, imgs[i].W,
                                                                         imgs[i].stride))]
            jobs = []
            for i in pending:
                im = imgs[i]
                pad = int(round(min(64, float(self.scrfd_edge_pad_frac) * max(im.W, im.H))))
                if pad > 0:
                    img_p = scratch_img("pad", i, lambda k: self._dev_rotate_pad(im, 0, pad, key=k))
                    jobs.append(((im.ptr, im.H, im.W, im.stride, "pad", pad, spec_dyn[i], float(probe_conf)), img_p,
                                 spec_dyn[i], probe_conf))
            self._fb_run(jobs)
            pending = [i for i in pending if not any(len(self._fb_cache.get(j[0], ((),))[0]) for j in jobs
                                                     if j[0][:4] == (imgs[i].ptr, imgs[i].H, imgs[i].W, imgs[i].stride))]
            self._prefetch_rotations_normal(idx, imgs, spec_dyn, set(pending), scratch_img)
            return
        if self.rot_adaptive:
            return   # rotation gating depends on the sequential hit history
        rr = self._prescan_rr
        probe_conf = max(0.02, float(getattr(self, "_probe_conf", 0.02)))
        plan = []
        for i in empty:
            if self._prescan_rr_mode == "rr":
                degs = ((90, 270)[rr % 2],)
                rr += 1
            else:
                degs = (90, 270)
            plan.append((i, degs))
        jobs = []
        for i, degs in plan:
            im = imgs[i]
            probe_dyn = _round32(max(320, min(spec_dyn[i], int(getattr(self, "_prescan_probe_imgsz", 384)))))
            for deg in degs:
                img_r = scratch_img("rot", i, lambda k: self._dev_rotate_pad(im, deg, 0, key=k))
                jobs.append(((im.ptr, im.H, im.W, im.stride, "rot", deg, 0, probe_dyn, float(probe_conf)), img_r,
                             probe_dyn, probe_conf))
        self._fb_run(jobs)
        jobs = []
        for i, degs in plan:
            im = imgs[i]
            probe_dyn = _round32(max(320, min(spec_dyn[i], int(getattr(self, "_prescan_probe_imgsz", 384)))))
            dyn = spec_dyn[i]
            L = max(im.H, im.W)
            heavy_cap = max(int(getattr(self, "_heavy_cap", 2048)), dyn)
            for deg in degs:
                pk = (im.ptr, im.H, im.W, im.stride, "rot", deg, 0, probe_dyn, float(probe_conf))
                hits = len(self._fb_cache.get(pk, ((),))[0])
                do_heavy = hits > 0 or self._prescan_escalate
                if hits == 0:
                    continue
                if deg == 180:
                    heavy = min(_round32(max(dyn, int(0.67 * L))), heavy_cap)
                else:
                    heavy = min(_round32(max(dyn, int(0.75 * L))), heavy_cap)
                override = getattr(self, "_high_180" if deg == 180 else "_high_90", None)
                if override and override > 0:
                    heavy = max(heavy, _round32(int(override)))
                heavy = min(heavy, int(getattr(self, "_heavy_cap", 2048)))
                D = heavy if do_heavy else dyn
                conf_deg = max(0.10, float(self.conf) * (0.8 if deg in (90, 270) else 0.6))
                img_h = scratch_img("rot", i, lambda k: self._dev_rotate_pad(im, deg, 24, key=k))
                jobs.append(((im.ptr, im.H, im.W, im.stride, "rot", deg, 24, D, float(conf_deg)), img_h, D, conf_deg))
        self._fb_run(jobs)

    def _detect_once(self, img: _DevImage, dyn: int, conf: float):
        if self.host_times is None:
            return self._detect_batch([img], dyn, conf)[0]
        t = time.perf_counter()   # (diagnostics: the synchronous detections inside the policy walk)
        r = self._detect_batch([img], dyn, conf)[0]
        self.host_times["inline_detect_within_policy"] = self.host_times.get("inline_detect_within_policy", 0.0) + \
            time.perf_counter() - t
        return r

    def _dev_rotate_pad(self, img: _DevImage, deg: int, pad: int, key: str) -> _DevImage:
        rh, rw = (img.W, img.H) if deg in (90, 270) else (img.H, img.W)
        OH, OW = rh + 2 * pad, rw + 2 * pad
        buf = self._ctx.scratch(key, OH * OW * 3)
        check(self._ctx.lib.pc_rotate_pad(self._ctx.handle, img.ptr, img.H, img.W, img.stride, int(deg), int(pad),
                                          buf.ptr), self._ctx.handle, "rotate_pad")
        return _DevImage(buf.ptr, OH, OW, OW * 3, buf)

    def _dev_resize(self, img: _DevImage, key: str, dsize: Optional[Tuple[int, int]] = None, fx: float = 0.0,
                    fy: float = 0.0, area: bool = False) -> _DevImage:
        """cv2.resize(img, dsize or None, fx, fy, INTER_AREA if area else INTER_LINEAR) on the device."""
        return dev_resize(self._ctx, img, key, dsize, fx, fy, area)

    def _cv_resize(self, img: _DevImage, p: dict, d_dst: int) -> None:
        cv_resize_into(self._ctx, img, p, d_dst)

    # ------------------------------------------------------------------ static helpers (reference API)
    _ARC_DST = imageops.ARC_DST

    @staticmethod
    def _canon_5pts(pts: np.ndarray) -> Optional[np.ndarray]:
        return imageops.canon_5pts(pts)

    @staticmethod
    def _iou(a, b):
        """face_embedder.py:2484-2494 (no +1)."""
        iw = max(0, min(a[2], b[2]) - max(a[0], b[0]))
        ih = max(0, min(a[3], b[3]) - max(a[1], b[1]))
        inter = iw * ih
        area_a = max(0, a[2] - a[0]) * max(0, a[3] - a[1])
        area_b = max(0, b[2] - b[0]) * max(0, b[3] - b[1])
        denom = area_a + area_b - inter
        return inter / denom if denom > 0 else 0.0

    @staticmethod
    def _nms_boxes(boxes, iou_thr=0.5):
        kept = []
        for b in sorted(boxes, key=lambda t: (t[2] - t[0]) * (t[3] - t[1]), reverse=True):
            if all(FaceEmbedder._iou(b, k) < iou_thr for k in kept):
                kept.append(b)
        return kept

    @staticmethod
    def best_face(faces):
        if not faces:
            return None
        return max(faces, key=lambda f: (f['quality'], (f['bbox'][2] - f['bbox'][0]) * (f['bbox'][3] - f['bbox'][1])))

    # ------------------------------------------------------------------ public API
    def extract(self, bgr_img: np.ndarray, *, imgsz: Optional[int] = None):
        """face_embedder.py:1663-1669 -> _extract_with_scrfd (:2095-2103)."""
        if bgr_img is None or bgr_img.size == 0:
            return []
        return self.extract_batch([bgr_img], imgsz=imgsz)[0]

    def extract_batch(self, frames: Sequence[np.ndarray], *, imgsz: Optional[int] = None,
                      dev_frames: Optional[Sequence[_DevImage]] = None, bank=None) -> List[list]:
        """Frame-order-exact batched extract: returns exactly what calling extract() on
        each frame in order would return (same state updates), with the 0-degree SCRFD
        passes, warps, quality and ArcFace runs of all frames batched on the device.
        bank: optional match.DeviceBank; each face dict then also carries
        'fd' = Processor._fd_min(feat, bank), computed on the device."""
        self._bank = bank
        self._fb_cache = {}
        n = len(frames) if dev_frames is None else len(dev_frames)
        if self.detector_backend == "yolo":   # face_embedder.py:1671-2093
            if dev_frames is not None:
                ims = list(dev_frames)
            else:
                ims = [None if f is None or f.size == 0 else self._upload(f, key=f"yf_frame{i}")
                       for i, f in enumerate(frames)]
            return self._extract_batch_yolo(ims, imgsz)
        imgs: List[Optional[_DevImage]] = []
        host_src: Dict[int, np.ndarray] = {}   # host frames not yet staged (device buffers reserved)
        for i in range(n):
            if dev_frames is not None:
                imgs.append(dev_frames[i])
            else:
                f = frames[i]
                if f is None or f.size == 0:
                    imgs.append(None)
                    continue
                if f.ndim != 3 or f.shape[2] != 3:
                    raise ValueError("expected an HxWx3 BGR uint8 image")
                buf = self._ctx.scratch(f"frame{i}", f.shape[0] * f.shape[1] * 3)
                imgs.append(_DevImage(buf.ptr, f.shape[0], f.shape[1], f.shape[1] * 3, buf))
                host_src[i] = f
        # speculative 0-degree pass for every frame at the det size implied by the current
        # state, enqueued chunk by chunk with its readback into pinned memory; the policy of
        # chunk c (host) then overlaps the device work of the later chunks, and ArcFace
        # launches as soon as a full batch of faces is known.
        ht = self.host_times
        tick = time.perf_counter
        t_prev = tick()

        def lap(key):
            nonlocal t_prev
            if ht is not None:
                t = tick()
                ht[key] = ht.get(key, 0.0) + (t - t_prev)
                t_prev = t
        spec_dyn = [self._dyn_for(im, imgsz) if im is not None else None for im in imgs]
        spec: List[Optional[tuple]] = [None] * n
        chunk = self._pipe_chunk if self._pipe_chunk > 0 else max(1, n)
        chunks = [list(range(c0, min(n, c0 + chunk))) for c0 in range(0, n, chunk)]
        det_pending: List[list] = [[] for _ in chunks]
        slot = 0

        def launch_det(ci: int) -> None:
            nonlocal slot
            if ci >= len(chunks):
                return
            staged = [i for i in chunks[ci] if i in host_src]
            if staged:
                # host frames of this chunk: pinned staging + H2D on the copy stream, which the
                # detection stream waits on; the copies of chunk c+1 overlap chunk c's detection
                for i in staged:
                    self._h2d.stage_frame(host_src.pop(i), imgs[i].ptr, self._stage_threads)
                self._ctx.wait_fence(self._h2d.fence(f"h2d{ci % 4}"))
            by_dyn: Dict[int, List[int]] = {}
            for i in chunks[ci]:
                if spec_dyn[i] is not None:
                    by_dyn.setdefault(spec_dyn[i], []).append(i)
            for d, idx in by_dyn.items():
                eng = self._engine(int(d))
                for s0 in range(0, len(idx), eng.max_batch):
                    sub = idx[s0:s0 + eng.max_batch]
                    pend = eng.detect_async([(imgs[i].ptr, imgs[i].H, imgs[i].W, imgs[i].stride) for i in sub],
                                            float(self.conf), slot=str(slot))
                    det_pending[ci].append((sub, eng, pend))
                    slot += 1
        # keep `ahead` detection chunks queued in front of the host so ArcFace batches
        # enqueued by the policy interleave with the remaining detection work
        ahead = max(1, self._pipe_ahead)
        for ci in range(ahead):
            launch_det(ci)
        lap("det_launch")
        faces_per_frame: List[list] = [[] for _ in range(n)]
        jobs: List[tuple] = []       # (frame index, (xi1, yi1, xi2, yi2), kps) not yet launched
        emb_pending: List[tuple] = []
        for ci, frames_c in enumerate(chunks):
            lap("host_other")
            for sub, eng, pend in det_pending[ci]:
                for i, r in zip(sub, eng.collect(pend)):
                    spec[i] = r
            lap("det_wait")
            if self._fb_prefetch:
                self._prefetch_fallbacks(frames_c, imgs, spec, spec_dyn)
                lap("fallback_prefetch")
            launch_det(ci + ahead)
            lap("det_launch")
            for i in frames_c:
                im = imgs[i]
                if im is None:
                    continue
                self._frame_idx += 1
                dyn = self._dyn_for(im, imgsz)
                self.spec_stats[0 if dyn == spec_dyn[i] else 1] += 1
                first = spec[i] if dyn == spec_dyn[i] else self._detect_once(im, dyn, float(self.conf))
                kept = self._scrfd_policy(im, dyn, first)
                faces_per_frame[i] = kept
                if self.state_trace is not None:
                    self.state_trace.append((i, self.policy_state()))
                jobs.extend(self._face_jobs(im, i, kept))
            lap("policy")
            per = self._embed_per()
            while len(jobs) >= per:
                emb_pending.append(self._embed_launch(imgs, jobs[:per], len(emb_pending)))
                jobs = jobs[per:]
            # chunk boundary: queue whole quanta of what is known behind the detections still
            # in flight, so the device goes from SCRFD straight into ArcFace (measured r02:
            # 3.2 ms of idle device per C3 step while the host filled the first full batch).
            # Embeddings do not depend on how faces are batched.
            q = min(self._embed_quantum, per)
            if q > 0 and ci + 1 < len(chunks) and len(jobs) >= q:
                k = len(jobs) // q * q
                emb_pending.append(self._embed_launch(imgs, jobs[:k], len(emb_pending)))
                jobs = jobs[k:]
            lap("embed_launch")
        if jobs:
            emb_pending.append(self._embed_launch(imgs, jobs, len(emb_pending)))
        lap("embed_launch")
        self._fb_cache = {}
        out: List[list] = [[] for _ in range(n)]
        for pend in emb_pending:
            self._embed_collect(pend, out)
        self._ctx.sync()
        self._ectx.sync()
        lap("embed_wait_collect")
        for lst in out:
            lst.sort(key=lambda f: (f['quality'], (f['bbox'][2] - f['bbox'][0]) * (f['bbox'][3] - f['bbox'][1])),
                     reverse=True)
        return out

    # ------------------------------------------------------------------ detector policy
    def policy_state(self) -> tuple:
        """The per-instance state the SCRFD policy carries from frame to frame
        (face_embedder.py:489-497): frame index, no-face streak, last face index, rotation
        cycle, pre-scan round-robin counter."""
        return (self._frame_idx, self._no_face_streak, self._last_face_idx, self._rot_cycle, self._prescan_rr)

    def set_policy_state(self, st: tuple) -> None:
        self._frame_idx, self._no_face_streak, self._last_face_idx, self._rot_cycle, self._prescan_rr = st

    def prescan_policy_key(self, state: tuple, active: bool, H: int, W: int) -> tuple:
        """What a fast pre-scan sample's extraction reads of the policy state, for the sharded
        pre-scan merge (prescan_shard.py): a speculative result is reused only when this key is
        the true stream's. With the pre-scan configuration (rot_adaptive off, gui_app.py:1164)
        the regime picks escalation / full rotation mode (_scrfd_policy, face_embedder.py:
        2330-2360: every empty sample probes rotations; "rr" mode probes (90, 270)[rr % 2]); the
        no-face streak enters only through `streak >= 3` in _dyn_for, and only where that
        changes the det size of this H x W sample. Adaptive rotation gates read the frame and
        last-face indices: then the whole state is the key."""
        if self.rot_adaptive or not self._fast_prescan:
            return (bool(active), tuple(state))
        im = _DevImage(0, int(H), int(W), int(W) * 3)
        saved = self._no_face_streak
        try:
            self._no_face_streak = 0
            d0 = self._dyn_for(im, None)
            self._no_face_streak = 3
            d3 = self._dyn_for(im, None)
        finally:
            self._no_face_streak = saved
        fi, streak, last, rc, rr = state
        return (bool(active), (streak >= 3) if d0 != d3 else None, None if active else rr % 2)

    @staticmethod
    def policy_transfer(spec_in: tuple, spec_out: tuple, true_in: tuple) -> tuple:
        """The true policy state after a sample whose extraction ran speculatively from
        spec_in to spec_out (same prescan_policy_key as true_in): the per-sample updates of
        _scrfd_policy replayed on the true state - the frame index advances by one, a found
        face resets the streak / rotation cycle and stamps the last-face index, an empty sample
        grows them, an "rr" probe advances the round-robin counter."""
        fi0, st0, lf0, rc0, rr0 = spec_in
        fi1, st1, lf1, rc1, rr1 = spec_out
        tfi, tst, tlf, trc, trr = true_in
        found = lf1 != lf0   # a 0-degree face stamps the last-face index (always < the frame index)
        return (tfi + (fi1 - fi0),
                0 if found else tst + (st1 - st0),
                tfi + (lf1 - fi0) if found else tlf,
                0 if found else trc + (rc1 - rc0),
                trr + (rr1 - rr0))

    def _dyn_for(self, im: _DevImage, imgsz: Optional[int]) -> int:
        """face_embedder.py:2190-2204."""
        H0, W0 = im.H, im.W
        dyn = int(imgsz) if (imgsz is not None and imgsz > 0) else 640
        if self._no_face_streak >= 3:
            dyn = min(dyn, self.fast_no_face_imgsz)
        if self._fast_prescan:
            dyn = min(dyn, int(getattr(self, "_prescan_probe_imgsz", 384)))
            if bool(getattr(self, "_prescan_no_upscale_det", True)):
                src_cap = max(320, (max(H0, W0) // 32) * 32)
                dyn = min(dyn, src_cap)
        return _round32(max(320, dyn))

    @staticmethod
    def _map_xy_from_rot(xr, yr, deg: int, W0: int, H0: int):
        if deg == 0:
            return xr, yr
        if deg == 90:
            return yr, H0 - 1 - xr
        if deg == 180:
            return W0 - 1 - xr, H0 - 1 - yr
        if deg == 270:
            return W0 - 1 - yr, xr
        return xr, yr

    @staticmethod
    def _accumulate0(bb: np.ndarray, kp: np.ndarray, W0: int, H0: int) -> List[tuple]:
        """The 0-degree _accumulate (face_embedder.py:2214-2239) of _scrfd_policy over all boxes of one SCRFD result
        at once (same truncation, clamping, size gate and crop-local f32 landmarks)."""
        if len(bb) == 0:
            return []
        xy = bb[:, :4].astype(np.int64)              # int(v): truncation toward zero
        xa1 = np.clip(np.minimum(xy[:, 0], xy[:, 2]), 0, W0 - 1)
        ya1 = np.clip(np.minimum(xy[:, 1], xy[:, 3]), 0, H0 - 1)
        xa2 = np.maximum(xa1 + 1, np.minimum(W0, np.maximum(xy[:, 0], xy[:, 2])))
        ya2 = np.maximum(ya1 + 1, np.minimum(H0, np.maximum(xy[:, 1], xy[:, 3])))
        keep = np.nonzero((xa2 - xa1 > 2) & (ya2 - ya1 > 2))[0]
        if keep.size == 0:
            return []
        off = np.stack([xa1, ya1], axis=1).astype(np.float64)[:, None, :]
        pts = (kp.astype(np.float64) - off).astype(np.float32)
        sc = bb[:, 4].astype(np.float64)
        return [(_IBox((int(xa1[i]), int(ya1[i]), int(xa2[i]), int(ya2[i])), bb[i, :4]), pts[i], float(sc[i]))
                for i in keep]

    def _scrfd_policy(self, im: _DevImage, dyn: int, first) -> List[tuple]:
        """face_embedder.py:2205-2443: from the 0-degree result through fallbacks to the
        cross-rotation NMS. Returns [((x1,y1,x2,y2), kps_local or None, score)]."""
        H0, W0 = im.H, im.W
        L = max(H0, W0)
        heavy_cap = max(int(getattr(self, "_heavy_cap", 2048)), dyn)
        heavy90 = min(_round32(max(dyn, int(0.75 * L))), heavy_cap)
        heavy180 = min(_round32(max(dyn, int(0.67 * L))), heavy_cap)
        dets: List[tuple] = []

        def accumulate(bb, kp, deg):
            x1, y1, x2, y2 = [int(v) for v in bb[:4]]
            x1o, y1o = self._map_xy_from_rot(x1, y1, deg, W0, H0)
            x2o, y2o = self._map_xy_from_rot(x2, y2, deg, W0, H0)
            xa1, ya1 = min(x1o, x2o), min(y1o, y2o)
            xa2, ya2 = max(x1o, x2o), max(y1o, y2o)
            xa1 = max(0, min(W0 - 1, xa1)); ya1 = max(0, min(H0 - 1, ya1))
            xa2 = max(xa1 + 1, min(W0, xa2)); ya2 = max(ya1 + 1, min(H0, ya2))
            if xa2 - xa1 <= 2 or ya2 - ya1 <= 2:
                return
            pts = None
            if kp is not None:
                flat = np.asarray(kp, dtype=np.float32).reshape(-1, 2)
                mapped = []
                for (px, py) in flat:
                    ox, oy = self._map_xy_from_rot(float(px), float(py), deg, W0, H0)
                    mapped.append([float(ox - xa1), float(oy - ya1)])
                pts = np.asarray(mapped[:5], dtype=np.float32) if len(mapped) >= 5 else None
            score = float(bb[4]) if len(bb) > 4 else 1.0
            fb = None
            if deg == 0:   # (the float box of an unrotated pass, for parity reports)
                fb = np.asarray(bb[:4], np.float64)
            dets.append((_IBox((xa1, ya1, xa2, ya2), fb), pts, score))

        bboxes, kpss = first
        if kpss is not None and len(kpss) == len(bboxes) and np.ndim(kpss) == 3 and np.shape(kpss)[1:] == (5, 2) \
                and np.ndim(bboxes) == 2 and np.shape(bboxes)[1] >= 5:
            dets.extend(self._accumulate0(np.asarray(bboxes), np.asarray(kpss, np.float32), W0, H0))
        else:
            for i, bb in enumerate(bboxes):
                accumulate(bb, None if kpss is None or i >= len(kpss) else kpss[i], 0)

        tta_scales = ()
        if not dets and not self._fast_prescan:
            tta_scales = tuple(self.scrfd_tta_scales) + ((1.25,) if max(W0, H0) <= 1920 else ())
            probe_conf = min(float(getattr(self, "conf", 0.5)), float(self.scrfd_probe_conf_cap))
            for s in tta_scales:
                if s == 1.0:
                    continue
                try:
                    dyn_s = _round32(min(self._heavy_cap, max(320, int(dyn * s))))
                    bb_s, kp_s = self._fb_detect(im, ("tta", s), dyn_s, probe_conf,
                                                 lambda: self._dev_resize(im, "tta", fx=s, fy=s, area=s < 1.0))
                except Exception:
                    bb_s, kp_s = None, None
                if bb_s is None or len(bb_s) == 0:
                    continue
                inv = 1.0 / s
                for i, bb in enumerate(bb_s):
                    kp = None if kp_s is None or i >= len(kp_s) else kp_s[i]
                    bb = np.asarray(bb).copy()
                    bb[:4] = np.asarray(bb[:4], dtype=np.float32) * inv
                    if kp is not None:
                        kp = np.asarray(kp, dtype=np.float32) * inv
                    accumulate(bb, kp, 0)
                if dets:
                    break
            if not dets:
                pad = int(round(min(64, float(self.scrfd_edge_pad_frac) * max(W0, H0))))
                if pad > 0:
                    try:
                        bb_p, kp_p = self._fb_detect(im, ("pad", pad), dyn, probe_conf,
                                                     lambda: self._dev_rotate_pad(im, 0, pad, key="edgepad"))
                    except Exception:
                        bb_p, kp_p = None, None
                    if bb_p is not None and len(bb_p) > 0:
                        for i, bb in enumerate(bb_p):
                            kp = None if kp_p is None or i >= len(kp_p) else kp_p[i]
                            bb = np.asarray(bb).copy()
                            bb[:4] -= np.array([pad, pad, pad, pad], dtype=np.float32)
                            bb[0] = max(0.0, min(float(W0 - 1), float(bb[0])))
                            bb[1] = max(0.0, min(float(H0 - 1), float(bb[1])))
                            bb[2] = max(bb[0] + 1.0, min(float(W0), float(bb[2])))
                            bb[3] = max(bb[1] + 1.0, min(float(H0), float(bb[3])))
                            if kp is not None:
                                kp = np.asarray(kp, dtype=np.float32).copy()
                                kp[..., 0] = np.clip(kp[..., 0] - pad, 0, W0 - 1)
                                kp[..., 1] = np.clip(kp[..., 1] - pad, 0, H0 - 1)
                            accumulate(bb, kp, 0)
        min_px = int(getattr(self, "scrfd_min_box_px", 8))
        dets = [d for d in dets if d[0][2] - d[0][0] >= min_px and d[0][3] - d[0][1] >= min_px]
        # rotation gating (face_embedder.py:2330-2360)
        if not dets:
            need_rot = False
            self._no_face_streak += 1
            if self.rot_adaptive:
                if (self._frame_idx - self._last_face_idx) <= self.rot_after_hit_frames:
                    need_rot = True
                elif ((self._frame_idx + (id(self) & 7)) % self.rot_every_n) == 0:
                    need_rot = True
            else:
                need_rot = True
        else:
            need_rot = False
            self._no_face_streak = 0
            self._last_face_idx = self._frame_idx
            self._rot_cycle = 0
        if self._fast_prescan:
            if dets:
                need_rot = False
            else:
                period = max(1, int(getattr(self, "_prescan_period", 3)))
                need_rot = need_rot or self._prescan_escalate or (((self._frame_idx + self._prescan_rr) % period) == 0)
        if self._fast_prescan and not dets and not need_rot:
            return []
        if not dets and need_rot:
            self._rot_cycle += 1
            if self._fast_prescan:
                rr = self._prescan_rr % 2
                if self._prescan_rr_mode == "rr":
                    rot_seq = ((90, 270)[rr],)
                    self._prescan_rr += 1
                else:
                    rot_seq = (90, 270)
            else:
                rot_seq = (90, 270, 180)
            for deg in rot_seq:
                probe_conf = max(0.02, float(getattr(self, "_probe_conf", 0.02)))
                probe_dyn = _round32(max(320, min(dyn, int(getattr(self, "_prescan_probe_imgsz", 384)))))
                probe_boxes, _ = self._fb_detect(im, ("rot", deg, 0), probe_dyn, probe_conf,
                                                 lambda: self._dev_rotate_pad(im, deg, 0, key="rot_probe"))
                probe_hits = len(probe_boxes) if probe_boxes is not None else 0
                do_heavy = (probe_hits > 0) or (self._fast_prescan and self._prescan_escalate) or \
                    (not self._fast_prescan)
                if self._fast_prescan and probe_hits == 0:
                    continue
                pad = 24
                rimg_make = lambda: self._dev_rotate_pad(im, deg, pad, key="rot_heavy")
                if self._fast_prescan:
                    heavy = heavy180 if deg == 180 else heavy90
                    override = getattr(self, "_high_180" if deg == 180 else "_high_90", None)
                    if override and override > 0:
                        heavy = max(heavy, _round32(int(override)))
                    heavy = min(heavy, int(getattr(self, "_heavy_cap", 2048)))
                    det_sizes = [dyn] if not do_heavy else [heavy]
                else:
                    full_sizes: List[int] = []
                    for base in (max(dyn, 1280), max(dyn, 1536)):
                        base = _round32(base)
                        if base not in full_sizes:
                            full_sizes.append(base)
                    det_sizes = full_sizes if do_heavy else [dyn]
                conf_deg = max(0.10, float(self.conf) * (0.8 if deg in (90, 270) else 0.6))
                rb = rk = None
                for det_size in det_sizes:
                    rb, rk = self._fb_detect(im, ("rot", deg, pad), det_size, conf_deg, rimg_make)
                    if rb is not None and len(rb) > 0:
                        break
                    rb = rk = None
                if rb is None or len(rb) == 0:
                    continue
                for i, bb in enumerate(rb):
                    kp = None if rk is None or i >= len(rk) else rk[i]
                    bb = np.asarray(bb).copy()
                    bb[:4] -= np.array([pad, pad, pad, pad], dtype=bb.dtype)
                    if kp is not None:
                        kp = np.asarray(kp).copy()
                        kp[..., 0] -= pad
                        kp[..., 1] -= pad
                    accumulate(bb, kp, deg)
                if dets:
                    break
        if not dets:
            return []
        dets = sorted(dets, key=lambda t: (t[2], (t[0][2] - t[0][0]) * (t[0][3] - t[0][1])), reverse=True)
        kept = []
        for box, pts, sc in dets:
            if all(self._iou(box, k[0]) < 0.45 for k in kept):
                kept.append((box, pts, sc))
        return kept

    # ------------------------------------------------------------------ align + embed
    @staticmethod
    def _face_jobs(im: _DevImage, fi: int, kept: list) -> List[tuple]:
        """Integer crop boxes of the kept detections (face_embedder.py:2445-2452), with the float
        box they are rounded from (parity reports: a box that differs by one pixel between two
        precisions has its float coordinate next to a .5)."""
        H0, W0 = im.H, im.W
        out = []
        for box, kps, _sc in kept:
            x1, y1, x2, y2 = box
            xi1 = max(0, min(W0 - 1, int(round(x1))))
            yi1 = max(0, min(H0 - 1, int(round(y1))))
            xi2 = max(xi1 + 1, min(W0, int(round(x2))))
            yi2 = max(yi1 + 1, min(H0, int(round(y2))))
            out.append((fi, (xi1, yi1, xi2, yi2), kps, getattr(box, "f", None)))
        return out

    def _do_flip(self) -> bool:
        return (not getattr(self, "_fast_prescan", False)) or getattr(self, "_prescan_escalate", False)

    def _embed_per(self) -> int:
        return self._arc.max_batch // 2 if self._do_flip() else self._arc.max_batch

    def _embed_launch(self, imgs: Sequence[Optional[_DevImage]], jobs: List[tuple], slot: int) -> tuple:
        """Enqueue crop + align/resize + quality + ArcFace (+ bank match) of at most one
        ArcFace batch of faces, and the readback into pinned memory."""
        m = len(jobs)
        ctx = self._ectx
        chips = ctx.scratch("chips", m * _ARC_SIDE * _ARC_SIDE * 3)
        chip_sz = _ARC_SIDE * _ARC_SIDE * 3
        has_k = [j for j in range(m) if jobs[j][2] is not None]
        valid = np.zeros((m,), bool)
        descs = []
        warps: List[WarpDesc] = []
        resize_jobs = []
        if has_k:
            cs, okc = imageops.canon_5pts_batch(np.stack([np.asarray(jobs[j][2], np.float32).reshape(5, 2)
                                                          if np.asarray(jobs[j][2]).shape == (5, 2)
                                                          else np.full((5, 2), np.nan, np.float32) for j in has_k]))
            aligned_idx = [j for j, o in zip(has_k, okc) if o]
            valid[aligned_idx] = True
            if aligned_idx:
                M, ok = imageops.align_matrices(cs[okc])
                sel = np.asarray(aligned_idx)[ok]
                if sel.size:
                    geo = np.array([(imgs[jobs[j][0]].ptr + jobs[j][1][1] * imgs[jobs[j][0]].stride + jobs[j][1][0] * 3,
                                     imgs[jobs[j][0]].stride, jobs[j][1][2] - jobs[j][1][0],
                                     jobs[j][1][3] - jobs[j][1][1]) for j in sel], dtype=np.int64).reshape(-1, 4)
                    descs.append(imageops.warp_descs(geo[:, 0], geo[:, 1], geo[:, 2], geo[:, 3], M[ok],
                                                     chips.ptr + sel.astype(np.int64) * chip_sz))
                resize_jobs.extend(int(j) for j in np.asarray(aligned_idx)[~ok])
        for j in range(m):
            if not valid[j]:
                fi, box, kps = jobs[j][:3]
                if kps is not None:
                    self._upright_by_eye_roll(imgs[fi], box, kps, chips.ptr + j * chip_sz, warps, resize_jobs, j)
                else:
                    resize_jobs.append(j)
        if warps:
            descs.append(np.frombuffer(b"".join(bytes(w) for w in warps), imageops.WARP_DESC_DTYPE))
        if descs:
            # (np.concatenate would canonicalise the padded record dtype: fill one array)
            arr = np.zeros(sum(len(d) for d in descs), imageops.WARP_DESC_DTYPE)
            o = 0
            for d in descs:
                arr[o:o + len(d)] = d
                o += len(d)
            assert arr.dtype.itemsize == 96
            check(ctx.lib.pc_warp_affine(ctx.handle, arr.ctypes.data_as(C.POINTER(WarpDesc)), len(arr)),
                  ctx.handle, "warp_affine")
        for j in resize_jobs:
            fi, (xi1, yi1, xi2, yi2), _ = jobs[j][:3]
            im = imgs[fi]
            crop = _DevImage(im.ptr + yi1 * im.stride + xi1 * 3, yi2 - yi1, xi2 - xi1, im.stride)
            self._resize_chip(crop, chips.ptr + j * chip_sz)
        qbuf = ctx.scratch("quality", m * 8)
        check(ctx.lib.pc_face_quality(ctx.handle, chips.ptr, m, _ARC_SIDE, qbuf.ptr), ctx.handle,
              "face_quality")
        do_flip = self._do_flip()
        fbuf = ctx.scratch("feats", m * self._arc_feat_dim * 4)
        if (2 * m if do_flip else m) > self._arc.max_batch:
            raise ValueError("embed launch larger than one ArcFace batch")
        self._arc.embed_device(chips.ptr, m, do_flip, fbuf.ptr)
        bank = getattr(self, "_bank", None)
        dbg = bool(getattr(self, "debug_chips", False))
        fd_bytes = m * 4 if bank is not None else 0
        sizes = [m * 8, m * self._arc_feat_dim * 4, fd_bytes, m * chip_sz if dbg else 0]
        pin = ctx.pinned(f"emb{slot}", sum(sizes))
        q = ctx.download_async(qbuf.ptr, pin, 0, (m,), np.float64)
        feats = ctx.download_async(fbuf.ptr, pin, sizes[0], (m, self._arc_feat_dim), np.float32)
        fd = None
        if bank is not None:
            dfd = ctx.scratch("fd", m * 4)
            didx = ctx.scratch("fd_idx", m * 4)
            bank.match_device(fbuf.ptr, m, dfd.ptr, didx.ptr, ctx=ctx)
            fd = ctx.download_async(dfd.ptr, pin, sizes[0] + sizes[1], (m,), np.float32)
        chip_h = None
        if dbg:
            chip_h = ctx.download_async(chips.ptr, pin, sizes[0] + sizes[1] + sizes[2],
                                              (m, _ARC_SIDE, _ARC_SIDE, 3), np.uint8)
        return ctx.fence(f"emb{slot}"), jobs, q, feats, fd, chip_h

    def _embed_collect(self, pend: tuple, out: List[list]) -> None:
        fence, jobs, q, feats, fd, chip_h = pend
        fence.wait()
        for j, (fi, (x1, y1, x2, y2), kps, fbox) in enumerate(jobs):
            face = {'bbox': np.array([x1, y1, x2, y2], dtype=np.int32), 'feat': feats[j].copy(),
                    'quality': float(q[j])}
            if fd is not None:
                face['fd'] = float(fd[j])
            if chip_h is not None:   # parity tests: the aligned chip and its landmarks
                face['chip'] = chip_h[j].copy()
                face['kps5'] = None if kps is None else np.asarray(kps, np.float32).copy()
                if fbox is not None:
                    face['bbox_f'] = fbox
            out[fi].append(face)

    def _resize_chip(self, crop: _DevImage, d_dst: int) -> None:
        """cv2.resize(face, (112,112), INTER_AREA if max(h,w) > 112 else INTER_LINEAR) (:2458-2460)."""
        p = imageops.resize_plan(crop.H, crop.W, (_ARC_SIDE, _ARC_SIDE), area=max(crop.H, crop.W) > _ARC_SIDE)
        cv_resize_into(self._ectx, crop, p, d_dst)   # embed stream (chips)

    def _upright_by_eye_roll(self, im: _DevImage, box, pts5, d_dst: int, warps: list, resize_jobs: list,
                             j: int) -> None:
        """face_embedder.py:1571-1647 on device: rotate the crop by the eye-line angle
        (>= 8 deg), re-canonicalise the rotated landmarks, then align or resize."""
        xi1, yi1, xi2, yi2 = box
        h, w = yi2 - yi1, xi2 - xi1
        src = im.ptr + yi1 * im.stride + xi1 * 3
        pts = np.asarray(pts5, dtype=np.float32)
        coords = pts[:5, :2].copy()
        if not np.isfinite(coords).all():
            resize_jobs.append(j)
            return
        coords[:, 0] = np.clip(coords[:, 0], 0.0, max(0, w - 1))
        coords[:, 1] = np.clip(coords[:, 1], 0.0, max(0, h - 1))
        vec = coords[1] - coords[0]
        if float(np.hypot(vec[0], vec[1])) < 1e-3:
            vec = coords[4] - coords[3]
            if float(np.hypot(vec[0], vec[1])) < 1e-3:
                resize_jobs.append(j)
                return
        angle = math.degrees(math.atan2(float(vec[1]), float(vec[0])))
        if angle < -90.0:
            angle += 180.0
        elif angle > 90.0:
            angle -= 180.0
        if abs(angle) < 8.0:
            resize_jobs.append(j)
            return
        angle = 90.0 if angle > 80.0 else (-90.0 if angle < -80.0 else angle)
        scale = 1.0 if max(h, w) <= 256 else 256.0 / float(max(h, w))
        # cv2.getRotationMatrix2D(center, -angle, scale)
        a = math.radians(-angle)
        alpha, beta = math.cos(a) * scale, math.sin(a) * scale
        cx, cy = w / 2.0, h / 2.0
        M = np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                      [-beta, alpha, beta * cx + (1 - alpha) * cy]], dtype=np.float64)
        ectx = self._ectx
        rot = ectx.scratch(f"roll{j}", w * h * 3)
        d = imageops.warp_desc(src, im.stride, w, h, M.reshape(-1), rot.ptr, out_w=w, out_h=h)
        check(ectx.lib.pc_warp_affine(ectx.handle, (WarpDesc * 1)(d), 1), ectx.handle, "warp_affine")
        pts_h = np.hstack([pts[:5, :2], np.ones((5, 1), dtype=np.float32)])
        pts_rot = (M @ pts_h.T).T.astype(np.float32)
        canon = imageops.canon_5pts(pts_rot)
        rimg = _DevImage(rot.ptr, h, w, w * 3, rot)
        if canon is not None:
            Ms, ok = imageops.align_matrices(canon[None].astype(np.float32))
            if ok[0]:
                warps.append(imageops.warp_desc(rot.ptr, w * 3, w, h, Ms[0].reshape(-1), d_dst))
                return
        self._resize_chip(rimg, d_dst)

    # ------------------------------------------------------------------ reference-compatible encode
    def _arcface_encode(self, bgr_list: List[np.ndarray]):
        """face_embedder.py:1290-1389 for host 112x112 chips (other sizes are resized
        on device first, as _arcface_preprocess does)."""
        if not bgr_list:
            return []
        m = len(bgr_list)
        chip_sz = _ARC_SIDE * _ARC_SIDE * 3
        ctx = self._ectx
        chips = ctx.scratch("enc_chips", m * chip_sz)
        for i, b in enumerate(bgr_list):
            b = np.ascontiguousarray(b, dtype=np.uint8)
            if b.shape[:2] == (_ARC_SIDE, _ARC_SIDE):
                ctx.upload(b, chips, offset=i * chip_sz)
            else:
                buf = ctx.scratch(f"enc_src{i}", b.nbytes)
                ctx.upload(b, buf)
                im = _DevImage(buf.ptr, b.shape[0], b.shape[1], b.strides[0], buf)
                self._resize_chip(im, chips.ptr + i * chip_sz)
        do_flip = (not getattr(self, "_fast_prescan", False)) or getattr(self, "_prescan_escalate", False)
        fbuf = ctx.scratch("enc_feats", m * self._arc_feat_dim * 4)
        per = self._arc.max_batch // 2 if do_flip else self._arc.max_batch
        for s in range(0, m, per):
            k = min(per, m - s)
            self._arc.embed_device(chips.ptr + s * chip_sz, k, do_flip, fbuf.ptr + s * self._arc_feat_dim * 4)
        return ctx.download(fbuf.ptr, (m, self._arc_feat_dim), np.float32)

    def _face_quality(self, bgr):
        b = np.ascontiguousarray(bgr, dtype=np.uint8)
        if b.shape[0] > 128 or b.shape[1] > 128 or b.shape[0] != b.shape[1]:
            raise ValueError("device face quality supports square chips up to 128 px")
        ctx = self._ectx
        d = ctx.scratch("q_chip", b.nbytes)
        ctx.upload(b, d)
        q = ctx.scratch("q_out", 8)
        check(ctx.lib.pc_face_quality(ctx.handle, d.ptr, 1, b.shape[0], q.ptr), ctx.handle)
        return float(ctx.download(q.ptr, (1,), np.float64)[0])
