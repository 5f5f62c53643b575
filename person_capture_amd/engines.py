"""Device engines behind the facades: ArcFace embedder, SCRFD detector and the
bank matcher, each a thin orchestration of C-ABI calls on one GpuContext."""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import models
from ._lib import PC_PREC_F16, PC_PREC_F16C8, PC_PREC_F16X3, PC_PREC_F32, LetterboxDesc, check, net_precision
from .runtime import DeviceBuffer, GpuContext, Net


class ArcFaceEngine:
    """IResNet embedder: u8 BGR chips (device) -> unit f32 embeddings, flip-TTA fused
    (FaceEmbedder._arcface_encode, face_embedder.py:1290-1389)."""

    def __init__(self, ctx: GpuContext, params: models.Params, depth: int = 100, precision: int = PC_PREC_F16,
                 max_batch: int = 256, graph: bool = False):
        self.ctx = ctx
        self.depth = depth
        self.precision = precision
        # PC_PREC_F16X3 / PC_PREC_F16C8: the split / f16c8 program on an f16 net (f32-class embeddings,
        # DESIGN.md §3.6-3.7)
        self.program = models.compile_iresnet(params, depth, split=precision == PC_PREC_F16X3,
                                              c8=precision == PC_PREC_F16C8)
        self.net = Net(ctx, self.program.serialize(), precision=net_precision(precision), max_batch=max_batch)
        self.dim = params["fc.weight"].shape[0]
        self.max_batch = max_batch
        self.absmax = None
        if precision == PC_PREC_F16C8:
            self.calibrate(calibration_chips())
        if graph:
            self.net.set_graph(True)

    def calibrate(self, chips_bgr: np.ndarray, headroom_log2: int = 5) -> None:
        """The f16c8 tensors' e4m3 scales from these chips (flip-TTA rows, as embedded): every
        activation may then grow 2^headroom_log2 past the calibration's largest before its e4m3
        bytes saturate (and degrade to f16 precision there, no further)."""
        chips = np.ascontiguousarray(chips_bgr, dtype=np.uint8)
        n = min(chips.shape[0], self.max_batch // 2)
        d = self.ctx.scratch("arc_calib_chips", chips[:n].nbytes)
        self.ctx.upload(chips[:n], d)
        x = self.ctx.scratch("arc_calib_input", 2 * n * 112 * 112 * 4 * 2)
        check(self.ctx.lib.pc_arcface_prep(self.ctx.handle, PC_PREC_F16X3, C.c_void_p(d.ptr), n, 112, 1,
                                           C.c_void_p(x.ptr)), self.ctx.handle, "arcface_prep")
        self.absmax = self.net.calibrate(x.ptr, 2 * n, headroom_log2, n_tensors=len(self.program.tensors))

    @property
    def flops_per_forward(self) -> float:
        return self.net.flops_per_image

    def embed_device(self, d_chips: int, n: int, flip: bool, d_out: int) -> None:
        """Enqueue: chips [n][112][112][3] u8 at d_chips -> d_out [n][dim] f32."""
        rows = 2 * n if flip else n
        if rows > self.max_batch:
            raise ValueError(f"ArcFace batch {rows} exceeds max_batch {self.max_batch}")
        check(self.ctx.lib.pc_arcface_embed(self.net.handle, C.c_void_p(int(d_chips)), int(n), 1 if flip else 0,
                                            C.c_void_p(int(d_out))), self.ctx.handle, "arcface_embed")

    def embed(self, chips_bgr: np.ndarray, flip: bool = True) -> np.ndarray:
        """Host convenience: chips [n][112][112][3] u8 -> [n][dim] unit f32 (chunks by max_batch)."""
        chips = np.ascontiguousarray(chips_bgr, dtype=np.uint8)
        n = chips.shape[0]
        if n == 0:
            return np.zeros((0, self.dim), np.float32)
        per = self.max_batch // 2 if flip else self.max_batch
        outs = []
        for s in range(0, n, per):
            part = chips[s:s + per]
            m = part.shape[0]
            d_in = self.ctx.scratch("arc_chips", part.nbytes)
            self.ctx.upload(part, d_in)
            d_out = self.ctx.scratch("arc_feat", m * self.dim * 4)
            self.embed_device(d_in.ptr, m, flip, d_out.ptr)
            outs.append(self.ctx.download(d_out.ptr, (m, self.dim), np.float32))
        return np.concatenate(outs, axis=0)


def calibration_chips(n: int = 16, seed: int = 20260518) -> np.ndarray:
    """Synthetic 112x112 chips for the f16c8 scale calibration: u8 noise (the bench's content) and
    smooth random fields at full contrast (camera-like images)."""
    rng = np.random.default_rng(seed)
    noise = rng.integers(0, 256, (n // 2, 112, 112, 3), dtype=np.uint8)
    f = rng.standard_normal((n - n // 2, 112 + 32, 112 + 32, 3))
    for ax in (1, 2):   # 17-tap box blur twice along each axis
        for _ in range(2):
            c = np.cumsum(f, axis=ax)
            f = (np.take(c, range(16, c.shape[ax]), axis=ax) - np.take(c, range(0, c.shape[ax] - 16), axis=ax)) / 16.0
    f = f[:, :112, :112]
    f = (f - f.mean(axis=(1, 2, 3), keepdims=True)) / (f.std(axis=(1, 2, 3), keepdims=True) + 1e-9)
    smooth = np.clip(np.rint(127.5 + 60.0 * f), 0, 255).astype(np.uint8)
    return np.concatenate([noise, smooth], axis=0)


class BankMatcher:
    """Batched Processor._fd_min (gui_app.py:660-674) on device."""

    def __init__(self, ctx: GpuContext):
        self.ctx = ctx

    def match_device(self, d_q: int, n: int, d_bank: int, b: int, dim: int, d_fd: int, d_idx: int) -> None:
        check(self.ctx.lib.pc_bank_match(self.ctx.handle, C.c_void_p(int(d_q)), int(n), C.c_void_p(int(d_bank)),
                                         int(b), int(dim), C.c_void_p(int(d_fd)), C.c_void_p(int(d_idx))),
              self.ctx.handle, "bank_match")

    def match(self, q: np.ndarray, bank: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        q = np.ascontiguousarray(q, dtype=np.float32)
        bank = np.ascontiguousarray(bank, dtype=np.float32).reshape(-1, q.shape[1]) if bank is not None and \
            np.asarray(bank).size else np.zeros((0, q.shape[1]), np.float32)
        n, dim = q.shape
        if n == 0:
            return np.zeros((0,), np.float32), np.zeros((0,), np.int32)
        dq = self.ctx.scratch("bm_q", q.nbytes)
        self.ctx.upload(q, dq)
        db = self.ctx.scratch("bm_bank", max(bank.nbytes, 4))
        if bank.size:
            self.ctx.upload(bank, db)
        dfd = self.ctx.scratch("bm_fd", n * 4)
        didx = self.ctx.scratch("bm_idx", n * 4)
        self.match_device(dq.ptr, n, db.ptr, bank.shape[0], dim, dfd.ptr, didx.ptr)
        fd = self.ctx.download(dfd.ptr, (n,), np.float32)
        idx = self.ctx.download(didx.ptr, (n,), np.int32)
        return fd, idx


def letterbox_geometry(H: int, W: int, D: int) -> Tuple[int, int, float]:
    """[ext] insightface SCRFD.detect sizing: keep aspect, fit into DxD."""
    im_ratio = float(H) / W
    model_ratio = 1.0
    if im_ratio > model_ratio:
        new_h = D
        new_w = int(new_h / im_ratio)
    else:
        new_w = D
        new_h = int(new_w * im_ratio)
    det_scale = float(new_h) / H
    return new_w, new_h, det_scale


def opencv_vresize_simd_end(width_bytes: int) -> int:
    """Byte index where OpenCV's 128-bit VResizeLinearVec_32s8u stops for a u8 row of
    width_bytes (16-byte loop, then 8-byte loop while x < width - 8); the remainder
    uses the scalar FixedPtCast path with different rounding."""
    x = (width_bytes // 16) * 16 if width_bytes >= 16 else 0
    while x < width_bytes - 8:
        x += 8
    return x


def make_letterbox_desc(d_src: int, H: int, W: int, row_stride: int, D: int) -> Tuple[LetterboxDesc, float]:
    new_w, new_h, det_scale = letterbox_geometry(H, W, D)
    d = LetterboxDesc()
    d.d_src = int(d_src)
    d.H, d.W, d.row_stride = H, W, row_stride
    d.new_w, d.new_h = new_w, new_h
    d.scale_x = 1.0 / (float(new_w) / W)
    d.scale_y = 1.0 / (float(new_h) / H)
    d.simd_end = opencv_vresize_simd_end(new_w * 3)
    return d, det_scale


class ScrfdEngine:
    """SCRFD detector at one square input size D (letterbox + net + decode + NMS on device)."""

    def __init__(self, ctx: GpuContext, params: models.Params, variant: str = "10g", D: int = 640,
                 precision: int = PC_PREC_F16, max_batch: int = 64, max_det: int = 256):
        self.ctx = ctx
        self.D = D
        self.variant = variant
        self.precision = precision
        # PC_PREC_F16X3: the split program on an f16 net (f32-class boxes and landmarks)
        self.program = models.compile_scrfd(params, variant, D, split=precision == PC_PREC_F16X3)
        self.net = Net(ctx, self.program.serialize(), precision=net_precision(precision), max_batch=max_batch)
        self.max_batch = max_batch
        self.max_det = max_det

    @property
    def flops_per_image(self) -> float:
        return self.net.flops_per_image

    def detect_device(self, descs: Sequence[LetterboxDesc], det_scales: Sequence[float], thresh: float,
                      nms_thresh: float = 0.4) -> Tuple[DeviceBuffer, DeviceBuffer, DeviceBuffer, DeviceBuffer]:
        n = len(descs)
        arr = (LetterboxDesc * n)(*descs)
        sc = (C.c_float * n)(*[float(s) for s in det_scales])
        dd = self.ctx.scratch(f"scrfd_dets{self.D}", n * self.max_det * 5 * 4)
        dk = self.ctx.scratch(f"scrfd_kps{self.D}", n * self.max_det * 10 * 4)
        dc = self.ctx.scratch(f"scrfd_cnt{self.D}", n * 4)
        dn = self.ctx.scratch(f"scrfd_ncand{self.D}", n * 4)
        check(self.ctx.lib.pc_scrfd_detect(self.net.handle, arr, n, self.D, C.c_float(thresh), C.c_float(nms_thresh),
                                           sc, self.max_det, C.c_void_p(dd.ptr), C.c_void_p(dk.ptr),
                                           C.c_void_p(dc.ptr), C.c_void_p(dn.ptr)), self.ctx.handle, "scrfd_detect")
        return dd, dk, dc, dn

    def read_results(self, bufs, n: int) -> List[Tuple[np.ndarray, np.ndarray]]:
        dd, dk, dc, dn = bufs
        cnt = self.ctx.download(dc.ptr, (n,), np.int32)
        dets = self.ctx.download(dd.ptr, (n, self.max_det, 5), np.float32)
        kps = self.ctx.download(dk.ptr, (n, self.max_det, 10), np.float32)
        return self._unpack(cnt, dets, kps)

    def _unpack(self, cnt, dets, kps) -> List[Tuple[np.ndarray, np.ndarray]]:
        if np.any(cnt > self.max_det):
            raise _MaxDetOverflow(int(cnt.max()))
        return [(dets[i, :int(cnt[i])].copy(), kps[i, :int(cnt[i])].reshape(-1, 5, 2).copy()) for i in range(len(cnt))]

    def _grow(self, need: int) -> None:
        self.max_det = max(need, 2 * self.max_det)

    def detect_async(self, d_frames: Sequence[Tuple[int, int, int, int]], thresh: float, slot: str,
                     nms_thresh: float = 0.4) -> list:
        """Enqueue detection of up to max_batch frames and the readback of its results
        into pinned memory; collect() waits for them. slot names the pinned buffers and
        fence (one per in-flight call)."""
        n = len(d_frames)
        if n > self.max_batch:
            raise ValueError(f"detect_async: {n} frames exceed max_batch {self.max_batch}")
        descs, scales = [], []
        for (ptr, H, W, rs) in d_frames:
            d, s = make_letterbox_desc(ptr, H, W, rs, self.D)
            descs.append(d)
            scales.append(s)
        dd, dk, dc, dn = self.detect_device(descs, scales, thresh, nms_thresh)
        md = self.max_det
        sizes = [n * 4, n * 4, n * md * 5 * 4, n * md * 10 * 4]
        pin = self.ctx.pinned(f"scrfd{self.D}_{slot}", sum(sizes))
        off = 0
        views = []
        for (buf, shape, dt), sz in zip(((dc, (n,), np.int32), (dn, (n,), np.int32), (dd, (n, md, 5), np.float32),
                                         (dk, (n, md, 10), np.float32)), sizes):
            views.append(self.ctx.download_async(buf.ptr, pin, off, shape, dt))
            off += sz
        fence = self.ctx.fence(f"scrfd{self.D}_{slot}")
        return [fence, n] + views + [(thresh, nms_thresh), list(d_frames)]

    def collect(self, pending) -> List[Tuple[np.ndarray, np.ndarray]]:
        fence, n, cnt, ncand, dets, kps = pending[:6]
        fence.wait()
        try:
            return self._unpack(cnt, dets, kps)
        except _MaxDetOverflow as e:
            # more faces kept than result rows: the device list is cut, so redo these frames
            # with room for all of them (the reference has no cap)
            self._grow(e.need)
            return self.detect_frames(pending[-1], thresh=pending[-2][0], nms_thresh=pending[-2][1])

    def detect_frames(self, d_frames: Sequence[Tuple[int, int, int, int]], thresh: float,
                      nms_thresh: float = 0.4) -> List[Tuple[np.ndarray, np.ndarray]]:
        """d_frames: (device ptr, H, W, row_stride) per frame (BGR u8)."""
        descs, scales = [], []
        for (ptr, H, W, rs) in d_frames:
            d, s = make_letterbox_desc(ptr, H, W, rs, self.D)
            descs.append(d)
            scales.append(s)
        res = []
        for s0 in range(0, len(descs), self.max_batch):
            while True:
                b = self.detect_device(descs[s0:s0 + self.max_batch], scales[s0:s0 + self.max_batch], thresh,
                                       nms_thresh)
                try:
                    res.extend(self.read_results(b, len(descs[s0:s0 + self.max_batch])))
                    break
                except _MaxDetOverflow as e:
                    self._grow(e.need)
        return res


class _MaxDetOverflow(Exception):
    def __init__(self, need: int):
        super().__init__(f"{need} detections kept")
        self.need = need
