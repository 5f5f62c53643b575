"""YOLOv8-face backend of FaceEmbedder (the reference default, Y8F_DEFAULT = 'yolov8l-face.pt',
face_embedder.py:33): detection + landmark alignment policy of FaceEmbedder.extract's YOLO
branch (face_embedder.py:1671-2093) and _redetect_align_on_rotations (:1475-1569), on the
MI355X.

ultralytics' `predict` (PoseModel, kpt_shape [5, 3]; `augment=True` is a no-op for pose
models in 8.3.205, DetectionModel._predict_augment reverts to single-scale) runs as one
C-ABI call per canvas (pc_yolo_pose_detect: LetterBox -> YOLOv8 conv program -> DFL decode
-> NMS -> scale_boxes, keypoint decode -> scale_coords -> visibility mask); the host walks
the same fallbacks as the reference: TTA scales 1.25/1.5, full-frame rotations 90/270/180
with probe and heavy sizes, arbitrary-angle affine rotations +-45/+-135 with a 114 border,
landmark-less re-detection on rotated crops; chips are aligned / eye-rolled / resized,
scored and embedded on the device.

Weights: the reference loads yolov8*-face.pt through ultralytics (a pickled model object,
which this build neither has nor unpickles); seeded synthetic weights of the same
architecture stand in (models_yolo.synth_yolov8_face).
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import imageops, models_yolo
from ._lib import PC_PREC_F16, WarpDesc, YoloLetterboxDesc, YoloScale, check, net_precision
from .engines import opencv_vresize_simd_end
from .runtime import GpuContext, Net

NKPT = 5
_ARC_SIDE = 112
_WEIGHTS: Dict[Tuple[str, int], dict] = {}


def yolo_face_weights(scale: str, seed: int = 0) -> dict:
    key = (scale, seed)
    if key not in _WEIGHTS:
        _WEIGHTS[key] = models_yolo.synth_yolov8_face(scale, seed=seed)
    return _WEIGHTS[key]


def check_imgsz(imgsz: int, stride: int = 32) -> int:
    """[ext] ultralytics check_imgsz for an int size: next multiple of the stride."""
    return max(int(math.ceil(int(imgsz) / stride) * stride), stride)


class YoloFaceEngine:
    """YOLOv8-face (Pose head) at one letterbox canvas Hp x Wp, up to max_batch frames per call."""

    def __init__(self, ctx: GpuContext, params: dict, scale: str, Hp: int, Wp: int, precision: int = PC_PREC_F16,
                 max_det: int = 80, max_batch: int = 1):
        self.ctx, self.Hp, self.Wp, self.max_det, self.max_batch = ctx, Hp, Wp, max_det, max(1, int(max_batch))
        self.program = models_yolo.compile_yolov8(params, scale, Hp, Wp, nc=1, kpt=(NKPT, 3))
        self.net = Net(ctx, self.program.serialize(), precision=precision, max_batch=self.max_batch)

    def predict(self, frame: Tuple[int, int, int, int], imgsz: int, conf: float, iou: float, max_det: int):
        """One ultralytics predict on a device frame (ptr, H, W, row_stride): returns (xyxy f32 [k][4],
        conf f32 [k], keypoints xy f32 [k][5][2]) in predict order."""
        return self.predict_many([frame], imgsz, conf, iou, max_det)[0]

    def predict_many(self, frames: Sequence[Tuple[int, int, int, int]], imgsz: int, conf: float, iou: float,
                     max_det: int) -> List[tuple]:
        """predict() of several frames that share this canvas: one letterbox + net + decode/NMS
        launch per max_batch frames, one readback of the counts and one of the detections."""
        out: List[tuple] = []
        for s0 in range(0, len(frames), self.max_batch):
            part = frames[s0:s0 + self.max_batch]
            n = len(part)
            d = (YoloLetterboxDesc * n)()
            sc = (YoloScale * n)()
            kpad = (C.c_float * (2 * n))()
            for i, (ptr, H, W, rs) in enumerate(part):
                new_w, new_h, top, left, Hp, Wp = models_yolo.letterbox_geometry(H, W, imgsz)
                if (Hp, Wp) != (self.Hp, self.Wp) or max_det > self.max_det:
                    raise ValueError("frame does not letterbox to this engine's canvas")
                d[i].d_src, d[i].H, d[i].W, d[i].row_stride = int(ptr), H, W, rs
                d[i].new_w, d[i].new_h, d[i].top, d[i].left = new_w, new_h, top, left
                d[i].scale_x, d[i].scale_y = 1.0 / (float(new_w) / W), 1.0 / (float(new_h) / H)
                d[i].simd_end = opencv_vresize_simd_end(new_w * 3)
                d[i].identity = 1 if (new_w, new_h) == (W, H) else 0
                gain, px, py = models_yolo.scale_geometry(Hp, Wp, H, W)
                sc[i].gain, sc[i].pad_x, sc[i].pad_y, sc[i].W0, sc[i].H0 = gain, float(px), float(py), float(W), float(H)
                kpad[2 * i], kpad[2 * i + 1] = (Wp - W * gain) / 2, (Hp - H * gain) / 2   # scale_coords: pad not rounded
            dd = self.ctx.scratch("yf_dets", n * max_det * 5 * 4)
            dk = self.ctx.scratch("yf_kpts", n * max_det * NKPT * 3 * 4)
            dc = self.ctx.scratch("yf_cnt", n * 4 + 4)
            check(self.ctx.lib.pc_yolo_pose_detect(self.net.handle, d, n, self.Hp, self.Wp, C.c_float(conf),
                                                   C.c_float(iou), sc, kpad, max_det, NKPT, C.c_void_p(dd.ptr),
                                                   C.c_void_p(dk.ptr), C.c_void_p(dc.ptr), None), self.ctx.handle,
                  "yolo_pose_detect")
            cnt = np.minimum(self.ctx.download(dc.ptr, (n,), np.int32), max_det)
            if cnt.max(initial=0) == 0:
                out.extend((np.zeros((0, 4), np.float32), np.zeros((0,), np.float32),
                            np.zeros((0, NKPT, 2), np.float32)) for _ in range(n))
                continue
            dets = self.ctx.download(dd.ptr, (n, max_det, 5), np.float32)
            kp = self.ctx.download(dk.ptr, (n, max_det, NKPT, 3), np.float32)
            for i in range(n):
                k = int(cnt[i])
                out.append((dets[i, :k, :4].copy(), dets[i, :k, 4].copy(), np.ascontiguousarray(kp[i, :k, :, :2])))
        return out


class YoloFaceBranch:
    """Mixin for FaceEmbedder: the YOLOv8-face extract path. Needs the FaceEmbedder device
    helpers (_ctx, _dev_resize, _dev_rotate_pad, _resize_chip, _upright_by_eye_roll, _arc, ...)."""

    def _init_yolo_face(self, model: str, seed: int) -> None:
        self.yolo_scale = models_yolo.yolo_scale_of(model.replace("-face", ""))
        self._yf_params = yolo_face_weights(self.yolo_scale, seed)
        self._yf_engines: Dict[Tuple[int, int], YoloFaceEngine] = {}
        self.weights_source["yolo_face"] = f"synthetic:yolov8{self.yolo_scale}-face:seed{seed}"

    # ---- ultralytics predict on a device image ----
    def _yf_engine(self, Hp: int, Wp: int) -> YoloFaceEngine:
        eng = self._yf_engines.get((Hp, Wp))
        if eng is None:
            # batch capacity for the speculative 0-degree pass of extract_batch; big fallback
            # canvases keep the activation footprint of a det_batch x 640 x 640 engine
            mb = max(1, min(self._det_batch, self._det_batch * 640 * 640 // (Hp * Wp)))
            eng = YoloFaceEngine(self._ctx, self._yf_params, self.yolo_scale, Hp, Wp, net_precision(self.det_precision),
                                 max_batch=mb)
            self._yf_engines[(Hp, Wp)] = eng
        return eng

    def _yf_predict(self, im, conf: float, imgsz: int, max_det: int, iou: float = 0.7):
        return self._yf_predict_many([im], conf, imgsz, max_det, iou)[0]

    def _yf_predict_many(self, ims, conf: float, imgsz: int, max_det: int, iou: float = 0.7) -> List[tuple]:
        """_yf_predict of several device images: grouped by letterbox canvas, batched per group."""
        imgsz = check_imgsz(imgsz)
        out: List[Optional[tuple]] = [None] * len(ims)
        groups: Dict[Tuple[int, int], List[int]] = {}
        for i, im in enumerate(ims):
            g = models_yolo.letterbox_geometry(im.H, im.W, imgsz)
            groups.setdefault((g[4], g[5]), []).append(i)
        for (Hp, Wp), idx in groups.items():
            res = self._yf_engine(Hp, Wp).predict_many([(ims[i].ptr, ims[i].H, ims[i].W, ims[i].stride) for i in idx],
                                                       imgsz, float(conf), float(iou), int(max_det))
            for i, r in zip(idx, res):
                out[i] = r
        return out

    # ---- chips ----
    def _yf_align(self, im, canon: np.ndarray, d_dst: int) -> None:
        """_align_by_5pts(img, canon) with img the whole device image (face_embedder.py:1465-1473)."""
        M, ok = imageops.align_matrices(np.asarray(canon, np.float32)[None])
        if ok[0]:
            d = imageops.warp_desc(im.ptr, im.stride, im.W, im.H, M[0].reshape(-1), d_dst)
            check(self._ctx.lib.pc_warp_affine(self._ctx.handle, (WarpDesc * 1)(d), 1), self._ctx.handle,
                  "warp_affine")
        else:
            self._resize_chip(im, d_dst)

    def _yf_eye_roll(self, im, pts5: np.ndarray, d_dst: int) -> None:
        """_upright_by_eye_roll(face_bgr, pts) on a device image."""
        warps: list = []
        resize_jobs: list = []
        self._upright_by_eye_roll(im, (0, 0, im.W, im.H), pts5, d_dst, warps, resize_jobs, 0)
        if warps:
            check(self._ctx.lib.pc_warp_affine(self._ctx.handle, (WarpDesc * 1)(warps[0]), 1), self._ctx.handle,
                  "warp_affine")
        for _ in resize_jobs:
            self._resize_chip(im, d_dst)

    def _yf_redetect_align_on_rotations(self, face, d_dst: int) -> bool:
        """face_embedder.py:1475-1569: YOLO on the face crop rotated 90 CW / 90 CCW / 180, the
        detection nearest the centre weighted with its confidence, canonical landmarks -> align."""
        h, w = face.H, face.W
        if h < 32 or w < 32:
            return False
        for deg in (90, 270, 180):
            img = self._dev_rotate_pad(face, deg, 0, key="yf_redet")
            H, W = img.H, img.W
            dyn = int(min(1280, max(320, max(H, W))))
            try:
                xyxy, confs, kps = self._yf_predict(img, 0.03, dyn, 60)
            except Exception:
                continue
            if len(kps) == 0:
                continue
            best_i = 0
            cxy = np.stack([(xyxy[:, 0] + xyxy[:, 2]) / np.float32(2), (xyxy[:, 1] + xyxy[:, 3]) / np.float32(2)], 1)
            cx, cy = W / 2.0, H / 2.0
            dist2 = (cxy[:, 0] - cx) ** 2 + (cxy[:, 1] - cy) ** 2
            if dist2.size:
                best_i = int(np.argmin(dist2))
                diag = math.hypot(W, H)
                dist_norm = np.sqrt(dist2[:confs.size])
                dist_norm = dist_norm / diag if diag > 0 else np.zeros_like(dist_norm)
                m = min(confs.size, dist_norm.size)
                if m > 0:
                    scores = 0.7 * confs[:m] - 0.3 * dist_norm[:m]
                    idx = int(np.argmax(scores))
                    best_i = idx if 0 <= idx < len(kps) else max(0, min(len(kps) - 1, idx))
            pts5 = kps[best_i][:5, :2].astype(np.float32)
            pts5[:, 0] = np.clip(pts5[:, 0], 0, W - 1)
            pts5[:, 1] = np.clip(pts5[:, 1], 0, H - 1)
            canon = imageops.canon_5pts(pts5)
            if canon is None:
                continue
            self._yf_align(img, canon, d_dst)
            return True
        return False

    def _yf_embed(self, m: int, chips_ptr: int):
        """quality + ArcFace (flip-TTA unless fast pre-scan) of m chips already on the device."""
        qbuf = self._ctx.scratch("yf_quality", m * 8)
        check(self._ctx.lib.pc_face_quality(self._ctx.handle, chips_ptr, m, _ARC_SIDE, qbuf.ptr), self._ctx.handle,
              "face_quality")
        fbuf = self._ctx.scratch("yf_feats", m * self._arc_feat_dim * 4)
        flip = self._do_flip()
        per = self._arc.max_batch // 2 if flip else self._arc.max_batch
        for s in range(0, m, per):
            k = min(per, m - s)
            self._arc.embed_device(chips_ptr + s * _ARC_SIDE * _ARC_SIDE * 3, k, flip,
                                   fbuf.ptr + s * self._arc_feat_dim * 4)
        fd = None
        bank = getattr(self, "_bank", None)
        if bank is not None:
            dfd = self._ctx.scratch("yf_fd", m * 4)
            didx = self._ctx.scratch("yf_fd_idx", m * 4)
            bank.match_device(fbuf.ptr, m, dfd.ptr, didx.ptr)
            fd = self._ctx.download(dfd.ptr, (m,), np.float32)
        q = self._ctx.download(qbuf.ptr, (m,), np.float64)
        feats = self._ctx.download(fbuf.ptr, (m, self._arc_feat_dim), np.float32)
        chips = self._ctx.download(chips_ptr, (m, _ARC_SIDE, _ARC_SIDE, 3), np.uint8) \
            if getattr(self, "debug_chips", False) else None
        return q, feats, fd, chips

    def _yf_faces(self, boxes: List[tuple], m_chips: int, chips_ptr: int) -> List[dict]:
        q, feats, fd, chips = self._yf_embed(m_chips, chips_ptr)
        out = []
        for i, (x1, y1, x2, y2) in enumerate(boxes):
            f = {"bbox": np.array([x1, y1, x2, y2], dtype=np.int32), "feat": feats[i].copy(), "quality": float(q[i])}
            if fd is not None:
                f["fd"] = float(fd[i])
            if chips is not None:
                f["chip"] = chips[i].copy()
            out.append(f)
        return out

    # ---- the YOLO branch of extract (face_embedder.py:1671-2093) ----
    @staticmethod
    def _yf_dyn(imgsz: Optional[int]) -> int:
        from .face_embedder import _round32
        dyn = int(imgsz) if (imgsz is not None and imgsz > 0) else 640
        return _round32(max(320, dyn))

    def _extract_batch_yolo(self, imgs, imgsz: Optional[int]) -> List[list]:
        """extract() of each frame in order (the branch's own state, _prescan_rr, advances frame by
        frame), with the 0-degree predicts of all frames batched per canvas up front (their inputs
        do not depend on any state) and one ArcFace/quality/bank pass over the chips of every frame
        whose faces came from that 0-degree pass."""
        dyn = self._yf_dyn(imgsz)
        live = [i for i, im in enumerate(imgs) if im is not None]
        first = dict(zip(live, self._yf_predict_many([imgs[i] for i in live], self.conf, dyn, 60, iou=0.30)))
        cap = sum(len(first[i][0]) for i in live)
        sink = {"chips": self._ctx.scratch("yf_chips_batch", max(1, cap) * _ARC_SIDE * _ARC_SIDE * 3), "used": 0,
                "cap": cap, "jobs": []}
        out: List[Optional[list]] = [[] for _ in imgs]
        for i in live:
            sink["frame"] = i
            r = self._extract_with_yolo(imgs[i], imgsz, first=first[i], sink=sink)
            out[i] = r   # None: deferred into the sink
        jobs = sink["jobs"]
        if jobs:
            m = sink["used"]
            faces = self._yf_faces([b for _, boxes in jobs for b in boxes], m, sink["chips"].ptr)
            k = 0
            for fi, boxes in jobs:
                lst = faces[k:k + len(boxes)]
                k += len(boxes)
                lst.sort(key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])),
                         reverse=True)
                out[fi] = lst
        return [o if o is not None else [] for o in out]

    def _extract_with_yolo(self, im, imgsz: Optional[int] = None, first=None, sink=None) -> Optional[List[dict]]:
        from .face_embedder import _DevImage, _round32
        H0, W0 = im.H, im.W
        dyn = self._yf_dyn(imgsz)
        L = max(H0, W0)
        heavy_cap = max(int(getattr(self, "_heavy_cap", 2048)), dyn)
        heavy_auto = min(_round32(max(dyn, int(0.75 * L))), heavy_cap)
        heavy_auto_180 = min(_round32(max(dyn, int(0.67 * L))), heavy_cap)
        chip_sz = _ARC_SIDE * _ARC_SIDE * 3
        xyxy, confs, kps0 = first if first is not None else self._yf_predict(im, self.conf, dyn, 60, iou=0.30)
        from_first = len(xyxy) > 0
        boxes = [tuple(int(v) for v in b) for b in xyxy]
        if not boxes and not self._fast_prescan:
            for s in (1.25, 1.5):
                img_s = self._dev_resize(im, "yf_tta", fx=s, fy=s, area=False)
                imgsz_s = max(320, int(dyn * s))
                imgsz_s = ((imgsz_s + 31) // 32) * 32
                try:
                    bx, cf, _ = self._yf_predict(img_s, min(self.conf, 0.10), imgsz_s, 80, iou=0.30)
                except Exception:
                    continue
                for j in range(len(bx)):
                    if float(cf[j]) < 0.05:
                        continue
                    x1s, y1s, x2s, y2s = (float(v) for v in bx[j])
                    x1 = max(0, min(W0 - 1, int(round(x1s / s))))
                    y1 = max(0, min(H0 - 1, int(round(y1s / s))))
                    x2 = max(x1 + 1, min(W0, int(round(x2s / s))))
                    y2 = max(y1 + 1, min(H0, int(round(y2s / s))))
                    boxes.append((x1, y1, x2, y2))
                if boxes:
                    break
        if not boxes:
            return self._yf_rotation_fallbacks(im, dyn, heavy_cap, heavy_auto, heavy_auto_180)
        boxes = self._nms_boxes(boxes, iou_thr=0.45)
        # keypoints of the 0-degree predict (res), in predict order, as the reference indexes them
        kps = kps0 if len(kps0) else None
        if kps is not None and len(kps) != len(boxes):
            kps = None
        defer = sink is not None and from_first and sink["used"] + len(boxes) <= sink["cap"]
        if defer:   # chips go to the batch buffer; embedding happens once for all frames
            base = sink["chips"].ptr + sink["used"] * chip_sz
        else:
            base = self._ctx.scratch("yf_chips", len(boxes) * chip_sz).ptr
        faces = []
        for i, (x1, y1, x2, y2) in enumerate(boxes):
            x1, y1 = max(0, x1), max(0, y1)
            x2, y2 = max(x1 + 1, x2), max(y1 + 1, y2)
            x2c, y2c = min(x2, W0), min(y2, H0)
            face = _DevImage(im.ptr + y1 * im.stride + x1 * 3, max(0, y2c - y1), max(0, x2c - x1), im.stride)
            d_dst = base + i * chip_sz
            if kps is not None and i < len(kps) and np.isfinite(kps[i]).all():
                pts = kps[i].astype(np.float32, copy=False)
                five = imageops.canon_5pts(pts[:5])
                if five is not None:
                    pts = five.copy()
                    pts[:, 0] -= float(x1)
                    pts[:, 1] -= float(y1)
                    pts[:, 0] = np.clip(pts[:, 0], 0.0, max(0, face.W - 1))
                    pts[:, 1] = np.clip(pts[:, 1], 0.0, max(0, face.H - 1))
                    self._yf_align(face, pts, d_dst)
                else:
                    pts = pts[:5].copy()
                    pts[:, 0] -= float(x1)
                    pts[:, 1] -= float(y1)
                    self._yf_eye_roll(face, pts, d_dst)
            else:
                if not self._yf_redetect_align_on_rotations(face, d_dst):
                    self._resize_chip(face, d_dst)
            faces.append((x1, y1, x2, y2))
        if defer:
            sink["jobs"].append((sink["frame"], faces))
            sink["used"] += len(faces)
            return None
        out = self._yf_faces(faces, len(faces), base)
        out.sort(key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])),
                 reverse=True)
        return out

    def _yf_single(self, img_r, xyxy, confs, kps, box_back, W0: int, H0: int) -> Optional[List[dict]]:
        """Best (max-conf) detection of a rotated/affine view -> one face (face_embedder.py:1878-1929)."""
        from .face_embedder import _DevImage
        idx = int(np.argmax(confs)) if len(confs) else 0
        x1r, y1r, x2r, y2r = [int(v) for v in xyxy[idx].tolist()]
        Hr, Wr = img_r.H, img_r.W
        x1r = max(0, min(Wr - 1, x1r))
        y1r = max(0, min(Hr - 1, y1r))
        x2r = max(x1r + 1, min(Wr, x2r))
        y2r = max(y1r + 1, min(Hr, y2r))
        chips = self._ctx.scratch("yf_chips", _ARC_SIDE * _ARC_SIDE * 3)
        done = False
        if kps is not None and len(kps) > idx:
            pts5 = kps[idx][:5, :2].astype(np.float32)
            pts5[:, 0] = np.clip(pts5[:, 0], 0, Wr - 1)
            pts5[:, 1] = np.clip(pts5[:, 1], 0, Hr - 1)
            canon = imageops.canon_5pts(pts5)
            if canon is not None:
                self._yf_align(img_r, canon, chips.ptr)
                done = True
        if not done:
            crop = _DevImage(img_r.ptr + y1r * img_r.stride + x1r * 3, y2r - y1r, x2r - x1r, img_r.stride)
            self._resize_chip(crop, chips.ptr)
        x1o, y1o, x2o, y2o = box_back(x1r, y1r, x2r, y2r)
        x1o = max(0, min(W0 - 1, x1o))
        y1o = max(0, min(H0 - 1, y1o))
        x2o = max(x1o + 1, min(W0, x2o))
        y2o = max(y1o + 1, min(H0, y2o))
        if (x2o - x1o) * (y2o - y1o) < 32 * 32:
            return None
        return self._yf_faces([(x1o, y1o, x2o, y2o)], 1, chips.ptr)

    def _yf_rotation_fallbacks(self, im, dyn: int, heavy_cap: int, heavy_auto: int, heavy_auto_180: int):
        """face_embedder.py:1761-2038: full-frame rotations, then affine +-45 / +-135."""
        H0, W0 = im.H, im.W
        if self._fast_prescan:
            full_sizes = [dyn]
        else:
            full_sizes = []
            for base in (max(dyn, 1280), max(dyn, 1536)):
                base = ((int(base) + 31) // 32) * 32
                if base not in full_sizes:
                    full_sizes.append(base)

        def back_rot(deg):
            def mp(xr, yr):
                if deg == 90:
                    return yr, H0 - 1 - xr
                if deg == 270:
                    return W0 - 1 - yr, xr
                return W0 - 1 - xr, H0 - 1 - yr

            def box(x1, y1, x2, y2):
                pts = [mp(x, y) for x, y in zip([x1, x2, x2, x1], [y1, y1, y2, y2])]
                xs, ys = [p[0] for p in pts], [p[1] for p in pts]
                return int(min(xs)), int(min(ys)), int(max(xs)), int(max(ys))
            return box

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
            img_r = self._dev_rotate_pad(im, deg, 0, key="yf_rot")
            try:
                probe = self._yf_predict(img_r, self._probe_conf, dyn, 40, iou=0.40)
                probe_hits = len(probe[0])
            except Exception:
                probe_hits = 0
            do_heavy = probe_hits > 0 or (self._fast_prescan and self._prescan_escalate) or not self._fast_prescan
            if self._fast_prescan:
                if deg == 180:
                    heavy, override = heavy_auto_180, self._high_180
                else:
                    heavy, override = heavy_auto, self._high_90
                if override and override > 0:
                    heavy = max(heavy, ((int(override) + 31) // 32) * 32)
                heavy = min(heavy, heavy_cap)
                det_sizes = [dyn] if not do_heavy else [heavy]
            else:
                det_sizes = full_sizes if do_heavy else [dyn]
            res = None
            for ds in det_sizes:
                try:
                    r = self._yf_predict(img_r, min(self.conf, 0.10), ds, 80, iou=0.30)
                except Exception:
                    continue
                if len(r[0]):
                    res = r
                    break
            if res is None:
                continue
            out = self._yf_single(img_r, res[0], res[1], res[2] if len(res[2]) else None, back_rot(deg), W0, H0)
            if out is not None:
                return out
        if self._fast_prescan:
            return []
        for ang in (45, -45, 135, -135):
            h, w = H0, W0
            a = math.radians(ang)
            alpha, beta = math.cos(a), math.sin(a)
            cx, cy = float(np.float32(w / 2.0)), float(np.float32(h / 2.0))
            M = np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                          [-beta, alpha, beta * cx + (1 - alpha) * cy]], dtype=np.float64)
            buf = self._ctx.scratch("yf_affine", w * h * 3)
            d = imageops.warp_desc(im.ptr, im.stride, w, h, M.reshape(-1), buf.ptr, out_w=w, out_h=h,
                                   border=imageops.border_constant(114))
            check(self._ctx.lib.pc_warp_affine(self._ctx.handle, (WarpDesc * 1)(d), 1), self._ctx.handle,
                  "warp_affine")
            from .face_embedder import _DevImage
            img_r = _DevImage(buf.ptr, h, w, w * 3, buf)
            res = None
            for ds in full_sizes:
                try:
                    r = self._yf_predict(img_r, min(self.conf, 0.10), ds, 80, iou=0.30)
                except Exception:
                    continue
                if len(r[0]):
                    res = r
                    break
            if res is None:
                continue

            def back_aff(x1, y1, x2, y2, M=M):
                A = np.vstack([M, [0, 0, 1]]).astype(np.float32)
                Minv = np.linalg.inv(A)[:2, :]
                pts = np.array([[x1, y1, 1], [x2, y1, 1], [x2, y2, 1], [x1, y2, 1]], dtype=np.float32).T
                back = Minv @ pts
                xs, ys = back[0], back[1]
                return int(np.floor(xs.min())), int(np.floor(ys.min())), int(np.ceil(xs.max())), int(np.ceil(ys.max()))
            out = self._yf_single(img_r, res[0], res[1], res[2] if len(res[2]) else None, back_aff, W0, H0)
            if out is not None:
                return out
        return []
