"""CPU oracle of FaceEmbedder's YOLOv8-face branch (test infrastructure only).

Restates person_capture/face_embedder.py:1671-2093 (extract, YOLO branch) and
:1475-1569 (_redetect_align_on_rotations) over an oracle `predict`: [ext] ultralytics
8.3.205 PoseModel predict = LetterBox (ref_algos.yolo_letterbox) -> fp32 torch forward
(nets_torch.yolov8_forward with the Pose head) -> ref_algos.yolo_postprocess (NMS,
scale_boxes, keypoint decode / scale_coords / visibility mask), returning
(res.boxes.xyxy, res.boxes.conf, res.keypoints.xy). ultralytics is not vendored and the
reference ships no fixtures for it: parity unpinned against ultralytics itself.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch

from . import cv_ops
from . import nets_torch as nt
from . import pipeline as op
from . import ref_algos as ra


def check_imgsz(imgsz: int, stride: int = 32) -> int:
    return max(int(math.ceil(int(imgsz) / stride) * stride), stride)


class OracleYoloFaceEmbedder:
    def __init__(self, yolo_params, scale: str, arc_params, depth: int, conf: float = 0.30):
        self.py, self.scale, self.p_a, self.depth = yolo_params, scale, arc_params, depth
        self.conf = float(conf)
        self._fast_prescan = False
        self._prescan_rr = 0
        self._prescan_rr_mode = "rr"
        self._prescan_escalate = False
        self._probe_conf = 0.03
        self._high_90 = 1536
        self._high_180 = 1280
        self._heavy_cap = 2048
        self.trace: List[str] = []

    def predict(self, img: np.ndarray, conf: float, imgsz: int, max_det: int, iou: float = 0.7):
        imgsz = check_imgsz(imgsz)
        canvas, (nw, nh, top, left, Hp, Wp) = ra.yolo_letterbox(img, imgsz)
        self.trace.append(f"predict{Hp}x{Wp}")
        x = torch.from_numpy(np.ascontiguousarray(canvas.transpose(2, 0, 1)[None]))
        heads = [h[0].numpy() for h in nt.yolov8_forward(self.py, self.scale, x, nc=1, kpt=(5, 3))]
        H, W = img.shape[:2]
        dets, kpts = ra.yolo_postprocess(heads, conf, iou, max_det, Hp, Wp, H, W, nk=15)
        return dets[:, :4].copy(), dets[:, 4].copy(), np.ascontiguousarray(kpts[..., :2])

    # ---- helpers ----
    def _embed(self, chips: List[np.ndarray]):
        c = np.stack(chips)
        flip = (not self._fast_prescan) or self._prescan_escalate
        e = nt.iresnet_forward(self.p_a, self.depth, nt.arcface_input_from_chips(c)).numpy()
        ef = nt.iresnet_forward(self.p_a, self.depth, nt.arcface_input_from_chips(c[:, :, ::-1])).numpy() \
            if flip else None
        return ra.arcface_postprocess(e, ef), [cv_ops.face_quality(x) for x in c]

    def _faces(self, boxes, chips):
        feats, q = self._embed(chips)
        return [{"bbox": np.array(b, np.int32), "feat": feats[i], "quality": float(q[i]), "chip": chips[i]}
                for i, b in enumerate(boxes)]

    def _redetect_align_on_rotations(self, face: np.ndarray) -> Optional[np.ndarray]:
        h, w = face.shape[:2]
        if h < 32 or w < 32:
            return None
        for deg in (90, 270, 180):
            img = op.rotate(face, deg)
            H, W = img.shape[:2]
            dyn = int(min(1280, max(320, max(H, W))))
            xyxy, confs, kps = self.predict(img, 0.03, dyn, 60)
            if len(kps) == 0:
                continue
            self.trace.append("redetect")
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
            canon = ra.canon_5pts(pts5)
            if canon is None:
                continue
            return op.align_by_5pts(img, canon)
        return None

    def _single(self, img_r, xyxy, confs, kps, back, W0, H0):
        idx = int(np.argmax(confs)) if len(confs) else 0
        x1r, y1r, x2r, y2r = [int(v) for v in xyxy[idx].tolist()]
        Hr, Wr = img_r.shape[:2]
        x1r = max(0, min(Wr - 1, x1r)); y1r = max(0, min(Hr - 1, y1r))
        x2r = max(x1r + 1, min(Wr, x2r)); y2r = max(y1r + 1, min(Hr, y2r))
        chip = None
        if kps is not None and len(kps) > idx:
            pts5 = kps[idx][:5, :2].astype(np.float32)
            pts5[:, 0] = np.clip(pts5[:, 0], 0, Wr - 1)
            pts5[:, 1] = np.clip(pts5[:, 1], 0, Hr - 1)
            canon = ra.canon_5pts(pts5)
            if canon is not None:
                chip = op.align_by_5pts(img_r, canon)
        if chip is None:
            chip = op.resize_for_arc(img_r[y1r:y2r, x1r:x2r])
        x1o, y1o, x2o, y2o = back(x1r, y1r, x2r, y2r)
        x1o = max(0, min(W0 - 1, x1o)); y1o = max(0, min(H0 - 1, y1o))
        x2o = max(x1o + 1, min(W0, x2o)); y2o = max(y1o + 1, min(H0, y2o))
        if (x2o - x1o) * (y2o - y1o) < 32 * 32:
            return None
        return self._faces([(x1o, y1o, x2o, y2o)], [chip])

    # ---- face_embedder.py:1671-2093 ----
    def extract(self, bgr: np.ndarray, *, imgsz: Optional[int] = None):
        if bgr is None or bgr.size == 0:
            return []
        self.trace = []
        H0, W0 = bgr.shape[:2]
        dyn = int(imgsz) if (imgsz is not None and imgsz > 0) else 640
        dyn = op._round32(max(320, dyn))
        L = max(H0, W0)
        heavy_cap = max(int(self._heavy_cap), dyn)
        heavy_auto = min(op._round32(max(dyn, int(0.75 * L))), heavy_cap)
        heavy_auto_180 = min(op._round32(max(dyn, int(0.67 * L))), heavy_cap)
        xyxy, confs, kps0 = self.predict(bgr, self.conf, dyn, 60, iou=0.30)
        boxes = [tuple(int(v) for v in b) for b in xyxy]
        if not boxes and not self._fast_prescan:
            for s in (1.25, 1.5):
                self.trace.append(f"tta{s}")
                img_s = cv_ops.resize(bgr, None, fx=s, fy=s, interpolation=cv_ops.INTER_LINEAR)
                imgsz_s = ((max(320, int(dyn * s)) + 31) // 32) * 32
                bx, cf, _ = self.predict(img_s, min(self.conf, 0.10), imgsz_s, 80, iou=0.30)
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
            return self._rotations(bgr, dyn, heavy_cap, heavy_auto, heavy_auto_180)
        boxes = ra.nms_boxes(boxes, iou_thr=0.45)
        kps = kps0 if len(kps0) else None
        if kps is not None and len(kps) != len(boxes):
            kps = None
        chips, faces = [], []
        for i, (x1, y1, x2, y2) in enumerate(boxes):
            x1, y1 = max(0, x1), max(0, y1)
            x2, y2 = max(x1 + 1, x2), max(y1 + 1, y2)
            face = bgr[y1:y2, x1:x2]
            if kps is not None and i < len(kps) and np.isfinite(kps[i]).all():
                pts = kps[i].astype(np.float32, copy=False)
                five = ra.canon_5pts(pts[:5])
                if five is not None:
                    pts = five.copy()
                    pts[:, 0] -= float(x1)
                    pts[:, 1] -= float(y1)
                    pts[:, 0] = np.clip(pts[:, 0], 0.0, max(0, face.shape[1] - 1))
                    pts[:, 1] = np.clip(pts[:, 1], 0.0, max(0, face.shape[0] - 1))
                    chip = op.align_by_5pts(face, pts)
                else:
                    self.trace.append("eyeroll")
                    pts = pts[:5].copy()
                    pts[:, 0] -= float(x1)
                    pts[:, 1] -= float(y1)
                    chip = op.upright_by_eye_roll(face, pts, self.trace)
            else:
                self.trace.append("nolandmarks")
                chip = self._redetect_align_on_rotations(face)
                if chip is None:
                    chip = op.resize_for_arc(face)
            faces.append((x1, y1, x2, y2))
            chips.append(chip)
        out = self._faces(faces, chips)
        out.sort(key=lambda f: (f["quality"], (f["bbox"][2] - f["bbox"][0]) * (f["bbox"][3] - f["bbox"][1])),
                 reverse=True)
        return out

    def _rotations(self, bgr, dyn, heavy_cap, heavy_auto, heavy_auto_180):
        H0, W0 = bgr.shape[:2]
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
            self.trace.append(f"rot{deg}")
            img_r = op.rotate(bgr, deg)
            probe_hits = len(self.predict(img_r, self._probe_conf, dyn, 40, iou=0.40)[0])
            do_heavy = probe_hits > 0 or (self._fast_prescan and self._prescan_escalate) or not self._fast_prescan
            if self._fast_prescan:
                heavy, override = (heavy_auto_180, self._high_180) if deg == 180 else (heavy_auto, self._high_90)
                if override and override > 0:
                    heavy = max(heavy, op._round32(int(override)))
                heavy = min(heavy, heavy_cap)
                det_sizes = [dyn] if not do_heavy else [heavy]
            else:
                det_sizes = full_sizes if do_heavy else [dyn]
            res = None
            for ds in det_sizes:
                r = self.predict(img_r, min(self.conf, 0.10), ds, 80, iou=0.30)
                if len(r[0]):
                    res = r
                    break
            if res is None:
                continue
            out = self._single(img_r, res[0], res[1], res[2] if len(res[2]) else None, back_rot(deg), W0, H0)
            if out is not None:
                return out
        if self._fast_prescan:
            return []
        for ang in (45, -45, 135, -135):
            self.trace.append(f"affine{ang}")
            h, w = H0, W0
            M = op.rotation_matrix_2d(w / 2.0, h / 2.0, ang, 1.0)
            img_r = cv_ops.warp_affine(bgr, M.reshape(-1), w, h, border=114 << 8)
            res = None
            for ds in full_sizes:
                r = self.predict(img_r, min(self.conf, 0.10), ds, 80, iou=0.30)
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
            out = self._single(img_r, res[0], res[1], res[2] if len(res[2]) else None, back_aff, W0, H0)
            if out is not None:
                return out
        return []
