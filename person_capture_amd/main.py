"""person_capture CLI (person_capture/main.py:146-358) on the MI355X build.

Same arguments, model construction (PersonDetector, FaceEmbedder, ReIDEmbedder with
ctx/device = --device), reference embeddings (best face of the reference image, ReID of its
largest person), per-frame loop (person boxes -> ReID of every crop, faces of every crop ->
distance to the reference face, combine_scores, accept if face or ReID passes its
threshold), crop geometry (expand_box_to_ratio with the face anchor and head bias,
enforce_scale_and_margins, optional sharpness gate) and the index.csv format.

Video / image IO: OpenCV is not part of this build (video decode is outside the
hot path), so --video / --ref also accept a .npy array (N x H x W x 3 BGR u8 / H x W x 3), a
directory of image files, any Pillow-readable image (--ref), or `synthetic:N:WxH` (seeded
frames, for plumbing runs); crops are written with Pillow (JPEG quality 95).
--device cpu raises like the reference's SCRFD / TensorRT-only paths do.
"""
from __future__ import annotations

import argparse
import csv
import os
from typing import Iterator, Tuple

import numpy as np

from .detectors import PersonDetector
from .face_embedder import FaceEmbedder
from .postmatch import INDEX_HEADER, calc_sharpness, combine_scores, enforce_scale_and_margins, index_row
from .reid_embedder import ReIDEmbedder
from .utils import ensure_dir, expand_box_to_ratio, parse_ratio


def _read_image(path: str) -> np.ndarray:
    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False)
    from PIL import Image
    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])


def load_image(path: str) -> np.ndarray:
    """main.py:109-113 (cv2.imread(IMREAD_COLOR) -> BGR)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"Cannot read image: {path}")
    return _read_image(path)


def iter_frames(video: str) -> Tuple[Iterator[np.ndarray], float, int]:
    """(frames, fps, count) of a .npy clip, a directory of images or synthetic:N:WxH."""
    if video.startswith("synthetic:"):
        _, n, wh = video.split(":")
        w, h = (int(v) for v in wh.lower().split("x"))
        n = int(n)
        return (np.random.default_rng(20260501 + i).integers(0, 256, (h, w, 3), dtype=np.uint8) for i in range(n)), 30.0, n
    if os.path.isdir(video):
        files = sorted(f for f in os.listdir(video) if not f.startswith("."))
        return (_read_image(os.path.join(video, f)) for f in files), 30.0, len(files)
    if video.endswith(".npy"):
        arr = np.load(video, mmap_mode="r", allow_pickle=False)
        return (np.ascontiguousarray(arr[i]) for i in range(arr.shape[0])), 30.0, int(arr.shape[0])
    raise RuntimeError(f"Cannot open video: {video} (this build reads .npy clips, image directories, synthetic:N:WxH)")


def _write_crop(path: str, bgr: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(bgr[..., ::-1])).save(path, quality=95)


def _write_annot(path: str, frame: np.ndarray, person, expanded, face_box, score, fd, rd) -> None:
    """Annotated frame as main.py:332-345 draws it (person box green, expanded crop box
    blue, face box red in BGR terms; score text) - PIL stands in for cv2 (absent here)."""
    from PIL import Image, ImageDraw
    img = Image.fromarray(np.ascontiguousarray(frame[..., ::-1]))
    d = ImageDraw.Draw(img)
    d.rectangle(person, outline=(0, 255, 0), width=2)
    d.rectangle(expanded, outline=(0, 0, 255), width=2)
    if face_box is not None:
        d.rectangle(face_box, outline=(255, 0, 0), width=2)
    d.text((15, 15), f"score={score:.3f} fd={fd if fd is not None else -1:.3f} rd={rd if rd is not None else -1:.3f}",
           fill=(255, 255, 255))
    img.save(path, quality=95)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument('--video', required=True, help='path to video file')
    ap.add_argument('--ref', required=True, help='reference image of the target person')
    ap.add_argument('--out', required=True, help='output directory')
    ap.add_argument('--ratio', default='2:3', help='crop aspect ratio W:H (e.g., 2:3)')
    ap.add_argument('--frame-stride', type=int, default=2, help='analyze every Nth frame')
    ap.add_argument('--min-det-conf', type=float, default=0.35, help='YOLO min confidence')
    ap.add_argument('--face-thresh', type=float, default=0.32, help='max cosine distance for face match')
    ap.add_argument('--reid-thresh', type=float, default=0.38, help='max cosine distance for reid match')
    ap.add_argument('--combine', default='min', choices=['min', 'avg', 'face_priority'])
    ap.add_argument('--device', default='cuda', choices=['cuda', 'cpu'])
    ap.add_argument('--save-annot', action='store_true', help='save annotated frames')
    ap.add_argument('--yolo', default='yolov8n.pt', help='ultralytics model name or path')
    ap.add_argument('--min-sharpness', type=float, default=0.0, help='minimum normalized sharpness; 0 disables the gate')
    args = ap.parse_args(argv)

    ensure_dir(args.out)
    crops_dir = os.path.join(args.out, 'crops')
    ann_dir = os.path.join(args.out, 'annot') if args.save_annot else None
    ensure_dir(crops_dir)
    if ann_dir:
        ensure_dir(ann_dir)
    det = PersonDetector(model_name=args.yolo, device=args.device)
    face = FaceEmbedder(ctx=args.device)
    reid = ReIDEmbedder(device=args.device)

    ref_img = load_image(args.ref)
    ref_face = FaceEmbedder.best_face(face.extract(ref_img))
    ref_face_feat = ref_face['feat'] if ref_face else None
    ref_persons = det.detect(ref_img, conf=0.1)
    if ref_persons:
        ref_persons.sort(key=lambda d: (d['xyxy'][2] - d['xyxy'][0]) * (d['xyxy'][3] - d['xyxy'][1]), reverse=True)
        rx1, ry1, rx2, ry2 = [int(v) for v in ref_persons[0]['xyxy']]
        ref_reid_feat = reid.extract([ref_img[ry1:ry2, rx1:rx2]])[0]
    else:
        ref_reid_feat = reid.extract([ref_img])[0]

    frames, fps, _total = iter_frames(args.video)
    ratio_w, ratio_h = parse_ratio(args.ratio)
    csv_path = os.path.join(args.out, 'index.csv')
    hit_count = 0
    refn = None if ref_face_feat is None else ref_face_feat / max(float(np.linalg.norm(ref_face_feat)), 1e-6)
    with open(csv_path, 'w', newline='') as csv_f:
        writer = csv.writer(csv_f)
        writer.writerow(INDEX_HEADER)
        for frame_idx, frame in enumerate(frames):
            if frame_idx % max(1, args.frame_stride) != 0:
                continue
            H, W = frame.shape[:2]
            persons = det.detect(frame, conf=args.min_det_conf)
            if not persons:
                continue
            crops, boxes = [], []
            for p in persons:
                x1, y1, x2, y2 = [int(v) for v in p['xyxy']]
                x1 = max(0, x1); y1 = max(0, y1); x2 = min(W - 1, x2); y2 = min(H - 1, y2)
                if x2 <= x1 + 2 or y2 <= y1 + 2:
                    continue
                crops.append(frame[y1:y2, x1:x2])
                boxes.append((x1, y1, x2, y2))
            reid_feats = reid.extract(crops) if crops else []
            face_map = {}
            # the per-crop face.extract calls of main.py:238-265, in order, batched on the device
            per_crop = face.extract_batch(crops) if crops else []
            for i, ffaces in enumerate(per_crop):
                bestf, bestf_fd = None, None
                if refn is not None and ffaces:
                    fw = [f for f in ffaces if f.get("feat") is not None]
                    if fw:
                        def _cosdist(f):
                            v = np.asarray(f["feat"], dtype=np.float32)
                            v = v / max(float(np.linalg.norm(v)), 1e-6)
                            return 1.0 - float(np.dot(v, refn))
                        bestf = min(fw, key=_cosdist)
                        bestf_fd = _cosdist(bestf)
                if bestf is None:
                    bestf = FaceEmbedder.best_face(ffaces)
                if bestf and refn is not None:
                    if bestf_fd is None and bestf.get("feat") is not None:
                        v = np.asarray(bestf["feat"], dtype=np.float32)
                        v = v / max(float(np.linalg.norm(v)), 1e-6)
                        bestf_fd = 1.0 - float(np.dot(v, refn))
                    if bestf_fd is not None:
                        face_map[i] = (bestf, bestf_fd)
            for i, feat in enumerate(reid_feats):
                rd = None
                if ref_reid_feat is not None:
                    rd = 1.0 - float(np.dot(feat / np.linalg.norm(feat), ref_reid_feat / np.linalg.norm(ref_reid_feat)))
                fd = face_map.get(i, (None, None))[1]
                score = combine_scores(fd, rd, mode=args.combine)
                accept = False
                if score is not None:
                    accept = (fd is not None and fd <= args.face_thresh) or (rd is not None and rd <= args.reid_thresh)
                if not accept:
                    continue
                x1, y1, x2, y2 = boxes[i]
                anchor, head_bias = None, 0.0
                bf = face_map.get(i, (None, None))[0]
                if bf is not None:
                    fb = bf['bbox']
                    anchor = (x1 + (fb[0] + fb[2]) / 2.0, y1 + (fb[1] + fb[3]) / 2.0)
                    head_bias = -(0.9 * (max(1.0, fb[3] - fb[1]) / max(1.0, y2 - y1)))
                ex1, ey1, ex2, ey2 = expand_box_to_ratio(x1, y1, x2, y2, ratio_w, ratio_h, W, H, anchor=anchor,
                                                         head_bias=head_bias)
                face_box_abs = None
                if bf is not None:
                    fb = bf['bbox']
                    face_box_abs = (x1 + fb[0], y1 + fb[1], x1 + fb[2], y1 + fb[3])
                ex1, ey1, ex2, ey2 = enforce_scale_and_margins((ex1, ey1, ex2, ey2), f"{ratio_w}:{ratio_h}", W, H,
                                                               face_box_abs)
                crop = frame[ey1:ey2, ex1:ex2]
                if args.min_sharpness > 0 and calc_sharpness(crop, face._ctx) < args.min_sharpness:
                    continue
                crop_img_path = os.path.join(crops_dir, f"f{frame_idx:08d}.jpg")
                _write_crop(crop_img_path, crop)
                hit_count += 1
                if ann_dir:
                    fbox = None
                    if bf is not None:
                        fb = bf['bbox']
                        fbox = (x1 + int(fb[0]), y1 + int(fb[1]), x1 + int(fb[2]), y1 + int(fb[3]))
                    _write_annot(os.path.join(ann_dir, f"f{frame_idx:08d}.jpg"), frame, (x1, y1, x2, y2),
                                 (ex1, ey1, ex2, ey2), fbox, score, fd, rd)
                writer.writerow(index_row(frame_idx, fps, score, fd, rd, (ex1, ey1, ex2, ey2),
                                          os.path.basename(crop_img_path)))
    print(f"Done. Hits: {hit_count}. Index: {csv_path}")
    return 0


if __name__ == '__main__':
    raise SystemExit(main())
