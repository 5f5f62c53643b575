"""BASELINE C1 plumbing: the person_capture CLI loop (main.py:146-358) end to end through the
MI355X facades on a 10-frame 640x360 synthetic clip with SCRFD-2.5G + ArcFace (the face model
selected by PERSON_CAPTURE_AMD_FACE_MODEL, as the reference's main.py takes FaceEmbedder's
default), YOLOv8n persons and the ReID tower; index.csv in the reference's format and one crop
per accepted row. Plus calc_sharpness's device INTER_AREA path against the oracle resize."""
import csv
import os

import numpy as np
import pytest

from oracle import cv_ops
from person_capture_amd import main as cli
from person_capture_amd import postmatch as pm

pytestmark = pytest.mark.gpu


def test_cli_c1_plumbing(gpu_ctx, monkeypatch, tmp_path):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_FACE_MODEL", "scrfd_2.5g_bnkps")
    ref = np.random.default_rng(20260501 + 3).integers(0, 256, (360, 640, 3), dtype=np.uint8)   # frame 3 of the clip
    np.save(tmp_path / "ref.npy", ref)
    out = tmp_path / "out"
    rc = cli.main(["--video", "synthetic:10:640x360", "--ref", str(tmp_path / "ref.npy"), "--out", str(out),
                   "--frame-stride", "1", "--face-thresh", "0.45", "--reid-thresh", "0.38", "--device", "cuda",
                   "--save-annot"])
    assert rc == 0
    rows = list(csv.reader(open(out / "index.csv")))
    assert rows[0] == pm.INDEX_HEADER
    crops = sorted(os.listdir(out / "crops"))
    print(f"{len(rows) - 1} accepted rows, {len(crops)} crop files")
    assert len(rows) > 1
    for r in rows[1:]:
        fi, x1, y1, x2, y2 = int(r[0]), int(r[5]), int(r[6]), int(r[7]), int(r[8])
        assert 0 <= fi < 10 and 0 <= x1 < x2 <= 640 and 0 <= y1 < y2 <= 360
        assert r[9] == f"f{fi:08d}.jpg" and r[9] in crops   # one file per frame, as main.py names them
    # --save-annot: one annotated full frame per accepted hit (main.py:332-345)
    assert sorted(os.listdir(out / "annot")) == crops


def test_sharpness_device_downscale(gpu_ctx):
    crop = np.random.default_rng(1).integers(0, 256, (400, 300, 3), dtype=np.uint8)
    got = pm.calc_sharpness(crop, gpu_ctx)
    g = pm.gray_u8(crop)
    g3 = np.repeat(g[..., None], 3, axis=2)
    small = cv_ops.resize(g3, (192, 256), interpolation=cv_ops.INTER_AREA)[..., 0]
    p = np.pad(small.astype(np.float32), 1, mode="reflect")
    lap = (p[1:-1, :-2] + p[1:-1, 2:] + p[:-2, 1:-1] + p[2:, 1:-1] - 4.0 * p[1:-1, 1:-1]).astype(np.float32)
    ref = float(np.var(lap)) / (float(np.mean(small)) ** 2 + 1e-6)
    assert got == ref
