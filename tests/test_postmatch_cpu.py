"""Post-match geometry (§8f rank 4) against the reference's own functions: main.py's
_enforce_scale_and_margins / _clip_to_frame and utils.detect_black_borders run by
tools/gen_golden.py into tests/golden/postmatch.npz; combine_scores and index.csv row format;
the CLI's --device cpu refusal (like the reference's SCRFD / TensorRT-only paths)."""
import os

import numpy as np
import pytest

from person_capture_amd import postmatch as pm

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "postmatch.npz")
RATIOS = ["2:3", "16:9", "1:1", "4:5"]


@pytest.fixture(scope="module")
def gold():
    return np.load(G, allow_pickle=False)


def test_enforce_scale_and_margins(gold):
    for row, out in zip(gold["esm_in"], gold["esm_out"]):
        x1, y1, x2, y2, r, W, H = (int(v) for v in row[:7])
        fb = None if row[7] < 0 else tuple(float(v) for v in row[7:11])
        assert pm.enforce_scale_and_margins((x1, y1, x2, y2), RATIOS[r], W, H, fb) == tuple(int(v) for v in out)


def test_clip_to_frame(gold):
    for row, out in zip(gold["clip_in"], gold["clip_out"]):
        assert pm.clip_to_frame(*[float(v) for v in row[:4]], int(row[4]), int(row[5])) == tuple(int(v) for v in out)


def test_detect_black_borders(gold):
    for i, out in enumerate(gold["bb_out"]):
        img = gold[f"border{i}"]
        assert pm.detect_black_borders(img, thr=int(out[4])) == tuple(int(v) for v in out[:4])
    assert pm.detect_black_borders(np.zeros((0, 0, 3), np.uint8)) == (0, 0, 0, 0)


def test_sharpness_small_crop_on_host():
    crop = np.random.default_rng(0).integers(0, 256, (120, 90, 3), dtype=np.uint8)
    g = pm.gray_u8(crop).astype(np.float64)
    p = np.pad(g, 1, mode="reflect")
    lap = p[1:-1, :-2] + p[1:-1, 2:] + p[:-2, 1:-1] + p[2:, 1:-1] - 4 * g
    ref = float(np.var(lap.astype(np.float32))) / (float(np.mean(pm.gray_u8(crop))) ** 2 + 1e-6)
    assert pm.calc_sharpness(crop) == pytest.approx(ref, rel=1e-6)
    assert pm.calc_sharpness(np.zeros((0, 0, 3), np.uint8)) == 0.0
    with pytest.raises(RuntimeError):
        pm.calc_sharpness(np.zeros((300, 300, 3), np.uint8))


def test_index_row_and_combine():
    assert pm.index_row(12, 30.0, 0.25, 0.25, None, (1, 2, 3, 4), "f00000012.jpg") == \
        [12, "0.400", "0.2500", "0.2500", "", 1, 2, 3, 4, "f00000012.jpg"]
    assert pm.combine_scores(None, None) is None
    assert pm.combine_scores(0.2, 0.5, "face_priority") == pytest.approx(0.7 * 0.2 + 0.3 * 0.5)


def test_cli_device_cpu_raises(tmp_path):
    from person_capture_amd import main as cli
    with pytest.raises(RuntimeError):
        cli.main(["--video", "synthetic:2:64x48", "--ref", str(tmp_path / "r.npy"), "--out", str(tmp_path / "o"),
                  "--device", "cpu"])
