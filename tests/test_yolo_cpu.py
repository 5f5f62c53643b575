"""CPU checks of the YOLOv8 person-detector build: the compiled program (in-place
concat slices, padded channel maps, fused Detect stems, BN eps 1e-3 folding) run
through the device-semantics emulator must match the literal oracle forward; the
ultralytics letterbox / scale_boxes geometry; the oracle post-processing contract."""
import numpy as np
import pytest
import torch

from oracle import nets_torch as nt
from oracle import ref_algos as ra
from person_capture_amd import models_yolo as my
from program_emulator import run_program


@pytest.fixture(scope="module")
def y8n():
    return my.synth_yolov8("n", seed=3)


def test_layer_table_yolov8n():
    L = my.yolo_layers("n")
    assert [l["cout"] for l in L[:10]] == [16, 32, 32, 64, 64, 128, 128, 256, 256, 256]
    assert [l.get("n") for l in L if l["type"] == "C2f"] == [1, 2, 2, 1, 1, 1, 1, 1]
    d = L[22]
    assert d["ch"] == [64, 128, 256] and d["c2b"] == 64 and d["c3"] == 80
    assert [l["cout"] for l in my.yolo_layers("s")[:2]] == [32, 64]


@pytest.mark.parametrize("Hp,Wp", [(128, 192), (96, 160)])
def test_yolo_program_matches_oracle(y8n, Hp, Wp):
    rng = np.random.default_rng(5)
    x = np.zeros((2, Hp, Wp, 4), np.float32)
    x[..., :3] = rng.integers(0, 256, (2, Hp, Wp, 3)).astype(np.float32) / 255.0
    ref = nt.yolov8_forward(y8n, "n", torch.from_numpy(np.ascontiguousarray(x[..., :3].transpose(0, 3, 1, 2))))
    P = my.compile_yolov8(y8n, "n", Hp, Wp)
    outs = run_program(P, x)
    assert len(outs) == 3
    for o, r in zip(outs, ref):
        got = o.permute(0, 2, 3, 1).numpy()
        r = r.numpy()
        assert got.shape == r.shape
        assert np.abs(got - r).max() / max(1.0, np.abs(r).max()) < 1e-4


def test_letterbox_geometry():
    # ultralytics LetterBox(auto=True, stride=32): 1080p -> 640x360 centred in 640x384
    assert my.letterbox_geometry(1080, 1920) == (640, 360, 12, 0, 384, 640)
    assert my.letterbox_geometry(2160, 3840) == (640, 360, 12, 0, 384, 640)
    assert my.letterbox_geometry(480, 640) == (640, 480, 0, 0, 480, 640)
    nw, nh, top, left, Hp, Wp = my.letterbox_geometry(1000, 333)
    assert (nh, Hp % 32, Wp % 32) == (640, 0, 0) and left + nw <= Wp
    # odd remainder splits round(d - 0.1) / round(d + 0.1)
    nw, nh, top, left, Hp, Wp = my.letterbox_geometry(500, 640)
    assert (Hp - nh - top) - top in (0, 1)
    g, px, py = my.scale_geometry(384, 640, 1080, 1920)
    assert abs(g - 1 / 3) < 1e-12 and (px, py) == (0, 12)


def test_yolo_letterbox_canvas():
    fr = np.random.default_rng(1).integers(0, 256, (90, 160, 3), dtype=np.uint8)
    img, (nw, nh, top, left, Hp, Wp) = ra.yolo_letterbox(fr)
    assert img.shape == (Hp, Wp, 3) and img.dtype == np.float32
    assert np.all(img[:top] == np.float32(114) / np.float32(255))
    # identity path when the frame already has the letterbox size
    fr2 = np.random.default_rng(2).integers(0, 256, (360, 640, 3), dtype=np.uint8)
    img2, g2 = ra.yolo_letterbox(fr2)
    assert g2[:2] == (640, 360)
    assert np.array_equal(img2[g2[2]:g2[2] + 360], fr2[..., ::-1].astype(np.float32) / np.float32(255))


def test_yolo_postprocess_contract():
    """Planted head maps: a strong class-0 anchor, a weaker overlapping one (suppressed
    at IoU 0.45), a class-3 anchor (filtered by classes=[0]) and a separate class-0 box."""
    heads = [np.full((h, w, 144), -20.0, np.float32) for h, w in ((48, 80), (24, 40), (12, 20))]
    for hd in heads:
        hd[..., :64] = 0.0
    def plant(lvl, y, x, cls, logit, bins=(3, 5, 3, 5)):
        hd = heads[lvl]
        hd[y, x, :64] = -8.0
        for k, b in enumerate(bins):
            hd[y, x, 16 * k + b] = 8.0
        hd[y, x, 64 + cls] = logit
    plant(0, 20, 30, 0, 3.0)
    plant(0, 20, 31, 0, 2.0)     # overlaps the first
    plant(0, 30, 60, 3, 5.0)     # not a person
    plant(1, 5, 5, 0, 1.0)
    d = ra.yolo_postprocess(heads, 0.35, 0.45, 40, 384, 640, 1080, 1920)
    assert d.shape == (2, 5)
    assert d[0, 4] > d[1, 4] > 0.35
    assert np.all(d[:, 0] >= 0) and np.all(d[:, 2] <= 1920) and np.all(d[:, 3] <= 1080)
    # box of the first: anchor (30.5, 20.5)*8 +- (3,5,3,5)*8 (DFL peak), scaled by 3, minus pad 12
    cx, cy = 30.5 * 8, 20.5 * 8
    np.testing.assert_allclose(d[0, :4], [(cx - 24) * 3, (cy - 40 - 12) * 3, (cx + 24) * 3, (cy + 40 - 12) * 3],
                               atol=0.05)
    assert len(ra.yolo_postprocess(heads, 0.99, 0.45, 40, 384, 640, 1080, 1920)) == 0


@pytest.fixture(scope="module")
def y8face():
    return my.synth_yolov8_face("n", seed=4)


def test_face_pose_layer_table():
    """yolov8-pose head (the YOLOv8-face models, kpt_shape [5, 3]): cv4 width max(ch0 // 4, 15)."""
    L = my.yolo_layers("l", 1, (5, 3))[22]
    assert L["type"] == "Pose" and L["nk"] == 15 and L["c4"] == max(L["ch"][0] // 4, 15) and L["nc"] == 1


@pytest.mark.parametrize("Hp,Wp", [(128, 192)])
def test_yolo_face_program_matches_oracle(y8face, Hp, Wp):
    """The Pose program's [DFL | cls | kpt] head maps against the literal oracle forward."""
    rng = np.random.default_rng(6)
    x = np.zeros((2, Hp, Wp, 4), np.float32)
    x[..., :3] = rng.integers(0, 256, (2, Hp, Wp, 3)).astype(np.float32) / 255.0
    ref = nt.yolov8_forward(y8face, "n", torch.from_numpy(np.ascontiguousarray(x[..., :3].transpose(0, 3, 1, 2))),
                            nc=1, kpt=(5, 3))
    outs = run_program(my.compile_yolov8(y8face, "n", Hp, Wp, nc=1, kpt=(5, 3)), x)
    for o, r in zip(outs, ref):
        got = o.permute(0, 2, 3, 1).numpy()
        r = r.numpy()
        assert got.shape == r.shape and r.shape[-1] == 64 + 1 + 15
        assert np.abs(got - r).max() / max(1.0, np.abs(r).max()) < 1e-4


def test_yolo_pose_postprocess_contract():
    """A planted face anchor: keypoints decode as (raw * 2 + anchor - 0.5) * stride, scale_coords
    with the unrounded pad, invisible points (sigmoid < 0.5) zeroed as Results.keypoints does."""
    heads = [np.full((h, w, 80), -20.0, np.float32) for h, w in ((48, 80), (24, 40), (12, 20))]
    hd = heads[0]
    hd[..., :64] = 0.0
    hd[20, 30, :64] = -8.0
    for k, b in enumerate((3, 5, 3, 5)):
        hd[20, 30, 16 * k + b] = 8.0
    hd[20, 30, 64] = 3.0
    raw = np.array([[0.1, 0.2, 4.0], [0.9, 0.2, 4.0], [0.5, 0.6, 4.0], [0.2, 0.9, -4.0], [0.8, 0.9, 4.0]],
                   np.float32)
    hd[20, 30, 65:] = raw.reshape(-1)
    d, k = ra.yolo_postprocess(heads, 0.3, 0.3, 60, 384, 640, 1080, 1920, nk=15)
    assert d.shape == (1, 5) and k.shape == (1, 5, 3)
    gain = 1 / 3
    for q in range(5):
        if raw[q, 2] < 0:
            assert k[0, q, 0] == 0 and k[0, q, 1] == 0
            continue
        x = (raw[q, 0] * 2 + 30) * 8
        y = (raw[q, 1] * 2 + 20) * 8
        assert abs(k[0, q, 0] - x / gain) < 1e-2 and abs(k[0, q, 1] - (y - 12) / gain) < 1e-2
