"""FaceEmbedder with the reference's model files present (§8f rank 1): scrfd_2.5g_bnkps.onnx
and arcface_r100.onnx (IResNet-50 here, the w600k_r50 fallback's depth, to keep the CPU
oracle quick) written in torch.onnx.export's layout by tests/onnx_export.py into a models
directory; the device path must give the oracle's boxes and embeddings computed from the
ORIGINAL (unexported) parameters: f32, boxes exact, chained embeddings within 1e-4."""
import numpy as np
import pytest

from oracle import nets_torch as nt
from oracle import pipeline as op
from oracle import ref_algos as ra
from person_capture_amd import face_embedder as fe_mod
from person_capture_amd import models, onnx_io
from onnx_export import iresnet_graph, scrfd_graph

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fuse", [True, False])
def test_face_embedder_loads_onnx_models(gpu_ctx, monkeypatch, tmp_path, fuse):
    ps = models.synth_scrfd("2.5g", seed=11)
    pa = models.synth_iresnet(50, seed=12)
    onnx_io.write_model(str(tmp_path / "scrfd_2.5g_bnkps.onnx"), scrfd_graph(ps, "2.5g", fuse_bn=fuse))
    onnx_io.write_model(str(tmp_path / "arcface_r100.onnx"), iresnet_graph(pa, 50, fuse_bn=fuse))
    monkeypatch.setenv("PERSON_CAPTURE_AMD_MODELS", str(tmp_path))
    monkeypatch.setenv("PERSON_CAPTURE_AMD_PRECISION", "f32")
    monkeypatch.setenv("PERSON_CAPTURE_AMD_REQUIRE_WEIGHTS", "1")
    fe = fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_2.5g_bnkps", conf=0.5)
    assert fe.weights_source["scrfd"].endswith("scrfd_2.5g_bnkps.onnx")
    assert fe.weights_source["arcface"].endswith("arcface_r100.onnx") and fe._arc_depth == 50
    fe.debug_chips = True
    frames = [np.random.default_rng(60 + i).integers(0, 256, (360, 640, 3), dtype=np.uint8) for i in range(2)]
    got = fe.extract_batch(frames)
    n = 0
    for frame, g in zip(frames, got):
        ref = op.extract_frame(frame, ps, "2.5g", pa, 50, conf=0.5, D=640)
        assert ref != op.NEEDS_FALLBACK and len(ref) == len(g)
        for a, b in zip(sorted(g, key=lambda f: tuple(f["bbox"])), sorted(ref, key=lambda f: tuple(f["bbox"]))):
            assert np.array_equal(a["bbox"], b["bbox"])
            e = nt.iresnet_forward(pa, 50, nt.arcface_input_from_chips(a["chip"][None])).numpy()
            ef = nt.iresnet_forward(pa, 50, nt.arcface_input_from_chips(a["chip"][None, :, ::-1])).numpy()
            assert np.abs(ra.arcface_postprocess(e, ef)[0] - a["feat"]).max() < 1e-4
            n += 1
    assert n >= 2


def test_missing_model_files_raise_when_required(gpu_ctx, monkeypatch, tmp_path):
    monkeypatch.setenv("PERSON_CAPTURE_AMD_MODELS", str(tmp_path))
    monkeypatch.setenv("PERSON_CAPTURE_AMD_REQUIRE_WEIGHTS", "1")
    with pytest.raises(RuntimeError, match="model files not found"):
        fe_mod.FaceEmbedder(ctx="cuda:0", yolo_model="scrfd_10g_bnkps")
