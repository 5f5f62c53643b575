"""ONNX weight loading (§8f rank 1): person_capture_amd.onnx_io decodes the protobuf wire
format without the `onnx` package, onnx_models maps the graph onto the IResNet / SCRFD
schemas. The files are written by tests/onnx_export.py in torch.onnx.export's layouts
(BatchNorm folded into the preceding Conv, and kept as separate nodes); the loaded
parameters must reproduce the original network's fp32 forward (oracle/nets_torch.py).
Parity against the real glintr100 / w600k_r50 / scrfd_*_bnkps files is unpinned: they are
not available offline."""
import numpy as np
import pytest
import torch

from oracle import nets_torch as nt
from person_capture_amd import models, onnx_io, onnx_models
from onnx_export import iresnet_graph, scrfd_graph


def test_wire_format_round_trip(tmp_path):
    g = onnx_io.Graph(nodes=[onnx_io.Node("Conv", ["x", "w"], ["y"], "c0", {"strides": [2, 2], "group": 1,
                                                                           "alpha": 0.5, "mode": b"nearest"})],
                      inits={"w": np.arange(24, dtype=np.float32).reshape(2, 3, 2, 2),
                             "shape": np.array([-1, 7], np.int64), "h": np.ones(3, np.float16)},
                      inputs=["x"], outputs=["y"])
    path = tmp_path / "m.onnx"
    onnx_io.write_model(str(path), g)
    r = onnx_io.read_model(str(path))
    assert [n.op for n in r.nodes] == ["Conv"] and r.nodes[0].inputs == ["x", "w"] and r.outputs == ["y"]
    assert r.nodes[0].attrs["strides"] == [2, 2] and r.nodes[0].attrs["group"] == 1
    assert abs(r.nodes[0].attrs["alpha"] - 0.5) < 1e-7 and r.nodes[0].attrs["mode"] == b"nearest"
    for k, v in g.inits.items():
        assert r.inits[k].dtype == v.dtype and np.array_equal(r.inits[k], v)
    assert r.inputs == ["x"]


@pytest.mark.parametrize("depth", [50, 100])
@pytest.mark.parametrize("fuse", [True, False])
def test_iresnet_from_onnx(tmp_path, depth, fuse):
    p = models.synth_iresnet(depth, seed=3)
    path = tmp_path / "arcface_r100.onnx"
    onnx_io.write_model(str(path), iresnet_graph(p, depth, fuse_bn=fuse))
    q, d, emb = onnx_models.load_arcface(str(path))
    assert d == depth and emb == 512
    x = torch.from_numpy(np.random.default_rng(0).standard_normal((2, 3, 112, 112)).astype(np.float32))
    a = nt.iresnet_forward(p, depth, x).numpy()
    b = nt.iresnet_forward(q, depth, x).numpy()
    assert np.abs(a - b).max() <= 1e-4 * np.abs(a).max()
    P = models.compile_iresnet(q, depth)   # and the device program compiles from them
    assert P.outputs


@pytest.mark.parametrize("variant", ["10g", "2.5g"])
@pytest.mark.parametrize("fuse", [True, False])
def test_scrfd_from_onnx(tmp_path, variant, fuse):
    p = models.synth_scrfd(variant, seed=2)
    path = tmp_path / f"scrfd_{variant}_bnkps.onnx"
    onnx_io.write_model(str(path), scrfd_graph(p, variant, fuse_bn=fuse))
    q, v = onnx_models.load_scrfd(str(path))
    assert v == variant
    x = torch.from_numpy(np.random.default_rng(1).standard_normal((1, 3, 160, 160)).astype(np.float32))
    for a, b in zip(nt.scrfd_forward(p, variant, x), nt.scrfd_forward(q, variant, x)):
        a, b = a.numpy(), b.numpy()
        assert np.abs(a - b).max() <= 1e-4 * max(1.0, np.abs(a).max())
    assert models.compile_scrfd(q, variant, 320).outputs


def test_mismatched_graph_is_rejected(tmp_path):
    p = models.synth_iresnet(50, seed=1, calibrate=False)
    g = iresnet_graph(p, 50)
    g.nodes = [n for n in g.nodes if n.op != "PRelu" or n is not g.nodes[1]]   # drop the stem PReLU
    with pytest.raises(ValueError, match="prelu"):
        onnx_models.iresnet_params(g)
    with pytest.raises(ValueError, match="no known depth"):
        g2 = iresnet_graph(p, 50)
        drop = [i for i, n in enumerate(g2.nodes) if n.op == "Conv"][5]
        del g2.nodes[drop]
        onnx_models.iresnet_params(g2)


def test_find_model_file(tmp_path, monkeypatch):
    f = tmp_path / "scrfd_10g_bnkps.onnx"
    f.write_bytes(b"x")
    monkeypatch.setenv("PERSON_CAPTURE_AMD_MODELS", str(tmp_path))
    assert onnx_models.find_model_file("scrfd_10g_bnkps.onnx") == str(f.resolve())
    assert onnx_models.find_model_file("missing_model.onnx") is None


def _ext_tensor(name: str, location: str, n: int) -> bytes:
    """TensorProto (wire format) of a float32 [n] tensor whose bytes live in an external file."""
    def entry(k, v):
        return onnx_io._ld(1, k.encode()) + onnx_io._ld(2, v.encode())
    body = b""
    body += onnx_io._key(1, 0) + onnx_io._enc_varint(n)          # dims
    body += onnx_io._key(2, 0) + onnx_io._enc_varint(1)          # data_type FLOAT
    body += onnx_io._ld(8, name.encode())
    body += onnx_io._ld(13, entry("location", location))
    body += onnx_io._ld(13, entry("length", str(4 * n)))
    body += onnx_io._key(14, 0) + onnx_io._enc_varint(1)         # data_location EXTERNAL
    return body


@pytest.mark.parametrize("loc", ["w.bin", "../escape.bin", "/etc/hostname", "sub/../w.bin"])
def test_external_data_stays_in_model_dir(tmp_path, loc):
    """External tensor data is read only from inside the model directory (as the onnx
    package enforces, CVE-2022-25882 / CVE-2024-27318); a truncated file is an error."""
    (tmp_path / "m").mkdir()
    np.arange(4, dtype=np.float32).tofile(tmp_path / "m" / "w.bin")
    np.arange(4, dtype=np.float32).tofile(tmp_path / "escape.bin")
    raw = _ext_tensor("w", loc, 4)
    if loc in ("w.bin", "sub/../w.bin"):
        if loc.startswith("sub"):
            (tmp_path / "m" / "sub").mkdir()
        name, arr = onnx_io._tensor(memoryview(raw), str(tmp_path / "m"))
        assert name == "w" and np.array_equal(arr, np.arange(4, dtype=np.float32))
    else:
        with pytest.raises(ValueError):
            onnx_io._tensor(memoryview(raw), str(tmp_path / "m"))
    with pytest.raises(ValueError):
        onnx_io._tensor(memoryview(_ext_tensor("w", "w.bin", 8)), str(tmp_path / "m"))
