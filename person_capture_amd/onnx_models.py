"""Map the reference's ONNX model files onto this build's parameter schemas (models.py).

The reference runs ``arcface_r100.onnx`` (glintr100 IResNet-100; w600k_r50 IResNet-50
fallback) and ``scrfd_10g_bnkps.onnx`` / ``scrfd_2.5g_bnkps.onnx`` through
onnxruntime + TensorRT (face_embedder.py:55-83, 598-606, 729-734, 893-895, 1102-1147);
their input names are probed at :1015-1017 and the ArcFace output width at :931-940.
Here only the weights matter: the graph is walked in file (= export, = forward) order,
each Conv is taken with the BatchNormalization / constant Mul that a non-fusing
exporter leaves behind it folded in, standalone BatchNormalization / PRelu / Gemm
(MatMul+Add) nodes are kept, and the resulting layer sequence is matched one by one
against the architecture's own layer list, checking every weight shape. A graph that
deviates (other widths, another block count, an op this mapping does not know) raises
ValueError naming the first layer that does not match.

The output is the unfolded parameter dict that models.compile_* and the CPU oracle
(oracle/nets_torch.py) take: a BatchNorm folded into a conv by the exporter becomes an
identity BatchNorm (weight 1, mean 0, var 1 - eps) carrying the conv bias.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import models
from .onnx_io import Graph, read_model

BN_EPS = models.BN_EPS

# reference file names (face_embedder.py:55-83)
SCRFD_FILES = {"10g": "scrfd_10g_bnkps.onnx", "2.5g": "scrfd_2.5g_bnkps.onnx"}
ARCFACE_ONNX = "arcface_r100.onnx"
ARCFACE_ALT = ("glintr100.onnx", "w600k_r50.onnx")


def find_model_file(name: str) -> Optional[str]:
    """The local part of the reference's _ensure_file (face_embedder.py:90-119): the path
    itself, then the name under the package directory, its parent, the running script's
    directory and PERSON_CAPTURE_AMD_MODELS. No download (there is no network here);
    None when absent."""
    p = Path(name)
    if p.exists():
        return str(p.resolve())
    pkg = Path(__file__).resolve().parent
    roots = [pkg, pkg.parent]
    try:
        roots.append(Path(sys.argv[0]).resolve().parent)
    except Exception:
        pass
    env = os.getenv("PERSON_CAPTURE_AMD_MODELS", "").strip()
    if env:
        roots.insert(0, Path(env))
    rel = p if not p.is_absolute() else Path(p.name)
    for base in roots:
        for cand in (base / rel, base / rel.name, base / "models" / rel.name):
            if cand.exists():
                return str(cand.resolve())
    return None


# ---------------------------------------------------------------------------
# graph -> layer sequence
# ---------------------------------------------------------------------------
class Layer:
    __slots__ = ("kind", "w", "b", "attrs", "node")

    def __init__(self, kind, w=None, b=None, attrs=None, node=""):
        self.kind, self.w, self.b, self.attrs, self.node = kind, w, b, attrs or {}, node

    def __repr__(self):
        return f"{self.kind}{'' if self.w is None else list(self.w.shape)}@{self.node}"


def _bn_affine(g: Graph, n) -> Tuple[np.ndarray, np.ndarray]:
    sc, bi, mean, var = (g.inits[n.inputs[i]].astype(np.float64) for i in range(1, 5))
    eps = float(n.attrs.get("epsilon", 1e-5))
    s = sc / np.sqrt(var + eps)
    return s, bi - mean * s


def layer_sequence(g: Graph) -> List[Layer]:
    """Conv (+ folded BN / scalar Mul), BN, PRelu, FC layers in graph order. Parameter-free
    ops (Relu, Add, pooling, Resize, Concat, Reshape, Transpose, Sigmoid, Flatten, ...)
    are skipped: the architecture's layer list fixes where they sit."""
    consumers: Dict[str, list] = {}
    for n in g.nodes:
        for i in n.inputs:
            consumers.setdefault(i, []).append(n)
    folded = set()
    seq: List[Layer] = []
    for n in g.nodes:
        if id(n) in folded:
            continue
        if n.op == "Conv":
            w = g.inits[n.inputs[1]].astype(np.float64)
            b = g.inits[n.inputs[2]].astype(np.float64) if len(n.inputs) > 2 and n.inputs[2] else np.zeros(w.shape[0])
            if int(n.attrs.get("group", 1)) != 1:
                raise ValueError(f"Conv {n.name}: grouped convolution is not part of these architectures")
            out = n.outputs[0]
            while True:
                cons = consumers.get(out, [])
                if len(cons) != 1:
                    break
                c = cons[0]
                if c.op == "BatchNormalization" and all(i in g.inits for i in c.inputs[1:5]):
                    s, t = _bn_affine(g, c)
                    w = w * s[:, None, None, None]
                    b = b * s + t
                elif c.op == "Mul" and any(i in g.inits and g.inits[i].size == 1 for i in c.inputs):
                    k = float([g.inits[i] for i in c.inputs if i in g.inits][0].reshape(()))
                    w, b = w * k, b * k
                else:
                    break
                folded.add(id(c))
                out = c.outputs[0]
            seq.append(Layer("conv", w, b, dict(n.attrs), n.name))
        elif n.op == "BatchNormalization":
            s, t = _bn_affine(g, n)
            seq.append(Layer("bn", s, t, dict(n.attrs), n.name))
        elif n.op == "PRelu":
            seq.append(Layer("prelu", g.inits[n.inputs[1]].astype(np.float64).reshape(-1), None, {}, n.name))
        elif n.op == "Gemm":
            w = g.inits[n.inputs[1]].astype(np.float64)
            if int(n.attrs.get("transB", 0)) == 0:
                w = w.T
            w = w * float(n.attrs.get("alpha", 1.0))
            b = g.inits[n.inputs[2]].astype(np.float64) * float(n.attrs.get("beta", 1.0)) \
                if len(n.inputs) > 2 else np.zeros(w.shape[0])
            seq.append(Layer("fc", w, b, {}, n.name))
        elif n.op == "MatMul" and n.inputs[1] in g.inits:
            w = g.inits[n.inputs[1]].astype(np.float64).T
            b = np.zeros(w.shape[0])
            cons = consumers.get(n.outputs[0], [])
            if len(cons) == 1 and cons[0].op == "Add" and any(i in g.inits for i in cons[0].inputs):
                b = [g.inits[i] for i in cons[0].inputs if i in g.inits][0].astype(np.float64).reshape(-1)
                folded.add(id(cons[0]))
            seq.append(Layer("fc", w, b, {}, n.name))
    return seq


class _Cursor:
    def __init__(self, seq: List[Layer], what: str):
        self.seq, self.i, self.what = seq, 0, what

    def take(self, kind: str, shape=None, label: str = "") -> Layer:
        if self.i >= len(self.seq):
            raise ValueError(f"{self.what}: graph ended before layer {label} ({kind})")
        L = self.seq[self.i]
        if L.kind != kind or (shape is not None and tuple(L.w.shape) != tuple(shape)):
            got = f"{L.kind} {None if L.w is None else tuple(L.w.shape)}"
            raise ValueError(f"{self.what}: layer {label} expected {kind} {shape}, graph has {got} at node "
                             f"{L.node!r} (position {self.i})")
        self.i += 1
        return L

    def peek(self) -> Optional[Layer]:
        return self.seq[self.i] if self.i < len(self.seq) else None

    def done(self):
        if self.i != len(self.seq):
            raise ValueError(f"{self.what}: {len(self.seq) - self.i} unexpected layers after the last one "
                             f"({self.seq[self.i]!r})")


def _bn_entry(p: Dict[str, np.ndarray], name: str, scale: np.ndarray, shift: np.ndarray) -> None:
    """Store an affine y = scale * x + shift as an eval BatchNorm (mean 0, var 1 - eps)."""
    c = scale.shape[0]
    p[name + ".weight"] = scale.astype(np.float32)
    p[name + ".bias"] = shift.astype(np.float32)
    p[name + ".running_mean"] = np.zeros(c, np.float32)
    p[name + ".running_var"] = np.full(c, 1.0 - BN_EPS, np.float32)


def _conv_bn(cur: _Cursor, p, wname: str, bnname: str, shape, label: str) -> None:
    L = cur.take("conv", shape, label)
    p[wname] = L.w.astype(np.float32)
    _bn_entry(p, bnname, np.ones(L.w.shape[0]), L.b)


# ---------------------------------------------------------------------------
# IResNet (arcface_r100.onnx = glintr100, w600k_r50.onnx)
# ---------------------------------------------------------------------------
def iresnet_depth_of(seq: List[Layer]) -> int:
    """Depth from the block count: 3 + 2 * sum(blocks) + downsample convs."""
    nconv = sum(1 for L in seq if L.kind == "conv")
    for depth, blocks in models.IRESNET_LAYERS.items():
        if nconv == 1 + 2 * sum(blocks) + len(blocks):
            return depth
    raise ValueError(f"IResNet: {nconv} convolutions match no known depth {sorted(models.IRESNET_LAYERS)}")


def iresnet_params(g: Graph, depth: Optional[int] = None) -> Tuple[Dict[str, np.ndarray], int]:
    """insightface arcface_torch IResNet (the glintr100 / w600k_r50 export) -> models.synth_iresnet
    schema. Layer order: conv1 (+bn1), prelu; per block bn1, conv1 (+bn2), prelu, conv2 (+bn3),
    [downsample conv (+bn)]; bn2, fc, features (BN1d, or folded into the FC by the exporter)."""
    seq = layer_sequence(g)
    depth = depth or iresnet_depth_of(seq)
    cur = _Cursor(seq, f"IResNet-{depth}")
    p: Dict[str, np.ndarray] = {}
    _conv_bn(cur, p, "conv1.weight", "bn1", (64, 3, 3, 3), "conv1")
    if cur.peek() is not None and cur.peek().kind == "bn":       # exporter kept bn1 separate
        L = cur.take("bn", None, "bn1")
        s0, t0 = p["bn1.weight"].astype(np.float64), p["bn1.bias"].astype(np.float64)
        _bn_entry(p, "bn1", s0 * L.w, t0 * L.w + L.b)
    p["prelu.weight"] = cur.take("prelu", None, "prelu").w.astype(np.float32)
    for pre, inp, pl, stride, ds in models.iresnet_blocks(depth):
        L = cur.take("bn", None, pre + ".bn1")
        if L.w.shape != (inp,):
            raise ValueError(f"IResNet-{depth}: {pre}.bn1 has {L.w.shape[0]} channels, expected {inp}")
        _bn_entry(p, pre + ".bn1", L.w, L.b)
        _conv_bn(cur, p, pre + ".conv1.weight", pre + ".bn2", (pl, inp, 3, 3), pre + ".conv1")
        p[pre + ".prelu.weight"] = cur.take("prelu", None, pre + ".prelu").w.astype(np.float32)
        L = cur.take("conv", (pl, pl, 3, 3), pre + ".conv2")
        if tuple(L.attrs.get("strides", [1, 1])) != (stride, stride):
            raise ValueError(f"IResNet-{depth}: {pre}.conv2 stride {L.attrs.get('strides')} != {stride}")
        p[pre + ".conv2.weight"] = L.w.astype(np.float32)
        _bn_entry(p, pre + ".bn3", np.ones(pl), L.b)
        if ds:
            _conv_bn(cur, p, pre + ".downsample.0.weight", pre + ".downsample.1", (pl, inp, 1, 1),
                     pre + ".downsample")
    L = cur.take("bn", None, "bn2")
    _bn_entry(p, "bn2", L.w, L.b)
    fc = cur.take("fc", None, "fc")
    if fc.w.shape[1] != 512 * 49:
        raise ValueError(f"IResNet-{depth}: fc has {fc.w.shape[1]} inputs, expected {512 * 49}")
    p["fc.weight"] = fc.w.astype(np.float32)
    p["fc.bias"] = fc.b.astype(np.float32)
    emb = fc.w.shape[0]
    nxt = cur.peek()
    if nxt is not None and nxt.kind == "bn":
        L = cur.take("bn", None, "features")
        _bn_entry(p, "features", L.w, L.b)
    else:
        _bn_entry(p, "features", np.ones(emb), np.zeros(emb))
    cur.done()
    return p, depth


# ---------------------------------------------------------------------------
# SCRFD (scrfd_10g_bnkps / scrfd_2.5g_bnkps)
# ---------------------------------------------------------------------------
def scrfd_variant_of(seq: List[Layer]) -> str:
    first = next(L for L in seq if L.kind == "conv")
    for v, cfg in models.SCRFD_CFG.items():
        if first.w.shape[0] == cfg["base"] // 2:
            return v
    raise ValueError(f"SCRFD: stem width {first.w.shape[0]} matches no known variant")


def scrfd_params(g: Graph, variant: Optional[str] = None) -> Tuple[Dict[str, np.ndarray], str]:
    """insightface SCRFD-*-BNKPS export -> models.synth_scrfd schema, in forward order: deep
    stem (3 conv+BN), BasicBlocks (conv1+bn1, conv2+bn2, [avg-down 1x1 conv+BN]), PAFPN
    (lateral 1x1 x3, fpn 3x3 x3, downsample 3x3/s2 x2, pafpn 3x3 x2), then per stride the
    stacked conv+BN, cls, reg (its Scale folded), kps convs."""
    seq = layer_sequence(g)
    variant = variant or scrfd_variant_of(seq)
    cfg = models.SCRFD_CFG[variant]
    cur = _Cursor(seq, f"SCRFD-{variant}")
    p: Dict[str, np.ndarray] = {}
    base = cfg["base"]
    for i, (ci, co) in enumerate([(3, base // 2), (base // 2, base // 2), (base // 2, base)]):
        _conv_bn(cur, p, f"backbone.stem.{3 * i}.weight", f"backbone.stem.{3 * i + 1}", (co, ci, 3, 3),
                 f"stem.{3 * i}")
    for pre, inp, pl, stride, ds in models.scrfd_blocks(cfg):
        _conv_bn(cur, p, pre + ".conv1.weight", pre + ".bn1", (pl, inp, 3, 3), pre + ".conv1")
        _conv_bn(cur, p, pre + ".conv2.weight", pre + ".bn2", (pl, pl, 3, 3), pre + ".conv2")
        if ds:
            _conv_bn(cur, p, pre + ".downsample.1.weight", pre + ".downsample.2", (pl, inp, 1, 1),
                     pre + ".downsample")
    nk = cfg["neck"]

    def biased(name, shape):
        L = cur.take("conv", shape, name)
        p[name + ".weight"] = L.w.astype(np.float32)
        p[name + ".bias"] = L.b.astype(np.float32)

    for i, c in enumerate(cfg["planes"][1:]):
        biased(f"neck.lateral_convs.{i}.conv", (nk, c, 1, 1))
    for i in range(3):
        biased(f"neck.fpn_convs.{i}.conv", (nk, nk, 3, 3))
    for i in range(2):
        biased(f"neck.downsample_convs.{i}.conv", (nk, nk, 3, 3))
    for i in range(2):
        biased(f"neck.pafpn_convs.{i}.conv", (nk, nk, 3, 3))
    ft, A = cfg["feat"], models.SCRFD_ANCHORS
    for s in models.SCRFD_STRIDES:
        for j in range(cfg["stacked"]):
            _conv_bn(cur, p, f"bbox_head.{s}.stack.{j}.conv.weight", f"bbox_head.{s}.stack.{j}.bn",
                     (ft, nk if j == 0 else ft, 3, 3), f"head.{s}.stack.{j}")
        biased(f"bbox_head.{s}.cls", (A, ft, 3, 3))
        biased(f"bbox_head.{s}.reg", (4 * A, ft, 3, 3))
        biased(f"bbox_head.{s}.kps", (10 * A, ft, 3, 3))
    cur.done()
    return p, variant


def load_arcface(path: str):
    """(params, depth, embedding width) of an ArcFace IResNet ONNX file."""
    p, depth = iresnet_params(read_model(path))
    return p, depth, int(p["fc.weight"].shape[0])


def load_scrfd(path: str):
    """(params, variant) of an SCRFD-BNKPS ONNX file."""
    return scrfd_params(read_model(path))
