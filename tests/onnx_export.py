"""Test infrastructure: write parameter dicts (models.py schema) as ONNX graphs laid out the way
torch.onnx.export writes the reference's model files (insightface exports glintr100 /
w600k_r50 from arcface_torch and the SCRFD-BNKPS models from mmdet with torch's exporter).

Two layouts per net: `fuse_bn=True` is torch's eval-mode export (a BatchNorm that directly
follows a Conv is folded into the Conv's weight and bias; other BatchNorms stay
BatchNormalization nodes), `fuse_bn=False` keeps every BatchNorm as its own node. The
parameter-free ops (Relu, Add, MaxPool, AveragePool, Resize, Flatten, Sigmoid, Reshape,
Transpose) are emitted too, so the loader is exercised on realistic graphs.
"""
from __future__ import annotations

import numpy as np

from person_capture_amd import models
from person_capture_amd.onnx_io import Graph, Node

EPS = 1e-5


class _B:
    def __init__(self, fuse_bn: bool):
        self.g = Graph(nodes=[], inits={}, inputs=["input.1"], outputs=[])
        self.fuse = fuse_bn
        self.k = 0

    def name(self):
        self.k += 1
        return str(self.k)

    def init(self, arr) -> str:
        n = f"w{self.name()}"
        arr = np.asarray(arr)
        self.g.inits[n] = np.ascontiguousarray(arr, dtype=np.int64 if arr.dtype.kind in "iu" else np.float32)
        return n

    def node(self, op, ins, **attrs) -> str:
        out = self.name()
        self.g.nodes.append(Node(op=op, inputs=list(ins), outputs=[out], name=f"{op}_{out}", attrs=attrs))
        return out

    def bn(self, x, p, name) -> str:
        return self.node("BatchNormalization", [x, self.init(p[name + ".weight"]), self.init(p[name + ".bias"]),
                                                self.init(p[name + ".running_mean"]),
                                                self.init(p[name + ".running_var"])], epsilon=EPS, momentum=0.9)

    def conv(self, x, w, b=None, stride=1, pad=None, bn=None, p=None) -> str:
        """Conv [+ BatchNorm `bn`]: folded into the conv when fusing (torch eval export)."""
        k = w.shape[2]
        pad = k // 2 if pad is None else pad
        attrs = dict(dilations=[1, 1], group=1, kernel_shape=[k, k], pads=[pad] * 4, strides=[stride, stride])
        w = np.asarray(w, np.float64)
        b = np.zeros(w.shape[0]) if b is None else np.asarray(b, np.float64)
        if bn is not None and self.fuse:
            s, t = models.bn_fold(p, bn)
            w, b = w * s[:, None, None, None], b * s + t
            return self.node("Conv", [x, self.init(w), self.init(b)], **attrs)
        y = self.node("Conv", [x, self.init(w), self.init(b)] if b.any() else [x, self.init(w)], **attrs)
        return self.bn(y, p, bn) if bn is not None else y


def iresnet_graph(p, depth: int, fuse_bn: bool = True) -> Graph:
    B = _B(fuse_bn)
    x = B.conv("input.1", p["conv1.weight"], bn="bn1", p=p)
    x = B.node("PRelu", [x, B.init(p["prelu.weight"].reshape(-1, 1, 1))])
    for pre, inp, pl, stride, ds in models.iresnet_blocks(depth):
        o = B.bn(x, p, pre + ".bn1")
        o = B.conv(o, p[pre + ".conv1.weight"], bn=pre + ".bn2", p=p)
        o = B.node("PRelu", [o, B.init(p[pre + ".prelu.weight"].reshape(-1, 1, 1))])
        o = B.conv(o, p[pre + ".conv2.weight"], stride=stride, bn=pre + ".bn3", p=p)
        idt = B.conv(x, p[pre + ".downsample.0.weight"], stride=stride, pad=0, bn=pre + ".downsample.1", p=p) \
            if ds else x
        x = B.node("Add", [o, idt])
    x = B.bn(x, p, "bn2")
    x = B.node("Flatten", [x], axis=1)
    x = B.node("Gemm", [x, B.init(p["fc.weight"]), B.init(p["fc.bias"])], alpha=1.0, beta=1.0, transB=1)
    x = B.bn(x, p, "features")
    B.g.outputs = [x]
    return B.g


def scrfd_graph(p, variant: str, fuse_bn: bool = True, reg_scale: float = 1.25) -> Graph:
    """mmdet SCRFD forward as exported: sigmoid scores and reshaped/transposed outputs
    score_8/16/32, bbox_*, kps_*; the reg conv is followed by its Scale (a scalar Mul:
    the weights written here are divided by `reg_scale`, so the folded result is p's)."""
    cfg = models.SCRFD_CFG[variant]
    B = _B(fuse_bn)
    x = "input.1"
    for i, s in enumerate((2, 1, 1)):
        x = B.conv(x, p[f"backbone.stem.{3 * i}.weight"], stride=s, bn=f"backbone.stem.{3 * i + 1}", p=p)
        x = B.node("Relu", [x])
    x = B.node("MaxPool", [x], kernel_shape=[3, 3], pads=[1, 1, 1, 1], strides=[2, 2])
    blocks = models.scrfd_blocks(cfg)
    outs = []
    for i, (pre, inp, pl, stride, ds) in enumerate(blocks):
        o = B.node("Relu", [B.conv(x, p[pre + ".conv1.weight"], stride=stride, bn=pre + ".bn1", p=p)])
        o = B.conv(o, p[pre + ".conv2.weight"], bn=pre + ".bn2", p=p)
        idt = x
        if ds:
            y = B.node("AveragePool", [x], kernel_shape=[stride, stride], strides=[stride, stride], ceil_mode=1,
                       count_include_pad=0) if stride > 1 else x
            idt = B.conv(y, p[pre + ".downsample.1.weight"], pad=0, bn=pre + ".downsample.2", p=p)
        x = B.node("Relu", [B.node("Add", [o, idt])])
        if i + 1 == len(blocks) or blocks[i + 1][0].split(".")[1] != pre.split(".")[1]:
            outs.append(x)
    ins = outs[1:]
    conv = lambda t, nm, s=1, pad=0: B.conv(t, p[nm + ".weight"], p[nm + ".bias"], stride=s, pad=pad)
    lat = [conv(ins[i], f"neck.lateral_convs.{i}.conv") for i in range(3)]
    for i in range(2, 0, -1):
        up = B.node("Resize", [lat[i], "", B.init(np.array([1, 1, 2, 2], np.float32))], mode="nearest")
        lat[i - 1] = B.node("Add", [lat[i - 1], up])
    inter = [conv(lat[i], f"neck.fpn_convs.{i}.conv", 1, 1) for i in range(3)]
    for i in range(2):
        inter[i + 1] = B.node("Add", [inter[i + 1], conv(inter[i], f"neck.downsample_convs.{i}.conv", 2, 1)])
    neck = [inter[0]] + [conv(inter[i], f"neck.pafpn_convs.{i - 1}.conv", 1, 1) for i in range(1, 3)]
    res = {"score": [], "bbox": [], "kps": []}
    for lvl, s in enumerate(models.SCRFD_STRIDES):
        h = neck[lvl]
        for j in range(cfg["stacked"]):
            h = B.node("Relu", [B.conv(h, p[f"bbox_head.{s}.stack.{j}.conv.weight"],
                                       bn=f"bbox_head.{s}.stack.{j}.bn", p=p)])
        cls = B.node("Sigmoid", [conv(h, f"bbox_head.{s}.cls", 1, 1)])
        reg = B.conv(h, p[f"bbox_head.{s}.reg.weight"] / reg_scale, p[f"bbox_head.{s}.reg.bias"] / reg_scale)
        reg = B.node("Mul", [reg, B.init(np.array(reg_scale, np.float32))])
        kps = conv(h, f"bbox_head.{s}.kps", 1, 1)
        for key, t, c in (("score", cls, 1), ("bbox", reg, 4), ("kps", kps, 10)):
            t = B.node("Transpose", [t], perm=[0, 2, 3, 1])
            res[key].append(B.node("Reshape", [t, B.init(np.array([-1, c], np.int64))]))
    B.g.outputs = res["score"] + res["bbox"] + res["kps"]
    return B.g
