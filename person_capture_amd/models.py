"""Conv architectures of the identity hot path: parameter schemas, synthetic
weights, and compilation into pcgpu programs.

Architectures (no weights ship with the reference):
  * ArcFace IResNet-100 / -50 — the network behind ``arcface_r100.onnx``
    (glintr100) / ``w600k_r50.onnx`` loaded at face_embedder.py:68-83, 729-734.
    insightface arcface_torch iresnet: conv3x3(3,64)+BN+PReLU, IBasicBlock
    stages [3,13,30,3] (r100) / [3,4,14,3] (r50) with widths 64..512, first block
    of every stage stride 2, then BN2d -> flatten(NCHW) -> FC(25088,512) -> BN1d.
  * SCRFD-10G-BNKPS / 2.5G-BNKPS — ``scrfd_10g_bnkps.onnx`` / ``scrfd_2.5g_bnkps.onnx``
    (face_embedder.py:55-65): ResNetV1e backbone (deep stem, avg-down shortcuts,
    BasicBlocks), PAFPN neck (start_level 1, 3 outputs, plain biased convs),
    per-stride heads (stacked conv+BN+ReLU, then cls/bbox/kps 3x3 convs,
    2 anchors per location).

Parameters use the frameworks' own (unfolded) parameterization — conv weights
[cout][cin][kh][kw], BN (weight, bias, running_mean, running_var, eps) — so the
CPU oracle (oracle/nets_torch.py) runs them literally while compile_*() applies
the inference-time algebra for the device. Synthetic weights are seeded
(He-normal convs, random affine BN) and their BN running statistics are
calibrated on seeded synthetic inputs so activations stay O(1) through 100
layers, as trained statistics would keep them.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from .program import (ACT_NONE, ACT_PRELU, ACT_RELU, BIAS_BORDER9, BIAS_CHANNEL, RES_SAME, RES_UP2, Program,
                      cpad, pack_conv_weights, pad_vec)

Params = Dict[str, np.ndarray]
BN_EPS = 1e-5

IRESNET_LAYERS = {100: [3, 13, 30, 3], 50: [3, 4, 14, 3], 34: [3, 4, 6, 3], 18: [2, 2, 2, 2]}
IRESNET_WIDTHS = [64, 128, 256, 512]

SCRFD_CFG = {
    # stage_blocks, stage_planes, base(stem) channels, neck out, head feat, stacked convs
    "10g": dict(blocks=(3, 4, 2, 3), planes=(56, 88, 88, 224), base=56, neck=56, feat=80, stacked=3),
    "2.5g": dict(blocks=(3, 5, 3, 2), planes=(24, 48, 48, 80), base=24, neck=24, feat=64, stacked=2),
}
SCRFD_STRIDES = (8, 16, 32)
SCRFD_ANCHORS = 2


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def bn_fold(p: Params, name: str) -> Tuple[np.ndarray, np.ndarray]:
    """Return (scale, shift) of an eval-mode BatchNorm as float64."""
    g = p[name + ".weight"].astype(np.float64)
    b = p[name + ".bias"].astype(np.float64)
    m = p[name + ".running_mean"].astype(np.float64)
    v = p[name + ".running_var"].astype(np.float64)
    s = g / np.sqrt(v + BN_EPS)
    return s, b - m * s


def _he(rng: np.random.Generator, shape, gain: float = 1.0) -> np.ndarray:
    fan_in = int(np.prod(shape[1:]))
    return (rng.standard_normal(shape) * gain * np.sqrt(2.0 / fan_in)).astype(np.float32)


def _bn_init(rng: np.random.Generator, p: Params, name: str, c: int, gamma=(0.8, 1.2)) -> None:
    p[name + ".weight"] = rng.uniform(gamma[0], gamma[1], c).astype(np.float32)
    p[name + ".bias"] = (rng.standard_normal(c) * 0.1).astype(np.float32)
    p[name + ".running_mean"] = np.zeros(c, np.float32)
    p[name + ".running_var"] = np.ones(c, np.float32)


# ---------------------------------------------------------------------------
# IResNet (ArcFace)
# ---------------------------------------------------------------------------
def iresnet_blocks(depth: int) -> List[Tuple[str, int, int, int, bool]]:
    """(prefix, inplanes, planes, stride, has_downsample) for every IBasicBlock."""
    out = []
    inpl = 64
    for li, (n, w) in enumerate(zip(IRESNET_LAYERS[depth], IRESNET_WIDTHS)):
        for bi in range(n):
            stride = 2 if bi == 0 else 1
            ds = bi == 0 and (stride != 1 or inpl != w)
            out.append((f"layer{li + 1}.{bi}", inpl, w, stride, ds))
            inpl = w
    return out


def synth_iresnet(depth: int = 100, seed: int = 0, calibrate: bool = True, emb: int = 512) -> Params:
    rng = np.random.default_rng(np.random.SeedSequence([20260501, depth, seed]))
    p: Params = {}
    p["conv1.weight"] = _he(rng, (64, 3, 3, 3))
    _bn_init(rng, p, "bn1", 64)
    p["prelu.weight"] = rng.uniform(0.1, 0.35, 64).astype(np.float32)
    for pre, inp, pl, stride, ds in iresnet_blocks(depth):
        _bn_init(rng, p, pre + ".bn1", inp)
        p[pre + ".conv1.weight"] = _he(rng, (pl, inp, 3, 3))
        _bn_init(rng, p, pre + ".bn2", pl)
        p[pre + ".prelu.weight"] = rng.uniform(0.1, 0.35, pl).astype(np.float32)
        p[pre + ".conv2.weight"] = _he(rng, (pl, pl, 3, 3))
        _bn_init(rng, p, pre + ".bn3", pl, gamma=(0.15, 0.35))
        if ds:
            p[pre + ".downsample.0.weight"] = _he(rng, (pl, inp, 1, 1))
            _bn_init(rng, p, pre + ".downsample.1", pl)
    _bn_init(rng, p, "bn2", 512)
    p["fc.weight"] = (rng.standard_normal((emb, 512 * 49)) / np.sqrt(512 * 49)).astype(np.float32)
    p["fc.bias"] = (rng.standard_normal(emb) * 0.01).astype(np.float32)
    _bn_init(rng, p, "features", emb)
    if calibrate:
        from .synth_calib import calibrate_iresnet
        imgs = rng.integers(0, 256, size=(2, 112, 112, 3), dtype=np.uint8)
        calibrate_iresnet(p, depth, imgs)
    return p


def compile_iresnet(p: Params, depth: int = 100, split: bool = False, c8: bool = False) -> Program:
    """IResNet -> program. Input: NHWC4 preprocessed chip (RGB, x/127.5-1, channel 3 = 0).
    split: the f16x3 form (program.Program) - every activation and weight hi + lo,
    f32-class embeddings on the f16 MFMA path. Its input is the centred chip x - 127.5 (exact in
    f16, where x/127.5 - 1 is not: that one rounding alone moved embeddings by ~2e-4,
    tools/emu_mixed_iresnet.py), with the 1/127.5 folded into the stem weights; the program
    flags it (Program.input_centered) and pc_arcface_embed preprocesses accordingly.
    c8: the f16c8 form (Program(c8=True)): the same f32-class embeddings from half
    the MFMA issues of split; the last trunk tensor stays split for the FC's split-K kernel."""
    split = split or c8
    P = Program(split=split, c8=c8)
    x = P.input_tensor(112, 112, 4)
    # stem: conv1 + bn1 + prelu, folded
    s, b = bn_fold(p, "bn1")
    w = p["conv1.weight"].astype(np.float64) * s[:, None, None, None]
    if split:
        P.input_centered = True
        w = w / 127.5
    w4 = np.zeros((64, 3, 3, 4))
    w4[:, :, :, :3] = np.transpose(w, (0, 2, 3, 1))
    t = P.act(112, 112, 64)
    P.stem(t, x, w4, b, stride=1, pad=1, slope=p["prelu.weight"], act=ACT_PRELU)
    H = 112
    for pre, inp, pl, stride, ds in iresnet_blocks(depth):
        # conv1: bn1 (pre-BN, folded with a border-class bias table) -> conv3x3 -> bn2 -> prelu
        s1, b1 = bn_fold(p, pre + ".bn1")
        s2, b2 = bn_fold(p, pre + ".bn2")
        W1 = p[pre + ".conv1.weight"].astype(np.float64)
        w1f = W1 * s1[None, :, None, None] * s2[:, None, None, None]
        npad = cpad(pl)
        # tab[rc][cc][co] = s2 * sum_{taps valid for class} sum_ci W1 * b1 + b2
        contrib = np.einsum("oikl,i->okl", W1, b1)   # [co][kh][kw]
        rows = [(1, 2), (0, 1, 2), (0, 1)]
        tab = np.zeros((3, 3, npad))
        for rc in range(3):
            for cc in range(3):
                v = contrib[:, list(rows[rc]), :][:, :, list(rows[cc])].sum(axis=(1, 2))
                tab[rc, cc, :pl] = s2 * v + b2
        y1 = P.act(H, H, pl)
        P.conv(y1, [(t, 3, 3, 1, 1, inp)], pack_conv_weights([w1f], [cpad(inp)], npad), pl,
               bias=tab.reshape(9, npad), bias_mode=BIAS_BORDER9, slope=pad_vec(p[pre + ".prelu.weight"], npad),
               act=ACT_PRELU)
        # conv2 (stride) -> bn3, + shortcut (identity, or downsample conv1x1/s + BN as a 2nd K-segment)
        Ho = H // stride
        s3, b3 = bn_fold(p, pre + ".bn3")
        w2f = p[pre + ".conv2.weight"].astype(np.float64) * s3[:, None, None, None]
        out = P.act(Ho, Ho, pl)
        if ds:
            sd, bd = bn_fold(p, pre + ".downsample.1")
            wdf = p[pre + ".downsample.0.weight"].astype(np.float64) * sd[:, None, None, None]
            P.conv(out, [(y1, 3, 3, stride, 1, pl), (t, 1, 1, stride, 0, inp)],
                   pack_conv_weights([w2f, wdf], [cpad(pl), cpad(inp)], npad), pl,
                   bias=pad_vec(b3 + bd, npad), bias_mode=BIAS_CHANNEL)
        else:
            P.conv(out, [(y1, 3, 3, stride, 1, pl)], pack_conv_weights([w2f], [cpad(pl)], npad), pl,
                   bias=pad_vec(b3, npad), bias_mode=BIAS_CHANNEL, res=t, res_mode=RES_SAME, act_after_res=0)
        t, H = out, Ho
    # bn2 -> flatten(NCHW) -> fc -> features(BN1d), as one 7x7 valid conv with split-K
    s2, b2 = bn_fold(p, "bn2")
    sf, bf = bn_fold(p, "features")
    Wfc = p["fc.weight"].astype(np.float64).reshape(-1, 512, 7, 7)   # [o][c][h][w] (NCHW flatten order)
    emb = Wfc.shape[0]
    wf = Wfc * s2[None, :, None, None] * sf[:, None, None, None]
    bias = sf * (np.einsum("ochw,c->o", Wfc, b2) + p["fc.bias"].astype(np.float64)) + bf
    e = P.act(1, 1, emb, is_f32=1)
    P.plain_split(t)
    P.conv(e, [(t, 7, 7, 1, 0, 512)], pack_conv_weights([wf], [512], cpad(emb)), emb,
           bias=pad_vec(bias, cpad(emb)), bias_mode=BIAS_CHANNEL, splitk=16)
    P.outputs = [e]
    return P


# ---------------------------------------------------------------------------
# SCRFD (ResNetV1e + PAFPN + SCRFDHead, BN + keypoints)
# ---------------------------------------------------------------------------
def scrfd_blocks(cfg: dict) -> List[Tuple[str, int, int, int, bool]]:
    out = []
    inpl = cfg["base"]
    for si, (n, pl) in enumerate(zip(cfg["blocks"], cfg["planes"])):
        for bi in range(n):
            stride = (1 if si == 0 else 2) if bi == 0 else 1
            ds = bi == 0 and (stride != 1 or inpl != pl)
            out.append((f"backbone.layer{si + 1}.{bi}", inpl, pl, stride, ds))
            inpl = pl
    return out


SCRFD_KPS_PRIOR = np.array([[-0.8, -0.6], [0.8, -0.6], [0.0, 0.2], [-0.6, 1.0], [0.6, 1.0]], np.float32)


def synth_scrfd(variant: str = "10g", seed: int = 0, calibrate: bool = True,
                target_per_image=(2.0, 1.5, 1.0)) -> Params:
    """Synthetic SCRFD weights. Head biases carry a face prior (boxes ~4 strides wide,
    canonical 5-point layout) so the downstream align/embed path is exercised the way
    real detections exercise it; the cls bias is calibrated so that ~target_per_image
    anchors per level pass score >= 0.5 on synthetic letterboxed frames."""
    cfg = SCRFD_CFG[variant]
    rng = np.random.default_rng(np.random.SeedSequence([20260502, len(variant), seed]))
    p: Params = {}
    base = cfg["base"]
    stem = [(3, base // 2), (base // 2, base // 2), (base // 2, base)]
    for i, (ci, co) in enumerate(stem):
        p[f"backbone.stem.{3 * i}.weight"] = _he(rng, (co, ci, 3, 3))
        _bn_init(rng, p, f"backbone.stem.{3 * i + 1}", co)
    for pre, inp, pl, stride, ds in scrfd_blocks(cfg):
        p[pre + ".conv1.weight"] = _he(rng, (pl, inp, 3, 3))
        _bn_init(rng, p, pre + ".bn1", pl)
        p[pre + ".conv2.weight"] = _he(rng, (pl, pl, 3, 3))
        _bn_init(rng, p, pre + ".bn2", pl, gamma=(0.3, 0.6))
        if ds:
            p[pre + ".downsample.1.weight"] = _he(rng, (pl, inp, 1, 1))
            _bn_init(rng, p, pre + ".downsample.2", pl)
    nk = cfg["neck"]
    ins = cfg["planes"][1:]
    for i, c in enumerate(ins):
        p[f"neck.lateral_convs.{i}.conv.weight"] = _he(rng, (nk, c, 1, 1), 0.7)
        p[f"neck.lateral_convs.{i}.conv.bias"] = (rng.standard_normal(nk) * 0.05).astype(np.float32)
        p[f"neck.fpn_convs.{i}.conv.weight"] = _he(rng, (nk, nk, 3, 3), 0.7)
        p[f"neck.fpn_convs.{i}.conv.bias"] = (rng.standard_normal(nk) * 0.05).astype(np.float32)
    for i in range(len(ins) - 1):
        p[f"neck.downsample_convs.{i}.conv.weight"] = _he(rng, (nk, nk, 3, 3), 0.5)
        p[f"neck.downsample_convs.{i}.conv.bias"] = (rng.standard_normal(nk) * 0.05).astype(np.float32)
        p[f"neck.pafpn_convs.{i}.conv.weight"] = _he(rng, (nk, nk, 3, 3), 0.7)
        p[f"neck.pafpn_convs.{i}.conv.bias"] = (rng.standard_normal(nk) * 0.05).astype(np.float32)
    ft = cfg["feat"]
    A = SCRFD_ANCHORS
    for s in SCRFD_STRIDES:
        for j in range(cfg["stacked"]):
            p[f"bbox_head.{s}.stack.{j}.conv.weight"] = _he(rng, (ft, nk if j == 0 else ft, 3, 3))
            _bn_init(rng, p, f"bbox_head.{s}.stack.{j}.bn", ft)
        p[f"bbox_head.{s}.cls.weight"] = _he(rng, (A, ft, 3, 3), 0.5)
        p[f"bbox_head.{s}.cls.bias"] = np.full(A, -4.0, np.float32)
        p[f"bbox_head.{s}.reg.weight"] = _he(rng, (4 * A, ft, 3, 3), 0.05)
        p[f"bbox_head.{s}.reg.bias"] = np.full(4 * A, 2.0, np.float32)
        p[f"bbox_head.{s}.kps.weight"] = _he(rng, (10 * A, ft, 3, 3), 0.05)
        kb = np.tile((SCRFD_KPS_PRIOR * 1.5).reshape(-1), A).astype(np.float32)
        p[f"bbox_head.{s}.kps.bias"] = kb
    if calibrate:
        from .synth_calib import calibrate_scrfd
        calibrate_scrfd(p, variant, rng, target_per_image)
    return p


def _conv_bn(P: Program, p: Params, x: int, wname: str, bnname: str, cin: int, cout: int, k: int, stride: int,
             act: int = ACT_RELU) -> int:
    s, b = bn_fold(p, bnname)
    w = p[wname].astype(np.float64) * s[:, None, None, None]
    H, W, _ = P.dims(x)
    pad = k // 2
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = P.act(Ho, Wo, cpad(cout))
    P.conv(out, [(x, k, k, stride, pad, cin)], pack_conv_weights([w], [cpad(cin)], cpad(cout)), cout,
           bias=pad_vec(b, cpad(cout)), act=act)
    return out


def _conv_bias(P: Program, p: Params, x: int, name: str, cin: int, cout: int, k: int, stride: int,
               res: int = None, res_mode: int = RES_SAME, out_f32: int = 0, extra=None) -> int:
    """Plain biased conv (no norm/act); optional residual add or second segment
    extra = (tensor, wname, bname, cin, k, stride)."""
    H, W, _ = P.dims(x)
    pad = k // 2
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = P.act(Ho, Wo, cpad(cout), is_f32=out_f32)
    ws = [p[name + ".weight"].astype(np.float64)]
    pads = [cpad(cin)]
    segs = [(x, k, k, stride, pad, cin)]
    bias = p[name + ".bias"].astype(np.float64)
    if extra is not None:
        xt, wn, bn, ci2, k2, s2 = extra
        ws.append(p[wn].astype(np.float64))
        pads.append(cpad(ci2))
        segs.append((xt, k2, k2, s2, k2 // 2, ci2))
        bias = bias + p[bn].astype(np.float64)
    P.conv(out, segs, pack_conv_weights(ws, pads, cpad(cout)), cout, bias=pad_vec(bias, cpad(cout)),
           res=res, res_mode=res_mode)
    return out


def compile_scrfd(p: Params, variant: str = "10g", D: int = 640, split: bool = False) -> Program:
    """SCRFD -> program for a DxD letterboxed input (NHWC4, (x-127.5)/128, RGB).
    Outputs (per stride 8/16/32): f32 [H][W][32] = cls logits(2) | bbox(8) | kps(20).
    split: the f16x3 form (program.Program): f32-class activations and weights on the f16
    MFMA path - the detector precision whose boxes and landmarks match the f32 path."""
    assert D % 32 == 0
    cfg = SCRFD_CFG[variant]
    P = Program(split=split)
    x = P.input_tensor(D, D, 4)
    base = cfg["base"]
    # deep stem: conv3x3/s2 (direct stem kernel) + 2 convs, then maxpool 3x3/s2
    s, b = bn_fold(p, "backbone.stem.1")
    w = p["backbone.stem.0.weight"].astype(np.float64) * s[:, None, None, None]
    w4 = np.zeros((base // 2, 3, 3, 4))
    w4[:, :, :, :3] = np.transpose(w, (0, 2, 3, 1))
    t = P.act(D // 2, D // 2, cpad(base // 2))
    P.stem(t, x, w4, b, stride=2, pad=1, act=ACT_RELU)
    t = _conv_bn(P, p, t, "backbone.stem.3.weight", "backbone.stem.4", base // 2, base // 2, 3, 1)
    t = _conv_bn(P, p, t, "backbone.stem.6.weight", "backbone.stem.7", base // 2, base, 3, 1)
    H = D // 4
    mp = P.act(H, H, cpad(base))
    P.maxpool(mp, t, 3, 2, 1)
    t = mp
    feats = []
    blocks = scrfd_blocks(cfg)
    stage_last = {}
    for i, (pre, inp, pl, stride, ds) in enumerate(blocks):
        stage_last[pre.split(".")[1]] = i
    for i, (pre, inp, pl, stride, ds) in enumerate(blocks):
        y1 = _conv_bn(P, p, t, pre + ".conv1.weight", pre + ".bn1", inp, pl, 3, stride)
        Hh, Ww, _ = P.dims(y1)
        s2, b2 = bn_fold(p, pre + ".bn2")
        w2 = p[pre + ".conv2.weight"].astype(np.float64) * s2[:, None, None, None]
        out = P.act(Hh, Ww, cpad(pl))
        if ds:
            sd, bd = bn_fold(p, pre + ".downsample.2")
            wd = p[pre + ".downsample.1.weight"].astype(np.float64) * sd[:, None, None, None]
            if stride == 2:
                # AvgPool2d(2,2,ceil,count_include_pad=False) + conv1x1 == conv2x2/s2 with W/4 (even H, W)
                wd = np.repeat(np.repeat(wd, 2, axis=2), 2, axis=3) / 4.0
                seg2 = (t, 2, 2, 2, 0, inp)
            else:
                seg2 = (t, 1, 1, 1, 0, inp)
            P.conv(out, [(y1, 3, 3, 1, 1, pl), seg2],
                   pack_conv_weights([w2, wd], [cpad(pl), cpad(inp)], cpad(pl)), pl,
                   bias=pad_vec(b2 + bd, cpad(pl)), act=ACT_RELU, act_after_res=1)
        else:
            P.conv(out, [(y1, 3, 3, 1, 1, pl)], pack_conv_weights([w2], [cpad(pl)], cpad(pl)), pl,
                   bias=pad_vec(b2, cpad(pl)), act=ACT_RELU, res=t, res_mode=RES_SAME, act_after_res=1)
        t = out
        if i == stage_last.get(pre.split(".")[1]):
            feats.append(t)
    # PAFPN (start_level=1): inputs = stage 2,3,4 outputs
    ins = feats[1:]
    chans = cfg["planes"][1:]
    nk = cfg["neck"]
    lat = [None] * 3
    lat[2] = _conv_bias(P, p, ins[2], "neck.lateral_convs.2.conv", chans[2], nk, 1, 1)
    lat[1] = _conv_bias(P, p, ins[1], "neck.lateral_convs.1.conv", chans[1], nk, 1, 1, res=lat[2], res_mode=RES_UP2)
    lat[0] = _conv_bias(P, p, ins[0], "neck.lateral_convs.0.conv", chans[0], nk, 1, 1, res=lat[1], res_mode=RES_UP2)
    inter = [None] * 3
    inter[0] = _conv_bias(P, p, lat[0], "neck.fpn_convs.0.conv", nk, nk, 3, 1)
    # inter[i+1] = fpn_conv(lat[i+1]) + downsample_conv(inter[i]): two K-segments, one launch
    inter[1] = _conv_bias(P, p, lat[1], "neck.fpn_convs.1.conv", nk, nk, 3, 1,
                          extra=(inter[0], "neck.downsample_convs.0.conv.weight", "neck.downsample_convs.0.conv.bias",
                                 nk, 3, 2))
    inter[2] = _conv_bias(P, p, lat[2], "neck.fpn_convs.2.conv", nk, nk, 3, 1,
                          extra=(inter[1], "neck.downsample_convs.1.conv.weight", "neck.downsample_convs.1.conv.bias",
                                 nk, 3, 2))
    outs = [inter[0],
            _conv_bias(P, p, inter[1], "neck.pafpn_convs.0.conv", nk, nk, 3, 1),
            _conv_bias(P, p, inter[2], "neck.pafpn_convs.1.conv", nk, nk, 3, 1)]
    # heads
    ft = cfg["feat"]
    A = SCRFD_ANCHORS
    results = []
    for lvl, s in enumerate(SCRFD_STRIDES):
        h = outs[lvl]
        cin = nk
        for j in range(cfg["stacked"]):
            h = _conv_bn(P, p, h, f"bbox_head.{s}.stack.{j}.conv.weight", f"bbox_head.{s}.stack.{j}.bn", cin, ft, 3, 1)
            cin = ft
        w = np.concatenate([p[f"bbox_head.{s}.cls.weight"], p[f"bbox_head.{s}.reg.weight"],
                            p[f"bbox_head.{s}.kps.weight"]], axis=0).astype(np.float64)
        bb = np.concatenate([p[f"bbox_head.{s}.cls.bias"], p[f"bbox_head.{s}.reg.bias"],
                             p[f"bbox_head.{s}.kps.bias"]]).astype(np.float64)
        co = w.shape[0]   # 2 + 8 + 20 = 30
        Hh, Ww, _ = P.dims(h)
        o = P.act(Hh, Ww, cpad(co), is_f32=1)
        P.conv(o, [(h, 3, 3, 1, 1, ft)], pack_conv_weights([w], [cpad(ft)], cpad(co)), co,
               bias=pad_vec(bb, cpad(co)))
        results.append(o)
    P.outputs = results
    return P
