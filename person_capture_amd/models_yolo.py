"""YOLOv8 person detector: architecture table, synthetic weights, and compilation
into a pcgpu program.

The reference's PersonDetector loads ``yolov8n.pt`` through [ext] ultralytics==8.3.205
(detectors.py:12-82, 84-269) and predicts with fused Conv+BN, fp16 on CUDA. The
architecture here is ultralytics' ``yolov8.yaml`` at scale n/s/m/l/x (parse_model:
channels make_divisible(min(c, max_channels) * width, 8), repeats
max(round(n * depth), 1)):

  backbone  Conv(64,3,2) Conv(128,3,2) C2f(128)x3 Conv(256,3,2) C2f(256)x6 Conv(512,3,2)
            C2f(512)x6 Conv(1024,3,2) C2f(1024)x3 SPPF(1024,5)
  head      Upsample Concat(6) C2f(512) Upsample Concat(4) C2f(256) Conv(256,3,2)
            Concat(12) C2f(512) Conv(512,3,2) Concat(9) C2f(1024) Detect(15,18,21)

Parameters follow the checkpoint's state-dict names (``model.{i}.conv.weight``,
``model.{i}.bn.*``, ``model.{i}.cv1.conv.weight``, ``model.{i}.m.{j}.cv1...``,
``model.22.cv2.{l}.{0,1,2}...``) with BatchNorm eps 1e-3 (ultralytics
initialize_weights). No checkpoint exists offline: weights are seeded, BN running
statistics calibrated on synthetic frames, and the class-0 (person) logit bias set so
that a few anchors per frame pass the detector threshold (synth_calib.calibrate_yolo).

Compilation (compile_yolov8): every Concat is a buffer whose channel slices the
producers write in place (Program.view), C2f's split is a channel view of its cv1
output, Upsample is an OP_UPSAMPLE into the concat slice, SPPF's three max-pools write
successive slices; every slice is padded to a multiple of 32 channels so each view
is a valid implicit-GEMM operand, and the consumers' weights are scattered onto the
padded channel positions. The Detect head's two first convs (box/cls) share one
launch; its outputs are f32 [H][W][64 DFL | nc class] per stride.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .program import ACT_NONE, ACT_SILU, RES_SAME, Program, cpad

Params = Dict[str, np.ndarray]
YOLO_BN_EPS = 1e-3
YOLO_NC = 80
REG_MAX = 16
YOLO_STRIDES = (8, 16, 32)
YOLO_SCALES = {"n": (0.33, 0.25, 1024), "s": (0.33, 0.50, 1024), "m": (0.67, 0.75, 768),
               "l": (1.00, 1.00, 512), "x": (1.00, 1.25, 512)}

_YAML = [  # (from, repeats, module, args) — ultralytics/cfg/models/v8/yolov8.yaml
    (-1, 1, "Conv", (64, 3, 2)), (-1, 1, "Conv", (128, 3, 2)), (-1, 3, "C2f", (128, True)),
    (-1, 1, "Conv", (256, 3, 2)), (-1, 6, "C2f", (256, True)), (-1, 1, "Conv", (512, 3, 2)),
    (-1, 6, "C2f", (512, True)), (-1, 1, "Conv", (1024, 3, 2)), (-1, 3, "C2f", (1024, True)),
    (-1, 1, "SPPF", (1024, 5)),
    (-1, 1, "Upsample", ()), ((-1, 6), 1, "Concat", ()), (-1, 3, "C2f", (512, False)),
    (-1, 1, "Upsample", ()), ((-1, 4), 1, "Concat", ()), (-1, 3, "C2f", (256, False)),
    (-1, 1, "Conv", (256, 3, 2)), ((-1, 12), 1, "Concat", ()), (-1, 3, "C2f", (512, False)),
    (-1, 1, "Conv", (512, 3, 2)), ((-1, 9), 1, "Concat", ()), (-1, 3, "C2f", (1024, False)),
    ((15, 18, 21), 1, "Detect", ()),
]


def yolo_scale_of(model_name: str) -> str:
    """'yolov8n.pt' -> 'n' (detectors.py:84-269 hub names); unknown names -> 'n'."""
    base = str(model_name).lower().rsplit("/", 1)[-1]
    for s in "nsmlx":
        if base.startswith(f"yolov8{s}"):
            return s
    return "n"


def yolo_layers(scale: str = "n", nc: int = YOLO_NC, kpt: Optional[Tuple[int, int]] = None) -> List[dict]:
    """Resolved layer table: type, inputs (absolute indices), channels, repeats. kpt = (nkpt, ndim)
    turns the Detect head into ultralytics' Pose head (yolov8-pose.yaml, the YOLOv8-face models:
    kpt_shape [5, 3]) with its cv4 keypoint branch of width c4 = max(ch[0] // 4, nkpt * ndim)."""
    depth, width, maxc = YOLO_SCALES[scale]
    div8 = lambda x: int(math.ceil(x / 8) * 8)
    out: List[dict] = []
    ch: List[int] = []
    for i, (f, n, m, args) in enumerate(_YAML):
        frm = [f] if isinstance(f, int) else list(f)
        frm = [i + j if j < 0 else j for j in frm]
        n = max(round(n * depth), 1) if n > 1 else n
        c1 = ch[frm[0]] if i > 0 else 3
        L = {"i": i, "type": m, "from": frm, "name": f"model.{i}"}
        if m in ("Conv", "C2f", "SPPF"):
            c2 = div8(min(args[0], maxc) * width)
            L.update(c1=c1, c2=c2)
            if m == "Conv":
                L.update(k=args[1], s=args[2])
            elif m == "C2f":
                L.update(n=n, shortcut=bool(args[1]))
            else:
                L.update(k=args[1])
        elif m == "Upsample":
            c2 = c1
        elif m == "Concat":
            c2 = sum(ch[j] for j in frm)
        else:  # Detect
            chs = [ch[j] for j in frm]
            c2b = max(16, chs[0] // 4, REG_MAX * 4)
            c3 = max(chs[0], min(nc, 100))
            L.update(ch=chs, c2b=c2b, c3=c3, nc=nc, nk=0)
            if kpt is not None:
                nk = kpt[0] * kpt[1]
                L.update(type="Pose", nk=nk, kpt=tuple(kpt), c4=max(chs[0] // 4, nk))
            c2 = 0
        L["cout"] = c2
        out.append(L)
        ch.append(c2)
    return out


# ---------------------------------------------------------------------------
# synthetic weights
# ---------------------------------------------------------------------------
def _he(rng, shape, gain=1.0):
    fan_in = int(np.prod(shape[1:]))
    return (rng.standard_normal(shape) * gain * np.sqrt(2.0 / fan_in)).astype(np.float32)


def _conv_init(rng, p: Params, name: str, c1: int, c2: int, k: int) -> None:
    p[name + ".conv.weight"] = _he(rng, (c2, c1, k, k))
    p[name + ".bn.weight"] = rng.uniform(0.8, 1.2, c2).astype(np.float32)
    p[name + ".bn.bias"] = (rng.standard_normal(c2) * 0.1).astype(np.float32)
    p[name + ".bn.running_mean"] = np.zeros(c2, np.float32)
    p[name + ".bn.running_var"] = np.ones(c2, np.float32)


# YOLOv8-face synthetic priors: a box ~2 strides wide and ~2.5 tall around the anchor and the
# 5 landmarks (eyes, nose, mouth corners) in strides from the anchor centre; the Pose head
# decodes x = (raw * 2 + anchor_x - 0.5) * stride, so raw = (offset + 0.5) / 2
FACE_BOX_PRIOR = (2.0, 2.5, 2.0, 2.5)
FACE_KPT_PRIOR = ((-0.7, -0.5), (0.7, -0.5), (0.0, 0.2), (-0.5, 0.9), (0.5, 0.9))


def synth_yolov8(scale: str = "n", seed: int = 0, calibrate: bool = True, target_per_image=(1.5, 0.8, 0.4),
                 nc: int = YOLO_NC, kpt: Optional[Tuple[int, int]] = None,
                 box_prior=(2.5, 4.5, 2.5, 4.5)) -> Params:
    """Seeded YOLOv8 weights (state-dict names of ultralytics' DetectionModel / PoseModel)."""
    rng = np.random.default_rng(np.random.SeedSequence([20260503, ord(scale), seed] + ([nc, 7] if kpt else [])))
    p: Params = {}
    for L in yolo_layers(scale, nc, kpt):
        nm, t = L["name"], L["type"]
        if t == "Conv":
            _conv_init(rng, p, nm, L["c1"], L["c2"], L["k"])
        elif t == "C2f":
            c = L["c2"] // 2
            _conv_init(rng, p, nm + ".cv1", L["c1"], 2 * c, 1)
            _conv_init(rng, p, nm + ".cv2", (2 + L["n"]) * c, L["c2"], 1)
            for j in range(L["n"]):
                _conv_init(rng, p, f"{nm}.m.{j}.cv1", c, c, 3)
                _conv_init(rng, p, f"{nm}.m.{j}.cv2", c, c, 3)
        elif t == "SPPF":
            c_ = L["c1"] // 2
            _conv_init(rng, p, nm + ".cv1", L["c1"], c_, 1)
            _conv_init(rng, p, nm + ".cv2", 4 * c_, L["c2"], 1)
        elif t in ("Detect", "Pose"):
            for lvl, x in enumerate(L["ch"]):
                _conv_init(rng, p, f"{nm}.cv2.{lvl}.0", x, L["c2b"], 3)
                _conv_init(rng, p, f"{nm}.cv2.{lvl}.1", L["c2b"], L["c2b"], 3)
                p[f"{nm}.cv2.{lvl}.2.weight"] = _he(rng, (4 * REG_MAX, L["c2b"], 1, 1), 0.3)
                # DFL prior: bins peaked near 2-3 strides sideways, 4-6 strides up/down (upright people)
                bins = np.arange(REG_MAX, dtype=np.float64)
                prior = []
                for mu in box_prior:
                    prior.append(-0.5 * ((bins - mu) / 1.2) ** 2)
                p[f"{nm}.cv2.{lvl}.2.bias"] = np.concatenate(prior).astype(np.float32)
                _conv_init(rng, p, f"{nm}.cv3.{lvl}.0", x, L["c3"], 3)
                _conv_init(rng, p, f"{nm}.cv3.{lvl}.1", L["c3"], L["c3"], 3)
                p[f"{nm}.cv3.{lvl}.2.weight"] = _he(rng, (L["nc"], L["c3"], 1, 1), 0.5)
                b = np.full(L["nc"], -12.0, np.float32)
                b[0] = -4.0
                p[f"{nm}.cv3.{lvl}.2.bias"] = b
                if t == "Pose":
                    _conv_init(rng, p, f"{nm}.cv4.{lvl}.0", x, L["c4"], 3)
                    _conv_init(rng, p, f"{nm}.cv4.{lvl}.1", L["c4"], L["c4"], 3)
                    p[f"{nm}.cv4.{lvl}.2.weight"] = _he(rng, (L["nk"], L["c4"], 1, 1), 0.05)
                    nkp, nd = L["kpt"]
                    kb = np.zeros((nkp, nd), np.float32)
                    for k in range(nkp):
                        dx, dy = FACE_KPT_PRIOR[k % len(FACE_KPT_PRIOR)]
                        kb[k, 0], kb[k, 1] = (dx + 0.5) / 2.0, (dy + 0.5) / 2.0
                        if nd == 3:
                            kb[k, 2] = 3.0   # visible (sigmoid 0.95)
                    p[f"{nm}.cv4.{lvl}.2.bias"] = kb.reshape(-1)
            p[nm + ".dfl.conv.weight"] = np.arange(REG_MAX, dtype=np.float32).reshape(1, REG_MAX, 1, 1)
    if calibrate:
        from .synth_calib import calibrate_yolo
        calibrate_yolo(p, scale, rng, target_per_image, nc=nc, kpt=kpt)
    return p


def synth_yolov8_face(scale: str = "l", seed: int = 0, calibrate: bool = True) -> Params:
    """Seeded YOLOv8-face weights (the reference default Y8F_DEFAULT = yolov8l-face.pt,
    face_embedder.py:33: a PoseModel, one class, kpt_shape [5, 3])."""
    return synth_yolov8(scale, seed, calibrate, target_per_image=(2.0, 1.0, 0.5), nc=1, kpt=(5, 3),
                        box_prior=FACE_BOX_PRIOR)


# ---------------------------------------------------------------------------
# compilation
# ---------------------------------------------------------------------------
def bn_fold_eps(p: Params, name: str, eps: float = YOLO_BN_EPS) -> Tuple[np.ndarray, np.ndarray]:
    g = p[name + ".weight"].astype(np.float64)
    b = p[name + ".bias"].astype(np.float64)
    m = p[name + ".running_mean"].astype(np.float64)
    v = p[name + ".running_var"].astype(np.float64)
    s = g / np.sqrt(v + eps)
    return s, b - m * s


ChanMap = List[Tuple[int, int]]   # (padded offset, true channels) segments of a tensor's channel axis


def _cols(cmap: ChanMap) -> np.ndarray:
    return np.concatenate([np.arange(o, o + n) for o, n in cmap]).astype(np.int64)


def pack_mapped(w: np.ndarray, cmap: ChanMap, cin_pad: int, npad: int,
                rows: Optional[np.ndarray] = None) -> np.ndarray:
    """[cout][cin][kh][kw] -> [npad][kh*kw*cin_pad]: true input channel i sits at the
    padded position _cols(cmap)[i], output channel o at row rows[o] (default o)."""
    cout, cin, kh, kw = w.shape
    cols = _cols(cmap)
    assert cols.size == cin, (cols.size, cin)
    rows = np.arange(cout) if rows is None else np.asarray(rows)
    t = np.zeros((npad, kh, kw, cin_pad), np.float64)
    t[rows[:, None, None, None], np.arange(kh)[None, :, None, None], np.arange(kw)[None, None, :, None],
      cols[None, None, None, :]] = np.transpose(w.astype(np.float64), (0, 2, 3, 1))
    return t.reshape(npad, kh * kw * cin_pad).astype(np.float32)


class _T:
    """A tensor of the program with its channel map."""
    __slots__ = ("t", "cmap")

    def __init__(self, t: int, cmap: ChanMap):
        self.t, self.cmap = t, cmap

    @property
    def ctrue(self) -> int:
        return sum(n for _, n in self.cmap)


def _conv(P: Program, p: Params, x: _T, name: str, c2: int, k: int, s: int, out: int, act: int = ACT_SILU,
          res: Optional[int] = None, rows: Optional[np.ndarray] = None, npad: Optional[int] = None,
          cout: Optional[int] = None, plain: bool = False) -> None:
    """ultralytics Conv (conv + BN(eps 1e-3) + SiLU, fused) or a plain biased Conv2d."""
    if plain:
        w = p[name + ".weight"].astype(np.float64)
        b = p[name + ".bias"].astype(np.float64)
    else:
        sc, b = bn_fold_eps(p, name + ".bn")
        w = p[name + ".conv.weight"].astype(np.float64) * sc[:, None, None, None]
    _, _, cin_pad = P.dims(x.t)
    npad = npad or cpad(c2)
    wp = pack_mapped(w, x.cmap, cin_pad, npad, rows)
    bias = np.zeros(npad)
    bias[np.arange(c2) if rows is None else np.asarray(rows)] = b
    P.conv(out, [(x.t, k, k, s, k // 2, x.ctrue)], wp, cout or c2, bias=bias, act=act, res=res,
           res_mode=RES_SAME, act_after_res=0, flops_cout=c2)


def compile_yolov8(p: Params, scale: str = "n", Hp: int = 384, Wp: int = 640, nc: int = YOLO_NC,
                   kpt: Optional[Tuple[int, int]] = None) -> Program:
    """YOLOv8 -> program for an Hp x Wp letterboxed canvas (NHWC4: RGB/255, channel 3 = 0).
    Outputs per stride 8/16/32: f32 [H][W][64 + nc (+ nk)] (DFL logits | class logits | raw
    keypoints of the Pose head)."""
    assert Hp % 32 == 0 and Wp % 32 == 0
    layers = yolo_layers(scale, nc, kpt)
    P = Program()
    xin = P.input_tensor(Hp, Wp, 4)
    # spatial size of every layer output
    hw: List[Tuple[int, int]] = []
    H, W = Hp, Wp
    for L in layers:
        if L["type"] == "Conv" and L["s"] == 2:
            H, W = H // 2, W // 2
        elif L["type"] == "Upsample":
            H, W = H * 2, W * 2
        elif L["type"] in ("Concat", "C2f", "SPPF", "Detect"):
            H, W = hw[L["from"][0]]
        hw.append((H, W))
    # concat buffers: producers write their slice in place
    dest: Dict[int, _T] = {}
    outs: Dict[int, _T] = {}
    for L in layers:
        if L["type"] != "Concat":
            continue
        H, W = hw[L["i"]]
        pads = [cpad(layers[j]["cout"]) for j in L["from"]]
        buf = P.act(H, W, sum(pads))
        off, cmap = 0, []
        for j, cp in zip(L["from"], pads):
            dest[j] = _T(P.view(buf, off, cp), [(0, layers[j]["cout"])])
            cmap.append((off, layers[j]["cout"]))
            off += cp
        outs[L["i"]] = _T(buf, cmap)

    def out_tensor(i: int) -> _T:
        if i in dest:
            return dest[i]
        H, W = hw[i]
        return _T(P.act(H, W, cpad(layers[i]["cout"])), [(0, layers[i]["cout"])])

    heads: List[int] = []
    for L in layers:
        i, t, nm = L["i"], L["type"], L["name"]
        H, W = hw[i]
        if t == "Concat":
            continue
        x = outs[L["from"][0]] if i > 0 else None
        if t == "Conv" and i == 0:
            y = out_tensor(i)
            sc, b = bn_fold_eps(p, nm + ".bn")
            w = p[nm + ".conv.weight"].astype(np.float64) * sc[:, None, None, None]
            w4 = np.zeros((L["c2"], 3, 3, 4))
            w4[:, :, :, :3] = np.transpose(w, (0, 2, 3, 1))
            P.stem(y.t, xin, w4, b, stride=L["s"], pad=1, act=ACT_SILU)
        elif t == "Conv":
            y = out_tensor(i)
            _conv(P, p, x, nm, L["c2"], L["k"], L["s"], y.t)
        elif t == "C2f":
            y = out_tensor(i)
            c = L["c2"] // 2
            cp = cpad(c)
            n = L["n"]
            Y = P.act(H, W, (2 + n) * cp)
            rows = np.concatenate([np.arange(c), cp + np.arange(c)])
            _conv(P, p, x, nm + ".cv1", 2 * c, 1, 1, P.view(Y, 0, 2 * cp), rows=rows, npad=2 * cp, cout=2 * cp)
            for j in range(n):
                src = _T(P.view(Y, (1 + j) * cp, cp), [(0, c)])
                t1 = _T(P.act(H, W, cp), [(0, c)])
                _conv(P, p, src, f"{nm}.m.{j}.cv1", c, 3, 1, t1.t)
                _conv(P, p, t1, f"{nm}.m.{j}.cv2", c, 3, 1, P.view(Y, (2 + j) * cp, cp),
                      res=src.t if L["shortcut"] else None)
            _conv(P, p, _T(Y, [(k * cp, c) for k in range(2 + n)]), nm + ".cv2", L["c2"], 1, 1, y.t)
        elif t == "SPPF":
            y = out_tensor(i)
            c_ = L["c1"] // 2
            cp = cpad(c_)
            Z = P.act(H, W, 4 * cp)
            _conv(P, p, x, nm + ".cv1", c_, 1, 1, P.view(Z, 0, cp))
            for j in range(3):
                P.maxpool(P.view(Z, (j + 1) * cp, cp), P.view(Z, j * cp, cp), L["k"], 1, L["k"] // 2)
            _conv(P, p, _T(Z, [(k * cp, c_) for k in range(4)]), nm + ".cv2", L["c2"], 1, 1, y.t)
        elif t == "Upsample":
            y = out_tensor(i)
            P.upsample2(y.t, x.t)
        elif t in ("Detect", "Pose"):
            c2b, c3, nc = L["c2b"], L["c3"], L["nc"]
            nk, c4 = L["nk"], L.get("c4", 0)
            bp, cp3, cp4 = cpad(c2b), cpad(c3), (cpad(c4) if nk else 0)
            for lvl, j in enumerate(L["from"]):
                xi = outs[j]
                Hl, Wl = hw[j]
                # cv2[l][0], cv3[l][0] (and cv4[l][0]) read the same input: one launch, rows [box | cls | kpt]
                branches = [("cv2", c2b, 0), ("cv3", c3, bp)] + ([("cv4", c4, bp + cp3)] if nk else [])
                h1 = P.act(Hl, Wl, bp + cp3 + cp4)
                ws, bs, rows = [], [], []
                for br, cw, off in branches:
                    sb, bb = bn_fold_eps(p, f"{nm}.{br}.{lvl}.0.bn")
                    ws.append(p[f"{nm}.{br}.{lvl}.0.conv.weight"].astype(np.float64) * sb[:, None, None, None])
                    bs.append(bb)
                    rows.append(off + np.arange(cw))
                rows = np.concatenate(rows)
                _, _, cin_pad = P.dims(xi.t)
                wp = pack_mapped(np.concatenate(ws, axis=0), xi.cmap, cin_pad, bp + cp3 + cp4, rows)
                bias = np.zeros(bp + cp3 + cp4)
                bias[rows] = np.concatenate(bs)
                P.conv(h1, [(xi.t, 3, 3, 1, 1, xi.ctrue)], wp, bp + cp3 + cp4, bias=bias, act=ACT_SILU,
                       flops_cout=c2b + c3 + (c4 if nk else 0))
                ctot = 4 * REG_MAX + nc + nk
                o = P.act(Hl, Wl, cpad(ctot), is_f32=1)
                # second conv of each branch, then its plain 1x1 into the output slice
                offs = [0, 4 * REG_MAX, 4 * REG_MAX + nc]
                outs_c = [4 * REG_MAX, nc, nk]
                for (br, cw, off), oo, oc in zip(branches, offs, outs_c):
                    cwp = cpad(cw)
                    hin = _T(P.view(h1, off, cwp), [(0, cw)])
                    h2 = _T(P.act(Hl, Wl, cwp), [(0, cw)])
                    _conv(P, p, hin, f"{nm}.{br}.{lvl}.1", cw, 3, 1, h2.t)
                    width = cpad(ctot) - oo if br != "cv2" else 4 * REG_MAX
                    _conv(P, p, h2, f"{nm}.{br}.{lvl}.2", oc, 1, 1, P.view(o, oo, width), act=ACT_NONE, plain=True)
                heads.append(P.view(o, 0, ctot))
            continue
        outs[i] = y
    P.outputs = heads
    return P


# ---------------------------------------------------------------------------
# host geometry: ultralytics LetterBox (auto, stride 32) and scale_boxes
# ---------------------------------------------------------------------------
def letterbox_geometry(H: int, W: int, imgsz: int = 640, stride: int = 32, auto: bool = True):
    """[ext] ultralytics LetterBox.__call__ (center=True, scaleup=True): returns
    (new_w, new_h, top, left, Hp, Wp)."""
    r = min(imgsz / H, imgsz / W)
    new_w, new_h = int(round(W * r)), int(round(H * r))
    dw, dh = imgsz - new_w, imgsz - new_h
    if auto:
        dw, dh = dw % stride, dh % stride
    dw /= 2
    dh /= 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return new_w, new_h, top, left, new_h + top + bottom, new_w + left + right


def scale_geometry(Hp: int, Wp: int, H: int, W: int) -> Tuple[float, int, int]:
    """[ext] ultralytics ops.scale_boxes: gain and (pad_x, pad_y)."""
    gain = min(Hp / H, Wp / W)
    pad_x = round((Wp - W * gain) / 2 - 0.1)
    pad_y = round((Hp - H * gain) / 2 - 0.1)
    return gain, int(pad_x), int(pad_y)
