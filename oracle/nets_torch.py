"""fp32 CPU forward passes of the conv networks (test infrastructure only).

Written directly from the architectures the reference loads (no folding, no
fusion): the GPU programs in person_capture_amd/models.py apply BN folding,
border bias tables, avg-down rewrites and segment fusion, and the parity tests
check them against these literal forwards.
  * IResNet: insightface arcface_torch iresnet.py (glintr100 / w600k_r50, loaded
    at person_capture/face_embedder.py:68-83, 729-734)
  * SCRFD: insightface/detection/scrfd (mmdet ResNetV1e + PAFPN + SCRFDHead),
    the scrfd_*_bnkps.onnx graphs loaded at face_embedder.py:55-65, 1102-1147
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


def _bn(p, name, x):
    T = lambda k: torch.from_numpy(p[name + k])
    return F.batch_norm(x, T(".running_mean"), T(".running_var"), T(".weight"), T(".bias"), False, 0.0, BN_EPS)


def iresnet_forward(p, depth, x_nchw: torch.Tensor) -> torch.Tensor:
    """x: [N,3,112,112] float32 (RGB, x/127.5-1). Returns raw embeddings [N,512]."""
    from person_capture_amd.models import iresnet_blocks  # block table only (names/strides)
    T = lambda k: torch.from_numpy(p[k])
    with torch.no_grad():
        x = F.conv2d(x_nchw, T("conv1.weight"), stride=1, padding=1)
        x = F.prelu(_bn(p, "bn1", x), T("prelu.weight"))
        for pre, inp, pl, stride, ds in iresnet_blocks(depth):
            identity = x
            out = _bn(p, pre + ".bn1", x)
            out = F.conv2d(out, T(pre + ".conv1.weight"), stride=1, padding=1)
            out = _bn(p, pre + ".bn2", out)
            out = F.prelu(out, T(pre + ".prelu.weight"))
            out = F.conv2d(out, T(pre + ".conv2.weight"), stride=stride, padding=1)
            out = _bn(p, pre + ".bn3", out)
            if ds:
                identity = _bn(p, pre + ".downsample.1", F.conv2d(x, T(pre + ".downsample.0.weight"), stride=stride))
            x = out + identity
        x = _bn(p, "bn2", x)
        x = torch.flatten(x, 1)
        x = F.linear(x, T("fc.weight"), T("fc.bias"))
        x = F.batch_norm(x, T("features.running_mean"), T("features.running_var"), T("features.weight"),
                         T("features.bias"), False, 0.0, BN_EPS)
    return x


def arcface_input_from_chips(chips_bgr_u8: np.ndarray) -> torch.Tensor:
    """face_embedder.py:1281-1288: BGR->RGB, astype(float32)/127.5 - 1.0, HWC->CHW."""
    rgb = chips_bgr_u8[..., ::-1]
    arr = rgb.astype(np.float32) / 127.5 - 1.0
    return torch.from_numpy(np.ascontiguousarray(np.transpose(arr, (0, 3, 1, 2))))


def scrfd_forward(p, variant, x_nchw: torch.Tensor):
    """x: [N,3,D,D] float32 blob ((x-127.5)/128, RGB). Returns per stride (8,16,32) the
    raw head tensors [N,H,W,30] = cls logits(2) | bbox(8) | kps(20) (channel order of
    the ONNX outputs after permute(0,2,3,1))."""
    from person_capture_amd.models import SCRFD_CFG, SCRFD_STRIDES, scrfd_blocks
    cfg = SCRFD_CFG[variant]
    T = lambda k: torch.from_numpy(p[k])
    with torch.no_grad():
        x = F.relu(_bn(p, "backbone.stem.1", F.conv2d(x_nchw, T("backbone.stem.0.weight"), stride=2, padding=1)))
        x = F.relu(_bn(p, "backbone.stem.4", F.conv2d(x, T("backbone.stem.3.weight"), padding=1)))
        x = F.relu(_bn(p, "backbone.stem.7", F.conv2d(x, T("backbone.stem.6.weight"), padding=1)))
        x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
        blocks = scrfd_blocks(cfg)
        outs = []
        for i, (pre, inp, pl, stride, ds) in enumerate(blocks):
            identity = x
            out = F.relu(_bn(p, pre + ".bn1", F.conv2d(x, T(pre + ".conv1.weight"), stride=stride, padding=1)))
            out = _bn(p, pre + ".bn2", F.conv2d(out, T(pre + ".conv2.weight"), padding=1))
            if ds:
                y = x
                if stride > 1:
                    y = F.avg_pool2d(x, kernel_size=stride, stride=stride, ceil_mode=True, count_include_pad=False)
                identity = _bn(p, pre + ".downsample.2", F.conv2d(y, T(pre + ".downsample.1.weight")))
            x = F.relu(out + identity)
            if i + 1 == len(blocks) or blocks[i + 1][0].split(".")[1] != pre.split(".")[1]:
                outs.append(x)
        inputs = outs[1:]
        conv = lambda t, nm, s=1, pad=0: F.conv2d(t, T(nm + ".weight"), T(nm + ".bias"), stride=s, padding=pad)
        laterals = [conv(inputs[i], f"neck.lateral_convs.{i}.conv") for i in range(3)]
        for i in range(2, 0, -1):
            laterals[i - 1] = laterals[i - 1] + F.interpolate(laterals[i], size=laterals[i - 1].shape[2:],
                                                              mode="nearest")
        inter = [conv(laterals[i], f"neck.fpn_convs.{i}.conv", 1, 1) for i in range(3)]
        for i in range(2):
            inter[i + 1] = inter[i + 1] + conv(inter[i], f"neck.downsample_convs.{i}.conv", 2, 1)
        neck = [inter[0]] + [conv(inter[i], f"neck.pafpn_convs.{i - 1}.conv", 1, 1) for i in range(1, 3)]
        res = []
        for lvl, s in enumerate(SCRFD_STRIDES):
            h = neck[lvl]
            for j in range(cfg["stacked"]):
                h = F.relu(_bn(p, f"bbox_head.{s}.stack.{j}.bn",
                               F.conv2d(h, T(f"bbox_head.{s}.stack.{j}.conv.weight"), padding=1)))
            cls = conv(h, f"bbox_head.{s}.cls", 1, 1)
            reg = conv(h, f"bbox_head.{s}.reg", 1, 1)
            kps = conv(h, f"bbox_head.{s}.kps", 1, 1)
            res.append(torch.cat([cls, reg, kps], dim=1).permute(0, 2, 3, 1).contiguous())
    return res


def yolov8_forward(p, scale, x_nchw: torch.Tensor, nc: int = 80, kpt=None):
    """YOLOv8 DetectionModel forward, unfused (Conv2d -> BatchNorm2d(eps 1e-3) -> SiLU), the
    module semantics of [ext] ultralytics 8.3.205 nn/modules (Conv, C2f, Bottleneck, SPPF,
    Concat, nn.Upsample, Detect) that detectors.py:271-296 runs. x: [N,3,H,W] RGB/255.
    Returns per stride (8,16,32) the raw Detect tensors [N,H,W,64+nc] = cat(cv2, cv3); with
    kpt = (nkpt, ndim) the Pose head's [N,H,W,64+nc+nkpt*ndim] = cat(cv2, cv3, cv4) (raw
    keypoints, decoded by ref_algos.yolo_postprocess)."""
    from person_capture_amd.models_yolo import YOLO_BN_EPS, yolo_layers  # layer table only
    T = lambda k: torch.from_numpy(p[k])

    def conv(t, name, k, s=1):
        y = F.conv2d(t, T(name + ".conv.weight"), stride=s, padding=k // 2)
        y = F.batch_norm(y, T(name + ".bn.running_mean"), T(name + ".bn.running_var"), T(name + ".bn.weight"),
                         T(name + ".bn.bias"), False, 0.0, YOLO_BN_EPS)
        return F.silu(y)

    with torch.no_grad():
        ys = []
        res = None
        for L in yolo_layers(scale, nc, kpt):
            t, nm = L["type"], L["name"]
            xi = ys[L["from"][0]] if L["i"] > 0 else x_nchw
            if t == "Conv":
                y = conv(xi, nm, L["k"], L["s"])
            elif t == "C2f":
                parts = list(conv(xi, nm + ".cv1", 1).chunk(2, 1))
                for j in range(L["n"]):
                    h = conv(conv(parts[-1], f"{nm}.m.{j}.cv1", 3), f"{nm}.m.{j}.cv2", 3)
                    parts.append(parts[-1] + h if L["shortcut"] else h)
                y = conv(torch.cat(parts, 1), nm + ".cv2", 1)
            elif t == "SPPF":
                parts = [conv(xi, nm + ".cv1", 1)]
                for _ in range(3):
                    parts.append(F.max_pool2d(parts[-1], kernel_size=L["k"], stride=1, padding=L["k"] // 2))
                y = conv(torch.cat(parts, 1), nm + ".cv2", 1)
            elif t == "Upsample":
                y = F.interpolate(xi, scale_factor=2.0, mode="nearest")
            elif t == "Concat":
                y = torch.cat([ys[j] for j in L["from"]], 1)
            else:
                res = []
                for lvl, j in enumerate(L["from"]):
                    b = conv(conv(ys[j], f"{nm}.cv2.{lvl}.0", 3), f"{nm}.cv2.{lvl}.1", 3)
                    b = F.conv2d(b, T(f"{nm}.cv2.{lvl}.2.weight"), T(f"{nm}.cv2.{lvl}.2.bias"))
                    c = conv(conv(ys[j], f"{nm}.cv3.{lvl}.0", 3), f"{nm}.cv3.{lvl}.1", 3)
                    c = F.conv2d(c, T(f"{nm}.cv3.{lvl}.2.weight"), T(f"{nm}.cv3.{lvl}.2.bias"))
                    parts = [b, c]
                    if L.get("nk"):
                        k = conv(conv(ys[j], f"{nm}.cv4.{lvl}.0", 3), f"{nm}.cv4.{lvl}.1", 3)
                        parts.append(F.conv2d(k, T(f"{nm}.cv4.{lvl}.2.weight"), T(f"{nm}.cv4.{lvl}.2.bias")))
                    res.append(torch.cat(parts, 1).permute(0, 2, 3, 1).contiguous())
                y = None
            ys.append(y)
    return res


def clip_vit_forward(p, name, x_nchw: torch.Tensor) -> torch.Tensor:
    """open_clip VisionTransformer.forward (no attn-pool, class-token pooling) + proj, as
    ReIDEmbedder.extract runs encode_image (reid_embedder.py:52-54; [ext] open-clip-torch
    3.2.0 transformer.py). x: [N,3,224,224] normalised. Returns [N,out] (before F.normalize)."""
    from person_capture_amd.models_clip import LN_EPS, clip_cfg   # config table only
    c = clip_cfg(name)
    T = lambda k: torch.from_numpy(p[k])
    w, heads = c["width"], c["heads"]
    d = w // heads
    with torch.no_grad():
        x = F.conv2d(x_nchw, T("visual.conv1.weight"), stride=c["patch"])          # [N,w,g,g]
        x = x.reshape(x.shape[0], w, -1).permute(0, 2, 1)                            # [N,g*g,w]
        cls = T("visual.class_embedding").view(1, 1, w).expand(x.shape[0], 1, w)
        x = torch.cat([cls, x], dim=1) + T("visual.positional_embedding")[None]
        x = F.layer_norm(x, (w,), T("visual.ln_pre.weight"), T("visual.ln_pre.bias"), LN_EPS)
        N, Tn, _ = x.shape
        for i in range(c["layers"]):
            pre = f"visual.transformer.resblocks.{i}"
            y = F.layer_norm(x, (w,), T(pre + ".ln_1.weight"), T(pre + ".ln_1.bias"), LN_EPS)
            qkv = F.linear(y, T(pre + ".attn.in_proj_weight"), T(pre + ".attn.in_proj_bias"))
            q, k, v = (qkv[..., j * w:(j + 1) * w].reshape(N, Tn, heads, d).transpose(1, 2) for j in range(3))
            a = torch.softmax((q @ k.transpose(-1, -2)) / np.sqrt(d), dim=-1) @ v
            a = a.transpose(1, 2).reshape(N, Tn, w)
            x = x + F.linear(a, T(pre + ".attn.out_proj.weight"), T(pre + ".attn.out_proj.bias"))
            y = F.layer_norm(x, (w,), T(pre + ".ln_2.weight"), T(pre + ".ln_2.bias"), LN_EPS)
            h = F.gelu(F.linear(y, T(pre + ".mlp.c_fc.weight"), T(pre + ".mlp.c_fc.bias")))
            x = x + F.linear(h, T(pre + ".mlp.c_proj.weight"), T(pre + ".mlp.c_proj.bias"))
        pooled = F.layer_norm(x[:, 0], (w,), T("visual.ln_post.weight"), T("visual.ln_post.bias"), LN_EPS)
        return pooled @ T("visual.proj")


def clip_preprocess_pil(bgr_u8: np.ndarray, side: int = 224) -> torch.Tensor:
    """reid_embedder.py:46-50 with the reference's own image stack: cv2.cvtColor(BGR2RGB)
    (a channel reversal), PIL.Image.fromarray, then the open_clip 'shortest' transform =
    torchvision Resize(side, BICUBIC) on PIL (Pillow Image.resize), CenterCrop(side),
    ToTensor, Normalize(OPENAI mean/std). Pillow is the real library here (pinned)."""
    from PIL import Image
    rgb = np.ascontiguousarray(bgr_u8[..., ::-1])
    h, w = rgb.shape[:2]
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = side, int(side * long / short)
    rw, rh = (new_short, new_long) if w <= h else (new_long, new_short)
    img = Image.fromarray(rgb)
    if (rw, rh) != (w, h):
        img = img.resize((rw, rh), Image.BICUBIC)
    top = int(round((rh - side) / 2.0))
    left = int(round((rw - side) / 2.0))
    img = img.crop((left, top, left + side, top + side))
    t = torch.from_numpy(np.array(img, np.uint8)).permute(2, 0, 1).contiguous().float().div(255)
    mean = torch.tensor([0.48145466, 0.4578275, 0.40821073], dtype=torch.float32).view(3, 1, 1)
    std = torch.tensor([0.26862954, 0.26130258, 0.27577711], dtype=torch.float32).view(3, 1, 1)
    return t.sub(mean).div(std)


def clip_patch_matrix(x_chw: torch.Tensor, patch: int = 14, kpad: int = 608) -> np.ndarray:
    """[3,224,224] -> the device input layout [1][257][kpad]: row 1 + py*g + px holds the
    patch in (kh, kw, c) order; row 0 and the padding columns are zero."""
    c, H, W = x_chw.shape
    g = H // patch
    a = x_chw.numpy().reshape(c, g, patch, g, patch).transpose(1, 3, 2, 4, 0).reshape(g * g, patch * patch * c)
    out = np.zeros((1, g * g + 1, kpad), np.float32)
    out[0, 1:, :a.shape[1]] = a
    return out
