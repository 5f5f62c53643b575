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
