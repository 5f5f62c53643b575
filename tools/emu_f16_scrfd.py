"""Where does SCRFD-10G's f16 landmark error enter? CPU emulation: every conv of the fp32
oracle (oracle/nets_torch.scrfd_forward) reads its input and weights rounded to f16 (the
device's f16 storage and weights, f32 accumulation), except the convs of one group kept in
f32. Metric: landmark/box regression error in pixels (x stride) at the anchors whose face
score passes 0.5, against the fp32 oracle. usage: python tools/emu_f16_scrfd.py [D]"""
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import torch
import torch.nn.functional as F

from oracle import nets_torch as nt
from person_capture_amd import models

_conv = F.conv2d


def _split(t):
    hi = t.half().float()
    return hi, (t - hi).half().float()


def run(p, x, keep32=lambda i: False, w16=True, a16=True, x3=False, w2=False, x3sel=None):
    i = [0]

    def conv(inp, w, b=None, *a, **k):
        j = i[0]
        i[0] += 1
        if x3 or (x3sel is not None and x3sel(j)):   # f16x3: hi*hi + lo*hi + hi*lo, f32 accumulation
            xh, xl = _split(inp)
            wh, wl = _split(w)
            return _conv(xh, wh, b, *a, **k) + _conv(xl, wh, None, *a, **k) + _conv(xh, wl, None, *a, **k)
        if w2:   # weights hi + lo, activations stored f16: x16*W_hi + x16*W_lo (2x K)
            xh = inp.half().float()
            wh, wl = _split(w)
            return _conv(xh, wh, b, *a, **k) + _conv(xh, wl, None, *a, **k)
        if not keep32(j):
            if a16:
                inp = inp.half().float()
            if w16:
                w = w.half().float()
        return _conv(inp, w, b, *a, **k)

    nt.F.conv2d = conv
    try:
        return nt.scrfd_forward(p, "10g", x), i[0]
    finally:
        nt.F.conv2d = _conv


def main():
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 640
    torch.set_num_threads(8)
    p = models.synth_scrfd("10g", seed=0) if hasattr(models, "synth_scrfd") else None
    img = np.random.default_rng(3).integers(0, 256, (D, D, 3), dtype=np.uint8)
    x = torch.from_numpy(((img[..., ::-1].astype(np.float32) - 127.5) / 128.0).transpose(2, 0, 1).copy())[None]
    ref, n = run(p, x, keep32=lambda i: True)
    print(f"{n} convs", flush=True)
    strides = (8, 16, 32)

    def err(out):
        e = []
        for s, r, o in zip(strides, ref, out):
            m = torch.sigmoid(r[..., 0:2]).amax(-1) > 0.5
            if m.any():
                e.append((o[..., 2:30][m] - r[..., 2:30][m]).abs().amax(-1) * s)
        e = torch.cat(e)
        return f"anchors {len(e)}  |d reg/kps| px median {e.median():.4f} p90 {e.quantile(0.9):.4f} max {e.max():.4f}"

    # conv index groups in scrfd_forward order: 3 stem, backbone blocks, neck, heads
    nb = len(models.scrfd_blocks(models.SCRFD_CFG["10g"]))
    nds = sum(1 for b in models.scrfd_blocks(models.SCRFD_CFG["10g"]) if b[4])
    bb_end = 3 + 2 * nb + nds
    neck_end = bb_end + 3 + 3 + 2 + 2
    groups = {"all f16": lambda i: False, "stem f32": lambda i: i < 3, "backbone f32": lambda i: i < bb_end,
              "first half backbone f32": lambda i: i < (3 + bb_end) // 2,
              "neck f32": lambda i: bb_end <= i < neck_end, "heads f32": lambda i: i >= neck_end}
    for name, k in groups.items():
        out, _ = run(p, x, keep32=k)
        print(f"{name:26s}: {err(out)}", flush=True)
    out, _ = run(p, x, w16=False)
    print(f"{'activations only f16':26s}: {err(out)}", flush=True)
    out, _ = run(p, x, a16=False)
    print(f"{'weights only f16':26s}: {err(out)}", flush=True)
    out, _ = run(p, x, w2=True)
    print(f"{'f16 acts, W hi+lo (2x K)':26s}: {err(out)}", flush=True)
    out, _ = run(p, x, x3=True)
    print(f"{'f16x3 (hi/lo split)':26s}: {err(out)}", flush=True)
    # mixed programs (r04): f16x3 on one group, plain f16 storage/weights elsewhere
    mixed = {"x3 stem+backbone": lambda i: i < bb_end, "x3 backbone+neck": lambda i: i < neck_end,
             "x3 all but heads": lambda i: i < neck_end, "x3 all but stem": lambda i: i >= 3,
             "x3 heads+neck": lambda i: i >= bb_end, "x3 2nd half bb+": lambda i: i >= (3 + bb_end) // 2}
    for name, k in mixed.items():
        out, _ = run(p, x, x3sel=k)
        print(f"{name:26s}: {err(out)}", flush=True)


if __name__ == "__main__":
    main()
