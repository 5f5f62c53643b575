"""Which IResNet convs must run split (f16x3) for the embedding to stay within 1e-4 of fp32?
CPU emulation of the device's folded program (pc_api.cpp IResNet program: folded weights,
f32 accumulation) where each storage / operand site is either f16 (one rounding) or split
(hi + lo f16 = 22 significant bits, emulated as f32). Sites per block: the residual stream
(`stream`: the tensor conv2's epilogue writes and the next block's conv1 / residual / shortcut
read), conv1's operand read of the stream (`in1`: hi only, or hi + lo = one extra MFMA term),
conv1's weights (`w1`), the intermediate (`y1`), conv2's weights (`w2`), the shortcut weights
(`wd`); net sites: stem weights / output, FC input / weights. Stages 1-4 = the 56/28/14/7 maps.
Metric: flip-TTA embeddings vs the fp32 oracle (1-cos, max |component|) and fd against a
planted bank like bench.plant_bank; plus the f16c8 program (emu_c8). usage:
python tools/emu_mixed_iresnet.py [n_chips] ["variant;variant"]"""
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import torch
import torch.nn.functional as F

from oracle.nets_torch import BN_EPS, arcface_input_from_chips, iresnet_forward
from person_capture_amd import models

SITES = ("x", "stem_w", "stem_out", "stream", "in1", "w1", "y1", "w2", "wd", "fc_in", "fc_w")


def bnf(p, name):
    s = p[name + ".weight"] / np.sqrt(p[name + ".running_var"] + BN_EPS)
    return s, p[name + ".bias"] - p[name + ".running_mean"] * s


def stage_of(pre):
    return int(pre.split(".")[0][5:])


def emu_forward(p, depth, x, split):
    """split(site, stage) -> True when that site is split (f32 class) at that stage (0 = stem,
    5 = FC)."""
    r16 = lambda t: t.half().float()
    R = lambda site, st, t: t if split(site, st) else r16(t)
    W = lambda site, st, a: R(site, st, torch.from_numpy(a.astype(np.float32)))
    T = lambda k: torch.from_numpy(p[k].astype(np.float32))
    c = lambda a: torch.from_numpy(np.asarray(a, np.float32))[None, :, None, None]
    with torch.no_grad():
        s, b = bnf(p, "bn1")
        w = p["conv1.weight"] * s[:, None, None, None]
        t = F.prelu(F.conv2d(R("x", 0, x), W("stem_w", 0, w), padding=1) + c(b), T("prelu.weight"))
        t = R("stem_out", 0, t)
        for pre, inp, pl, stride, ds in models.iresnet_blocks(depth):
            st = stage_of(pre)
            s1, b1 = bnf(p, pre + ".bn1")
            s2, b2 = bnf(p, pre + ".bn2")
            W1 = p[pre + ".conv1.weight"]
            w1f = W1 * s1[None, :, None, None] * s2[:, None, None, None]
            tin = R("in1", st, t)
            ones = torch.ones((1, inp) + tuple(t.shape[2:]))
            tab = F.conv2d(ones * c(b1), torch.from_numpy(W1.astype(np.float32)), padding=1)
            tab = tab * c(s2) + c(b2)
            y1 = F.conv2d(tin, W("w1", st, w1f), padding=1) + tab
            y1 = R("y1", st, F.prelu(y1, T(pre + ".prelu.weight")))
            s3, b3 = bnf(p, pre + ".bn3")
            w2f = p[pre + ".conv2.weight"] * s3[:, None, None, None]
            o = F.conv2d(y1, W("w2", st, w2f), stride=stride, padding=1) + c(b3)
            if ds:
                sd, bd = bnf(p, pre + ".downsample.1")
                wdf = p[pre + ".downsample.0.weight"] * sd[:, None, None, None]
                o = o + F.conv2d(tin, W("wd", st, wdf), stride=stride) + c(bd)
            else:
                o = o + t
            t = R("stream", st, o)
        s2, b2 = bnf(p, "bn2")
        sf, bf = bnf(p, "features")
        Wfc = p["fc.weight"].reshape(-1, 512, 7, 7)
        wf = Wfc * s2[None, :, None, None] * sf[:, None, None, None]
        bias = sf * (np.einsum("ochw,c->o", Wfc, b2) + p["fc.bias"]) + bf
        e = F.conv2d(R("fc_in", 5, t), W("fc_w", 5, wf)).flatten(1) + \
            torch.from_numpy(bias.astype(np.float32))
    return e


def q8(t):
    """e4m3 (OCP e4m3fn) with one power-of-two scale per tensor putting its max in [224, 448)."""
    m = t.abs().max().clamp_min(1e-30)
    e = torch.floor(torch.log2(448.0 / m))
    return (t * 2 ** e).to(torch.float8_e4m3fn).float() * 2 ** (-e)


def emu_c8(p, depth, x):
    """The f16c8 program: every activation stored as f16 hi + e4m3 lo, every conv
    x_hi*W_hi (f16 operands, f32 accumulate) + q8(x_lo)*q8(W_hi) + q8(x_hi)*q8(W_lo); exact
    centred input; FC input kept split (f32 class)."""
    def conv(t, w, **kw):
        th = t.half().float()
        wh = w.half().float()
        return F.conv2d(th, wh, **kw) + F.conv2d(q8(t - th), q8(wh), **kw) + F.conv2d(q8(th), q8(w - wh), **kw)

    def store(t):
        h = t.half().float()
        return h + q8(t - h)
    T = lambda k: torch.from_numpy(p[k].astype(np.float32))
    c = lambda a: torch.from_numpy(np.asarray(a, np.float32))[None, :, None, None]
    W = lambda a: torch.from_numpy(a.astype(np.float32))
    with torch.no_grad():
        s, b = bnf(p, "bn1")
        t = store(F.prelu(F.conv2d(x, W(p["conv1.weight"] * s[:, None, None, None]), padding=1) + c(b),
                          T("prelu.weight")))
        for pre, inp, pl, stride, ds in models.iresnet_blocks(depth):
            s1, b1 = bnf(p, pre + ".bn1")
            s2, b2 = bnf(p, pre + ".bn2")
            W1 = p[pre + ".conv1.weight"]
            ones = torch.ones((1, inp) + tuple(t.shape[2:]))
            tab = F.conv2d(ones * c(b1), W(W1), padding=1) * c(s2) + c(b2)
            y1 = store(F.prelu(conv(t, W(W1 * s1[None, :, None, None] * s2[:, None, None, None]), padding=1) + tab,
                               T(pre + ".prelu.weight")))
            s3, b3 = bnf(p, pre + ".bn3")
            o = conv(y1, W(p[pre + ".conv2.weight"] * s3[:, None, None, None]), stride=stride, padding=1) + c(b3)
            if ds:
                sd, bd = bnf(p, pre + ".downsample.1")
                o = o + conv(t, W(p[pre + ".downsample.0.weight"] * sd[:, None, None, None]), stride=stride) + c(bd)
            else:
                o = o + t
            t = store(o)
        s2, b2 = bnf(p, "bn2")
        sf, bf = bnf(p, "features")
        Wfc = p["fc.weight"].reshape(-1, 512, 7, 7)
        wf = Wfc * s2[None, :, None, None] * sf[:, None, None, None]
        bias = sf * (np.einsum("ochw,c->o", Wfc, b2) + p["fc.bias"]) + bf
        return F.conv2d(t, W(wf)).flatten(1) + torch.from_numpy(bias.astype(np.float32))


def tta(fwd, chips):
    x = arcface_input_from_chips(chips)
    e = fwd(x) + fwd(torch.flip(x, dims=[3]))
    return (e / e.norm(dim=1, keepdim=True)).numpy()


def rule(sites=(), stages=(0, 1, 2, 3, 4, 5)):
    sites, stages = set(sites), set(stages)
    return lambda site, st: site in sites and st in stages


BLK = ["stream", "in1", "y1", "w1", "w2", "wd"]
NET = ["x", "stem_w", "stem_out", "fc_in", "fc_w"]
VARIANTS = {
    "acts split, weights f16 (2 MFMA)": rule(["x", "stem_out", "stream", "in1", "y1", "fc_in"]),
    "weights split, acts f16 (2 MFMA)": rule(["x", "stem_w", "w1", "w2", "wd", "fc_w"]),
    "x3 all but y1 (conv2 2 MFMA)": rule(NET + ["stream", "in1", "w1", "w2", "wd"]),
    "net sites only": rule(NET),
    "net + stream": rule(NET + ["stream"]),
    "net + stream+in1": rule(NET + ["stream", "in1"]),
    "net + stream+in1+w1+wd": rule(NET + ["stream", "in1", "w1", "wd"]),
    "net + stream+in1+w1+w2+wd": rule(NET + ["stream", "in1", "w1", "w2", "wd"]),
    "net + blk stages 1": lambda s, st: s in NET or (s in BLK and st in (1,)),
    "net + blk stages 1,2": lambda s, st: s in NET or (s in BLK and st in (1, 2)),
    "net + blk stages 1,2,4": lambda s, st: s in NET or (s in BLK and st in (1, 2, 4)),
    "net + blk stages 1,2 + stream": lambda s, st: s in NET or s == "stream" or (s in BLK and st in (1, 2)),
    "net + blk stages 1,2 + stream+in1": lambda s, st: s in NET or s in ("stream", "in1") or (s in BLK and st in (1, 2)),
    "net + blk 1,2,4 + stream+in1": lambda s, st: s in NET or s in ("stream", "in1") or (s in BLK and st in (1, 2, 4)),

    # round 6: one operand of the 14x14x256 stage (stage 3: 58 of the 100 convs, 46 % of the x3 time)
    # in f16 (2 MFMAs per product there), everything else split
    "all split but w1,w2 at st3": lambda s, st: not (s in ("w1", "w2") and st == 3),
    "all split but w2 at st3": lambda s, st: not (s == "w2" and st == 3),
    "all split but w1 at st3": lambda s, st: not (s == "w1" and st == 3),
    "all split but y1 at st3": lambda s, st: not (s == "y1" and st == 3),
    "all split but in1 at st3": lambda s, st: not (s == "in1" and st == 3),
    "all split but y1 at st2,3": lambda s, st: not (s == "y1" and st in (2, 3)),
    "all split": lambda s, st: True,
    "f16": rule(),
    "stream": rule(["stream"]),
    "stream+in1": rule(["stream", "in1"]),
    "stream+w1+w2+wd": rule(["stream", "w1", "w2", "wd"]),
    "stream+in1+w1+w2+wd": rule(["stream", "in1", "w1", "w2", "wd"]),
    "stream+in1+y1+w1+w2+wd (x3 all)": rule(["stream", "in1", "y1", "w1", "w2", "wd"]),
    "all sites split": rule(SITES),
    "stream+fc": rule(["stream", "fc_in", "fc_w"]),
    "stream+in1+fc": rule(["stream", "in1", "fc_in", "fc_w"]),
    "stream+in1+w1+wd+fc": rule(["stream", "in1", "w1", "wd", "fc_in", "fc_w"]),
    "stream+in1+w1+w2+wd+fc": rule(["stream", "in1", "w1", "w2", "wd", "fc_in", "fc_w"]),
}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    only = sys.argv[2].split(";") if len(sys.argv) > 2 else None
    depth = 100
    torch.set_num_threads(8)
    p = {k: v.astype(np.float64) if v.dtype == np.float32 else v
         for k, v in models.synth_iresnet(depth, seed=0).items()}
    p32 = {k: v.astype(np.float32) for k, v in p.items()}
    chips = np.random.default_rng(7).integers(0, 256, (n, 112, 112, 3), dtype=np.uint8)
    ref = tta(lambda x: iresnet_forward(p32, depth, x), chips)
    rng = np.random.default_rng(1)
    mean = ref.mean(0)
    bank = []
    for k in range(8):
        v = ref[k % n] - 0.3 * mean + (0.1 + 0.1 * k) * rng.standard_normal(512) / np.sqrt(512.0)
        bank.append(v / np.linalg.norm(v))
    bank = np.array(bank, np.float32)
    fd = lambda e: (1.0 - e @ bank.T).min(1)
    fd_ref = fd(ref)
    runs = [(k, (lambda x, fn=fn: emu_forward(p, depth, x, fn))) for k, fn in VARIANTS.items()]
    runs.append(("f16c8 (e4m3 corrections, lo stored e4m3)", lambda x: emu_c8(p, depth, x)))
    for name, fwd in runs:
        if only and not any(o == name for o in only):
            continue
        e = tta(fwd, chips)
        d = np.abs(fd(e) - fd_ref)
        nd = np.linalg.norm(e.astype(np.float64) - ref, axis=1)
        print(f"{name:34s}: |dfd| med {np.median(d):.2e} max {d.max():.2e}; |de|max "
              f"{np.abs(e - ref).max():.2e}; ||de|| med {np.median(nd):.2e} max {nd.max():.2e}",
              flush=True)


if __name__ == "__main__":
    main()
