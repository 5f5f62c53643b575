"""Where does the f16 IResNet's error enter? CPU emulation of the device's folded f16
compute (pc_api.cpp IResNet program: folded weights in f16, f32 accumulation, f16 storage
of every activation) against the fp32 oracle (oracle/nets_torch.iresnet_forward), with
one storage choice changed at a time. Inputs: u8 noise chips (the bench's frames are u8
noise, so its face chips are too); metric: the flip-TTA embedding's fd against a planted
bank built like bench.plant_bank. usage: python tools/emu_f16_iresnet.py [n_chips] [depth]"""
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import numpy as np
import torch
import torch.nn.functional as F

from oracle.nets_torch import BN_EPS, arcface_input_from_chips, iresnet_forward
from person_capture_amd import models


def bnf(p, name):
    s = p[name + ".weight"] / np.sqrt(p[name + ".running_var"] + BN_EPS)
    return s, p[name + ".bias"] - p[name + ".running_mean"] * s


def emu_forward(p, depth, x, act16=True, w16=True, res32=False, y1_32=False):
    r = (lambda t: t.half().float()) if act16 else (lambda t: t)
    rw = (lambda a: torch.from_numpy(a.astype(np.float32)).half().float()) if w16 else \
        (lambda a: torch.from_numpy(a.astype(np.float32)))
    T = lambda k: torch.from_numpy(p[k].astype(np.float32))
    c = lambda a: torch.from_numpy(np.asarray(a, np.float32))[None, :, None, None]
    with torch.no_grad():
        s, b = bnf(p, "bn1")
        w = p["conv1.weight"] * s[:, None, None, None]
        t = F.prelu(F.conv2d(r(x), rw(w), padding=1) + c(b), T("prelu.weight"))
        t = r(t)
        for pre, inp, pl, stride, ds in models.iresnet_blocks(depth):
            s1, b1 = bnf(p, pre + ".bn1")
            s2, b2 = bnf(p, pre + ".bn2")
            W1 = p[pre + ".conv1.weight"]
            w1f = W1 * s1[None, :, None, None] * s2[:, None, None, None]
            tin = r(t)
            ones = torch.ones((1, inp) + tuple(t.shape[2:]))
            tab = F.conv2d(ones * c(b1),
                           torch.from_numpy(W1.astype(np.float32)), padding=1)
            tab = tab * c(s2) + c(b2)
            y1 = F.conv2d(tin, rw(w1f), padding=1) + tab
            y1 = F.prelu(y1, T(pre + ".prelu.weight"))
            y1 = y1 if y1_32 else r(y1)
            s3, b3 = bnf(p, pre + ".bn3")
            w2f = p[pre + ".conv2.weight"] * s3[:, None, None, None]
            o = F.conv2d(r(y1), rw(w2f), stride=stride, padding=1) + c(b3)
            if ds:
                sd, bd = bnf(p, pre + ".downsample.1")
                wdf = p[pre + ".downsample.0.weight"] * sd[:, None, None, None]
                o = o + F.conv2d(tin, rw(wdf), stride=stride) + c(bd)
            else:
                o = o + (t if res32 else tin)
            t = o if res32 else r(o)
        s2, b2 = bnf(p, "bn2")
        sf, bf = bnf(p, "features")
        Wfc = p["fc.weight"].reshape(-1, 512, 7, 7)
        wf = Wfc * s2[None, :, None, None] * sf[:, None, None, None]
        bias = sf * (np.einsum("ochw,c->o", Wfc, b2) + p["fc.bias"]) + bf
        e = F.conv2d(r(t), rw(wf)).flatten(1) + torch.from_numpy(bias.astype(np.float32))
    return e


def tta(fwd, chips):
    x = arcface_input_from_chips(chips)
    e = fwd(x) + fwd(torch.flip(x, dims=[3]))
    return (e / e.norm(dim=1, keepdim=True)).numpy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    torch.set_num_threads(8)
    p = {k: v.astype(np.float64) if v.dtype == np.float32 else v for k, v in models.synth_iresnet(depth, seed=0).items()}
    p32 = {k: v.astype(np.float32) for k, v in p.items()}
    chips = np.random.default_rng(7).integers(0, 256, (n, 112, 112, 3), dtype=np.uint8)
    ref = tta(lambda x: iresnet_forward(p32, depth, x), chips)
    # planted bank like bench.plant_bank: rows from these faces minus 0.3 of the mean plus noise
    rng = np.random.default_rng(1)
    mean = ref.mean(0)
    bank = []
    for k in range(8):
        v = ref[k % n] - 0.3 * mean + (0.1 + 0.1 * k) * rng.standard_normal(512) / np.sqrt(512.0)
        bank.append(v / np.linalg.norm(v))
    bank = np.array(bank, np.float32)
    fd = lambda e: (1.0 - e @ bank.T).min(1)
    fd_ref = fd(ref)
    print(f"fd (f32) spread over faces: min {fd_ref.min():.4f} median {np.median(fd_ref):.4f} "
          f"max {fd_ref.max():.4f}; 1-cos(face_i, mean face) median {np.median(1 - ref @ (mean / np.linalg.norm(mean))):.2e}")
    variants = {
        "emu f32 (folding only)": dict(act16=False, w16=False),
        "device f16": dict(),
        "f16, weights f32": dict(w16=False),
        "f16, residual stream f32": dict(res32=True),
        "f16, residual + y1 f32": dict(res32=True, y1_32=True),
    }
    for name, kw in variants.items():
        e = tta(lambda x: emu_forward(p, depth, x, **kw), chips)
        d = np.abs(fd(e) - fd_ref)
        cs = 1.0 - (e * ref).sum(1)
        print(f"{name:28s}: |dfd| median {np.median(d):.2e} max {d.max():.2e}; 1-cos(e, e32) median "
              f"{np.median(cs):.2e} max {cs.max():.2e}", flush=True)


if __name__ == "__main__":
    main()
