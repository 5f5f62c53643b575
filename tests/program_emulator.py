"""CPU (torch fp32) interpreter of pcgpu programs — test infrastructure.

Executes the serialized op list exactly as the device executor defines it
(csrc/pc_api.cpp + pc_conv*.hip / pc_ops.hip semantics: K-segments, border-class
bias, activation before/after the residual, nearest-2x residual, split-K, stem,
max-pool, upsample, layernorm, attention) over buffer-level tensor views, so the
inference-time algebra in person_capture_amd/models*.py (BN folding, pre-BN border
tables, avg-down rewrite, PAFPN fusions, in-place concatenation slices, padded
channel maps) can be checked against the literal oracle nets without a GPU.
"""
import numpy as np
import torch
import torch.nn.functional as F

from person_capture_amd import program as pg


def _act(y, act, slope):
    if act == pg.ACT_RELU:
        return F.relu(y)
    if act == pg.ACT_PRELU:
        return torch.where(y > 0, y, y * slope.view(1, -1, 1, 1))
    if act == pg.ACT_SILU:
        return F.silu(y)
    if act == pg.ACT_GELU:
        return F.gelu(y)
    return y


def run_program(P: pg.Program, x_nhwc: np.ndarray):
    """x_nhwc: [N][H][W][C] input (padded channels). Returns list of outputs NCHW (the
    output tensors' channels)."""
    N = x_nhwc.shape[0]
    inp = torch.from_numpy(np.ascontiguousarray(np.transpose(x_nhwc, (0, 3, 1, 2)))).float()
    bufs = {}
    A = [torch.from_numpy(a.astype(np.float32)) for a in P.arrays]

    tsplit = getattr(P, "tsplit", [0] * len(P.tensors))

    def read(t):
        """The tensor's values (a split tensor: hi + lo, exact in f32)."""
        vb, H, W, C, cs, off, _ = P.tensors[t]
        if vb < 0:
            return inp[:, off:off + C]
        x = bufs[vb][:, off:off + C]
        if tsplit[t]:
            return x[:, :C // 2] + x[:, C // 2:]
        return x

    def read_k(t):
        """The channels a conv's K walks: a split tensor's virtual [hi, lo, hi]."""
        vb, H, W, C, cs, off, _ = P.tensors[t]
        if tsplit[t]:
            x = bufs[vb][:, off:off + C]
            return torch.cat([x[:, :C // 2], x[:, C // 2:], x[:, :C // 2]], 1)
        return read(t)

    def write(t, y):
        vb, H, W, C, cs, off, _ = P.tensors[t]
        if vb not in bufs:
            bufs[vb] = torch.zeros(N, cs, H, W)
        if tsplit[t]:   # device epilogue: hi = f16(v), lo = f16(v - hi)
            h = C // 2
            v = y[:, :h].float()
            hi = v.half().float()
            bufs[vb][:, off:off + h] = hi
            bufs[vb][:, off + h:off + C] = (v - hi).half().float()
            return
        bufs[vb][:, off:off + C] = y[:, :C]

    def logical_c(t):
        C = P.tensors[t][3]
        return C // 2 if tsplit[t] else C

    for w in P.ops:
        if w[0] == pg.OP_CONV:
            npad, ktot = w[14], w[15]
            Wm = A[w[13]].view(npad, ktot)
            acc = None
            k0 = 0
            for s in range(w[2]):
                t, kh, kw, st, pd = w[3 + 5 * s: 8 + 5 * s]
                X = read_k(t)
                cp = X.shape[1]
                n = kh * kw * cp
                ws = Wm[:, k0:k0 + n].reshape(npad, kh, kw, cp).permute(0, 3, 1, 2).contiguous()
                k0 += n
                y = F.conv2d(X, ws, stride=st, padding=pd)
                acc = y if acc is None else acc + y
            Ho, Wo = acc.shape[2], acc.shape[3]
            if w[17] >= 0:
                b = A[w[17]]
                if w[18] == pg.BIAS_BORDER9:
                    t0, kh0, kw0, st0, pd0 = w[3:8]
                    X0 = read(t0)
                    H, Wd = X0.shape[2], X0.shape[3]
                    b9 = b.view(3, 3, npad)
                    ih0 = torch.arange(Ho) * st0 - pd0
                    iw0 = torch.arange(Wo) * st0 - pd0
                    rc = torch.where(ih0 < 0, 0, torch.where(ih0 + kh0 - 1 >= H, 2, 1))
                    cc = torch.where(iw0 < 0, 0, torch.where(iw0 + kw0 - 1 >= Wd, 2, 1))
                    acc = acc + b9[rc[:, None], cc[None, :]].permute(2, 0, 1)[None]
                else:
                    acc = acc + b.view(1, -1, 1, 1)
            slope = A[w[19]] if w[19] >= 0 else None
            act = w[20]
            res = read(w[21]) if w[21] >= 0 else None
            if res is not None and w[22] == pg.RES_UP2:
                res = F.interpolate(res, size=(Ho, Wo), mode="nearest")
            if not w[23]:
                acc = _act(acc, act, slope)
            if res is not None:
                k = min(res.shape[1], acc.shape[1])
                acc = acc.clone()
                acc[:, :k] = acc[:, :k] + res[:, :k]
            if w[23]:
                acc = _act(acc, act, slope)
            C = logical_c(w[1])
            out = torch.zeros(N, C, Ho, Wo)
            k = min(C, npad)
            out[:, :k] = acc[:, :k]
            out[:, w[16]:] = 0
            write(w[1], out)
        elif w[0] == pg.OP_STEM:
            X = read(w[2])
            cout = w[8]
            wt = A[w[7]].view(cout, 3, 3, 4).permute(0, 3, 1, 2).contiguous()
            if tsplit[w[1]]:   # split stem: x * W_hi + x * W_lo (the input is exact in f16)
                whi = wt.half().float()
                y = F.conv2d(X, whi, stride=w[5], padding=w[6]) + \
                    F.conv2d(X, (wt - whi).half().float(), stride=w[5], padding=w[6])
                y = y + A[w[9]].view(1, -1, 1, 1)
            else:
                y = F.conv2d(X, wt, stride=w[5], padding=w[6]) + A[w[9]].view(1, -1, 1, 1)
            y = _act(y, w[11], A[w[10]] if w[10] >= 0 else None)
            cp = logical_c(w[1])
            out = torch.zeros(y.shape[0], cp, y.shape[2], y.shape[3])
            out[:, :cout] = y
            write(w[1], out)
        elif w[0] == pg.OP_MAXPOOL:
            write(w[1], F.max_pool2d(read(w[2]), w[3], w[4], w[5]))
        elif w[0] == pg.OP_UPSAMPLE:
            write(w[1], F.interpolate(read(w[2]), scale_factor=2.0, mode="nearest"))
        elif w[0] == pg.OP_LAYERNORM:
            X = read(w[2])                           # [N][C][H][W]
            C = w[8]
            x = X[:, :C].permute(0, 2, 3, 1).reshape(N, -1, C)
            if w[5] >= 0:
                x = x + A[w[5]].view(w[6], C)[None]
            eps = float(np.int32(w[7]).view(np.float32))
            y = F.layer_norm(x, (C,), A[w[3]], A[w[4]], eps)
            H, W = X.shape[2], X.shape[3]
            Cout = P.tensors[w[1]][3]
            out = torch.zeros(N, Cout, H, W)
            out[:, :C] = y.view(N, H, W, C).permute(0, 3, 1, 2)
            write(w[1], out)
        elif w[0] == pg.OP_ATTENTION:
            X = read(w[2])
            heads, d = w[3], w[4]
            E = heads * d
            Tn = X.shape[2] * X.shape[3]
            x = X.permute(0, 2, 3, 1).reshape(N, Tn, -1)
            q, k, v = (x[..., i * E:(i + 1) * E].reshape(N, Tn, heads, d).transpose(1, 2) for i in range(3))
            a = torch.softmax((q * (1.0 / np.sqrt(d))) @ k.transpose(-1, -2), dim=-1) @ v
            y = a.transpose(1, 2).reshape(N, Tn, E)
            write(w[1], y.view(N, X.shape[2], X.shape[3], E).permute(0, 3, 1, 2))
        else:
            raise ValueError(f"unknown op {w[0]}")
    return [read(o) for o in P.outputs]
