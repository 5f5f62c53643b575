"""Serialized network programs for the gfx950 executor (pcgpu.h: pc_net_create).

A program is the host-side description of one conv network after all
inference-time algebra has been applied (BN folded into weights/biases, the
IResNet pre-BN folded with a per-border-class bias table, ResNetV1e avg-down
shortcuts rewritten as 2x2/s2 convs, PAFPN top-down/bottom-up adds expressed as
residual epilogues or second K-segments). The device executor
(csrc/pc_api.cpp) only sees CONV / STEM / MAXPOOL ops over NHWC tensor views.

Binary format (little-endian int32 words, then float32 data):
  magic 'PCNT', version 1, n_buf, n_tensor, n_array, n_op, n_out, input_tensor
  buffers : n_buf   x [elems_per_image lo, hi, is_f32, 0]
  tensors : n_tensor x [buf, H, W, C, cs, coff, is_f32, split]
            (split bit 0: f16x3 tensor, C physical channels = [hi | lo] halves of C/2, DESIGN.md §3.6;
             bit 1, input tensor only: centred u8 input x - 127.5, Program.input_centered;
             bit 2: f16c8 tensor, the second half e4m3 [lo8 | hi8] per 32 channels, Program(c8=True))
  arrays  : n_array x [offset lo, hi, count lo, hi]   (in floats, into data)
  outputs : n_out tensor ids
  ops     : n_op x 32 words (layouts below, mirrored in pc_api.cpp)
  data    : float32
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

OP_CONV, OP_STEM, OP_MAXPOOL, OP_UPSAMPLE, OP_LAYERNORM, OP_ATTENTION = 1, 2, 3, 4, 5, 6
ACT_NONE, ACT_RELU, ACT_PRELU, ACT_SILU, ACT_GELU = 0, 1, 2, 3, 4
BIAS_NONE, BIAS_CHANNEL, BIAS_BORDER9 = 0, 1, 2
RES_NONE, RES_SAME, RES_UP2 = 0, 1, 2


def cpad(c: int, m: int = 32) -> int:
    return (int(c) + m - 1) // m * m


class Program:
    """Builder for a pcgpu network program.

    split=True builds the f16x3 form: every f16 activation is stored as
    two f16 halves [hi | lo] (x = hi + lo, f32-class precision), and every conv that reads
    one walks K as [hi, lo, hi] per tap against weights [W_hi, W_hi, W_lo], so the device
    accumulates x_hi*W_hi + x_lo*W_hi + x_hi*W_lo in f32 (the dropped x_lo*W_lo is ~2^-22
    relative). The models compile unchanged: act() allocates the halves and conv()
    expands the weight columns."""

    def __init__(self, split: bool = False, c8: bool = False) -> None:
        """c8: the f16c8 form - split storage whose second half holds e4m3 bytes
        [lo8 | hi8] per 32 channels; convs read it as x_hi*W_hi (f16 MFMA) + one block-scaled e4m3
        MFMA for x_lo*W_hi + x_hi*W_lo. Every split activation of 64-channel blocks is f16c8 unless
        plain_split() marks it (a tensor read by an op without the f16c8 path)."""
        self.split = bool(split) or bool(c8)
        self.c8 = bool(c8)
        self.tc8: List[int] = []                  # per tensor: 1 = f16c8
        self.vbufs: List[List[int]] = []          # [elems_per_image, is_f32]
        self.tensors: List[List[int]] = []        # [vbuf, H, W, C, cs, coff, is_f32]  (C, cs physical)
        self.tsplit: List[int] = []               # per tensor: 1 = f16x3 split
        self.arrays: List[np.ndarray] = []
        self.ops: List[List[int]] = []
        self.outputs: List[int] = []
        self.input: Optional[int] = None
        # the input holds the centred u8 image (x - 127.5, exact in f16) instead of the model's own
        # normalisation; the scale is folded into the first op (models.compile_iresnet(split=True))
        self.input_centered = False
        self.flops_per_image = 0.0

    # ---- tensors -------------------------------------------------------
    def input_tensor(self, H: int, W: int, C: int) -> int:
        t = len(self.tensors)
        self.tensors.append([-1, H, W, C, C, 0, 0])
        self.tsplit.append(0)
        self.tc8.append(0)
        self.input = t
        return t

    def act(self, H: int, W: int, C: int, is_f32: int = 0) -> int:
        """Activation of C (padded) channels; in a split program an f16 one holds 2C."""
        sp = 1 if (self.split and not is_f32) else 0
        Cp = C * (2 if sp else 1)
        vb = len(self.vbufs)
        self.vbufs.append([H * W * Cp, is_f32])
        t = len(self.tensors)
        self.tensors.append([vb, H, W, Cp, Cp, 0, is_f32])
        self.tsplit.append(sp)
        self.tc8.append(1 if (sp and self.c8 and C % 32 == 0) else 0)
        return t

    def plain_split(self, t: int) -> None:
        """Keep tensor t in the f16x3 [hi | lo] form in an f16c8 program."""
        self.tc8[t] = 0

    def view(self, t: int, coff: int, C: int) -> int:
        """Channel slice [coff, coff+C) of tensor t (same buffer and pixel stride):
        concatenations are written and read in place."""
        vb, H, W, C0, cs, off, f32 = self.tensors[t]
        assert not self.tsplit[t], "channel views of split tensors are not supported"
        assert coff + C <= C0
        self.tensors.append([vb, H, W, C, cs, off + coff, f32])
        self.tsplit.append(0)
        self.tc8.append(0)
        return len(self.tensors) - 1

    def dims(self, t: int) -> Tuple[int, int, int]:
        """(H, W, logical channels): a split tensor's C counts one half."""
        T = self.tensors[t]
        return T[1], T[2], T[3] // 2 if self.tsplit[t] else T[3]

    def arr(self, a: np.ndarray) -> int:
        self.arrays.append(np.ascontiguousarray(a, dtype=np.float32).reshape(-1))
        return len(self.arrays) - 1

    # ---- ops -----------------------------------------------------------
    def conv(self, out: int, segs: Sequence[Tuple[int, int, int, int, int, int]], w_packed: np.ndarray,
             cout: int, bias: Optional[np.ndarray] = None, bias_mode: int = BIAS_CHANNEL,
             slope: Optional[np.ndarray] = None, act: int = ACT_NONE, res: Optional[int] = None,
             res_mode: int = RES_SAME, act_after_res: int = 0, splitk: int = 1,
             flops_cout: Optional[int] = None) -> None:
        """segs: (tensor, KH, KW, stride, pad, cin_true) per K-segment (max 2).
        flops_cout: true output channels for the FLOP count when the packed weight rows
        interleave padding (outputs split into padded channel slices)."""
        assert 1 <= len(segs) <= 2
        if any(self.tsplit[s[0]] for s in segs):
            w_packed = self._split_columns(w_packed, segs)
        npad, ktot = w_packed.shape
        w = [0] * 32
        w[0] = OP_CONV
        w[1] = out
        w[2] = len(segs)
        for i, (t, kh, kw, s, p, _cin) in enumerate(segs):
            w[3 + 5 * i: 8 + 5 * i] = [t, kh, kw, s, p]
            w[25 + i] = _cin
        w[13] = self.arr(w_packed)
        w[14] = npad
        w[15] = ktot
        w[16] = cout
        w[17] = self.arr(bias) if bias is not None else -1
        w[18] = bias_mode if bias is not None else BIAS_NONE
        w[19] = self.arr(slope) if slope is not None else -1
        w[20] = act
        w[21] = res if res is not None else -1
        w[22] = res_mode if res is not None else RES_NONE
        w[23] = act_after_res
        w[24] = splitk
        w[27] = int(flops_cout) if flops_cout else 0
        self.ops.append(w)
        oh, ow, _ = self.dims(out)
        fc = flops_cout or cout
        for (t, kh, kw, s, p, cin) in segs:
            self.flops_per_image += 2.0 * oh * ow * fc * kh * kw * cin

    def _split_columns(self, w_packed: np.ndarray, segs) -> np.ndarray:
        """[npad][sum KH*KW*C] -> split segments' columns as [W_hi | W_hi | W_lo] per tap
        (f32 values exactly representable in f16: the device's f16 upload is exact)."""
        w32 = np.asarray(w_packed, dtype=np.float32)
        npad = w32.shape[0]
        cols, k0 = [], 0
        for (t, kh, kw, _s, _p, _cin) in segs:
            cp = self.dims(t)[2]
            n = kh * kw * cp
            blk = w32[:, k0:k0 + n]
            k0 += n
            if self.tsplit[t]:
                taps = blk.reshape(npad, kh * kw, cp)
                hi = taps.astype(np.float16).astype(np.float32)
                lo = (taps - hi).astype(np.float16).astype(np.float32)
                blk = np.concatenate([hi, hi, lo], axis=2).reshape(npad, kh * kw * 3 * cp)
            cols.append(blk)
        assert k0 == w32.shape[1], "packed weight columns do not match the segments"
        return np.concatenate(cols, axis=1)

    def stem(self, out: int, x: int, w: np.ndarray, bias: np.ndarray, stride: int, pad: int,
             slope: Optional[np.ndarray] = None, act: int = ACT_NONE, cin_true: int = 3) -> None:
        """w: [cout][3][3][4] folded filter (input channel 3 is padding)."""
        cout = w.shape[0]
        _, _, cp = self.dims(out)
        ops = [0] * 32
        ops[0] = OP_STEM
        ops[1:13] = [out, x, 3, 3, stride, pad, self.arr(w), cout, self.arr(bias),
                     self.arr(slope) if slope is not None else -1, act, cp]
        ops[13] = cin_true
        self.ops.append(ops)
        oh, ow, _ = self.dims(out)
        self.flops_per_image += 2.0 * oh * ow * cout * 9 * cin_true

    def maxpool(self, out: int, x: int, k: int, s: int, p: int) -> None:
        ops = [0] * 32
        ops[0:6] = [OP_MAXPOOL, out, x, k, s, p]
        self.ops.append(ops)

    def upsample2(self, out: int, x: int) -> None:
        """Nearest-neighbour x2 (nn.Upsample(scale_factor=2, mode='nearest')) into out."""
        ops = [0] * 32
        ops[0:3] = [OP_UPSAMPLE, out, x]
        self.ops.append(ops)

    def layernorm(self, out: int, x: int, gamma: np.ndarray, beta: np.ndarray, eps: float = 1e-5,
                  add: Optional[np.ndarray] = None) -> None:
        """Per-pixel LayerNorm over the C true channels of x (f32 statistics). `add`
        ([rows][C], rows = pixels per image) is added to x first (positional table)."""
        ops = [0] * 32
        _, _, C = self.dims(x)
        ops[0:8] = [OP_LAYERNORM, out, x, self.arr(gamma), self.arr(beta),
                    self.arr(add) if add is not None else -1, int(add.shape[0]) if add is not None else 0,
                    int(np.float32(eps).view(np.int32))]
        ops[8] = int(gamma.shape[0])
        self.ops.append(ops)

    def attention(self, out: int, qkv: int, heads: int, head_dim: int) -> None:
        """Multi-head self-attention over the W tokens of each image: qkv [T][3*h*d]
        (q | k | v, head-major inside each) -> out [T][h*d], softmax(q k^T / sqrt(d)) v."""
        ops = [0] * 32
        ops[0:5] = [OP_ATTENTION, out, qkv, heads, head_dim]
        self.ops.append(ops)
        H, W, _ = self.dims(qkv)
        T = H * W
        self.flops_per_image += 4.0 * T * T * heads * head_dim

    # ---- serialization --------------------------------------------------
    def _op_io(self, w: List[int]) -> Tuple[List[int], int]:
        if w[0] == OP_CONV:
            ins = [w[3 + 5 * i] for i in range(w[2])]
            if w[21] >= 0:
                ins.append(w[21])
            return ins, w[1]
        return [w[2]], w[1]

    def _assign_buffers(self) -> Tuple[List[List[int]], List[int]]:
        """Liveness-based reuse of activation buffers (same dtype pool)."""
        nv = len(self.vbufs)
        first = [None] * nv
        last = [-1] * nv
        for i, w in enumerate(self.ops):
            ins, out = self._op_io(w)
            vb = self.tensors[out][0]
            if vb >= 0 and first[vb] is None:
                first[vb] = i
            for t in ins:
                vb = self.tensors[t][0]
                if vb >= 0:
                    last[vb] = max(last[vb], i)
        for t in self.outputs:
            vb = self.tensors[t][0]
            if vb >= 0:
                last[vb] = len(self.ops) + 1
        phys: List[List[int]] = []     # [elems, is_f32, busy_until]
        mapping = [-1] * nv
        order = sorted([v for v in range(nv) if first[v] is not None], key=lambda v: first[v])
        for v in order:
            elems, f32 = self.vbufs[v]
            lastv = max(last[v], first[v])
            best = -1
            for j, (pe, pf, busy) in enumerate(phys):
                if pf == f32 and busy < first[v]:
                    if best < 0 or abs(pe - elems) < abs(phys[best][0] - elems):
                        best = j
            if best < 0:
                phys.append([elems, f32, lastv])
                best = len(phys) - 1
            else:
                phys[best][0] = max(phys[best][0], elems)
                phys[best][2] = lastv
            mapping[v] = best
        return phys, mapping

    def serialize(self) -> bytes:
        assert self.input is not None and self.outputs
        phys, mapping = self._assign_buffers()
        words: List[int] = [0x544E4350, 1, len(phys), len(self.tensors), len(self.arrays), len(self.ops),
                            len(self.outputs), self.input]
        for elems, f32, _ in phys:
            words += [elems & 0xFFFFFFFF, elems >> 32, f32, 0]
        for i, ((vb, H, W, C, cs, coff, f32), sp, c8) in enumerate(zip(self.tensors, self.tsplit, self.tc8)):
            if i == self.input and self.input_centered:
                sp |= 2
            if c8:
                sp |= 4
            words += [mapping[vb] if vb >= 0 else -1, H, W, C, cs, coff, f32, sp]
        off = 0
        for a in self.arrays:
            n = a.size
            words += [off & 0xFFFFFFFF, off >> 32, n & 0xFFFFFFFF, n >> 32]
            off += n
        words += list(self.outputs)
        for w in self.ops:
            assert len(w) == 32
            words += w
        head = struct.pack("<%di" % len(words), *[int(x) if x < 2**31 else int(x) - 2**32 for x in words])
        data = np.concatenate(self.arrays).astype("<f4").tobytes() if self.arrays else b""
        return head + data


def pack_conv_weights(ws: Sequence[np.ndarray], cin_pads: Sequence[int], npad: int) -> np.ndarray:
    """[cout][cin][kh][kw] per segment -> [npad][sum_s kh*kw*cin_pad_s], K = tap-major, channel-minor."""
    cols = []
    for w, cp in zip(ws, cin_pads):
        cout, cin, kh, kw = w.shape
        t = np.zeros((npad, kh, kw, cp), dtype=np.float64)
        t[:cout, :, :, :cin] = np.transpose(w, (0, 2, 3, 1))
        cols.append(t.reshape(npad, kh * kw * cp))
    return np.concatenate(cols, axis=1).astype(np.float32)


def pad_vec(v: np.ndarray, n: int) -> np.ndarray:
    out = np.zeros((n,), dtype=np.float64)
    out[: v.shape[0]] = v
    return out
