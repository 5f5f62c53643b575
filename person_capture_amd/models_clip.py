"""OpenCLIP ViT image tower for ReIDEmbedder: architecture, synthetic weights and
compilation into a pcgpu program.

The reference embeds person crops with ``open_clip.create_model_and_transforms(
'ViT-L-14', pretrained='laion2b_s32b_b82k')`` and ``encode_image`` (reid_embedder.py:
19-57, [ext] open-clip-torch==3.2.0). ViT-L/14 @224: conv1 14x14/14 3->1024 (no bias),
class token + learned positional embedding (257 tokens), ln_pre, 24 residual blocks
(x += out_proj(MHA(ln_1(x))) with 16 heads of 64; x += c_proj(GELU(c_fc(ln_2(x))))
with MLP 4096), ln_post on the class token, @ proj (1024x768). Parameters use the
open_clip state-dict names (``visual.transformer.resblocks.{i}.attn.in_proj_weight`` ...).
No weights exist offline (pretrained tags are downloaded by the reference), so they are
seeded with open_clip's own init scheme (VisionTransformer.init_parameters std values).

Device program (compile_clip_vit): tokens are the pixels of a 1 x 257 image, so
every linear layer is a 1x1 implicit-GEMM conv on the MFMA engine with its bias,
GELU and residual add fused in the epilogue; the patch embedding is a 1x1 conv over
the patch matrix the preprocessing kernel writes ([257][608]: 14*14*3 = 588 columns
padded to 608, token 0 zero), the class/positional embedding is the additive table of
the ln_pre LayerNorm op, attention is OP_ATTENTION, and the final projection is a 1x1
conv with stride 257 that reads only the class token of every image.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from .program import ACT_GELU, ACT_NONE, BIAS_CHANNEL, RES_SAME, Program, cpad

Params = Dict[str, np.ndarray]

CLIP_CFGS = {
    # width, layers, heads, mlp, output dim, patch, image size
    "ViT-L-14": dict(width=1024, layers=24, heads=16, mlp=4096, out=768, patch=14, image=224),
    "ViT-B-16": dict(width=768, layers=12, heads=12, mlp=3072, out=512, patch=16, image=224),
    # reduced-depth towers for parity tests (same kernels and shapes per layer)
    "ViT-L-14-d2": dict(width=1024, layers=2, heads=16, mlp=4096, out=768, patch=14, image=224),
    "ViT-tiny-14": dict(width=128, layers=2, heads=2, mlp=512, out=64, patch=14, image=224),
}
LN_EPS = 1e-5


def clip_cfg(name: str) -> dict:
    if name not in CLIP_CFGS:
        raise RuntimeError(f"ReID model '{name}' is not part of this MI355X build (have: {sorted(CLIP_CFGS)})")
    c = dict(CLIP_CFGS[name])
    if c["patch"] != 14 or c["image"] != 224:
        raise RuntimeError(f"ReID model '{name}': only 14-pixel patches at 224 are implemented")
    return c


def synth_clip_vit(name: str = "ViT-L-14", seed: int = 0) -> Params:
    c = clip_cfg(name)
    w, L, ps, od = c["width"], c["layers"], c["patch"], c["out"]
    rng = np.random.default_rng(np.random.SeedSequence([20260504, w, L, seed]))
    f = lambda shape, std: (rng.standard_normal(shape) * std).astype(np.float32)
    scale = w ** -0.5
    attn_std = w ** -0.5
    proj_std = (w ** -0.5) * ((2 * L) ** -0.5)
    fc_std = (2 * w) ** -0.5
    p: Params = {}
    p["visual.conv1.weight"] = f((w, 3, ps, ps), (3 * ps * ps) ** -0.5)
    p["visual.class_embedding"] = f((w,), scale)
    p["visual.positional_embedding"] = f(((c["image"] // ps) ** 2 + 1, w), scale)
    ln = lambda name: (p.__setitem__(name + ".weight", rng.uniform(0.8, 1.2, w).astype(np.float32)),
                       p.__setitem__(name + ".bias", f((w,), 0.05)))
    ln("visual.ln_pre")
    for i in range(L):
        pre = f"visual.transformer.resblocks.{i}"
        ln(pre + ".ln_1")
        p[pre + ".attn.in_proj_weight"] = f((3 * w, w), attn_std)
        p[pre + ".attn.in_proj_bias"] = f((3 * w,), 0.02)
        p[pre + ".attn.out_proj.weight"] = f((w, w), proj_std)
        p[pre + ".attn.out_proj.bias"] = f((w,), 0.02)
        ln(pre + ".ln_2")
        p[pre + ".mlp.c_fc.weight"] = f((c["mlp"], w), fc_std)
        p[pre + ".mlp.c_fc.bias"] = f((c["mlp"],), 0.02)
        p[pre + ".mlp.c_proj.weight"] = f((w, c["mlp"]), proj_std)
        p[pre + ".mlp.c_proj.bias"] = f((w,), 0.02)
    ln("visual.ln_post")
    p["visual.proj"] = f((w, od), scale)
    return p


def _lin(P: Program, out: int, x: int, W: np.ndarray, b, act: int = ACT_NONE, res: int = None,
         stride: int = 1) -> None:
    """y = act(x @ W^T + b) (+ res) as a 1x1 conv over the token axis."""
    cout, cin = W.shape
    _, _, cp = P.dims(x)
    npad = cpad(cout)
    wp = np.zeros((npad, cp), np.float32)
    wp[:cout, :cin] = W
    bias = None
    if b is not None:
        bias = np.zeros(npad, np.float64)
        bias[:cout] = b
    P.conv(out, [(x, 1, 1, stride, 0, cin)], wp, cout, bias=bias, bias_mode=BIAS_CHANNEL, act=act, res=res,
           res_mode=RES_SAME, act_after_res=0)


def compile_clip_vit(p: Params, name: str = "ViT-L-14") -> Program:
    """Image tower -> program. Input: patch matrix [1][T][608] (see module doc). Output:
    f32 [1][1][out_dim] per image (before F.normalize)."""
    c = clip_cfg(name)
    w, L, heads, od = c["width"], c["layers"], c["heads"], c["out"]
    g = c["image"] // c["patch"]
    T = g * g + 1
    K = 3 * c["patch"] ** 2
    P = Program()
    x_in = P.input_tensor(1, T, cpad(K))
    # patch embedding: conv1 weight [w][3][14][14] -> [w][(kh*14 + kw)*3 + c]
    Wc = np.transpose(p["visual.conv1.weight"], (0, 2, 3, 1)).reshape(w, K)
    e = P.act(1, T, w)
    _lin(P, e, x_in, Wc, None)
    x = P.act(1, T, w)
    add = p["visual.positional_embedding"].astype(np.float64).copy()
    add[0] += p["visual.class_embedding"]
    P.layernorm(x, e, p["visual.ln_pre.weight"], p["visual.ln_pre.bias"], LN_EPS, add=add)
    for i in range(L):
        pre = f"visual.transformer.resblocks.{i}"
        y = P.act(1, T, w)
        P.layernorm(y, x, p[pre + ".ln_1.weight"], p[pre + ".ln_1.bias"], LN_EPS)
        qkv = P.act(1, T, 3 * w)
        _lin(P, qkv, y, p[pre + ".attn.in_proj_weight"], p[pre + ".attn.in_proj_bias"])
        a = P.act(1, T, w)
        P.attention(a, qkv, heads, w // heads)
        x2 = P.act(1, T, w)
        _lin(P, x2, a, p[pre + ".attn.out_proj.weight"], p[pre + ".attn.out_proj.bias"], res=x)
        y2 = P.act(1, T, w)
        P.layernorm(y2, x2, p[pre + ".ln_2.weight"], p[pre + ".ln_2.bias"], LN_EPS)
        h = P.act(1, T, c["mlp"])
        _lin(P, h, y2, p[pre + ".mlp.c_fc.weight"], p[pre + ".mlp.c_fc.bias"], act=ACT_GELU)
        x3 = P.act(1, T, w)
        _lin(P, x3, h, p[pre + ".mlp.c_proj.weight"], p[pre + ".mlp.c_proj.bias"], res=x2)
        x = x3
    yl = P.act(1, T, w)
    P.layernorm(yl, x, p["visual.ln_post.weight"], p["visual.ln_post.bias"], LN_EPS)
    o = P.act(1, 1, cpad(od), is_f32=1)
    _lin(P, o, yl, p["visual.proj"].T.copy(), None, stride=T)   # class token only
    P.outputs = [P.view(o, 0, od)]
    return P
