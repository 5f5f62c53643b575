"""ReIDEmbedder — drop-in for person_capture/reid_embedder.py on the MI355X.

Same class name, constructor keywords (device='cuda', model_name='ViT-L-14',
pretrained='laion2b_s32b_b82k', progress=None), ``device`` attribute and
``extract(bgr_list)`` contract (reid_embedder.py:10-57): L2-normalised float32
embeddings, one per non-empty crop (None / empty crops are skipped, so the output
can be shorter than the input), ``[]`` for an empty list.

Per call the reference converts every crop on the CPU (cvtColor, PIL, open_clip
preprocess), stacks them, copies the batch to the GPU and runs encode_image in fp32.
Here one C-ABI call (pc_clip_embed) does it all on the device: the Pillow bicubic
resample + centre crop + normalise kernel writes the ViT patch matrix, the image
tower runs as MFMA 1x1 convs + LayerNorm/attention kernels, and F.normalize finishes.

Weights: the laion2b checkpoint is downloaded by open_clip in the reference; none
exists offline, so seeded weights with open_clip's init scheme are used
(models_clip.synth_clip_vit). ``pretrained`` is kept for signature compatibility.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import models_clip
from ._lib import PC_PREC_F16, PC_PREC_F32, CropDesc, check
from .runtime import GpuContext, Net

_WEIGHTS: Dict[Tuple[str, int], dict] = {}


def _precision() -> int:
    """f32 by default: the reference runs encode_image in fp32 (reid_embedder.py:53-55) and
    no TensorRT engine exists for it. PERSON_CAPTURE_AMD_REID_PRECISION=f16 opts into the
    f16 tower (narrower than the reference: tests/test_gpu_reid.py bounds it)."""
    v = os.getenv("PERSON_CAPTURE_AMD_REID_PRECISION", "f32")
    return PC_PREC_F16 if v.strip().lower() in ("f16", "fp16", "float16", "half") else PC_PREC_F32


def clip_weights(name: str, seed: int = 0) -> dict:
    key = (name, seed)
    if key not in _WEIGHTS:
        _WEIGHTS[key] = models_clip.synth_clip_vit(name, seed=seed)
    return _WEIGHTS[key]


class ClipEngine:
    """OpenCLIP image tower on one GPU context (crops on device -> unit embeddings)."""

    def __init__(self, ctx: GpuContext, params: dict, name: str, precision: int = PC_PREC_F16, max_batch: int = 32):
        self.ctx, self.name, self.max_batch = ctx, name, max_batch
        self.program = models_clip.compile_clip_vit(params, name)
        self.net = Net(ctx, self.program.serialize(), precision=precision, max_batch=max_batch)
        self.dim = models_clip.clip_cfg(name)["out"]

    @property
    def flops_per_image(self) -> float:
        return self.net.flops_per_image

    def embed_device(self, crops: Sequence[Tuple[int, int, int, int]], d_out: int) -> None:
        """crops: (device ptr, H, W, row_stride) BGR u8 -> d_out [n][dim] f32 (enqueued)."""
        n = len(crops)
        if n > self.max_batch:
            raise ValueError(f"ReID batch {n} exceeds max_batch {self.max_batch}")
        arr = (CropDesc * n)()
        for i, (ptr, H, W, rs) in enumerate(crops):
            arr[i].d_src, arr[i].H, arr[i].W, arr[i].row_stride = int(ptr), int(H), int(W), int(rs)
        check(self.ctx.lib.pc_clip_embed(self.net.handle, arr, n, C.c_void_p(int(d_out))), self.ctx.handle,
              "clip_embed")


class ReIDEmbedder:
    """
    Body embedding via an OpenCLIP ViT image tower on the MI355X.
    Defaults to ViT-L-14; returns L2-normalized embeddings as np.float32.
    """

    def __init__(self, device: str = 'cuda', model_name: str = 'ViT-L-14', pretrained: str = 'laion2b_s32b_b82k',
                 progress=None):
        s = str(device)
        if not s.startswith("cuda"):
            raise RuntimeError("ReIDEmbedder on this build runs on the MI355X HIP device only (device='cuda').")
        idx = int(s.split(":", 1)[1]) if ":" in s and s.split(":", 1)[1].isdigit() else 0
        self.device = 'cuda'
        self.model_name = model_name
        self.pretrained = pretrained
        models_clip.clip_cfg(model_name)   # RuntimeError for towers this build does not have
        from .face_embedder import get_context
        self._ctx = get_context(idx)
        seed = int(os.getenv("PERSON_CAPTURE_AMD_SEED", "0"))
        if callable(progress):
            progress(f"pcgpu: synthetic weights for OpenCLIP {model_name} (no {pretrained} checkpoint offline)")
        self._engine = ClipEngine(self._ctx, clip_weights(model_name, seed), model_name, _precision(),
                                  int(os.getenv("PERSON_CAPTURE_AMD_REID_BATCH", "32")))
        self.dim = self._engine.dim

    def extract_device(self, crops: Sequence[Tuple[int, int, int, int]]) -> np.ndarray:
        """Crops already in HBM: (ptr, H, W, row_stride) -> [n][dim] unit f32."""
        n = len(crops)
        out = np.zeros((n, self.dim), np.float32)
        per = self._engine.max_batch
        for s0 in range(0, n, per):
            part = crops[s0:s0 + per]
            d = self._ctx.scratch("reid_feat", len(part) * self.dim * 4)
            self._engine.embed_device(part, d.ptr)
            out[s0:s0 + len(part)] = self._ctx.download(d.ptr, (len(part), self.dim), np.float32)
        return out

    def extract(self, bgr_list):
        if not bgr_list:
            return []
        crops = [b for b in bgr_list if b is not None and getattr(b, "size", 0) != 0]
        if not crops:
            return []
        per = self._engine.max_batch
        feats: List[np.ndarray] = []
        for s0 in range(0, len(crops), per):
            part = crops[s0:s0 + per]
            devs = []
            for k, b in enumerate(part):
                a = np.ascontiguousarray(b, dtype=np.uint8)
                d = self._ctx.scratch(f"reid_crop{k}", a.nbytes)
                self._ctx.upload(a, d)
                devs.append((d.ptr, a.shape[0], a.shape[1], a.strides[0]))
            feats.extend(self.extract_device(devs))
        return [f for f in feats]
