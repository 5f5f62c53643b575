"""Reference-bank matching.

Host functions with the exact semantics of Processor._fd_min
(gui_app.py:660-674) and Processor._stream_ref_bank_update (gui_app.py:922-986)
— they run in frame order on the host, where the reference runs them — plus
DeviceBank, the batched on-device form of _fd_min (pc_bank_match) used by the
batched extract path and the frame-shard runner.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from ._lib import check
from .runtime import GpuContext


def fd_min(feat, ref_bank) -> float:
    """1 - max cosine similarity of a face feature against a bank of unit rows; 9.0 when
    either side is missing or the bank is empty (gui_app.py:660-674)."""
    if feat is None or ref_bank is None:
        return 9.0
    vec = np.asarray(feat, dtype=np.float32).reshape(-1)
    vec = vec / max(float(np.linalg.norm(vec)), 1e-6)
    bank = np.asarray(ref_bank, dtype=np.float32)
    if bank.ndim == 1:
        return 1.0 - float(np.dot(vec, bank))
    if bank.size == 0:
        return 9.0
    sims = bank @ vec
    return 9.0 if sims.size == 0 else 1.0 - float(np.max(sims))


def stream_ref_bank_update(ref_bank_list: List[np.ndarray], ref_face_feat: Optional[np.ndarray], vec_new,
                           quality_val: float, *, cap: int = 64, dedup_cos: float = 0.968,
                           rep_margin: float = 0.010, weights=(0.70, 0.25, 0.05)
                           ) -> Tuple[Optional[np.ndarray], str, Optional[int]]:
    """Grow / dedup / replace-worst update of the reference bank (gui_app.py:922-986);
    config values are passed explicitly instead of read from a SessionConfig."""
    if vec_new is None:
        return ref_face_feat, "skip", None
    cap = max(1, int(cap))
    w_anchor, w_div, w_q = weights
    v = np.asarray(vec_new, dtype=np.float32).reshape(-1)
    norm = float(np.linalg.norm(v))
    if norm <= 1e-6:
        return ref_face_feat, "skip", None
    v = v / norm
    bank = np.asarray(ref_face_feat if ref_face_feat is not None else ref_bank_list, dtype=np.float32)
    if bank.ndim == 1:
        bank = bank.reshape(1, -1)
    if bank.size == 0:
        ref_bank_list.append(v)
        return np.vstack(ref_bank_list).astype(np.float32), "added", None
    sims = bank @ v
    if sims.size > 0 and float(sims.max()) >= dedup_cos:
        return ref_face_feat, "dup", None
    anchor = bank[0]
    cos_anchor = max(-1.0, min(1.0, float(np.dot(anchor, v))))
    fd_anchor = float(np.sqrt(max(0.0, 2.0 - 2.0 * cos_anchor)))
    nn_sim = float(sims.max()) if sims.size else 0.0
    q_term = float(min(max(quality_val or 0.0, 0.0), 1000.0) / 300.0)
    s_new = w_anchor * (1.0 - fd_anchor) + w_div * (1.0 - nn_sim) + w_q * q_term
    if len(ref_bank_list) < cap:
        ref_bank_list.append(v)
        return np.vstack(ref_bank_list).astype(np.float32), "added", None
    gram = bank @ bank.T
    np.fill_diagonal(gram, -1.0)
    nn_each = gram.max(axis=1)
    cos_each = np.clip(bank @ anchor, -1.0, 1.0)
    fd_each = np.sqrt(np.maximum(0.0, 2.0 - 2.0 * cos_each))
    s_bank = w_anchor * (1.0 - fd_each) + w_div * (1.0 - nn_each)
    worst = int(np.argmin(s_bank))
    if s_new > float(s_bank[worst]) + rep_margin:
        ref_bank_list[worst] = v
        return np.vstack(ref_bank_list).astype(np.float32), "replaced", worst
    return ref_face_feat, "skip", None


class DeviceBank:
    """A reference bank resident in HBM ([B][D] f32 unit rows) and the batched fd kernel."""

    def __init__(self, ctx: GpuContext, bank: Optional[np.ndarray] = None):
        self.ctx = ctx
        self.rows = 0
        self.dim = 0
        self._buf = None
        if bank is not None:
            self.set(bank)

    def set(self, bank: np.ndarray) -> None:
        """bank: [B][D] unit rows, or one 1-D row (the reference's _fd_min then takes 1 - dot).
        A 1-D empty bank is rejected: the reference's np.dot((D,), (0,)) raises there."""
        b = np.ascontiguousarray(bank, dtype=np.float32)
        if b.ndim == 1:
            if b.size == 0:
                raise ValueError("1-D empty reference bank (shapes not aligned)")
            b = b.reshape(1, -1)
        if b.ndim != 2:
            raise ValueError(f"reference bank must be 1-D or 2-D, got shape {b.shape}")
        self.rows, self.dim = b.shape
        self._buf = self.ctx.alloc(max(b.nbytes, 16))
        if b.size:
            self.ctx.upload(b, self._buf)
            self.ctx.sync()   # other streams (the face embedder's embed stream) read the rows

    def match_device(self, d_feats: int, n: int, d_fd: int, d_idx: int, feat_dim: int = 512, ctx=None) -> None:
        """fd[i] = Processor._fd_min(feats[i], bank) for n device feature rows of feat_dim f32,
        on the stream of `ctx` (default: the bank's own context; the bank rows are on the
        device before set() returns, so any stream may read them)."""
        if self.rows and self.dim != feat_dim:
            raise ValueError(f"bank rows have {self.dim} dims, features {feat_dim} (shapes not aligned)")
        c = self.ctx if ctx is None else ctx
        check(c.lib.pc_bank_match(c.handle, d_feats, int(n), self._buf.ptr, int(self.rows),
                                  int(feat_dim), d_fd, d_idx), c.handle, "bank_match")
