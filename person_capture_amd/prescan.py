"""Pre-scan driver: the sampling loop of Processor._prescan (gui_app.py:1101-1668) over
device-resident frames, batched speculatively on the MI355X.

Per sample (gui_app.py:1468-1622): the escalation hint follows the `active` span state
(`_prescan_rr_mode = "full" if active else "rr"`, set_prescan_hint(escalate=active)); the
fd9 skip gate (after `prescan_fd9_grace` samples with no match, only every
`prescan_fd9_probe_period`-th sample is extracted while idle); an extracted sample is
downscaled to `prescan_max_width` with INTER_AREA (:1505-1507, on the device), run through
FaceEmbedder.extract, each face matched against the live bank (_fd_min), confident
good-quality faces grow the bank (_stream_ref_bank_update with the add cooldown), and the
best distance drives the enter/exit hysteresis that builds the keep-spans (pad, min length,
merge), closed at the end and bridged over short gaps (:1648-1668).

The loop is sequential: sample k+1's detector settings, skip decision and bank depend on
sample k. It runs in chunks: the driver predicts the gate decisions and hints of the next
`batch` samples assuming the current regime holds (idle without a match stays idle; a
match keeps the span open), runs all predicted extractions in ONE FaceEmbedder.extract_batch
(downscale, SCRFD, align, ArcFace batched on the device), then replays the host logic
sample by sample. At the first sample whose real state differs from the prediction, the
chunk is cut there: the FaceEmbedder's per-frame policy state is restored from its state
trace and the next chunk starts at that sample. Results are therefore identical to the
sequential loop; a regime change only costs the tail of one chunk.

Not here (GUI/IO plumbing outside the per-frame hot path): the command queue (pause, seek,
step, live cfg edits), decoder seeking, previews and progress signals, and the edge
refinement re-scan (:1670-) which reuses this same per-sample step at a finer stride.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .match import fd_min, stream_ref_bank_update


@dataclass
class PrescanConfig:
    """The SessionConfig fields the loop reads (gui_app.py:554-590 defaults)."""
    prescan_stride: int = 24
    prescan_max_width: int = 416
    prescan_face_conf: float = 0.5
    prescan_fd_enter: float = 0.45
    prescan_fd_add: float = 0.22
    prescan_fd_exit: float = 0.52
    prescan_add_cooldown_samples: int = 5
    prescan_rot_probe_period: int = 3
    prescan_probe_imgsz: int = 512
    prescan_no_upscale_det: bool = True
    prescan_probe_conf: float = 0.03
    prescan_heavy_90: int = 1536
    prescan_heavy_180: int = 1280
    prescan_min_segment_sec: float = 1.0
    prescan_pad_sec: float = 1.5
    prescan_bridge_gap_sec: float = 1.0
    prescan_exit_cooldown_sec: float = 0.50
    prescan_bank_max: int = 64
    prescan_diversity_dedup_cos: float = 0.968
    prescan_replace_margin: float = 0.010
    prescan_fd9_skip: bool = True
    prescan_fd9_grace: int = 1
    prescan_fd9_probe_period: int = 2
    prescan_weights: Tuple[float, float, float] = (0.70, 0.25, 0.05)
    face_quality_min: float = 70.0


@dataclass
class SampleRecord:
    idx: int            # frame index
    extracted: bool
    best: float         # best fd of the sample (9.0 when skipped or no face)
    n_faces: int
    bank_action: str    # last bank action of the sample ("" when none)
    active: bool        # span state after the sample


class _LoopState:
    __slots__ = ("active", "start", "neg_run", "fd9_streak", "last_add_sample", "spans", "bank_list", "bank",
                 "processed", "added", "last_found")

    def __init__(self, ref_feat):
        if ref_feat is None:
            self.bank_list: List[np.ndarray] = []
        else:
            arr = np.asarray(ref_feat, dtype=np.float32)
            if arr.ndim == 1:
                arr = arr.reshape(1, -1)
            arr = arr / np.maximum(np.linalg.norm(arr, axis=1, keepdims=True), 1e-6)
            self.bank_list = [row.copy() for row in arr]
        self.bank = np.vstack(self.bank_list).astype(np.float32) if self.bank_list else None
        self.active = False
        self.start = 0
        self.neg_run = 0
        self.fd9_streak = 0
        self.last_add_sample = -10 ** 9
        self.spans: List[Tuple[int, int]] = []
        self.processed = 0
        self.added = 0
        self.last_found = False   # did the last extracted sample have a face with a finite fd

    def copy(self) -> "_LoopState":
        c = _LoopState.__new__(_LoopState)
        for k in self.__slots__:
            v = getattr(self, k)
            setattr(c, k, list(v) if isinstance(v, list) else v)
        return c


@dataclass
class SpecRecord:
    """One speculatively extracted sample of a pre-scan shard (prescan_shard.py): the regime
    it ran under (span open: escalation + full rotation mode), the FaceEmbedder policy state
    before and after it, and its faces (host dicts: bbox, kps5, feat, quality)."""
    pos: int
    active: bool
    state_in: tuple
    state_out: tuple
    faces: list
    dims: Tuple[int, int] = (0, 0)   # (H, W) of the sample after the pre-scan downscale


class PrescanRunner:
    """Processor._prescan's sampling loop for one FaceEmbedder (SCRFD backend)."""

    def __init__(self, face, cfg: PrescanConfig, fps: float, total_frames: int, ref_feat=None, batch: int = 32):
        self.face, self.cfg, self.fps, self.total = face, cfg, float(fps), int(total_frames)
        self.ref_feat = ref_feat
        self.batch = max(1, int(batch))
        self.records: List[SampleRecord] = []
        self.chunks = 0
        self.cuts = 0
        self.spec: Optional[List[SpecRecord]] = None   # run(..., speculate=True) fills it
        self.initial_state: Optional[tuple] = None

    def samples(self) -> List[int]:
        """Frame index of every sample position (gui_app.py:1468: range(0, total, stride))."""
        return list(range(0, self.total, max(1, int(self.cfg.prescan_stride))))

    def setup_face(self) -> None:
        """The FaceEmbedder configuration of a pre-scan (gui_app.py:1162-1196)."""
        f = self.face
        self._apply_face_cfg()
        f.configure_rotation_strategy(adaptive=False)
        f.set_prescan_fast(True, mode="rr")
        f.set_prescan_hint(escalate=False)
        self._apply_face_cfg()

    def extract_one(self, frame_at, pos: int, active: bool, state: tuple):
        """Sample `pos` extracted under the given regime and policy state (the sharded
        merge's re-extraction). Returns (faces, policy state after)."""
        f = self.face
        f.set_policy_state(state)
        f._prescan_rr_mode = "full" if active else "rr"
        f.set_prescan_hint(escalate=active)
        im = frame_at(self.samples()[pos])
        if not hasattr(im, "ptr"):
            im = f._upload(np.ascontiguousarray(im), key="prescan_src0")
        im = self._downscale(im, 0)
        res = f.extract_batch([None], dev_frames=[im])
        return res[0], f.policy_state()

    def spec_chunk(self, frame_at, st: "_LoopState", k: int, stop: int):
        """One speculative chunk from sample position k (at most `batch` positions, < stop) under
        the current regime and the FaceEmbedder's current policy state: the gate decisions are
        predicted assuming the last extracted sample's outcome repeats, every predicted extraction
        runs in ONE extract_batch. Returns (plan [(pos, skip)], regime, policy state before,
        {pos: faces}, {pos: policy state after}, {pos: (H, W) after the downscale})."""
        f = self.face
        samples = self.samples()
        sim = st.copy()
        plan = []   # (sample position, skip)
        for j in range(k, min(stop, k + self.batch)):
            skip, _ = self._gate(sim)
            plan.append((j, skip))
            # regime assumption: the last extracted sample's outcome repeats (faces with a finite
            # distance keep the fd9 streak at 0, an empty sample grows it; skipped samples grow it)
            sim.fd9_streak = 0 if (not skip and sim.last_found) else sim.fd9_streak + 1
        active0 = st.active
        f._prescan_rr_mode = "full" if active0 else "rr"
        f.set_prescan_hint(escalate=active0)
        todo = [j for j, skip in plan if not skip]
        srcs = []
        for j in todo:
            im = frame_at(samples[j])
            if not hasattr(im, "ptr"):
                im = f._upload(np.ascontiguousarray(im), key=f"prescan_src{j % self.batch}")
            srcs.append(im)
        ims = self._downscale_many(srcs, [j - k for j in todo])
        state0 = f.policy_state()
        f.state_trace = []
        try:
            res = f.extract_batch([None] * len(ims), dev_frames=ims) if ims else []
        finally:
            trace = f.state_trace
            f.state_trace = None
        by_pos = {j: r for j, r in zip(todo, res)}
        state_after = {todo[t]: s for t, (_, s) in enumerate(trace)}
        dims = {j: (int(im.H), int(im.W)) for j, im in zip(todo, ims)}
        self.chunks += 1
        return plan, active0, state0, by_pos, state_after, dims

    def close(self, st: "_LoopState") -> List[Tuple[int, int]]:
        """End of the loop: close an open span at the last frame, then bridge short gaps
        (gui_app.py:1648-1668)."""
        c = self.cfg
        if st.active:
            pad = int(round(c.prescan_pad_sec * self.fps))
            min_len = int(round(c.prescan_min_segment_sec * self.fps))
            s, e = max(0, st.start - pad), self.total - 1
            if e - s + 1 >= min_len:
                if st.spans and s <= st.spans[-1][1] + 1:
                    st.spans[-1] = (st.spans[-1][0], max(st.spans[-1][1], e))
                else:
                    st.spans.append((s, e))
        spans = st.spans
        if spans and c.prescan_bridge_gap_sec > 0:
            gap = int(round(c.prescan_bridge_gap_sec * self.fps))
            bridged = []
            cs, ce = spans[0]
            for s, e in spans[1:]:
                if s - ce <= gap:
                    ce = max(ce, e)
                else:
                    bridged.append((cs, ce))
                    cs, ce = s, e
            bridged.append((cs, ce))
            spans = bridged
        return spans

    # ---- FaceEmbedder runtime configuration (gui_app.py:1162-1196) ----
    def _apply_face_cfg(self) -> None:
        f, c = self.face, self.cfg
        f.conf = min(0.95, max(0.01, float(c.prescan_face_conf)))
        f._probe_conf = float(c.prescan_probe_conf)
        f._prescan_period = int(c.prescan_rot_probe_period)
        f._prescan_probe_imgsz = int(c.prescan_probe_imgsz)
        f._prescan_no_upscale_det = bool(c.prescan_no_upscale_det)
        f._high_90 = int(c.prescan_heavy_90)
        f._high_180 = int(c.prescan_heavy_180)

    def _gate(self, st: _LoopState) -> Tuple[bool, bool]:
        """(skip_extract, gate_active) of the fd9 skip gate (gui_app.py:1479-1492)."""
        c = self.cfg
        if (not st.active) and c.prescan_fd9_skip:
            grace = max(0, int(c.prescan_fd9_grace))
            period = max(1, int(c.prescan_fd9_probe_period))
            if st.fd9_streak >= grace:
                return (st.fd9_streak % period) != 0, True
        return False, False

    def _downscale_many(self, ims, ks):
        """_downscale of a chunk's samples: the frames wider than prescan_max_width in one batched
        INTER_AREA launch (face_embedder.dev_resize_batch), the same bytes as one resize each."""
        from .face_embedder import dev_resize_batch
        Wmax = int(self.cfg.prescan_max_width)
        out = list(ims)
        wide = [t for t, im in enumerate(ims) if im.W > Wmax]
        by_dims = {}
        for t in wide:
            by_dims.setdefault((ims[t].H, ims[t].W), []).append(t)
        for (H, W), ts in by_dims.items():
            nh = int(round(H * (Wmax / float(W))))
            res = dev_resize_batch(self.face._ctx, [ims[t] for t in ts], [f"prescan{ks[t]}" for t in ts], (Wmax, nh))
            for t, r in zip(ts, res):
                out[t] = r
        return out

    def _downscale(self, im, k: int):
        """gui_app.py:1505-1507: INTER_AREA to prescan_max_width when wider."""
        Wmax = int(self.cfg.prescan_max_width)
        if im.W > Wmax:
            nh = int(round(im.H * (Wmax / float(im.W))))
            return self.face._dev_resize(im, f"prescan{k}", dsize=(Wmax, nh), area=True)
        return im

    def _finish_sample(self, st: _LoopState, idx: int, sample_idx: int, faces, extracted: bool) -> SampleRecord:
        """Bank growth, fd9 streak and span hysteresis of one sample (gui_app.py:1512-1622)."""
        c = self.cfg
        best = 9.0
        action = ""
        if extracted:
            for f in faces:
                feat = f.get("feat")
                if feat is None:
                    continue
                fd = fd_min(feat, st.bank)
                best = min(best, fd)
                if fd <= float(c.prescan_fd_add) and (sample_idx - st.last_add_sample) >= int(
                        c.prescan_add_cooldown_samples) and f.get("quality", 1e9) >= c.face_quality_min:
                    st.bank, action, _ = stream_ref_bank_update(
                        st.bank_list, st.bank, feat, float(f.get("quality", 0.0)), cap=int(c.prescan_bank_max),
                        dedup_cos=float(c.prescan_diversity_dedup_cos), rep_margin=float(c.prescan_replace_margin),
                        weights=tuple(c.prescan_weights))
                    if action in ("added", "replaced"):
                        st.last_add_sample = sample_idx
                        st.added += action == "added"
        st.fd9_streak = st.fd9_streak + 1 if best >= 8.99 else 0
        if extracted:
            st.last_found = best < 8.99
        stride = max(1, int(c.prescan_stride))
        pad = int(round(c.prescan_pad_sec * self.fps))
        min_len = int(round(c.prescan_min_segment_sec * self.fps))
        if best <= float(c.prescan_fd_enter):
            if not st.active:
                st.active = True
                st.fd9_streak = 0
                st.start = idx
            st.neg_run = 0
        elif st.active:
            st.neg_run += 1
            exit_cool = int(round(max(0.0, float(c.prescan_exit_cooldown_sec)) * self.fps))
            if st.neg_run * stride >= exit_cool or best >= float(c.prescan_fd_exit):
                s = max(0, st.start - pad)
                e = min(self.total - 1, idx + pad)
                if e - s + 1 >= min_len:
                    if st.spans and s <= st.spans[-1][1] + 1:
                        st.spans[-1] = (st.spans[-1][0], max(st.spans[-1][1], e))
                    else:
                        st.spans.append((s, e))
                st.active = False
                st.neg_run = 0
                st.fd9_streak = 0
        n = len(faces) if extracted else 0
        return SampleRecord(idx, extracted, float(best), n, action, st.active)

    def run(self, frame_at: Callable[[int], object], positions: Optional[range] = None,
            speculate: bool = False) -> Tuple[List[Tuple[int, int]], Optional[np.ndarray]]:
        """frame_at(frame_index) -> the frame as a device image (face_embedder._DevImage) or a host
        BGR array. Returns (spans, updated bank) like Processor._prescan.
        positions: run only these sample positions (a contiguous shard of the sample list, as
        if the clip started there); speculate: record every extracted sample as a SpecRecord
        in self.spec (regime, policy state in / out, faces) for the sharded merge."""
        f, c = self.face, self.cfg
        self.setup_face()
        self.initial_state = f.policy_state()
        samples = self.samples()
        pos = range(len(samples)) if positions is None else positions
        if speculate:
            self.spec = []
        st = _LoopState(self.ref_feat)
        k = pos.start
        while k < pos.stop:
            plan, active0, state0, by_pos, state_after, dims = self.spec_chunk(frame_at, st, k, pos.stop)
            # ---- replay; cut at the first divergence ----
            last_state = state0
            cut = None
            for j, skip_pred in plan:
                skip, _ = self._gate(st)
                if skip != skip_pred or st.active != active0:
                    cut = j
                    break
                rec = self._finish_sample(st, samples[j], st.processed, by_pos.get(j, []), not skip)
                st.processed += 1
                self.records.append(rec)
                if not skip:
                    if speculate:
                        self.spec.append(SpecRecord(j, active0, last_state, state_after[j], _host_faces(by_pos[j]),
                                                    dims[j]))
                    last_state = state_after[j]
            if cut is not None:
                self.cuts += 1
                k = cut
            else:
                k = plan[-1][0] + 1
            f.set_policy_state(last_state)
        spans = self.close(st)
        f.set_prescan_fast(False)
        f.set_prescan_hint(escalate=False)
        self.final_state = st
        return spans, st.bank


def _host_faces(faces) -> list:
    """The parts of extract()'s face dicts the pre-scan loop and its merge read (picklable
    host values: no chips or device handles)."""
    keep = ("bbox", "kps5", "feat", "quality", "score")
    return [{k: f[k] for k in keep if k in f} for f in faces]


def run_cached(runner: "PrescanRunner", frame_at, video, refs="", cache_dir: str = "prescan_cache",
               mode: str = "auto", settings=None):
    """Processor._prescan's cache wrapper (gui_app.py:847-920 around the sampling loop): a hit
    returns the stored spans and bank without touching a frame; a miss runs the loop and stores
    its result. `settings`: the SessionConfig-like source of the key (default: the runner's
    PrescanConfig, other keys at SessionConfig defaults). Returns (spans, bank, hit)."""
    from . import prescan_cache as pcache
    if settings is None:
        settings = _runner_settings(runner)
    meta = pcache.cache_meta(settings, video, refs, runner.fps, runner.total)
    root = pcache.cache_root(cache_dir)
    hit, spans, bank = pcache.load(root, meta, mode)
    if hit:
        return spans, bank, True
    spans, bank = runner.run(frame_at)
    try:   # a read-only or full cache dir must not lose the computed result (gui_app.py:919)
        pcache.save(root, meta, spans, bank, mode)
    except Exception as e:   # noqa: BLE001 - the reference logs and continues the same way
        runner.cache_error = f"{type(e).__name__}: {e}"
    return spans, bank, False


def _runner_settings(runner: "PrescanRunner") -> dict:
    """Cache-key settings of a runner: its PrescanConfig fields plus the face backend that
    actually ran (face_model / use_arcface are key fields, gui_app.py:821-825), so caches of
    different detectors never collide."""
    from dataclasses import asdict
    s = asdict(runner.cfg)
    face = getattr(runner, "face", None)
    model = getattr(face, "detector_backend", None)
    if model == "scrfd" or model is None:
        variant = getattr(face, "scrfd_variant", "10g")
        model = {"10g": "scrfd_10g_bnkps", "2.5g": "scrfd_2.5g_bnkps"}.get(variant, f"scrfd_{variant}")
    elif model == "yolo":   # the model name the FaceEmbedder was built with
        model = os.path.basename(str(getattr(face, "_scrfd_model_path", "") or "yolov8-face"))
    s["face_model"] = model
    s["use_arcface"] = bool(getattr(face, "use_arcface", True))
    return s


def prescan_sequential(face, cfg: PrescanConfig, fps: float, total_frames: int, frame_at, ref_feat=None):
    """The same loop one sample per extract (batch 1): the reference's own order, for tests."""
    r = PrescanRunner(face, cfg, fps, total_frames, ref_feat=ref_feat, batch=1)
    out = r.run(frame_at)
    return out, r
