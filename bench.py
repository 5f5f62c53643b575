#!/usr/bin/env python3
"""Benchmark: frames/sec of detect + embed + match @1080p (BASELINE.json `metric`).

Workload (BASELINE.json configs[2], the single-GPU config the metric is quoted
on): a batch of 64 synthetic 1080p BGR frames resident in HBM; one step =
FaceEmbedder.extract_batch over the batch (SCRFD-10G letterbox + detect + NMS,
5-point align, quality, ArcFace-R100 with flip-TTA, L2) + cosine match of every
face against a 32-entry reference bank on the device. Seeded synthetic
weights (no checkpoints exist offline). Frames shard across ranks with no
collective (weak scaling): each rank runs its own batch; value = all frames /
max-over-ranks time.

Also reported: roofline of the dominant kernel family (the MFMA implicit-GEMM
convs of both networks: algorithmic FLOPs / HIP-event time of their launches
inside the timed region) and a bounded CPU baseline (the oracle port of the same
pipeline, rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F16_TFLOPS = 2500.0   # MI355X dense fp16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_F32_TFLOPS = 157.3


def _dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        from person_capture_amd.shard import dist_timeout
        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank, timeout=dist_timeout())
    return world, rank, local


def _device(local: int) -> int:
    from person_capture_amd.shard import device_for_rank
    return device_for_rank(local)


def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _max_over_ranks(world, v: float) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum_over_ranks(world, v: float) -> float:
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def synth_frames(rank: int, n: int, H: int = 1080, W: int = 1920) -> np.ndarray:
    """np.random.default_rng(seed=20260501 + frame_idx) u8 BGR frames."""
    out = np.empty((n, H, W, 3), np.uint8)
    for i in range(n):
        out[i] = np.random.default_rng(20260501 + rank * 1_000_000 + i).integers(0, 256, (H, W, 3), dtype=np.uint8)
    return out


def synth_bank(n: int, dim: int = 512) -> np.ndarray:
    b = np.random.default_rng(20260503).standard_normal((n, dim)).astype(np.float32)
    return b / np.linalg.norm(b, axis=1, keepdims=True)


def plant_bank(res, bank_h: np.ndarray) -> int:
    """Plant a quarter of the bank (in place) from the faces of a first pass; returns the count."""
    feats = [f["feat"] for r in res for f in r]
    n_plant = min(len(feats), len(bank_h) // 4)
    if n_plant:
        rng = np.random.default_rng(20260504)
        mean = np.mean(feats, axis=0)
        for k, i in enumerate(rng.choice(len(feats), n_plant, replace=False)):
            v = feats[i] - 0.3 * mean + (0.1 + 0.1 * k) * rng.standard_normal(512).astype(np.float32) / np.sqrt(512.0)
            bank_h[k] = v / np.linalg.norm(v)
    return n_plant


def cpu_baseline(frames: np.ndarray, fe, bank: np.ndarray, n_sample: int, n_sample_1t: int):
    """The oracle port of the same pipeline on the host cores, bounded sample: all-core
    (16 threads, the box's CPU share) and single-thread (the reference CLI pins torch and
    OpenCV to one thread, main.py:3-6,14)."""
    import torch
    from oracle import pipeline as op

    def run(threads, n):
        torch.set_num_threads(threads)
        t0 = time.perf_counter()
        faces = 0
        for i in range(n):
            r = op.extract_frame(frames[i], fe._scrfd_params, fe.scrfd_variant, fe._arc_params, fe._arc_depth,
                                 conf=fe.conf, D=640, bank=bank)
            faces += 0 if r == op.NEEDS_FALLBACK else len(r)
        return n / (time.perf_counter() - t0), faces, time.perf_counter() - t0

    threads = min(16, os.cpu_count() or 1)
    v, faces, dt = run(threads, n_sample)
    out = {"value": round(v, 4), "unit": "frames/s", "cores": threads, "kind": "port",
           "host_cpu_count": os.cpu_count(),
           "sample": f"{n_sample} of the bench's 1080p frames through oracle/pipeline.extract_frame "
                     f"(fp32 torch-CPU SCRFD-10G + ArcFace-R100 flip-TTA, numpy/C post), {faces} faces, "
                     f"{dt:.1f} s at {threads} threads"}
    if n_sample_1t > 0:
        v1, faces1, dt1 = run(1, n_sample_1t)
        out["value_1_thread"] = round(v1, 4)
        out["sample_1_thread"] = f"first {n_sample_1t} frames, {faces1} faces, {dt1:.1f} s at 1 thread"
    torch.set_num_threads(threads)
    return out


def f16_parity(fe16, devs, bank_h, conf: float = 0.5) -> dict:
    """Outside the timed region: the same frames through an f32 FaceEmbedder (the parity mode,
    itself checked against the fp32 CPU oracle in tests/test_gpu_bench_config.py) against the
    f16 throughput mode, face by face (nearest box): how many decisions f16 changes, and where
    the difference enters. f16 is the precision of the reference's TensorRT engines
    (face_embedder.py:1058). Attribution: the f16 pass's own chips are embedded again by the
    f32 ArcFace, which separates the ArcFace error (same chip, f16 vs f32 net) from the
    detection error (SCRFD f16 landmarks -> a different aligned chip)."""
    from person_capture_amd.face_embedder import FaceEmbedder
    from person_capture_amd.match import DeviceBank

    def run(fe, bank):
        fe.debug_chips = True
        try:
            r = fe.extract_batch([None] * len(devs), dev_frames=devs, bank=bank)
        finally:
            fe.debug_chips = False
        fe._ctx.sync()
        fe._ectx.sync()
        return r

    res16 = run(fe16, DeviceBank(fe16._ctx, bank_h))
    old = {k: os.environ.get(k) for k in ("PERSON_CAPTURE_AMD_PRECISION", "PERSON_CAPTURE_AMD_DET_PRECISION")}
    for k in old:
        os.environ[k] = "f32"
    try:
        fe32 = FaceEmbedder(ctx=f"cuda:{_device(int(os.environ.get('LOCAL_RANK', '0')))}",
                            yolo_model="scrfd_10g_bnkps", conf=conf)
        res32 = run(fe32, DeviceBank(fe32._ctx, bank_h))
        chips16 = [f["chip"] for r in res16 for f in r]
        e32_on16 = fe32._arc.embed(np.stack(chips16), flip=True) if chips16 else np.zeros((0, 512), np.float32)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    fd_arc32 = iter((1.0 - e32_on16 @ bank_h.T).min(1).tolist() if len(chips16) else [])
    for r in res16:
        for f in r:
            f["fd_arc32"] = next(fd_arc32)
    n = count_mis = box_mis = acc_mis = acc_mis_45 = chip_same = arc_flip = 0
    worst_fd = worst_arc = 0.0
    kps_d = []
    near = []
    for a16, a32 in zip(res16, res32):
        count_mis += abs(len(a16) - len(a32))
        for b in a32:
            n += 1
            a = min(a16, key=lambda f: int(np.abs(f["bbox"].astype(np.int64) - b["bbox"]).sum())) if a16 else None
            if a is None:
                box_mis += 1
                continue
            if not np.array_equal(a["bbox"], b["bbox"]):
                box_mis += 1
            if a["kps5"] is not None and b["kps5"] is not None:
                kps_d.append(float(np.abs(a["kps5"] - b["kps5"]).max()))
            chip_same += int(np.array_equal(a["chip"], b["chip"]))
            d = abs(float(a["fd"]) - float(b["fd"]))
            worst_fd = max(worst_fd, d)
            worst_arc = max(worst_arc, abs(float(a["fd"]) - a["fd_arc32"]))
            arc_flip += (a["fd"] <= 0.32) != (a["fd_arc32"] <= 0.32)
            if (a["fd"] <= 0.32) != (b["fd"] <= 0.32):
                acc_mis += 1
                near.append(round(abs(float(b["fd"]) - 0.32), 5))
            acc_mis_45 += (a["fd"] <= 0.45) != (b["fd"] <= 0.45)
    kps_d = np.array(kps_d) if kps_d else np.zeros(1)
    return {"reference": "same frames, f32 parity mode on the device", "faces_f32": n,
            "face_count_mismatch": count_mis, "box_mismatch": box_mis, "accept_mismatch_0.32": acc_mis,
            "accept_mismatch_0.45": acc_mis_45, "accept_mismatch_frac_0.32": round(acc_mis / max(1, n), 4),
            "max_fd_diff": round(worst_fd, 6), "flipped_faces_f32_distance_to_0.32": sorted(near),
            "attribution": {
                "chips_identical": chip_same,
                "kps_abs_diff_px": {"median": round(float(np.median(kps_d)), 5), "max": round(float(kps_d.max()), 5)},
                "arcface_only_max_fd_diff": round(worst_arc, 6),
                "arcface_only_accept_flips_0.32": arc_flip,
                "note": "arcface_only: f16 fd vs the f32 ArcFace on the f16 pass's own chips; the rest of the "
                        "difference enters through the SCRFD f16 landmarks (a different aligned chip; the "
                        "bench frames are u8 noise, so a sub-pixel landmark shift resamples the chip)"}}


def smooth_parity(fe16, frames: np.ndarray, bank_rows: int) -> dict:
    """The f16-vs-f32 comparison on the bench frames low-pass filtered (Gaussian, sigma 1.5 px):
    u8 noise frames resample to unrelated chips under a sub-pixel landmark shift, smooth
    frames (like camera images) do not. Same planted-bank construction, own bank."""
    from scipy.ndimage import gaussian_filter
    from person_capture_amd.face_embedder import _DevImage
    from person_capture_amd.match import DeviceBank
    sm = np.empty_like(frames)
    for i, f in enumerate(frames):   # blur, then restore contrast about the noise mean 127.5
        g = gaussian_filter(f.astype(np.float32), sigma=(1.5, 1.5, 0))
        sm[i] = np.clip(np.rint(128.0 + 2.5 * (g - 127.5)), 0, 255).astype(np.uint8)
    ctx = fe16._ctx
    d = ctx.alloc(sm.nbytes)
    ctx.upload(sm, d)
    fsz = sm[0].nbytes
    H, W = sm.shape[1:3]
    devs = [_DevImage(d.ptr + i * fsz, H, W, W * 3) for i in range(len(sm))]
    bank_h = synth_bank(bank_rows)
    conf0 = fe16.conf
    fe16.conf = 0.8   # the synthetic SCRFD fires on ~380 anchors of a smooth 1080p frame at 0.5, ~6 at 0.8
    try:
        first = fe16.extract_batch([None] * len(devs), dev_frames=devs, bank=DeviceBank(ctx, bank_h))
        plant_bank(first, bank_h)
        r = f16_parity(fe16, devs, bank_h, conf=0.8)
    finally:
        fe16.conf = conf0
    r.pop("flipped_faces_f32_distance_to_0.32", None)
    r["frames"] = "bench frames, Gaussian sigma 1.5 px, contrast x2.5 about 127.5; SCRFD conf 0.8"
    ctx.sync()
    d.free()
    return r


def _kernel_of(code: float, cfg: float) -> str:
    """Planner code of a profiled conv launch (pc_net_profile_ops) -> kernel instantiation."""
    c = int(code)
    if c == 300:
        return "conv_chain (resident IResNet block chain, pc_conv_chain.hip)"
    if c >= 200:
        return f"conv_t2d (2-D block kernel, variant {c - 200})"
    if c >= 100:
        return f"conv_fast tile cfg {c - 100} (pc_conv_fast.hip kFastCfgs)"
    if c >= 0:
        return f"conv_halo tile {c}"
    return f"conv_igemm tile cfg {int(cfg)}"


def dominant_conv(nets, names) -> dict:
    """The conv kernel instantiation with the largest total HIP-event time over the timed
    region (per-launch records of every profiled net), with its algorithmic FLOPs per launch
    and average launch duration: the roofline line is this kernel's."""
    agg = {}
    total = 0.0
    for n, name in zip(nets, names):
        for op, kind, ms, fl, code, cfg in n.profile_ops():
            if fl <= 0:
                continue
            k = (name, int(code), int(cfg) if code < 0 else -1)
            a = agg.setdefault(k, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += ms
            a[2] += fl
            total += ms
    if not agg:
        return {"kernel": None, "code": None, "launches": 0, "avg_us": None, "flops_per_launch": None,
                "achieved_tflops": 0.0, "share": None}
    (name, code, cfg), (cnt, ms, fl) = max(agg.items(), key=lambda kv: kv[1][1])
    return {"kernel": f"{_kernel_of(code, cfg)} in {name}" + (
                " = conv_fast<f16,256,224,128,4,2,2,1> (ArcFace 14x14x256 layers)" if code == 113 else ""),
            "code": code, "launches": cnt, "avg_us": round(ms * 1e3 / cnt, 2), "flops_per_launch": round(fl / cnt),
            "achieved_tflops": round(fl / (ms * 1e-3) / 1e12, 2), "share": round(ms / total, 4)}


def load_traffic():
    """HBM bytes per conv launch from the round's rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (tools/pmc_traffic.py writes bench_traffic.json at the repo root, next to this file, so
    it travels to the GPU box)."""
    tpath = os.path.join(ROOT, "bench_traffic.json")
    if not os.path.isfile(tpath):
        return None, None
    try:
        t = json.load(open(tpath))
    except Exception:
        return None, None
    return t.get("conv_hbm_bytes_per_launch"), t.get("dominant")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bank", type=int, default=32)
    ap.add_argument("--cpu-sample", type=int, default=48)
    ap.add_argument("--cpu-sample-1t", type=int, default=4)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the f16-vs-f32 decision parity pass")
    ap.add_argument("--precision", default="f16", choices=["f16", "f32"])
    ap.add_argument("--frames", default="resident", choices=["resident", "host", "per-frame"],
                    help="C3 frame source: resident in HBM (the headline), host arrays through extract_batch "
                         "(H2D inside the timed region), or one extract() per host frame")
    ap.add_argument("--det-size", type=int, default=640, help="C3 --frames per-frame: extract(imgsz=...)")
    ap.add_argument("--face-model", default="scrfd_10g_bnkps",
                    help="C3 FaceEmbedder detector (yolov8l-face.pt: the reference default an unchanged main.py gets)")
    ap.add_argument("--face-conf", type=float, default=0.5,
                    help="C3 SCRFD threshold (the synthetic SCRFD-10G fires on ~1000 anchors of a 1080p noise frame "
                         "at D=1408 and 0.5; 0.75 gives a handful, as at D=640 and 0.5)")
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c4", "c5"],
                    help="c3: BASELINE configs[2] (the metric's config, default); c2: ArcFace-R100 embed only at "
                         "batch 256 (the north star's MFMA target); c4: full path with YOLOv8n "
                         "persons + per-crop SCRFD/ArcFace + CLIP ReID; c5: 4K pre-scan (INTER_AREA 416 wide, "
                         "SCRFD @384, 1 ArcFace forward, 1024-entry bank)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N self-launch: kill every rank if the job runs longer (seconds)")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)   # launcher test hook
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the rank launcher, dist init and the timing/reduction protocol only")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # --gpus N without torch.distributed.run: start N fresh rank processes (this process has not
        # touched the GPU) and exit with their status
        from person_capture_amd.shard import spawn_local_ranks
        sys.exit(spawn_local_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus,
                                   timeout=args.launch_timeout))
    if args.dry_run:
        return main_dry(args)
    if args.workload == "c2":
        return main_c2(args)
    if args.workload != "c3":
        return main_other(args)

    world, rank, local = _dist_init()
    local = _device(local)
    os.environ.setdefault("PERSON_CAPTURE_AMD_PRECISION", args.precision)
    os.environ.setdefault("PERSON_CAPTURE_AMD_DET_BATCH", str(args.batch))
    os.environ.setdefault("PERSON_CAPTURE_AMD_ARC_BATCH", "512")
    from person_capture_amd._lib import PC_PREC_F32
    from person_capture_amd.face_embedder import FaceEmbedder, _DevImage
    from person_capture_amd.match import DeviceBank, fd_min

    fe = FaceEmbedder(ctx=f"cuda:{local}", yolo_model=args.face_model, conf=args.face_conf)
    frames = synth_frames(rank, args.batch)
    ctx = fe._ctx
    dframes = ctx.alloc(frames.nbytes)
    ctx.upload(frames, dframes)
    fsz = frames[0].nbytes
    devs = [_DevImage(dframes.ptr + i * fsz, 1080, 1920, 1920 * 3) for i in range(args.batch)]
    bank_h = synth_bank(args.bank)
    bank = DeviceBank(ctx, bank_h)
    ctx.sync()

    host_list = list(frames)

    def step():
        if args.frames == "host":
            # caller frames in pageable host memory: pinned staging + H2D inside the timed region
            return fe.extract_batch(host_list, bank=bank)
        if args.frames == "per-frame":
            # an unchanged caller (main.py:246, gui_app.py:6045): extract() one host frame at a
            # time, fd against the bank on the host as the reference's Processor does
            out = []
            for f in host_list:
                faces = fe.extract(f, imgsz=args.det_size)
                for fc in faces:
                    fc["fd"] = fd_min(fc["feat"], bank_h)
                out.append(faces)
            return out
        return fe.extract_batch([None] * args.batch, dev_frames=devs, bank=bank)

    res = step()
    # plant a quarter of the bank with embeddings of faces the pipeline finds in these frames
    # (a reference bank is built from the target's own faces, gui_app.py:922-986) so the
    # accept path runs too; the rest stay random rows. The synthetic (untrained) embedder's
    # outputs share a large common component, so the planted rows carry 0.3 of the mean
    # removed plus noise of growing strength (as tests/test_gpu_bench_config.planted_bank):
    # the distances then straddle the CLI's 0.32 threshold instead of accepting every face.
    n_plant = plant_bank(res, bank_h)
    if n_plant:
        bank = DeviceBank(ctx, bank_h)
    for _ in range(args.warmup):
        res = step()
    nfaces = sum(len(r) for r in res)
    accept = sum(1 for r in res for f in r if f["fd"] <= 0.45)
    accept_cli = sum(1 for r in res for f in r if f["fd"] <= 0.32)
    if fe.detector_backend == "yolo":
        det_nets = [e.net for e in fe._yf_engines.values()]
        net_names = tuple(f"yolo-face{k}" for k in range(len(det_nets))) + ("arcface",)
    else:
        det_nets = [e.net for e in fe._scrfd_engines.values()] if args.frames == "per-frame" else [fe._engine(640).net]
        net_names = tuple("scrfd" if k == 0 else f"scrfd{k}" for k in range(len(det_nets))) + ("arcface",)
    nets = det_nets + [fe._arc.net]
    if not os.getenv("PC_BENCH_NOPROF"):
        for n in nets:
            n.profile(True)
    if fe.host_times is not None:
        fe.host_times.clear()
    _barrier(world)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    t1 = time.perf_counter()
    _barrier(world)
    elapsed = _max_over_ranks(world, t1 - t0)
    prof = [n.profile_read() for n in nets]
    dom = dominant_conv(nets, net_names)
    for n in nets:
        n.profile(False)
    if fe.host_times is not None:
        print("host phases ms/step: " + ", ".join(f"{k} {v * 1e3 / args.steps:.2f}" for k, v in fe.host_times.items()),
              file=sys.stderr)
    conv_ms = sum(p["conv_ms"] for p in prof)
    conv_launches = sum(p["conv_launches"] for p in prof)
    conv_flops = sum(p["conv_flops"] for p in prof)
    total_frames = _sum_over_ranks(world, args.batch * args.steps)
    value = total_frames / elapsed
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    peak = PEAK_F16_TFLOPS if args.precision == "f16" else PEAK_F32_TFLOPS
    traffic, dominant = load_traffic()
    out = {
        "metric": "frames/sec detect+embed+match @1080p, 1/2/4/8 GPU; MFMA util %",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (seeded u8 1080p frames, seeded synthetic SCRFD-10G/IResNet-100 weights)",
        "config": {"workload": "C3: SCRFD-10G detect + ArcFace-R100 embed (flip-TTA) + cosine match vs "
                               f"{args.bank}-embedding bank, 1080p, batch {args.batch} frames per GPU",
                   "frames_per_step_per_gpu": args.batch, "det_size": args.det_size, "face_model": args.face_model, "face_conf": args.face_conf, "bank": args.bank,
                   "frames": {"resident": "resident in HBM before the timed region",
                              "host": "pageable host arrays, extract_batch: pinned staging + H2D timed",
                              "per-frame": "pageable host arrays, one extract() per frame (unchanged callers), "
                                           "host fd"}[args.frames],
                   "faces_per_frame": round(nfaces / args.batch, 3), "accepted_faces_per_step": accept,
                   "accepted_faces_per_step_cli_0.32": accept_cli, "bank_planted_rows": n_plant,
                   "detector_dtype": "f32" if fe.det_precision == PC_PREC_F32 else "f16",
                   "parallelism": f"frame-shard x{world} (no collective)"},
        "roofline": {"bound": "mfma", "achieved": dom["achieved_tflops"], "peak": peak, "unit": "TFLOP/s",
                     "frac": round(dom["achieved_tflops"] / peak, 4),
                     "traffic": (dominant or {}).get("hbm_bytes_per_launch") if dom["code"] == 113 else None,
                     "kernel": dom["kernel"], "kernel_launches": dom["launches"],
                     "kernel_avg_launch_us": dom["avg_us"], "kernel_flops_per_launch": dom["flops_per_launch"],
                     "kernel_share_of_conv_time": dom["share"],
                     "conv_family": {"achieved": round(achieved, 2), "frac": round(achieved / peak, 4),
                                     "traffic_mean_per_launch": traffic},
                     "launches": conv_launches, "avg_launch_us": round(conv_ms * 1e3 / max(1, conv_launches), 2),
                     "flops_per_launch": round(conv_flops / max(1, conv_launches)),
                     "conv_share_of_step": round(conv_ms * 1e-3 / (t1 - t0), 4),
                     "streams": 2 if fe._ectx is not fe._ctx else 1,
                     "streams_note": "ArcFace (embed stream) runs beside SCRFD (detection stream): the conv "
                                     "event spans of the two overlap, so conv_share_of_step can exceed 1 and a "
                                     "launch's duration includes the co-running kernels' share of the CUs",
                     "per_net": {name: {"conv_ms_per_step": round(p_["conv_ms"] / args.steps, 3),
                                        "tflops": round(p_["conv_flops"] / (p_["conv_ms"] * 1e-3) / 1e12, 1)
                                        if p_["conv_ms"] > 0 else None}
                                 for name, p_ in zip(net_names, prof)},
                     "traffic_unit": "HBM bytes per launch of the dominant kernel (rocprofv3 FETCH_SIZE x2 + "
                                     "WRITE_SIZE, bench_traffic.json); conv_family.traffic_mean_per_launch: the mean "
                                     "over all conv launches",
                     "dominant_kernel_rocprof": dominant},
        "cpu_baseline": None,
    }
    if rank == 0 and args.precision == "f16" and not args.no_parity and args.frames == "resident" and \
            fe.detector_backend == "scrfd":
        out["parity"] = f16_parity(fe, devs, bank_h)
        # the same pipeline with the detector in f32 (PERSON_CAPTURE_AMD_DET_PRECISION=f32): f32
        # landmarks give the f32 chips; its throughput and decisions, measured here too
        old_dp = os.environ.get("PERSON_CAPTURE_AMD_DET_PRECISION")
        os.environ["PERSON_CAPTURE_AMD_DET_PRECISION"] = "f32"
        try:
            fe_d = FaceEmbedder(ctx=f"cuda:{local}", yolo_model="scrfd_10g_bnkps", conf=0.5)
        finally:
            if old_dp is None:
                os.environ.pop("PERSON_CAPTURE_AMD_DET_PRECISION", None)
            else:
                os.environ["PERSON_CAPTURE_AMD_DET_PRECISION"] = old_dp
        run_d = lambda: fe_d.extract_batch([None] * args.batch, dev_frames=devs, bank=bank)
        run_d()
        fe_d._ctx.sync()
        t0 = time.perf_counter()
        for _ in range(3):
            run_d()
        fe_d._ctx.sync()
        fe_d._ectx.sync()
        fps_d = 3 * args.batch / (time.perf_counter() - t0)
        pd = f16_parity(fe_d, devs, bank_h)
        out["parity"]["detector_f32_mode"] = {
            "frames_per_s": round(fps_d, 2), "steps": 3,
            **{k: pd[k] for k in ("face_count_mismatch", "box_mismatch", "accept_mismatch_0.32",
                                  "accept_mismatch_0.45", "accept_mismatch_frac_0.32", "max_fd_diff")},
            "chips_identical": pd["attribution"]["chips_identical"],
            "note": "SCRFD f32 + ArcFace f16 (env PERSON_CAPTURE_AMD_DET_PRECISION=f32): identical chips, the "
                    "remaining flips are the f16 ArcFace's"}
        out["parity"]["smooth_frames"] = smooth_parity(fe, frames, args.bank)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(frames, fe, bank_h, args.cpu_sample, args.cpu_sample_1t)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def _timed(world, ctx, steps, step):
    _barrier(world)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    t1 = time.perf_counter()
    _barrier(world)
    return _max_over_ranks(world, t1 - t0), t1 - t0


def main_c2(args):
    """C2 (BASELINE configs[1]): ArcFace-R100 embed only, batch 256 aligned 112x112 faces, f16,
    one GPU per rank. One step = pc_arcface_embed over 256 device-resident u8 chips (preprocess
    -> IResNet-100 -> L2) without flip, i.e. 256 forward rows: the batch the north star's
    '>= 50 % MFMA at batch 256' is quoted on. The flip-TTA form the reference's
    _arcface_encode runs (face_embedder.py:1290-1389: 256 faces = 512 rows) is timed beside it
    (flip_tta). roofline: the whole network's algorithmic FLOPs / step time (all of its MFMA
    work), plus the dominant kernel's own launch rate."""
    world, rank, local = _dist_init()
    local = _device(local)
    from person_capture_amd import models
    from person_capture_amd._lib import PC_PREC_F16, PC_PREC_F32
    from person_capture_amd.engines import ArcFaceEngine
    from person_capture_amd.runtime import GpuContext
    B = 256
    ctx = GpuContext(local)
    prec = PC_PREC_F16 if args.precision == "f16" else PC_PREC_F32
    eng = ArcFaceEngine(ctx, models.synth_iresnet(100, seed=0), 100, precision=prec, max_batch=2 * B)
    chips = np.random.default_rng(20260505 + rank).integers(0, 256, (B, 112, 112, 3), dtype=np.uint8)
    d_chips = ctx.upload(chips)
    d_out = ctx.alloc(B * eng.dim * 4)
    for _ in range(max(1, args.warmup)):
        eng.embed_device(d_chips.ptr, B, False, d_out.ptr)
        eng.embed_device(d_chips.ptr, B, True, d_out.ptr)
    ctx.sync()
    elapsed, _ = _timed(world, ctx, args.steps, lambda: eng.embed_device(d_chips.ptr, B, False, d_out.ptr))
    t_flip, _ = _timed(world, ctx, args.steps, lambda: eng.embed_device(d_chips.ptr, B, True, d_out.ptr))
    # per-launch split of one profiled step (HIP events on the net's stream)
    eng.net.profile(True)
    eng.embed_device(d_chips.ptr, B, False, d_out.ptr)
    dom = dominant_conv([eng.net], ("arcface",))
    recs = eng.net.profile_ops()
    eng.net.profile(False)
    peak = PEAK_F16_TFLOPS if args.precision == "f16" else PEAK_F32_TFLOPS
    fl = eng.flops_per_forward * B
    ms = elapsed / args.steps * 1e3
    net_tf = fl / (ms * 1e-3) / 1e12
    split = {}
    for op, kind, t, f, code, cfg in recs:
        k = _kernel_of(code, cfg) if f > 0 else "other"
        a = split.setdefault(k, [0, 0.0, 0.0])
        a[0] += 1; a[1] += t; a[2] += f
    total_faces = _sum_over_ranks(world, B * args.steps)
    out = {
        "metric": "ArcFace-R100 embeddings/sec at batch 256 (C2); MFMA util %",
        "value": round(total_faces / elapsed, 2), "unit": "faces/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (seeded u8 112x112 chips, seeded synthetic IResNet-100 weights)",
        "config": {"workload": "C2: ArcFace-R100 embed only, batch 256 aligned 112x112 faces (256 forward rows), "
                               "preprocess + IResNet-100 + L2 on device", "batch": B,
                   "parallelism": f"replica x{world} (no collective)"},
        "roofline": {"bound": "mfma", "achieved": round(net_tf, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(net_tf / peak, 4), "traffic": None,
                     "scope": "whole IResNet-100 forward: algorithmic conv FLOPs of 256 rows / step time "
                              f"({fl / 1e12:.3f} TFLOP per step)",
                     "dominant_kernel": dom,
                     "per_kernel": {k: {"launches": v[0], "ms": round(v[1], 4),
                                        "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1) if v[1] > 0 and v[2] > 0
                                        else None} for k, v in sorted(split.items(), key=lambda kv: -kv[1][1])}},
        "flip_tta": {"faces_per_step": B, "rows": 2 * B, "ms_per_step": round(t_flip / args.steps * 1e3, 4),
                     "faces_per_s": round(_sum_over_ranks(world, B * args.steps) / t_flip, 2),
                     "tflops": round(2 * fl / (t_flip / args.steps) / 1e12, 2)},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main_dry(args):
    """The multi-rank protocol without a GPU (CPU test of the launcher): every rank
    'processes' its contiguous share of a batch with a host stand-in, then the same
    barrier / max-over-ranks time / sum-over-ranks frames reduction as the real run."""
    from person_capture_amd.shard import shard_indices
    if args.fail_rank >= 0 and int(os.environ.get("RANK", "0")) == args.fail_rank:
        sys.exit(1)   # launcher test: this rank dies before the rendezvous
    world, rank, local = _dist_init()
    total = args.batch * max(1, world)
    mine = shard_indices(total, rank, world)
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sum(i * i for i in mine)
    t1 = time.perf_counter()
    _barrier(world)
    elapsed = max(_max_over_ranks(world, t1 - t0), 1e-9)
    frames = _sum_over_ranks(world, len(mine) * args.steps)
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": frames / elapsed, "unit": "frames/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "frames": frames, "local_rank": local}),
              flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main_other(args):
    """C4 (full path) and C5 (4K pre-scan): secondary workloads, same JSON contract."""
    world, rank, local = _dist_init()
    local = _device(local)
    os.environ.setdefault("PERSON_CAPTURE_AMD_PRECISION", args.precision)
    os.environ.setdefault("PERSON_CAPTURE_AMD_DET_BATCH", str(args.batch))
    os.environ.setdefault("PERSON_CAPTURE_AMD_ARC_BATCH", "512")
    from person_capture_amd._lib import PC_PREC_F32
    from person_capture_amd.face_embedder import FaceEmbedder, _DevImage
    from person_capture_amd.match import DeviceBank

    fe = FaceEmbedder(ctx=f"cuda:{local}", yolo_model="scrfd_10g_bnkps", conf=0.5)
    ctx = fe._ctx
    H, W = (1080, 1920) if args.workload == "c4" else (2160, 3840)
    frames = synth_frames(rank, args.batch, H, W)
    dframes = ctx.alloc(frames.nbytes)
    ctx.upload(frames, dframes)
    fsz = frames[0].nbytes
    devs = [_DevImage(dframes.ptr + i * fsz, H, W, W * 3) for i in range(args.batch)]
    bank_n = args.bank if args.workload == "c4" else 1024
    bank = DeviceBank(ctx, synth_bank(bank_n))
    stats = {}
    nets = [fe._arc.net]
    if args.workload == "c4":
        from person_capture_amd.detectors import PersonDetector
        from person_capture_amd.reid_embedder import ReIDEmbedder
        det = PersonDetector("yolov8n.pt", device=f"cuda:{local}")
        # the untrained synthetic SCRFD fires on ~150 anchors of a bilinearly upscaled person crop
        # at 0.5 (it was calibrated on native-scale frames); 0.75 gives a few faces per crop as a
        # trained detector would. Real weights need no such knob.
        fe.conf = 0.75
        reid = ReIDEmbedder(device=f"cuda:{local}")
        stats["reid_dtype"] = "f32" if reid._engine.net.precision == 1 else "f16"
        dtuples = [(d.ptr, H, W, W * 3) for d in devs]

        def step():
            persons = det.detect_device(dtuples, conf=0.35)
            crops = []
            for d, dets in zip(devs, persons):
                for x1, y1, x2, y2, _ in dets:   # main.py:231-236
                    x1, y1 = max(0, int(x1)), max(0, int(y1))
                    x2, y2 = min(W - 1, int(x2)), min(H - 1, int(y2))
                    if x2 <= x1 + 2 or y2 <= y1 + 2:
                        continue
                    crops.append(_DevImage(d.ptr + y1 * d.stride + x1 * 3, y2 - y1, x2 - x1, d.stride))
            faces = fe.extract_batch([None] * len(crops), dev_frames=crops, bank=bank) if crops else []
            feats = reid.extract_device([(c.ptr, c.H, c.W, c.stride) for c in crops])
            stats["persons"] = len(crops)
            stats["faces"] = sum(len(f) for f in faces)
            return feats
        nets += [fe._engine(640).net, reid._engine.net]
        wl = (f"C4: YOLOv8n persons + SCRFD-10G@640 per person crop + ArcFace-R100 flip-TTA + CLIP ViT-L/14 ReID "
              f"per crop + match vs {bank_n}-embedding bank, 1080p, batch {args.batch} frames per GPU")
    else:
        # the pre-scan driver (Processor._prescan's sampling loop, person_capture_amd/prescan.py):
        # the resident 4K frames are the sampled frames of a clip at stride 24 (gui_app.py:555),
        # downscaled to 416 wide on the device, fast pre-scan SCRFD + ArcFace, fd against the
        # 1024-row bank, bank growth and span hysteresis replayed in sample order
        from person_capture_amd.prescan import PrescanConfig, PrescanRunner
        pcfg = PrescanConfig()
        stride = pcfg.prescan_stride
        bank_h = synth_bank(bank_n)
        # plant a quarter of the bank from faces of the first samples (downscaled as the driver
        # does) so spans open and the escalated two-forward path is timed too
        r0 = PrescanRunner(fe, pcfg, 30.0, args.batch * stride, ref_feat=None, batch=args.batch)
        ims = [r0._downscale(devs[i], i) for i in range(min(16, len(devs)))]
        fe.set_prescan_fast(True, mode="rr")
        seed_res = fe.extract_batch([None] * len(ims), dev_frames=ims)
        fe.set_prescan_fast(False)
        stats["bank_planted_rows"] = plant_bank(seed_res, bank_h)

        def step():
            r = PrescanRunner(fe, pcfg, 30.0, args.batch * stride, ref_feat=bank_h, batch=args.batch)
            spans, _ = r.run(lambda idx: devs[idx // stride])
            stats["faces"] = sum(x.n_faces for x in r.records)
            stats["extracted_samples"] = sum(1 for x in r.records if x.extracted)
            stats["driver_chunks"], stats["driver_cuts"], stats["spans"] = r.chunks, r.cuts, len(spans)
            return spans
        wl = (f"C5: pre-scan driver over 4K frames sampled at stride {stride} -> INTER_AREA 416 wide, fast pre-scan "
              f"SCRFD-10G, ArcFace-R100 (1 forward, 2 while a span is active), fd vs {bank_n}-embedding bank, "
              f"batch {args.batch} samples per GPU")
    for k in range(args.warmup):
        t = time.perf_counter()
        step()
        ctx.sync()
        print(f"[bench {args.workload}] warmup {k}: {time.perf_counter() - t:.3f} s {stats}", file=sys.stderr,
              flush=True)
    if args.workload == "c5":
        nets += [e.net for e in fe._scrfd_engines.values()]
    for n in nets:
        n.profile(True)
    elapsed, local_dt = _timed(world, ctx, args.steps, step)
    prof = [n.profile_read() for n in nets]
    for n in nets:
        n.profile(False)
    conv_ms = sum(p["conv_ms"] for p in prof)
    conv_flops = sum(p["conv_flops"] for p in prof)
    conv_launches = sum(p["conv_launches"] for p in prof)
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    peak = PEAK_F16_TFLOPS if args.precision == "f16" else PEAK_F32_TFLOPS
    total_frames = _sum_over_ranks(world, args.batch * args.steps)
    out = {
        "metric": "frames/sec detect+embed+match @1080p, 1/2/4/8 GPU; MFMA util %" if args.workload == "c4"
        else "frames/sec pre-scan detect+embed+match @4K, 1/2/4/8 GPU; MFMA util %",
        "value": round(total_frames / elapsed, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (seeded u8 frames, seeded synthetic weights of every net)",
        "config": {"workload": wl, "frames_per_step_per_gpu": args.batch, "bank": bank_n,
                   **{k: v for k, v in stats.items()}, "parallelism": f"frame-shard x{world} (no collective)"},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": None,
                     "kernel": "implicit-GEMM MFMA convs (all nets, ViT linears as 1x1)", "launches": conv_launches,
                     "avg_launch_us": round(conv_ms * 1e3 / max(1, conv_launches), 2),
                     "conv_share_of_step": round(conv_ms * 1e-3 / local_dt, 4)},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
