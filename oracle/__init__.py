"""CPU oracle for the person_capture identity hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything from this package, and only as the checker (or the timed CPU
baseline). The product (person_capture_amd) never imports it; its GPU path has
no CPU fallback.

Contents
  ref_algos.py   numpy restatements of the reference's host-side algorithms
                 (match, bank growth, landmark canonicalisation, IoU/NMS, SCRFD
                 decode, ArcFace post-processing), each citing the reference
                 file:line it follows; pinned against golden vectors generated
                 from the reference itself (tests/golden, tools/gen_golden.py).
  cv_ops.c       C restatement of the OpenCV 4.9 u8 image arithmetic the path
                 uses (resize INTER_LINEAR/INTER_AREA, warpAffine, BGR2GRAY,
                 Laplacian variance). OpenCV itself is absent: parity unpinned
                 against OpenCV, bit-exact against the GPU kernels.
  nets_torch.py  fp32 torch-CPU forward of IResNet / SCRFD from unfolded params.
"""
