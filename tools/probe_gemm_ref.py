"""Reference point for the conv engine: torch.matmul (hipBLASLt) f16 on the GEMM shapes of
the ArcFace-r100 b256 3x3 layers as plain GEMMs (im2col already materialised; no epilogue),
HIP-event timed. Not on the product path: a ceiling estimate for the implicit-GEMM kernels."""
import torch

SHAPES = [("s3 14x14x256", 50176, 256, 2304), ("s2 28x28x128", 200704, 128, 1152),
          ("s1 56x56x64", 802816, 64, 576), ("s4 7x7x512", 12544, 512, 4608)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name:14s} M={M} N={N} K={K}: {ms * 1e3:8.1f} us  {2 * M * N * K / ms / 1e9:7.1f} TFLOP/s", flush=True)
