"""MI355X-native (gfx950) implementation of person_capture's per-frame identity
hot path: SCRFD face detect -> 5-point align -> ArcFace embed -> L2 -> cosine
bank match (+ YOLO person detect and ReID body embed), behind the reference's
FaceEmbedder / PersonDetector / ReIDEmbedder class surfaces.

Device work runs in hand-written HIP kernels (csrc/, built into lib/libpcgpu.so)
called through the C ABI in include/pcgpu.h. There is no CPU fallback.
"""
__version__ = "0.1.0"
