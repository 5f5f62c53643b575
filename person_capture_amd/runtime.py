"""Thin Python handles over the pcgpu C ABI: a per-GPU context, device buffers
and compiled networks. No torch types cross the boundary; device memory is
owned by the native library (hipMalloc) and addressed by integer pointers."""
from __future__ import annotations

import atexit
import ctypes as C
import weakref
from typing import Dict, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import PC_PREC_F16, PC_PREC_F32, check


class DeviceBuffer:
    """A raw device allocation owned by a GpuContext."""

    def __init__(self, ctx: "GpuContext", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(ctx.lib.pc_device_alloc(ctx.handle, max(self.nbytes, 16), C.byref(p)), ctx.handle, "alloc")
        self.ptr = int(p.value)

    def free(self) -> None:
        if self.ptr and self.ctx.handle:
            self.ctx.lib.pc_device_free(self.ctx.handle, C.c_void_p(self.ptr))
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) viewed as a flat uint8 numpy array."""

    def __init__(self, ctx: "GpuContext", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(ctx.lib.pc_host_alloc(ctx.handle, max(self.nbytes, 16), C.byref(p)), ctx.handle, "host_alloc")
        self.ptr = int(p.value)
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))

    def view(self, shape, dtype, offset: int = 0) -> np.ndarray:
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        if offset + n > self.nbytes:
            raise ValueError("pinned view out of range")
        return self.array[offset:offset + n].view(dtype).reshape(shape)

    def free(self) -> None:
        if self.ptr and self.ctx.handle:
            self.array = None
            self.ctx.lib.pc_host_free(self.ctx.handle, C.c_void_p(self.ptr))
        self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Fence:
    """A HIP event recorded on the context stream (host waits for the work before it)."""

    def __init__(self, ctx: "GpuContext"):
        self.ctx = ctx
        h = C.c_void_p()
        check(ctx.lib.pc_fence_create(ctx.handle, C.byref(h)), ctx.handle, "fence_create")
        self.handle = h

    def record(self) -> "Fence":
        check(self.ctx.lib.pc_fence_record(self.ctx.handle, self.handle), self.ctx.handle, "fence_record")
        return self

    def wait(self) -> None:
        check(self.ctx.lib.pc_fence_wait(self.ctx.handle, self.handle), self.ctx.handle, "fence_wait")

    def __del__(self):
        try:
            if self.handle and self.ctx.handle:
                self.ctx.lib.pc_fence_destroy(self.ctx.handle, self.handle)
        except Exception:
            pass


# Every live context, closed at interpreter exit before the HIP runtime's own teardown: a native
# object destroyed from a garbage-collection finaliser after the runtime is gone (or after its
# context) is what aborted the r04n suite process at exit (teardown order).
_LIVE_CONTEXTS: "weakref.WeakSet[GpuContext]" = weakref.WeakSet()


@atexit.register
def _close_all_contexts() -> None:
    for c in list(_LIVE_CONTEXTS):
        try:
            c.close()
        except Exception:
            pass


class GpuContext:
    """One context per (GPU, consumer): stream, zero page, staging ring. Nets created on it are
    destroyed before it (close() closes them first; pc_net_destroy needs its context)."""

    def __init__(self, device_id: int = 0):
        self.lib = _lib.load()
        self.device_id = int(device_id)
        h = C.c_void_p()
        rc = self.lib.pc_ctx_create(self.device_id, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"pcgpu: cannot create a context on HIP device {device_id} (status {rc})")
        self.handle = h
        self._keep = []   # host arrays referenced by in-flight async copies
        self._bufs: Dict[str, DeviceBuffer] = {}
        self._pinned: Dict[str, PinnedBuffer] = {}
        self._fences: Dict[str, Fence] = {}
        self._nets: "weakref.WeakSet[Net]" = weakref.WeakSet()
        _LIVE_CONTEXTS.add(self)

    def close(self) -> None:
        if self.handle:
            for n in list(self._nets):
                n.close()
            self._bufs.clear()
            self._pinned.clear()
            self._fences.clear()
            self.lib.pc_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- memory ----
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def scratch(self, key: str, nbytes: int) -> DeviceBuffer:
        """A named, growable scratch buffer (reused across calls)."""
        b = self._bufs.get(key)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                self.sync()
            b = DeviceBuffer(self, max(int(nbytes), 256))
            self._bufs[key] = b
        return b

    def pinned(self, key: str, nbytes: int) -> PinnedBuffer:
        """A named, growable pinned host buffer. The caller owns the ordering: a buffer
        may only be reused once the fence covering its last copy has been waited on."""
        b = self._pinned.get(key)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                self.sync()
            b = PinnedBuffer(self, max(int(nbytes), 4096))
            self._pinned[key] = b
        return b

    def fence(self, key: str) -> Fence:
        """Record (and return) the named fence on the context stream."""
        f = self._fences.get(key)
        if f is None:
            f = self._fences[key] = Fence(self)
        return f.record()

    def download_async(self, ptr: int, pin: PinnedBuffer, offset: int, shape, dtype) -> np.ndarray:
        """Stream-ordered D2H into pinned memory; the returned view is valid after a
        later fence on this context has been waited on."""
        out = pin.view(shape, dtype, offset)
        if out.nbytes:
            check(self.lib.pc_copy_d2h(self.handle, C.c_void_p(pin.ptr + offset), C.c_void_p(int(ptr)), out.nbytes),
                  self.handle, "d2h")
        return out

    def upload(self, arr: np.ndarray, dst: Optional[DeviceBuffer] = None, offset: int = 0) -> DeviceBuffer:
        a = np.ascontiguousarray(arr)
        if dst is None:
            dst = self.alloc(a.nbytes)
        check(self.lib.pc_copy_h2d(self.handle, C.c_void_p(dst.ptr + offset), a.ctypes.data_as(C.c_void_p), a.nbytes),
              self.handle, "h2d")
        self._keep.append(a)
        return dst

    def stage_frame(self, img: np.ndarray, d_dst: int, threads: int = 4) -> None:
        """Host image [H][W][C] u8 (row-strided views allowed) -> d_dst packed, through the
        native pinned staging ring (pc_frame_stage); the array may be reused on return."""
        if (img.ndim != 3 or img.dtype != np.uint8 or img.strides[2] != 1 or img.strides[1] != img.shape[2]
                or img.strides[0] < img.shape[1] * img.shape[2]):
            img = np.ascontiguousarray(img, dtype=np.uint8)
        row = img.shape[1] * img.shape[2]
        check(self.lib.pc_frame_stage(self.handle, C.c_void_p(int(d_dst)), C.c_void_p(img.ctypes.data), row,
                                      img.shape[0], img.strides[0], int(threads)), self.handle, "frame_stage")

    def wait_fence(self, fence: "Fence") -> None:
        """Work enqueued on this context from now on waits for `fence` (another context's)."""
        check(self.lib.pc_ctx_wait_fence(self.handle, fence.handle), self.handle, "wait_fence")

    def download(self, ptr: int, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        if out.nbytes:
            check(self.lib.pc_copy_d2h(self.handle, out.ctypes.data_as(C.c_void_p), C.c_void_p(int(ptr)), out.nbytes),
                  self.handle, "d2h")
        self.sync()
        return out

    def memset(self, ptr: int, value: int, nbytes: int) -> None:
        check(self.lib.pc_memset(self.handle, C.c_void_p(int(ptr)), int(value), int(nbytes)), self.handle, "memset")

    def sync(self) -> None:
        check(self.lib.pc_ctx_sync(self.handle), self.handle, "sync")
        self._keep.clear()

    def set_priority(self, priority: int) -> None:
        """Re-create this context's stream at a HIP priority (lower = higher; clamped)."""
        check(self.lib.pc_ctx_set_priority(self.handle, int(priority)), self.handle, "set_priority")

    @property
    def stream(self) -> int:
        return int(self.lib.pc_ctx_stream(self.handle) or 0)


class Net:
    """A compiled network resident on one GPU (weights + activation buffers)."""

    def __init__(self, ctx: GpuContext, program: bytes, precision: int = PC_PREC_F16, max_batch: int = 1):
        self.ctx = ctx
        self.precision = int(precision)
        self.max_batch = int(max_batch)
        buf = C.create_string_buffer(program, len(program))
        h = C.c_void_p()
        check(ctx.lib.pc_net_create(ctx.handle, buf, len(program), self.precision, self.max_batch, C.byref(h)),
              ctx.handle, "net_create")
        self.handle = h
        ctx._nets.add(self)
        d = (C.c_int32 * 4)()
        check(ctx.lib.pc_net_input_dims(h, d), ctx.handle, "input_dims")
        self.input_dims = tuple(d)
        fl = C.c_double()
        nl = C.c_int32()
        ctx.lib.pc_net_stats(h, C.byref(fl), C.byref(nl))
        self.flops_per_image = fl.value
        self.launches = nl.value

    @property
    def act_itemsize(self) -> int:
        return 4 if self.precision == PC_PREC_F32 else 2

    def close(self) -> None:
        # a closed context has destroyed its nets already (GpuContext.close)
        if getattr(self, "handle", None) and self.ctx.handle:
            self.ctx.lib.pc_net_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def chain_info(self) -> Tuple[int, int, int]:
        """(resident block chains, batch from which they run, images per round of workgroups)."""
        mb, pr = C.c_int32(), C.c_int32()
        k = self.ctx.lib.pc_net_chain_info(self.handle, C.byref(mb), C.byref(pr))
        if k < 0:
            check(-k, self.ctx.handle, "chain_info")
        return k, mb.value, pr.value

    def set_chain_min_batch(self, min_batch: int) -> None:
        """Batch from which the resident block chains run (<= 0: never)."""
        k = self.ctx.lib.pc_net_set_chain_min_batch(self.handle, int(min_batch))
        if k < 0:
            check(-k, self.ctx.handle, "set_chain_min_batch")

    def set_graph(self, enable: bool, max_batch: Optional[int] = None) -> None:
        """HIP-graph capture / replay of net runs (of at most max_batch images when given)."""
        check(self.ctx.lib.pc_net_set_graph(self.handle, 1 if enable else 0), self.ctx.handle, "set_graph")
        if max_batch is not None:
            check(self.ctx.lib.pc_net_set_graph_max_batch(self.handle, int(max_batch)), self.ctx.handle,
                  "set_graph_max_batch")

    def calibrate(self, d_input: int, batch: int, headroom_log2: int = 5, n_tensors: int = 0) -> Optional[np.ndarray]:
        """pc_net_calibrate: the f16c8 tensors' e4m3 scales from one run over `batch` images at
        d_input. Returns the measured max |x| per tensor when n_tensors is given."""
        buf = (C.c_float * n_tensors)() if n_tensors else None
        check(self.ctx.lib.pc_net_calibrate(self.handle, C.c_void_p(int(d_input)), int(batch), int(headroom_log2), buf),
              self.ctx.handle, "net_calibrate")
        return np.frombuffer(buf, dtype=np.float32).copy() if n_tensors else None

    def profile(self, enable: bool) -> None:
        check(self.ctx.lib.pc_net_profile(self.handle, 1 if enable else 0), self.ctx.handle, "profile")

    def profile_read(self) -> dict:
        out = (C.c_double * 5)()
        check(self.ctx.lib.pc_net_profile_read(self.handle, out), self.ctx.handle, "profile_read")
        return {"conv_ms": out[0], "conv_launches": int(out[1]), "conv_flops": out[2], "other_ms": out[3],
                "other_launches": int(out[4])}

    def profile_ops(self, max_recs: int = 65536) -> np.ndarray:
        """[n][6]: op index, kind, ms, flops, halo tile (-1 = igemm), igemm tile (profiled runs)."""
        out = (C.c_double * (6 * max_recs))()
        k = self.ctx.lib.pc_net_profile_ops(self.handle, out, max_recs)
        if k < 0:
            check(-k, self.ctx.handle, "profile_ops")
        return np.frombuffer(out, dtype=np.float64, count=6 * k).reshape(k, 6).copy()

    def run(self, d_input: int, batch: int) -> None:
        check(self.ctx.lib.pc_net_run(self.handle, C.c_void_p(int(d_input)), int(batch)), self.ctx.handle, "net_run")

    def output(self, i: int) -> Tuple[int, Tuple[int, int, int, int, int]]:
        p = C.c_void_p()
        d = (C.c_int32 * 5)()
        check(self.ctx.lib.pc_net_output(self.handle, i, C.byref(p), d), self.ctx.handle, "net_output")
        return int(p.value), tuple(d)

    def read_output(self, i: int, batch: int) -> np.ndarray:
        """Download output i as float32 [batch][H][W][C] (channel padding dropped by caller)."""
        ptr, (H, W, Cc, cs, is_f32) = self.output(i)
        dt = np.float32 if is_f32 else np.float16
        raw = self.ctx.download(ptr, (batch, H, W, cs), dt)
        return raw[..., :Cc].astype(np.float32)
