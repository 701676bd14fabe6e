"""Minimal ctypes binding of the HIP runtime (libamdhip64) -- device memory,
streams and events for the device-resident path, bench and tests.

This is plumbing, not a compatibility layer: it binds the same
libamdhip64.so.7 the engine library links, so buffers and streams created
here are directly usable by fd_ed25519_amd_verify_dev.  (PyTorch-ROCm ships
its own HIP runtime build; loading both in one process makes whichever comes
second see no GPU, so the GPU path here does not go through torch.)
"""
import ctypes
import os

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is not None:
        return _hip
    cands = [os.environ.get("FD_AMD_HIP_LIB"), "/opt/rocm/lib/libamdhip64.so.7", "libamdhip64.so.7"]
    last = None
    for c in cands:
        if not c:
            continue
        try:
            H = ctypes.CDLL(c, mode=ctypes.RTLD_GLOBAL)
            break
        except OSError as e:
            last = e
    else:
        raise RuntimeError("libamdhip64 not found: %s" % last)
    vp, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    H.hipGetDeviceCount.argtypes = [ctypes.POINTER(i)]
    H.hipSetDevice.argtypes = [i]
    H.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    H.hipFree.argtypes = [vp]
    H.hipMemcpy.argtypes = [vp, vp, sz, i]
    H.hipMemcpyAsync.argtypes = [vp, vp, sz, i, vp]
    H.hipMemset.argtypes = [vp, i, sz]
    H.hipMemsetAsync.argtypes = [vp, i, sz, vp]
    H.hipDeviceSynchronize.argtypes = []
    H.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    H.hipStreamDestroy.argtypes = [vp]
    H.hipStreamSynchronize.argtypes = [vp]
    H.hipEventCreate.argtypes = [ctypes.POINTER(vp)]
    H.hipEventDestroy.argtypes = [vp]
    H.hipEventRecord.argtypes = [vp, vp]
    H.hipEventSynchronize.argtypes = [vp]
    H.hipStreamWaitEvent.argtypes = [vp, vp, u]
    H.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
    H.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, u]
    H.hipHostFree.argtypes = [vp]
    H.hipGetErrorString.argtypes = [i]
    H.hipGetErrorString.restype = ctypes.c_char_p
    H.hipDeviceGetName = getattr(H, "hipDeviceGetName", None)
    if H.hipDeviceGetName is not None:
        H.hipDeviceGetName.argtypes = [ctypes.c_char_p, i, i]
    _hip = H
    return H


H2D, D2H, D2D = 1, 2, 3


def check(rc, what=""):
    if rc != 0:
        raise RuntimeError("HIP error %d (%s) in %s" % (rc, hip().hipGetErrorString(rc).decode(), what))


def device_count():
    n = ctypes.c_int(0)
    rc = hip().hipGetDeviceCount(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(d):
    check(hip().hipSetDevice(int(d)), "hipSetDevice")


def device_name(d=0):
    H = hip()
    if H.hipDeviceGetName is None:
        return "unknown"
    buf = ctypes.create_string_buffer(256)
    if H.hipDeviceGetName(buf, 256, int(d)) != 0:
        return "unknown"
    return buf.value.decode()


def synchronize():
    check(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceBuffer:
    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(hip().hipMalloc(ctypes.byref(p), max(self.nbytes, 1)), "hipMalloc(%d)" % self.nbytes)
        self.ptr = p.value

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        if a.nbytes:
            check(hip().hipMemcpy(b.ptr, a.ctypes.data, a.nbytes, H2D), "hipMemcpy H2D")
        return b

    def to_array(self, dtype, count):
        out = np.zeros(count, dtype)
        if out.nbytes:
            check(hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H), "hipMemcpy D2H")
        return out

    def zero(self):
        check(hip().hipMemset(self.ptr, 0, max(self.nbytes, 1)), "hipMemset")

    def free(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc), viewable as a numpy array."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(hip().hipHostMalloc(ctypes.byref(p), max(self.nbytes, 1), 0), "hipHostMalloc(%d)" % self.nbytes)
        self.ptr = p.value

    def array(self, dtype=np.uint8):
        n = self.nbytes // np.dtype(dtype).itemsize
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr)).view(dtype)[:n]

    def free(self):
        if self.ptr:
            hip().hipHostFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def h2d_bandwidth(nbytes=256 << 20, reps=5):
    """Measured pinned host -> device copy rate in GB/s (the PCIe ceiling
    the host-staged paths are priced against)."""
    src, dst, st = PinnedBuffer(nbytes), DeviceBuffer(nbytes), Stream()
    e0, e1 = Event(), Event()
    H = hip()
    check(H.hipMemcpyAsync(dst.ptr, src.ptr, nbytes, H2D, st.handle), "hipMemcpyAsync")
    st.synchronize()
    e0.record(st)
    for _ in range(reps):
        check(H.hipMemcpyAsync(dst.ptr, src.ptr, nbytes, H2D, st.handle), "hipMemcpyAsync")
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_ms(e1)
    st.destroy(); src.free(); dst.free()
    return nbytes * reps / (ms * 1e-3) / 1e9


class Stream:
    def __init__(self):
        s = ctypes.c_void_p()
        check(hip().hipStreamCreate(ctypes.byref(s)), "hipStreamCreate")
        self.handle = s.value

    def synchronize(self):
        check(hip().hipStreamSynchronize(self.handle), "hipStreamSynchronize")

    def wait(self, event):
        """Later work on this stream waits for `event`'s latest record."""
        check(hip().hipStreamWaitEvent(self.handle, event.handle, 0), "hipStreamWaitEvent")

    def destroy(self):
        if self.handle:
            hip().hipStreamDestroy(self.handle)
            self.handle = None


class Event:
    def __init__(self):
        e = ctypes.c_void_p()
        check(hip().hipEventCreate(ctypes.byref(e)), "hipEventCreate")
        self.handle = e.value

    def record(self, stream):
        check(hip().hipEventRecord(self.handle, stream.handle if isinstance(stream, Stream) else stream), "hipEventRecord")

    def synchronize(self):
        check(hip().hipEventSynchronize(self.handle), "hipEventSynchronize")

    def elapsed_ms(self, later):
        f = ctypes.c_float()
        check(hip().hipEventElapsedTime(ctypes.byref(f), self.handle, later.handle), "hipEventElapsedTime")
        return f.value
