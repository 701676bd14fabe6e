"""Python mirror of the reference's ed25519 API over the MI355X engine.

Reference interface: src/ballet/ed25519/fd_ed25519.h (fd_ed25519_verify,
fd_ed25519_sign, fd_ed25519_public_from_private, fd_ed25519_strerror,
FD_ED25519_SUCCESS / ERR_SIG / ERR_PUBKEY / ERR_MSG).  Same names, same
argument meaning, same codes.  Everything here is a thin ctypes layer over
firedancer_amd/libfd_ed25519_amd.so (include/fd_ed25519_amd.h); the verify
work always runs in the HIP kernels.  If the library is missing this module
raises at import of the first call -- there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

FD_ED25519_SUCCESS = 0
FD_ED25519_ERR_SIG = -1
FD_ED25519_ERR_PUBKEY = -2
FD_ED25519_ERR_MSG = -3
FD_ED25519_SIG_SZ = 64
MSG_MAX = 1232

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FD_AMD_LIB") or os.path.join(_HERE, "libfd_ed25519_amd.so")   # override: A/B builds only

_lib = None

c_ulong_p = ctypes.POINTER(ctypes.c_ulong)
c_void_pp = ctypes.POINTER(ctypes.c_void_p)


def lib():
    """Load the engine library (once).  Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            "firedancer_amd: %s missing -- build it with __graft_entry__.build() "
            "(the verify engine is HIP-only; there is no CPU path)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    vp, ul, ui, i = ctypes.c_void_p, ctypes.c_ulong, ctypes.c_uint, ctypes.c_int
    L.fd_ed25519_verify.argtypes = [vp, ul, vp, vp, vp]
    L.fd_ed25519_verify.restype = i
    L.fd_ed25519_strerror.argtypes = [i]
    L.fd_ed25519_strerror.restype = ctypes.c_char_p
    L.fd_ed25519_public_from_private.argtypes = [vp, vp, vp]
    L.fd_ed25519_public_from_private.restype = vp
    L.fd_ed25519_sign.argtypes = [vp, vp, ul, vp, vp, vp]
    L.fd_ed25519_sign.restype = vp
    L.fd_ed25519_amd_new.argtypes = [i, ul, ul]
    L.fd_ed25519_amd_new.restype = vp
    L.fd_ed25519_amd_delete.argtypes = [vp]
    L.fd_ed25519_amd_delete.restype = None
    L.fd_ed25519_amd_verify_batch.argtypes = [vp, ul, c_void_pp, c_ulong_p, c_void_pp, c_void_pp, vp]
    L.fd_ed25519_amd_verify_batch.restype = i
    L.fd_ed25519_amd_verify_soa.argtypes = [vp, ul, vp, vp, vp, vp, vp, ul, vp]
    L.fd_ed25519_amd_verify_soa.restype = i
    L.fd_ed25519_amd_workspace_footprint.argtypes = [ul]
    L.fd_ed25519_amd_workspace_footprint.restype = ul
    L.fd_ed25519_amd_verify_dev.argtypes = [ul, vp, vp, vp, vp, vp, vp, vp, vp]
    L.fd_ed25519_amd_verify_dev.restype = i
    L.fd_ed25519_amd_verify_dev_ev.argtypes = [ul, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.fd_ed25519_amd_verify_dev_ev.restype = i
    L.fd_ed25519_amd_work_stats_dev.argtypes = [ul, vp, vp, vp]
    L.fd_ed25519_amd_work_stats_dev.restype = i
    L.fd_ed25519_amd_debug_digits_dev.argtypes = [ul, vp, vp, vp, vp]
    L.fd_ed25519_amd_debug_digits_dev.restype = i
    L.fd_ed25519_amd_version.argtypes = []
    L.fd_ed25519_amd_version.restype = ctypes.c_char_p
    L.fd_ed25519_amd_sign_batch.argtypes = [ul, vp, vp, vp, vp, vp, vp, i]
    L.fd_ed25519_amd_sign_batch.restype = i
    L.fd_ed25519_amd_verify_txns.argtypes = [vp, ul, vp, vp, vp, ul, vp, vp, vp]
    L.fd_ed25519_amd_verify_txns.restype = i
    L.fd_txn_amd_parse_dev.argtypes = [ul, vp, vp, vp, vp, vp, ul, vp]
    L.fd_txn_amd_parse_dev.restype = i
    L.fd_ed25519_amd_sign_dev.argtypes = [ul, vp, vp, vp, vp, vp, vp, vp]
    L.fd_ed25519_amd_sign_dev.restype = i
    L.fd_ed25519_amd_set_small_batch_max.argtypes = [ul]
    L.fd_ed25519_amd_set_small_batch_max.restype = None
    L.fd_ed25519_amd_set_latency_batch_max.argtypes = [ul]
    L.fd_ed25519_amd_set_latency_batch_max.restype = None
    L.fd_ed25519_amd_set_pool_batch_min.argtypes = [ul]
    L.fd_ed25519_amd_set_pool_batch_min.restype = None
    L.fd_ed25519_amd_debug_set_pool_iter_cap.argtypes = [ul]
    L.fd_ed25519_amd_debug_set_pool_iter_cap.restype = None
    L.fd_verify_amd_tile_new.argtypes = [i, ul, ul, ul, ul]
    L.fd_verify_amd_tile_new.restype = vp
    L.fd_verify_amd_tile_cfg_default.argtypes = [vp]
    L.fd_verify_amd_tile_cfg_default.restype = None
    L.fd_verify_amd_tile_new_cfg.argtypes = [vp]
    L.fd_verify_amd_tile_new_cfg.restype = vp
    L.fd_verify_amd_tile_set_trace.argtypes = [vp, vp, ul]
    L.fd_verify_amd_tile_set_trace.restype = None
    L.fd_verify_amd_tile_set_verdict_log.argtypes = [vp, vp, ul]
    L.fd_verify_amd_tile_set_verdict_log.restype = None
    L.fd_verify_amd_tile_cut.argtypes = [vp, ul, ul, ul, i, ul, i]
    L.fd_verify_amd_tile_cut.restype = ul
    L.fd_verify_amd_tile_mode.argtypes = [i, i, ctypes.c_double, ctypes.c_double, ctypes.c_double]
    L.fd_verify_amd_tile_mode.restype = i

    L.fd_verify_amd_tile_pack.argtypes = [vp, ul, i, c_ulong_p]
    L.fd_verify_amd_tile_pack.restype = ul
    L.fd_verify_amd_tile_out_chunk0.argtypes = [vp]
    L.fd_verify_amd_tile_out_chunk0.restype = vp
    L.fd_verify_amd_tile_out_data_sz.argtypes = [vp]
    L.fd_verify_amd_tile_out_data_sz.restype = ul
    L.fd_ed25519_amd_host_register.argtypes = [vp, ul]
    L.fd_ed25519_amd_host_register.restype = i
    L.fd_ed25519_amd_host_unregister.argtypes = [vp]
    L.fd_ed25519_amd_host_unregister.restype = i
    L.fd_ed25519_amd_verify_soa_registered.argtypes = [vp, ul, vp, vp, vp, vp, vp, ul, vp]
    L.fd_ed25519_amd_verify_soa_registered.restype = i
    L.fd_ed25519_amd_multi_new.argtypes = [vp, ul, ul, ul]
    L.fd_ed25519_amd_multi_new.restype = vp
    L.fd_ed25519_amd_multi_delete.argtypes = [vp]
    L.fd_ed25519_amd_multi_delete.restype = None
    L.fd_ed25519_amd_multi_ndev.argtypes = [vp]
    L.fd_ed25519_amd_multi_ndev.restype = ul
    L.fd_ed25519_amd_shard_range.argtypes = [ul, ul, ul, c_ulong_p, c_ulong_p]
    L.fd_ed25519_amd_shard_range.restype = None
    L.fd_ed25519_amd_multi_verify_soa.argtypes = [vp, ul, vp, vp, vp, vp, vp, ul, vp]
    L.fd_ed25519_amd_multi_verify_soa.restype = i
    L.fd_ed25519_amd_multi_verify_txns.argtypes = [vp, ul, vp, vp, vp, ul, vp, vp, vp]
    L.fd_ed25519_amd_multi_verify_txns.restype = i
    L.fd_ed25519_amd_txn_slots.argtypes = [ul, vp, vp, vp, vp]
    L.fd_ed25519_amd_txn_slots.restype = ul
    L.fd_verify_amd_tile_register_dcache.argtypes = [vp, vp, ul]
    L.fd_verify_amd_tile_register_dcache.restype = i
    L.fd_verify_amd_tile_set_framing.argtypes = [vp, i]
    L.fd_verify_amd_tile_set_framing.restype = i
    L.fd_verify_amd_tile_delete.argtypes = [vp]
    L.fd_verify_amd_tile_delete.restype = None
    L.fd_verify_amd_tile_run.argtypes = [vp, vp, ul, vp, ul, vp, vp, ul, ul, vp, ul, vp, vp, vp, ul]
    L.fd_verify_amd_tile_run.restype = i
    L.fd_verify_amd_tickcount.argtypes = []
    L.fd_verify_amd_tickcount.restype = ui
    L.fd_verify_amd_bench_stream.argtypes = [i, ul, ul, ctypes.c_double, i, ul, ul, vp, vp, vp, vp, vp, vp, vp, ul,
                                             ul, vp]
    L.fd_verify_amd_bench_stream.restype = i
    # entry points added in round 6 (an A/B build of an earlier round, FD_AMD_LIB, lacks them)
    opt = {"fd_ed25519_amd_dropin_set_device": ([i], i), "fd_ed25519_amd_dropin_device": ([], i),
           "fd_ed25519_amd_dropin_pick": ([ctypes.POINTER(i), i, i, ul], i),
           "fd_verify_amd_tile_level": ([i, i] + [ctypes.c_double] * 5, i),
           "fd_verify_amd_tile_level_step": ([i, i, ul, ul, ctypes.POINTER(ul)], i)}
    for name, (args, res) in opt.items():
        if hasattr(L, name) or not os.environ.get("FD_AMD_LIB"):
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
    _lib = L
    return L


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else ctypes.c_void_p(0)


def _u8(b):
    return np.frombuffer(bytes(b), np.uint8)


# ---------------------------------------------------------------- reference API

def strerror(err):
    """fd_ed25519_strerror (fd_ed25519.h:108-109)."""
    return lib().fd_ed25519_strerror(int(err)).decode()


def verify(msg, sig, public_key):
    """fd_ed25519_verify (fd_ed25519.h:96-101): returns 0 or FD_ED25519_ERR_*.
    Runs on the GPU as a batch of one."""
    m = bytes(msg)
    s = bytes(sig)
    p = bytes(public_key)
    assert len(s) == 64 and len(p) == 32
    mb = ctypes.create_string_buffer(m, max(len(m), 1))
    return lib().fd_ed25519_verify(mb if m else None, len(m), s, p, None)


DROPIN_AUTO = -1


def dropin_set_device(device):
    """fd_ed25519_amd_dropin_set_device: the calling thread's device for
    verify() (DROPIN_AUTO: the default rule).  Raises on a bad device."""
    rc = lib().fd_ed25519_amd_dropin_set_device(int(device))
    if rc:
        raise EngineError("fd_ed25519_amd_dropin_set_device(%d) rc=%d" % (device, rc))


def dropin_device():
    """The device of the calling thread's drop-in engine (-1 before its first call)."""
    return int(lib().fd_ed25519_amd_dropin_device())


def dropin_pick(dev_node, cpu_node, ordinal):
    """fd_ed25519_amd_dropin_pick: the default device rule (pure)."""
    a = (ctypes.c_int * max(len(dev_node), 1))(*dev_node)
    return int(lib().fd_ed25519_amd_dropin_pick(a, len(dev_node), int(cpu_node), int(ordinal)))


def public_from_private(private_key):
    """fd_ed25519_public_from_private (fd_ed25519.h:40-44)."""
    out = ctypes.create_string_buffer(32)
    lib().fd_ed25519_public_from_private(out, bytes(private_key), None)
    return out.raw


def sign(msg, public_key, private_key):
    """fd_ed25519_sign (fd_ed25519.h:71-78) -> 64-byte signature."""
    out = ctypes.create_string_buffer(64)
    m = bytes(msg)
    lib().fd_ed25519_sign(out, m if m else None, len(m), bytes(public_key), bytes(private_key), None)
    return out.raw


def sign_batch(prv, blob, msg_off, msg_sz, nthread=None):
    """Keygen + sign n messages on host threads: prv (n,32) u8 -> pub (n,32), sig (n,64)."""
    prv = np.ascontiguousarray(prv, np.uint8)
    n = prv.shape[0]
    blob = np.ascontiguousarray(blob, np.uint8)
    off = np.ascontiguousarray(msg_off, np.uint32)
    sz = np.ascontiguousarray(msg_sz, np.uint32)
    pub = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    if nthread is None:
        nthread = min(16, os.cpu_count() or 1)
    rc = lib().fd_ed25519_amd_sign_batch(n, _ptr(prv), _ptr(blob), _ptr(off), _ptr(sz), _ptr(pub), _ptr(sig), nthread)
    assert rc == 0
    return pub, sig


# ---------------------------------------------------------------- batch engine

class EngineError(RuntimeError):
    pass


class Engine:
    """fd_ed25519_amd_t: one engine per device (multi-GPU = one per device)."""

    def __init__(self, device=0, batch_max=1 << 16, blob_max=None):
        if blob_max is None:
            blob_max = max(batch_max * 256, MSG_MAX)
        self._h = lib().fd_ed25519_amd_new(int(device), int(batch_max), int(blob_max))
        if not self._h:
            raise EngineError("fd_ed25519_amd_new(device=%d) failed (no HIP device?)" % device)
        self.device = device

    def close(self):
        if self._h:
            lib().fd_ed25519_amd_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def verify_soa(self, pub, sig, msg_off, msg_sz, blob):
        pub = np.ascontiguousarray(pub, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        off = np.ascontiguousarray(msg_off, np.uint32)
        sz = np.ascontiguousarray(msg_sz, np.uint32)
        blob = np.ascontiguousarray(blob, np.uint8)
        n = int(pub.shape[0])
        err = np.zeros(n, np.int8)
        rc = lib().fd_ed25519_amd_verify_soa(self._h, n, _ptr(pub), _ptr(sig), _ptr(off), _ptr(sz),
                                             _ptr(blob), int(blob.size), _ptr(err))
        if rc:
            raise EngineError("fd_ed25519_amd_verify_soa rc=%d" % rc)
        return err

    def verify_soa_registered(self, pub, sig, msg_off, msg_sz, blob, err=None):
        """fd_ed25519_amd_verify_soa_registered: every plane must lie in memory
        registered with host_register (see RegisteredPlanes); no host copy."""
        n = int(pub.shape[0])
        if err is None:
            err = np.zeros(n, np.int8)
        rc = lib().fd_ed25519_amd_verify_soa_registered(self._h, n, _ptr(pub), _ptr(sig), _ptr(msg_off), _ptr(msg_sz),
                                                        _ptr(blob), int(blob.size), _ptr(err))
        if rc:
            raise EngineError("fd_ed25519_amd_verify_soa_registered rc=%d" % rc)
        return err

    def verify_batch(self, msgs, sigs, pubs):
        """Pointer-array form: lists of bytes-like."""
        n = len(msgs)
        keep = [bytes(m) for m in msgs] + [bytes(s) for s in sigs] + [bytes(p) for p in pubs]
        bufs = [ctypes.create_string_buffer(b, max(len(b), 1)) for b in keep]
        mp = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs[:n]])
        sp = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs[n:2 * n]])
        pp = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs[2 * n:]])
        sz = (ctypes.c_ulong * max(n, 1))(*[len(b) for b in keep[:n]])
        err = np.zeros(max(n, 1), np.int8)
        rc = lib().fd_ed25519_amd_verify_batch(self._h, n, mp, sz, sp, pp, _ptr(err))
        if rc:
            raise EngineError("fd_ed25519_amd_verify_batch rc=%d" % rc)
        return err[:n]

    def verify_txns(self, payload, txn_off, txn_sz, want_sigs=False):
        """Wire-format transaction batch (include/fd_txn_amd.h): parse on the
        GPU, verify every signature (multi-signer rule), one verdict per
        transaction in {0, -1, -2, -3, FD_TXN_AMD_ERR_PARSE}.  With
        want_sigs, also returns (sig_base, sig_err)."""
        return _verify_txns(lib().fd_ed25519_amd_verify_txns, self._h, payload, txn_off, txn_sz, want_sigs)


def txn_slots(payload, txn_off, txn_sz):
    """fd_ed25519_amd_txn_slots: (tbase[txn_cnt+1], total signature slots)."""
    payload = np.ascontiguousarray(payload, np.uint8)
    off = np.ascontiguousarray(txn_off, np.uint32)
    sz = np.ascontiguousarray(txn_sz, np.uint32)
    base = np.zeros(off.size + 1, np.uint32)
    tot = lib().fd_ed25519_amd_txn_slots(int(off.size), _ptr(payload), _ptr(off), _ptr(sz), _ptr(base))
    return base, int(tot)


def _verify_txns(fn, h, payload, txn_off, txn_sz, want_sigs):
    payload = np.ascontiguousarray(payload, np.uint8)
    off = np.ascontiguousarray(txn_off, np.uint32)
    sz = np.ascontiguousarray(txn_sz, np.uint32)
    n = int(off.size)
    terr = np.zeros(max(n, 1), np.int8)
    base = serr = None
    if want_sigs:
        # sig_err is sized by the engine's own slot rule (overlapping or
        # repeated txn_off entries reserve slots more than once)
        base, tot = txn_slots(payload, off, sz)
        serr = np.zeros(max(tot, 1), np.int8)
    rc = fn(h, n, _ptr(payload), _ptr(off), _ptr(sz), int(payload.size), _ptr(terr),
            _ptr(base) if want_sigs else None, _ptr(serr) if want_sigs else None)
    if rc:
        raise EngineError("verify_txns rc=%d" % rc)
    if want_sigs:
        return terr[:n], base, serr[:int(base[-1])]
    return terr[:n]


def shard_range(n, ndev, r):
    """fd_ed25519_amd_shard_range: engine r's contiguous shard [lo, hi) of n."""
    lo, hi = ctypes.c_ulong(), ctypes.c_ulong()
    lib().fd_ed25519_amd_shard_range(int(n), int(ndev), int(r), ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


class MultiEngine:
    """fd_ed25519_amd_multi_t: one engine + one persistent host thread per
    entry of `devices` (repeats allowed); a batch is split into contiguous
    shards verified concurrently, no collective."""

    def __init__(self, devices, batch_max=1 << 16, blob_max=None):
        if blob_max is None:
            blob_max = max(batch_max * 256, MSG_MAX)
        dv = np.ascontiguousarray(devices, np.int32)
        self._h = lib().fd_ed25519_amd_multi_new(_ptr(dv), int(dv.size), int(batch_max), int(blob_max))
        if not self._h:
            raise EngineError("fd_ed25519_amd_multi_new(%r) failed" % (list(devices),))
        self.ndev = int(lib().fd_ed25519_amd_multi_ndev(self._h))

    def close(self):
        if self._h:
            lib().fd_ed25519_amd_multi_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def verify_soa(self, pub, sig, msg_off, msg_sz, blob):
        pub = np.ascontiguousarray(pub, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        off = np.ascontiguousarray(msg_off, np.uint32)
        sz = np.ascontiguousarray(msg_sz, np.uint32)
        blob = np.ascontiguousarray(blob, np.uint8)
        n = int(pub.shape[0])
        err = np.zeros(max(n, 1), np.int8)
        rc = lib().fd_ed25519_amd_multi_verify_soa(self._h, n, _ptr(pub), _ptr(sig), _ptr(off), _ptr(sz), _ptr(blob),
                                                   int(blob.size), _ptr(err))
        if rc:
            raise EngineError("fd_ed25519_amd_multi_verify_soa rc=%d" % rc)
        return err[:n]

    def verify_txns(self, payload, txn_off, txn_sz, want_sigs=False):
        return _verify_txns(lib().fd_ed25519_amd_multi_verify_txns, self._h, payload, txn_off, txn_sz, want_sigs)


class RegisteredPlanes:
    """Page-aligned copies of numpy arrays, registered with
    fd_ed25519_amd_host_register (inputs of Engine.verify_soa_registered);
    planes[k] is the registered copy of arrays[k].  close() unregisters."""

    def __init__(self, *arrays):
        self._raw = []
        self.planes = []
        for a in arrays:
            a = np.ascontiguousarray(a)
            nb = (max(a.nbytes, 1) + 4095) & ~4095
            raw = np.zeros(nb + 4096, np.uint8)
            o = (-raw.ctypes.data) % 4096
            region = raw[o:o + nb]
            b = region[:a.nbytes].view(a.dtype).reshape(a.shape)
            b[...] = a
            host_register(region)
            self._raw.append(region)
            self.planes.append(b)

    def __getitem__(self, k):
        return self.planes[k]

    def close(self):
        for r in self._raw:
            host_unregister(r)
        self._raw = []


def host_register(arr):
    """Pin a numpy array's memory for fd_ed25519_amd_verify_soa_registered."""
    rc = lib().fd_ed25519_amd_host_register(_ptr(arr), int(arr.nbytes))
    if rc:
        raise EngineError("fd_ed25519_amd_host_register rc=%d" % rc)


def host_unregister(arr):
    rc = lib().fd_ed25519_amd_host_unregister(_ptr(arr))
    if rc:
        raise EngineError("fd_ed25519_amd_host_unregister rc=%d" % rc)


# ---------------------------------------------------------------- device-resident path

def workspace_footprint(n):
    return int(lib().fd_ed25519_amd_workspace_footprint(int(n)))


def verify_dev(n, d_pub, d_sig, d_off, d_sz, d_blob, d_err, d_ws, stream=0):
    """All arguments are device pointers (ints, e.g. torch tensor .data_ptr());
    enqueued on `stream` (hipStream_t as int), not synchronised."""
    rc = lib().fd_ed25519_amd_verify_dev(int(n), d_pub, d_sig, d_off, d_sz, d_blob, d_err, d_ws, stream)
    if rc:
        raise EngineError("fd_ed25519_amd_verify_dev rc=%d" % rc)


def verify_dev_ev(n, d_pub, d_sig, d_off, d_sz, d_blob, d_err, d_ws, stream, events):
    """verify_dev recording 4 HIP events (hip.Event) around/between the
    three kernels on `stream`."""
    arr = None
    if events is not None:
        arr = (ctypes.c_void_p * 4)(*[e.handle for e in events])
    rc = lib().fd_ed25519_amd_verify_dev_ev(int(n), d_pub, d_sig, d_off, d_sz, d_blob, d_err, d_ws, stream, arr)
    if rc:
        raise EngineError("fd_ed25519_amd_verify_dev_ev rc=%d" % rc)


def work_stats_dev(n, d_ws, d_stats, stream=0):
    rc = lib().fd_ed25519_amd_work_stats_dev(int(n), d_ws, d_stats, stream)
    if rc:
        raise EngineError("fd_ed25519_amd_work_stats_dev rc=%d" % rc)


def debug_digits_dev(n, d_ws, d_dig, d_top, stream=0):
    rc = lib().fd_ed25519_amd_debug_digits_dev(int(n), d_ws, d_dig, d_top, stream)
    if rc:
        raise EngineError("fd_ed25519_amd_debug_digits_dev rc=%d" % rc)


def sign_dev(n, d_prv, d_off, d_sz, d_blob, d_pub, d_sig, stream=0):
    """GPU keygen + sign on device buffers (fd_ed25519_amd_sign_dev)."""
    rc = lib().fd_ed25519_amd_sign_dev(int(n), d_prv, d_off, d_sz, d_blob, d_pub, d_sig, stream)
    if rc:
        raise EngineError("fd_ed25519_amd_sign_dev rc=%d" % rc)


def sign_batch_gpu(prv, blob, msg_off, msg_sz):
    """Host arrays in, (pub, sig) out, signed on the GPU (k_sign)."""
    from . import hip
    prv = np.ascontiguousarray(prv, np.uint8)
    n = prv.shape[0]
    if not n:
        return np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8)
    d = [hip.DeviceBuffer.from_array(np.ascontiguousarray(a)) for a in
         (prv, np.asarray(msg_off, np.uint32), np.asarray(msg_sz, np.uint32), np.asarray(blob, np.uint8))]
    d_pub, d_sig = hip.DeviceBuffer(32 * n), hip.DeviceBuffer(64 * n)
    st = hip.Stream()
    sign_dev(n, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d_pub.ptr, d_sig.ptr, st.handle)
    st.synchronize()
    return d_pub.to_array(np.uint8, 32 * n).reshape(n, 32), d_sig.to_array(np.uint8, 64 * n).reshape(n, 64)


def set_small_batch_max(n):
    """Batches of at most n signatures use the 4-lane latency kernel (k_dsm4)."""
    lib().fd_ed25519_amd_set_small_batch_max(int(n))


def set_latency_batch_max(n):
    """Batches of at most n signatures use the 8-lane latency kernel (k_dsm8)."""
    lib().fd_ed25519_amd_set_latency_batch_max(int(n))


def set_pool_batch_min(n):
    """Throughput batches of at least n signatures use the pooled kernel (k_dsmp)."""
    lib().fd_ed25519_amd_set_pool_batch_min(int(n))


VERDICT_DEVICE = -128   # FD_ED25519_AMD_VERDICT_DEVICE: k_dsmp's step guard tripped


def device_numa_node(device):
    """fd_ed25519_amd_device_numa_node: the NUMA node of HIP device `device` (-1 unknown)."""
    f = lib().fd_ed25519_amd_device_numa_node
    f.restype = ctypes.c_int
    return int(f(int(device)))


def debug_set_pool_iter_cap(cap):
    """Debug: cap k_dsmp's step guard at `cap` steps per wave (0 restores it)."""
    lib().fd_ed25519_amd_debug_set_pool_iter_cap(int(cap))


def select_dsm_kernel(name):
    """Force one double-scalar-mult kernel for every batch size (tests):
    'k_dsm', 'k_dsmp', 'k_dsm4', 'k_dsm8'; 'default' restores the size rule."""
    big = (1 << 32) - 1
    small, lat, pool = {"k_dsm": (0, 0, big), "k_dsmp": (0, 0, 0), "k_dsm4": (big, 0, big),
                        "k_dsm8": (big, big, big),
                        "default": (SMALL_BATCH_MAX_DEFAULT, LATENCY_BATCH_MAX_DEFAULT, POOL_BATCH_MIN_DEFAULT)}[name]
    set_small_batch_max(small)
    set_latency_batch_max(lat)
    set_pool_batch_min(pool)


SMALL_BATCH_MAX_DEFAULT = 16384
LATENCY_BATCH_MAX_DEFAULT = 8192
POOL_BATCH_MIN_DEFAULT = 1 << 19   # k_dsmp from 2^19 signatures
FD_TXN_AMD_ERR_PARSE = -4
FD_TXN_MAX_SZ = 3570


def txn_parse_dev(txn_cnt, d_payload, d_toff, d_tsz, d_fp, d_out=None, out_stride=0, stream=0):
    """Device batch parse (fd_txn_amd_parse_dev): footprints (and optionally
    fd_txn_t descriptors, out_stride apart) of txn_cnt wire transactions."""
    rc = lib().fd_txn_amd_parse_dev(int(txn_cnt), d_payload, d_toff, d_tsz, d_fp, d_out, int(out_stride), stream)
    if rc:
        raise EngineError("fd_txn_amd_parse_dev rc=%d" % rc)


def version():
    return lib().fd_ed25519_amd_version().decode()
