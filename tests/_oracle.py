"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST CHECKER ONLY.

The oracle is the clean-room C restatement of the reference verdict function
(oracle/fd_ed25519_oracle.c); it is used here to check the HIP engine, never
as the thing measured or shipped.  oracle/_ref/libfdref.so (the reference's
own sources, compiled) is bound too when present, as a second checker.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libfdref.so")

_o = None
_r = None


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def oracle():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle/liboracle.so missing: run __graft_entry__.build()")
        L = ctypes.CDLL(ORACLE_SO)
        vp = ctypes.c_void_p
        L.oracle_ed25519_verify.argtypes = [vp, ctypes.c_size_t, vp, vp]
        L.oracle_ed25519_verify.restype = ctypes.c_int
        L.oracle_ed25519_verify_batch.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_ed25519_verify_batch.restype = ctypes.c_int
        L.oracle_sha512.argtypes = [vp, ctypes.c_size_t, vp]
        L.oracle_sha512.restype = None
        L.oracle_sc_reduce.argtypes = [vp, vp]
        L.oracle_sc_reduce.restype = None
        L.oracle_stream_gen.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_int, vp, vp, vp, vp, vp, vp]
        L.oracle_stream_gen.restype = ctypes.c_uint64
        L.oracle_txn_parse.argtypes = [vp, ctypes.c_ulong, vp, vp]
        L.oracle_txn_parse.restype = ctypes.c_ulong
        L.oracle_txn_parse_fail_line.argtypes = [vp, ctypes.c_ulong]
        L.oracle_txn_parse_fail_line.restype = ctypes.c_ulong
        L.oracle_txn_verify_batch.argtypes = [ctypes.c_ulong, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_txn_verify_batch.restype = ctypes.c_int
        _o = L
    return _o


def ref():
    """The compiled reference (None when oracle/_ref was not built)."""
    global _r
    if _r is None and os.path.exists(REF_SO):
        L = ctypes.CDLL(REF_SO)
        vp = ctypes.c_void_p
        L.fd_sha512_new.argtypes = [vp]
        L.fd_sha512_new.restype = vp
        L.fd_sha512_join.argtypes = [vp]
        L.fd_sha512_join.restype = vp
        L.fd_ed25519_verify.argtypes = [vp, ctypes.c_ulong, vp, vp, vp]
        L.fd_ed25519_verify.restype = ctypes.c_int
        _r = L
    return _r


def verify(msg, sig, pub):
    m = bytes(msg)
    return oracle().oracle_ed25519_verify(m if m else None, len(m), bytes(sig), bytes(pub))


def verify_batch(batch, nthread=None, stats=False):
    n = len(batch)
    err = np.zeros(n, np.int8)
    st = np.zeros((n, 3), np.uint32) if stats else None
    if nthread is None:
        nthread = min(16, os.cpu_count() or 1)
    oracle().oracle_ed25519_verify_batch(
        n, _p(np.ascontiguousarray(batch.pub)), _p(np.ascontiguousarray(batch.sig)),
        _p(np.ascontiguousarray(batch.msg_off)), _p(np.ascontiguousarray(batch.msg_sz)),
        _p(np.ascontiguousarray(batch.blob)), _p(err), _p(st) if stats else None, nthread)
    return (err, st) if stats else err


def sha512(data):
    out = ctypes.create_string_buffer(64)
    d = bytes(data)
    oracle().oracle_sha512(d if d else None, len(d), out)
    return out.raw


def sc_reduce(b64):
    out = ctypes.create_string_buffer(32)
    oracle().oracle_sc_reduce(out, bytes(b64))
    return out.raw


def ref_verify(msg, sig, pub):
    R = ref()
    if R is None:
        return None
    if not hasattr(ref_verify, "_sha"):
        buf = ctypes.create_string_buffer(256 + 128)
        addr = (ctypes.addressof(buf) + 127) & ~127
        ref_verify._buf = buf
        ref_verify._sha = R.fd_sha512_join(R.fd_sha512_new(addr))
    m = bytes(msg)
    return R.fd_ed25519_verify(m if m else None, len(m), bytes(sig), bytes(pub), ref_verify._sha)


def stream_inputs(seed, count, szlo, szhi, mixed):
    """Draw-for-draw regeneration of oracle/vecgen.h streams (unsigned)."""
    prv = np.zeros((count, 32), np.uint8)
    blob = np.zeros(count * max(szhi, 1) + 1, np.uint8)
    off = np.zeros(count, np.uint32)
    sz = np.zeros(count, np.uint32)
    fk = np.zeros(count, np.uint8)
    fp = np.zeros(count, np.uint32)
    used = oracle().oracle_stream_gen(seed, count, szlo, szhi, int(mixed), _p(prv), _p(blob), _p(off), _p(sz),
                                      _p(fk), _p(fp))
    return prv, blob[:used + 1], off, sz, fk, fp


def txn_parse(payload):
    """oracle fd_txn_parse: (footprint, descriptor bytes[:footprint], fail line)."""
    p = bytes(payload)
    buf = ctypes.create_string_buffer(3570 + 16)
    fp = oracle().oracle_txn_parse(p if p else None, len(p), buf, None)
    line = 0 if fp else oracle().oracle_txn_parse_fail_line(p if p else None, len(p))
    return int(fp), buf.raw[:fp], int(line)


def txn_verify_batch(payload, txn_off, txn_sz, nthread=None):
    """Multi-signer verdicts: (txn_err, sig_base, sig_err) -- the rule of
    fd_ed25519_amd_verify_txns on the CPU oracle."""
    payload = np.ascontiguousarray(payload, np.uint8)
    off = np.ascontiguousarray(txn_off, np.uint32)
    sz = np.ascontiguousarray(txn_sz, np.uint32)
    n = off.size
    terr = np.zeros(max(n, 1), np.int8)
    base = np.zeros(n + 1, np.uint32)
    serr = np.zeros(max(payload.size // 65 + 1, 1), np.int8)
    if nthread is None:
        nthread = min(16, os.cpu_count() or 1)
    oracle().oracle_txn_verify_batch(n, _p(payload), _p(off), _p(sz), _p(terr), _p(base), _p(serr), nthread)
    return terr[:n], base, serr[:int(base[-1])]
