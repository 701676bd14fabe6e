"""Synthetic workloads for the bench and the tests (BASELINE.json configs),
signed on the GPU (fd_ed25519_amd_sign_dev; byte-identical to the host and
reference signers) so large batches cost seconds, not minutes.

    sig_batch(n, msg_sz, seed)          configs[1]: single-signer, fixed size
    txn_batch(n_sigs, seed, ...)        configs[3]: multi-signer transactions,
                                        64..1232-B messages (legacy + v0)
"""
import ctypes

import numpy as np

from . import ed25519, hip


def sig_batch(n, msg_sz, seed):
    """n fresh keypairs, random msg_sz-byte messages, signed on the GPU.
    Returns host arrays (pub, sig, off, sz, blob)."""
    rng = np.random.default_rng(seed)
    prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    blob = rng.integers(0, 256, n * msg_sz + 1, dtype=np.uint8)
    off = (np.arange(n, dtype=np.uint64) * msg_sz).astype(np.uint32)
    sz = np.full(n, msg_sz, np.uint32)
    pub, sig = ed25519.sign_batch_gpu(prv, blob, off, sz)
    return pub, sig, off, sz, blob


def _bind():
    L = ed25519.lib()
    if not hasattr(L, "_synth_bound"):
        vp, ul, ui = ctypes.c_void_p, ctypes.c_ulong, ctypes.c_uint
        L.fd_ed25519_amd_synth_txns.argtypes = [ul, ul, ui, ui, ui, ui, vp, ul, vp, ul, vp, vp, vp, vp, vp]
        L.fd_ed25519_amd_synth_txns.restype = ul
        L.fd_ed25519_amd_txn_slots.argtypes = [ul, vp, vp, vp, vp]
        L.fd_ed25519_amd_txn_slots.restype = ul
        L.fd_ed25519_amd_txn_workspace_footprint.argtypes = [ul, ul]
        L.fd_ed25519_amd_txn_workspace_footprint.restype = ul
        L.fd_ed25519_amd_verify_txns_dev.argtypes = [ul, ul, vp, vp, vp, vp, vp, vp, vp, vp]
        L.fd_ed25519_amd_verify_txns_dev.restype = ctypes.c_int
        L._synth_bound = True
    return L


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def txn_batch(n_sigs, seed, nsig_lo=1, nsig_hi=12, msg_lo=64, msg_hi=1232):
    """Wire-format multi-signer transactions holding about n_sigs
    signatures, every signature valid.  Returns (payload, txn_off, txn_sz,
    tbase) with tbase the engine's signature-slot numbering."""
    L = _bind()
    rng = np.random.default_rng(seed)
    mean = (nsig_lo + nsig_hi) / 2.0
    txn_cnt = max(1, int(n_sigs / mean))
    cap_sigs = txn_cnt * nsig_hi
    prv = rng.integers(0, 256, (cap_sigs, 32), dtype=np.uint8)
    z = np.zeros(cap_sigs, np.uint32)
    pub, _ = ed25519.sign_batch_gpu(prv, np.zeros(8, np.uint8), z, z)       # keygen
    payload = np.zeros(txn_cnt * 1232 + 8, np.uint8)
    toff = np.zeros(txn_cnt, np.uint32)
    tsz = np.zeros(txn_cnt, np.uint32)
    smo = np.zeros(cap_sigs, np.uint32)
    sms = np.zeros(cap_sigs, np.uint32)
    sat = np.zeros(cap_sigs, np.uint32)
    ns = L.fd_ed25519_amd_synth_txns(seed, txn_cnt, nsig_lo, nsig_hi, msg_lo, msg_hi, _p(pub), cap_sigs,
                                     _p(payload), payload.size, _p(toff), _p(tsz), _p(smo), _p(sms), _p(sat))
    assert ns > 0
    used = int(toff[-1]) + int(tsz[-1])
    payload = payload[:used + 8]
    _, sig = ed25519.sign_batch_gpu(prv[:ns], payload, smo[:ns], sms[:ns])
    idx = sat[:ns].astype(np.int64)[:, None] + np.arange(64)[None, :]
    payload[idx] = sig
    tbase = np.zeros(txn_cnt + 1, np.uint32)
    L.fd_ed25519_amd_txn_slots(txn_cnt, _p(payload), _p(toff), _p(tsz), _p(tbase))
    return payload, toff, tsz, tbase


class TxnDevice:
    """A transaction batch resident in HBM + its workspace (bench path)."""

    def __init__(self, payload, toff, tsz, tbase):
        L = _bind()
        self.txn_cnt = int(toff.size)
        self.slot_cnt = int(tbase[-1])
        self.d = {k: hip.DeviceBuffer.from_array(np.ascontiguousarray(v)) for k, v in
                  dict(payload=payload, toff=toff, tsz=tsz, tbase=tbase).items()}
        self.d_terr = hip.DeviceBuffer(max(self.txn_cnt, 1))
        self.d_serr = hip.DeviceBuffer(max(self.slot_cnt, 1))
        self.d_ws = hip.DeviceBuffer(L.fd_ed25519_amd_txn_workspace_footprint(self.txn_cnt, self.slot_cnt))

    def run(self, stream):
        rc = _bind().fd_ed25519_amd_verify_txns_dev(
            self.txn_cnt, self.slot_cnt, self.d["payload"].ptr, self.d["toff"].ptr, self.d["tsz"].ptr,
            self.d["tbase"].ptr, self.d_terr.ptr, self.d_serr.ptr, self.d_ws.ptr, stream)
        if rc:
            raise ed25519.EngineError("fd_ed25519_amd_verify_txns_dev rc=%d" % rc)

    def verdicts(self):
        return self.d_terr.to_array(np.int8, self.txn_cnt), self.d_serr.to_array(np.int8, self.slot_cnt)
