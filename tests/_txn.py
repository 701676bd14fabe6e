"""Transaction test helpers: the committed parse fixtures and a synthetic
multi-signer transaction builder.

tests/golden/txn_mutations.bin is written by oracle/gen_txn_golden.c from
the COMPILED REFERENCE fd_txn_parse (src/ballet/txn/fd_txn_parse.c) over the
reference's own fixtures (src/ballet/txn/fixtures/transaction{1,2,3}.bin,
kept verbatim inside the file as data) and a deterministic mutation list
(mutation_list below, mirrored from gen_txn_golden.c: mutations()).
"""
import os
import struct

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "txn_mutations.bin")
FNV0 = 0xcbf29ce484222325
FNV_P = 0x100000001b3
M64 = (1 << 64) - 1


def fnv(h, data):
    for b in bytes(data):
        h = ((h ^ b) * FNV_P) & M64
    return h


class Fixture:
    def __init__(self, payload, digest, footprints, lines):
        self.payload = payload
        self.digest = digest
        self.footprint = footprints
        self.line = lines


def load_fixtures():
    raw = open(GOLD, "rb").read()
    assert raw[:12] == b"FDTXNGOLDEN1"
    nfix = struct.unpack_from("<I", raw, 16)[0]
    at = 24
    out = []
    for _ in range(nfix):
        sz, nmut = struct.unpack_from("<II", raw, at)
        dig = struct.unpack_from("<Q", raw, at + 8)[0]
        at += 16
        payload = raw[at:at + sz]
        at += sz
        rec = np.frombuffer(raw, np.uint16, 2 * nmut, at).reshape(nmut, 2)
        at += 4 * nmut
        out.append(Fixture(payload, dig, rec[:, 0].astype(np.uint32), rec[:, 1].astype(np.uint32)))
    return out


def mutation_list(payload):
    """(payload bytes) for every mutation, in gen_txn_golden.c order: per
    position i the values o^1, o^0x80, o+1, 0x00, 0xff that differ from o,
    then every truncation length 0..sz-1."""
    p = bytearray(payload)
    out = []
    for i, o in enumerate(payload):
        for v in (o ^ 1, o ^ 0x80, (o + 1) & 0xff, 0x00, 0xff):
            if v == o:
                continue
            p[i] = v
            out.append(bytes(p))
        p[i] = o
    for L in range(len(payload)):
        out.append(bytes(payload[:L]))
    return out


def pack(payloads):
    """Concatenate payloads -> (blob u8, off u32, sz u32); blob 4-byte padded."""
    sz = np.array([len(p) for p in payloads], np.uint32)
    off = np.zeros(len(payloads), np.uint32)
    if len(payloads):
        off[1:] = np.cumsum(sz[:-1], dtype=np.uint64).astype(np.uint32)
    blob = np.frombuffer(b"".join(payloads) + b"\0" * 4, np.uint8).copy()
    return blob, off, sz


def cu16(v):
    if v < 0x80:
        return bytes([v])
    if v < 0x4000:
        return bytes([0x80 | (v & 0x7f), v >> 7])
    return bytes([0x80 | (v & 0x7f), 0x80 | ((v >> 7) & 0x7f), v >> 14])


def message(rng, pubs, msg_len, v0, nx):
    """A well-formed message (fd_txn.h layout) whose signer addresses are
    `pubs` followed by nx other accounts, padded with one instruction's data
    to about msg_len bytes (never below the fixed part)."""
    nsig = len(pubs)
    nacct = nsig + nx
    head = (b"\x80" if v0 else b"") + bytes([nsig, int(rng.integers(0, nsig)), int(rng.integers(0, nx + 1))])
    accts = b"".join(bytes(p) for p in pubs) + rng.integers(0, 256, 32 * nx, dtype=np.uint8).tobytes()
    body = head + cu16(nacct) + accts + rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    tail = cu16(0) if v0 else b""
    # one instruction: program index, two account indices, data
    fixed = len(body) + 1 + 1 + 1 + 2 + len(tail)
    dlen = max(0, msg_len - fixed - 3)
    ins = bytes([int(rng.integers(1, nacct))]) + cu16(2) + bytes([0, nacct - 1]) + cu16(dlen) + \
        rng.integers(0, 256, dlen, dtype=np.uint8).tobytes()
    return body + cu16(1) + ins + tail


def build_txns(seed, count, nsig_lo=1, nsig_hi=12, msg_lo=64, msg_hi=1232, v0_frac=0.5, mtu=1232):
    """count signed multi-signer transactions: (payloads, signer count per txn).
    Every signature is valid (signed by the product's host signer)."""
    from firedancer_amd import ed25519
    rng = np.random.default_rng(seed)
    nsig = rng.integers(nsig_lo, nsig_hi + 1, count)
    tot = int(nsig.sum())
    prv = rng.integers(0, 256, (tot, 32), dtype=np.uint8)
    z = np.zeros(tot, np.uint32)
    pub, _ = ed25519.sign_batch(prv, np.zeros(1, np.uint8), z, z)
    msgs, k = [], 0
    for t in range(count):
        n = int(nsig[t])
        room = mtu - 1 - 64 * n
        ml = int(min(room, rng.integers(msg_lo, msg_hi + 1)))
        nx = 1 if n >= 10 else int(rng.integers(1, 4))
        m = message(rng, pub[k:k + n], ml, rng.random() < v0_frac, nx)
        assert 1 + 64 * n + len(m) <= mtu, (n, len(m))
        msgs.append(m)
        k += n
    blob = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    mlen = np.array([len(m) for m in msgs], np.uint32)
    moff = np.concatenate([[0], np.cumsum(mlen)[:-1]]).astype(np.uint32)
    sig_off = np.repeat(moff, nsig)
    sig_sz = np.repeat(mlen, nsig)
    pub2, sig = ed25519.sign_batch(prv, blob, sig_off, sig_sz)
    assert np.array_equal(pub, pub2)
    payloads, k = [], 0
    for t in range(count):
        n = int(nsig[t])
        payloads.append(bytes([n]) + sig[k:k + n].tobytes() + msgs[t])
        k += n
    return payloads, nsig
