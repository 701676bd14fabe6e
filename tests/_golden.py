"""Reader for the committed golden fixtures (tests/golden/).

The fixtures are DATA: inputs and the reference's expected verdict codes,
generated in the build container by oracle/gen_golden.c against the compiled
reference (see tests/golden/README.md).  Format (little endian):

  magic[16] "FDED25519GOLD1\\0\\0", u32 count, u32 reserved,
  count x { pub[32], sig[64], u32 sz, i8 expect, u8 cls, u16 0, msg[sz] }
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")
VECTORS = os.path.join(GOLDEN_DIR, "ed25519_vectors.bin")
STREAMS = os.path.join(GOLDEN_DIR, "ed25519_streams.jsonl")

CLASSES = [
    "valid", "flip_sig", "flip_msg", "flip_pub", "s_window", "s_range", "malleate",
    "offcurve_a", "offcurve_r", "small_order", "noncanon", "false_reject", "random",
    "rfc8032", "mainnet", "zero_msg", "max_msg",
]


class Batch:
    """SoA batch in the engine's input layout."""

    def __init__(self, pub, sig, msg_off, msg_sz, blob, expect=None, cls=None):
        self.pub = pub            # (n, 32) uint8
        self.sig = sig            # (n, 64) uint8
        self.msg_off = msg_off    # (n,) uint32
        self.msg_sz = msg_sz      # (n,) uint32
        self.blob = blob          # (total,) uint8
        self.expect = expect      # (n,) int8 or None
        self.cls = cls            # (n,) uint8 or None

    def __len__(self):
        return int(self.pub.shape[0])

    def msg(self, i):
        o = int(self.msg_off[i])
        return bytes(self.blob[o:o + int(self.msg_sz[i])])


def load_vectors(path=VECTORS):
    raw = open(path, "rb").read()
    assert raw[:14] == b"FDED25519GOLD1", "bad golden magic"
    n = int.from_bytes(raw[16:20], "little")
    pos = 24
    pub = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    sz = np.zeros(n, np.uint32)
    off = np.zeros(n, np.uint32)
    exp = np.zeros(n, np.int8)
    cls = np.zeros(n, np.uint8)
    chunks = []
    total = 0
    for i in range(n):
        pub[i] = np.frombuffer(raw, np.uint8, 32, pos)
        sig[i] = np.frombuffer(raw, np.uint8, 64, pos + 32)
        s = int.from_bytes(raw[pos + 96:pos + 100], "little")
        exp[i] = np.int8(np.uint8(raw[pos + 100]).view(np.int8))
        cls[i] = raw[pos + 101]
        pos += 104
        chunks.append(raw[pos:pos + s])
        sz[i] = s
        off[i] = total
        total += s
        pos += s
    assert pos == len(raw)
    blob = np.frombuffer(b"".join(chunks) + b"\0", np.uint8).copy()
    return Batch(pub, sig, off, sz, blob, exp, cls)


def load_streams(path=STREAMS):
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


def fnv1a64(codes):
    h = 0xCBF29CE484222325
    for c in np.asarray(codes, np.int8).view(np.uint8).tolist():
        h = ((h ^ c) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h
