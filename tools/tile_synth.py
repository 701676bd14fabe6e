"""Measurement aid: k_tile_persist's chunk pipeline alone (fd_amd_tile_synth:
frags already in device memory, no host hand-off).  Per configuration the
launch time, the time per chunk per wave and the verdict check.  Runs on the
diagnostics library (FD_AMD_DIAG build; the product library does not carry
k_tile_synth):
    python -m firedancer_amd.build --diag && python tools/tile_synth.py"""
import ctypes
import json
import os
import sys

os.environ.setdefault("FD_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "firedancer_amd", "libfd_ed25519_amd_diag.so"))

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, workload  # noqa: E402

FR = 1408
m = 4096
pub, sig, off, sz, blob = workload.sig_batch(m, 200, 9)
frames = np.zeros((m, FR), np.uint8)
frames[:, :32] = pub
frames[:, 32:96] = sig
for i in range(m):
    frames[i, 96:96 + sz[i]] = blob[off[i]:off[i] + sz[i]]
fsz = (96 + sz).astype(np.uint32)
L = ed25519.lib()
L.fd_amd_tile_synth.restype = ctypes.c_int
# (waves, iters, eight, where): where 1 ring, 2 results, 4 frames (coherent), 8 frames (non-coherent)
# in mapped host memory, 16 a wave polling host words meanwhile
cfgs = [(2048, 4, 0, 0), (2048, 4, 0, 1), (2048, 4, 0, 2), (2048, 4, 0, 4), (2048, 4, 0, 8),
        (2048, 4, 0, 16), (2048, 4, 0, 31 & ~8), (2048, 16, 1, 0), (2048, 16, 1, 31 & ~8)]
if len(sys.argv) > 1:
    cfgs = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
for waves, iters, eight, where in cfgs:
    k = {0: 64, 1: 8, 2: 16}[eight]
    n = waves * iters * k
    v = np.zeros(n, np.int8)
    ms = ctypes.c_double(0)
    rc = L.fd_amd_tile_synth(0, waves, iters, eight, where, frames.ctypes.data_as(ctypes.c_void_p), m,
                             fsz.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ms), v.ctypes.data_as(ctypes.c_void_p))
    if rc:
        raise SystemExit("fd_amd_tile_synth rc=%d" % rc)
    print(json.dumps(dict(waves=waves, iters=iters, eight=eight, where=where, ms=round(ms.value, 3),
                          ms_per_chunk=round(ms.value / iters, 3), frags_per_s=round(n / ms.value * 1e3),
                          ok=int((v == 0).sum()), bad=int((v != 0).sum()))), flush=True)
