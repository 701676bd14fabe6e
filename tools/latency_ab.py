"""Latency-path A/B on the diagnostics library (fd_amd_latency_ab): one
4096-signature batch resident in HBM through k_front + k_dsm8, launched on
a stream or replayed from a captured hipGraph, completion seen through
hipEventSynchronize or by spinning on the verdicts in mapped memory.
    python -m firedancer_amd.build --diag && python tools/latency_ab.py [n] [iters]"""
import ctypes
import json
import os
import sys

os.environ.setdefault("FD_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "firedancer_amd", "libfd_ed25519_amd_diag.so"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from firedancer_amd import ed25519, workload  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 400
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 11)
L = ed25519.lib()
out = (ctypes.c_double * 16)()
vp = ctypes.c_void_p
arr = [np.ascontiguousarray(a) for a in (pub, sig, off, sz, blob)]
rc = L.fd_amd_latency_ab(ctypes.c_int(0), ctypes.c_uint32(n), *[vp(a.ctypes.data) for a in arr],
                         ctypes.c_uint64(arr[4].nbytes), ctypes.c_uint32(iters), out)
if rc:
    raise SystemExit("fd_amd_latency_ab rc=%d" % rc)
names = ("stream launches + hipEventSynchronize", "stream launches + spin on mapped verdicts",
         "hipGraph + hipEventSynchronize", "hipGraph + spin on mapped verdicts")
for m, name in enumerate(names):
    print(json.dumps({"n": n, "iters": iters, "mode": m, "path": name, "p50_us": round(out[4 * m], 1),
                      "p99_us": round(out[4 * m + 1], 1), "min_us": round(out[4 * m + 2], 1),
                      "gpu_p50_us": round(out[4 * m + 3], 1)}), flush=True)
