"""Scout-stop experiment (profiles/r06_scout_stop_fix.txt):
one saturated zero-copy tile run of `frags` frags per library build, straight
through the C ABI with ctypes (any round's build: only fd_ed25519_amd_sign_batch
and fd_verify_amd_bench_stream are bound), in its own process per build.  A
build whose scout stops returns FD_ED25519_AMD_ERR_DEVICE (the tile's watchdog
message goes to stderr).  One JSON line per run.

usage: python tools/scout_touch_probe.py <frags> lib1.so [lib2.so ...]
"""
import ctypes
import json
import os
import subprocess
import sys

CHILD = r'''
import ctypes, json, sys, time
import numpy as np
L = ctypes.CDLL(sys.argv[1])
vp, ul = ctypes.c_void_p, ctypes.c_ulong
n = 1 << 14
rng = np.random.default_rng(5)
prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
blob = rng.integers(0, 256, n * 200 + 1, dtype=np.uint8)
off = (np.arange(n) * 200).astype(np.uint32)
sz = np.full(n, 200, np.uint32)
pub = np.zeros((n, 32), np.uint8)
sig = np.zeros((n, 64), np.uint8)
p = lambda a: vp(a.ctypes.data)
L.fd_ed25519_amd_sign_batch.argtypes = [ul, vp, vp, vp, vp, vp, vp, ctypes.c_int]
L.fd_ed25519_amd_sign_batch(n, p(prv), p(blob), p(off), p(sz), p(pub), p(sig), 8)
L.fd_verify_amd_bench_stream.argtypes = [ctypes.c_int, ul, ul, ctypes.c_double, ctypes.c_int, ul, ul, vp, vp, vp, vp, vp,
                                         vp, vp, ul, ul, vp]
out = (ctypes.c_double * 64)()
t0 = time.time()
rc = L.fd_verify_amd_bench_stream(0, 16384, 0, 0.0, 1, 0, n, p(pub), p(sig), p(off), p(sz), p(blob), None, None,
                                  int(sys.argv[2]), 0, out)
print(json.dumps({"rc": rc, "s": round(time.time() - t0, 3), "mfps": round(out[0] / 1e6, 2) if rc == 0 else None,
                  "published": int(out[5]) if rc == 0 else None}))
'''

if __name__ == "__main__":
    frags, libs = int(sys.argv[1]), sys.argv[2:]
    for lib in libs:
        try:
            q = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(lib), str(frags)], capture_output=True,
                               text=True, timeout=120)
            last = q.stdout.strip().splitlines()[-1] if q.stdout.strip() else "{}"
            r = json.loads(last)
            r.update(lib=lib, exit=q.returncode, stderr=q.stderr.strip()[-400:])
        except subprocess.TimeoutExpired:
            r = {"lib": lib, "exit": "timeout"}
        print(json.dumps(r), flush=True)
        if r.get("exit") == "timeout":
            sys.exit(1)   # a run the watchdog did not end: start nothing more on the GPU
