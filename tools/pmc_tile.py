"""PMC helper: one saturated persistent-tile run (zero copy, 2^20 frags or argv[2])
and, for comparison, one resident batch of 2^18 through the batch kernels
(k_prep, k_decomp, k_dsm forced).  Run under rocprofv3 --pmc.
    python tools/pmc_tile.py [tile|batch|both]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, hip, tango, workload  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "both"
frags = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
pub, sig, off, sz, blob = workload.sig_batch(1 << 16, 200, 9)
if what in ("tile", "both"):
    r = tango.bench_stream(0, 16384, 0, pub, sig, off, sz, blob, frags, zero_copy=True)
    print("tile", {k: round(v) for k, v in r.items()}, flush=True)
if what in ("batch", "both"):
    n = 1 << 18
    p2, s2, o2, z2, b2 = workload.sig_batch(n, 200, 10)
    d = [hip.DeviceBuffer.from_array(a) for a in (p2, s2, o2, z2, b2)]
    err, ws = hip.DeviceBuffer(n), hip.DeviceBuffer(ed25519.workspace_footprint(n))
    ed25519.select_dsm_kernel("k_dsm")
    st = hip.Stream()
    ed25519.verify_dev(n, *[x.ptr for x in d], err.ptr, ws.ptr, st.handle)
    st.synchronize()
    print("batch ok", int((err.to_array(np.int8, n) == 0).sum()), flush=True)
