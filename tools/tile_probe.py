"""Streaming-tile probe (A/B and profiling aid): one bench_stream run per
argument set, printed as JSON lines: saturated, then paced at half the
saturated rate.  HIP's hardware-queue setting is left as the box has it
(FD_PROBE_HW_QUEUES sets GPU_MAX_HW_QUEUES for an A/B).
    python tools/tile_probe.py BATCH_MAX FRAGS [zc] [check] [write]"""
import hashlib
import json
import os
import sys

import numpy as np

if os.environ.get("FD_PROBE_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["FD_PROBE_HW_QUEUES"]

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import tango, workload  # noqa: E402

bmax, nf = int(sys.argv[1]), int(sys.argv[2])
flags = set(sys.argv[3:])
m = 1 << 14
pub, sig, off, sz, blob = workload.sig_batch(m, 200, 9)
kw = {}
if "check" in flags:
    tag = np.array([int.from_bytes(hashlib.sha512(bytes(sig[i][:32]) + bytes(pub[i]) +
                                                  bytes(blob[off[i]:off[i] + sz[i]])).digest()[:8], "little")
                    for i in range(m)], np.uint64)
    kw = dict(expect_err=np.zeros(m, np.int8), expect_tag=tag)
sat = None
for rate in (0.0, None):
    if rate is None:
        rate = 0.5 * sat
    r = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, nf if rate == 0.0 else int(min(nf, rate * 0.5)) or 1,
                           rate=rate, zero_copy="zc" in flags, writes="write" in flags, sample_bytes=True, **kw)
    sat = sat or r["frags_per_s"]
    print(json.dumps(dict(bmax=bmax, rate=round(rate), flags=sorted(flags), **{k: round(v, 3) for k, v in r.items()})),
          flush=True)
