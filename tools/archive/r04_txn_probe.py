"""TXN-framed frags through the tile's batch path at several batch_max
values (signatures per batch), saturated, zero copy, every published
transaction checked (verdict, first signature's tag, order)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from firedancer_amd import ed25519, tango, workload  # noqa: E402
import bench  # noqa: E402

payload, toff, tsz, _ = workload.txn_batch(1 << 17, 777)
payload = payload.copy()
rng = np.random.default_rng(56)
for t in rng.choice(toff.size, toff.size // 10, replace=False):
    payload[int(toff[t]) + 1 + int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
eng = ed25519.Engine(device=0, batch_max=1 << 16, blob_max=payload.size + 64)
terr = eng.verify_txns(payload, toff, tsz)
eng.close()
tag = np.array([bench._txn_first_tag(payload[int(o):int(o) + int(z)]) for o, z in zip(toff, tsz)], np.uint64)
pool = (np.zeros((toff.size, 32), np.uint8), np.zeros((toff.size, 64), np.uint8), toff, tsz, payload)
spt = float(ed25519.txn_slots(payload, toff, tsz)[1]) / toff.size
for bmax in (4096, 16384, 65536):
    r = tango.bench_stream(0, bmax, 0, *pool, 1 << 20, zero_copy=True, txn=True, expect_err=terr, expect_tag=tag,
                           sample_bytes=True)
    print(json.dumps({"batch_max": bmax, "txns_per_s": round(r["frags_per_s"]), "verifies_per_s": round(r["frags_per_s"] * spt),
                      "mismatches": int(r["mismatches"]), "checked": int(r["checked"]), "mean_batch": r["mean_batch"]}),
          flush=True)
