"""GPU parity sweep at scale: the engine vs the CPU oracle on the very streams
of oracle/PARITY_LOG.md (regenerated draw for draw from oracle/vecgen.h,
signed on the GPU -- byte-identical to the reference signer -- and given the
same 10 % single-bit flips).  Every verdict is compared with the oracle run on
the box's host cores, and each stream's code histogram with the reference's
histogram recorded in PARITY_LOG.md.  Stream k forces kernel k % 3 (k_dsm,
k_dsm4, k_dsm8) for every chunk, or FD_SWEEP_KERNEL (e.g. k_dsmp) for all.

usage: python tools/gpu_sweep.py [stream[:kernel]...] > gpurun_out/sweep.jsonl
       (e.g. `0:k_dsmp 1:k_dsm8`; a bare index uses FD_SWEEP_KERNEL or k % 3)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402

import _golden  # noqa: E402
import _oracle  # noqa: E402
from firedancer_amd import ed25519  # noqa: E402

N = 1 << 24
# (seed, szlo, szhi, reference histogram 0/-1/-2/-3) -- oracle/PARITY_LOG.md, round 1 session 2
STREAMS = [
    (70001, 0, 256, (15099845, 4359, 417727, 1255285)),
    (70002, 0, 256, (15099308, 4293, 417235, 1256380)),
    (70003, 64, 1232, (15102417, 4231, 416592, 1253976)),
    (70004, 64, 1232, (15101907, 4296, 416799, 1254214)),
    (70005, 0, 1232, (15099668, 4443, 417441, 1255664)),
    (70006, 0, 1232, (15100150, 4222, 418938, 1253906)),
]


CH = 1 << 21   # signatures per sub-batch: keeps every blob under the SoA API's 32-bit offsets


def run(k, kern=None):
    seed, szlo, szhi, ref_hist = STREAMS[k]
    t0 = time.time()
    rs = (seed * 0x2545F4914F6CDD1D + 1) & 0xFFFFFFFFFFFFFFFF   # check_vs_ref.c's seeding
    prv, blob, _, sz, fk, fp = _oracle.stream_inputs(rs, N, szlo, szhi, True)
    off64 = np.zeros(N, np.int64)
    off64[1:] = np.cumsum(sz[:-1], dtype=np.int64)      # the generator's u32 offsets wrap past 4 GB
    kern = kern or os.environ.get("FD_SWEEP_KERNEL") or ("k_dsm", "k_dsm4", "k_dsm8")[k % 3]
    ed25519.select_dsm_kernel(kern)
    eng = ed25519.Engine(device=0, batch_max=1 << 20, blob_max=(1 << 20) * max(szhi, 1))
    err = np.zeros(N, np.int8)
    exp = np.zeros(N, np.int8)
    t_gpu = t_cpu = 0.0
    for c0 in range(0, N, CH):
        c1 = min(N, c0 + CH)
        base = int(off64[c0])
        b = blob[base:int(off64[c1 - 1] + sz[c1 - 1]) + 1]
        o = (off64[c0:c1] - base).astype(np.uint32)
        z = sz[c0:c1]
        pub, sig = ed25519.sign_batch_gpu(prv[c0:c1], b, o, z)
        f, p = fk[c0:c1], fp[c0:c1]
        byte, bit = np.divmod(p.astype(np.int64), 8)
        flip = (np.uint8(1) << bit.astype(np.uint8))
        i1, i2, i3 = (np.nonzero(f == c)[0] for c in (1, 2, 3))
        sig[i1, byte[i1]] ^= flip[i1]
        b[o[i2].astype(np.int64) + byte[i2]] ^= flip[i2]
        pub[i3, byte[i3]] ^= flip[i3]
        t1 = time.time()
        err[c0:c1] = eng.verify_soa(pub, sig, o, z, b)
        t_gpu += time.time() - t1
        t2 = time.time()
        exp[c0:c1] = _oracle.verify_batch(_golden.Batch(pub, sig, o, z, b))
        t_cpu += time.time() - t2
        print("  stream %d: %d/%d" % (seed, c1, N), file=sys.stderr, flush=True)
    eng.close()
    ed25519.select_dsm_kernel("default")
    hist = tuple(int((err == -c).sum()) for c in range(4))
    bad = np.nonzero(err != exp)[0]
    false_rej = int(((fk == 0) & (err == -3)).sum())
    return {"seed": seed, "szlo": szlo, "szhi": szhi, "signatures": N,
            "kernel": kern, "mismatches_vs_oracle": int(bad.size),
            "first_mismatches": [int(i) for i in bad[:5]], "hist": hist,
            "hist_equals_reference": hist == ref_hist, "false_rejects": false_rej,
            "total_s": round(time.time() - t0, 1), "gpu_verify_s": round(t_gpu, 2), "oracle_s": round(t_cpu, 1)}


if __name__ == "__main__":
    ks = [(int(a.split(":")[0]), a.split(":")[1] if ":" in a else None) for a in sys.argv[1:]] \
        or [(k, None) for k in range(len(STREAMS))]
    for k, kern in ks:
        r = run(k, kern)
        print(json.dumps(r), flush=True)
        if r["mismatches_vs_oracle"] or not r["hist_equals_reference"]:
            sys.exit(1)
