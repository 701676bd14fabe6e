"""GPU parity sweep at scale through the streaming tile's kernel
(k_tile_persist): the streams of oracle/PARITY_LOG.md, regenerated draw for
draw (oracle/vecgen.h), signed on the GPU and given the same 10 % single-bit
flips as tools/gpu_sweep.py, are laid out as tango frags (pub | sig | msg in
a dcache, metadata in an mcache) and run through fd_verify_amd_tile_run
twice -- every chunk forced to 8-lane latency chunks, then to 64-frag
throughput chunks (cfg.chunk_mode) -- in copy mode (or zero copy).  The tile's verdict log
(fd_verify_amd_tile_set_verdict_log) is compared with the CPU oracle on every
signature, and each stream's code histogram with the reference's histogram
recorded in oracle/PARITY_LOG.md.

usage: python tools/gpu_sweep_tile.py [--zero-copy] [stream indices...] > gpurun_out/sweep_tile.jsonl
(--zero-copy: the tile's GPU gathers every frag from the mapped region instead of the host copying it)
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
from firedancer_amd import ed25519, tango  # noqa: E402
from gpu_sweep import STREAMS, N, CH  # noqa: E402

SUB = 1 << 20          # frags per tile run
MODES = ((tango.CHUNK_LATENCY, "latency"), (tango.CHUNK_THROUGHPUT, "throughput"), (tango.CHUNK_QUAD, "quad"))
# the AUTO rule (the product default) on request only: FD_SWEEP_TILE_MODES=auto
if "auto" in os.environ.get("FD_SWEEP_TILE_MODES", "").split(","):
    MODES = MODES + ((tango.CHUNK_AUTO, "auto"),)
# copy mode with the copy helper (cfg.copy_cpu) on the last CPU this process may use, when FD_SWEEP_TILE_HELPER=1
HELPER = {"copy_cpu": max(os.sched_getaffinity(0))} if os.environ.get("FD_SWEEP_TILE_HELPER") else {}
if os.environ.get("FD_SWEEP_TILE_MODES"):   # e.g. "quad" or "latency,quad"
    MODES = tuple(m for m in MODES if m[1] in os.environ["FD_SWEEP_TILE_MODES"].split(","))


def frames(pub, sig, o, z, b):
    """A dcache holding frag i = pub | sig | msg at chunk c[i] (compact
    layout, 64-B chunks), and the chunk and size of every frag."""
    n = pub.shape[0]
    fsz = 96 + z.astype(np.int64)
    nch = (fsz + 63) // 64
    c = np.zeros(n, np.int64)
    c[1:] = np.cumsum(nch[:-1])
    region = tango._aligned(int((c[-1] + nch[-1] + 2) * 64), 4096)
    base = c * 64
    region[base[:, None] + np.arange(32)] = pub
    region[base[:, None] + 32 + np.arange(64)] = sig
    step = 1 << 16
    for a in range(0, n, step):
        e = min(n, a + step)
        zz = z[a:e].astype(np.int64)
        tot = int(zz.sum())
        if not tot:
            continue
        oo = o[a:e].astype(np.int64)
        src = np.repeat(oo - np.concatenate(([0], np.cumsum(zz)[:-1])), zz) + np.arange(tot)
        dst = np.repeat(base[a:e] + 96 - np.concatenate(([0], np.cumsum(zz)[:-1])), zz) + np.arange(tot)
        region[dst] = b[src]
    return region, c.astype(np.uint32), fsz.astype(np.uint16)


def run_tile(tile, region, chunk, fsz, zero_copy=False):
    n = chunk.size
    depth = 1
    while depth < n:
        depth <<= 1
    mc = tango.mcache_new(depth)
    mc["seq"][:n] = np.arange(n, dtype=np.uint64)
    mc["chunk"][:n] = chunk
    mc["sz"][:n] = fsz
    mc["ctl"][:n] = 3
    out = tango.mcache_new(depth)
    log = np.full(n, 99, np.int8)
    if zero_copy:
        tile.register_dcache(region)   # the GPU gathers each frag from the mapped region itself
    tile.set_verdict_log(log)
    diag, _ = tile.run(mc, region, 0, out, 0, n)
    tile.set_verdict_log(None)
    assert diag["in_cnt"] == n and diag["ha_filt_cnt"] == 0 and diag["bad_frag_cnt"] == 0 and diag["ovrn_cnt"] == 0
    assert diag["out_cnt"] + diag["sv_filt_cnt"] == n
    return log, diag


def run(k, tiles):
    seed, szlo, szhi, ref_hist = STREAMS[k]
    t0 = time.time()
    rs = (seed * 0x2545F4914F6CDD1D + 1) & 0xFFFFFFFFFFFFFFFF   # check_vs_ref.c's seeding
    prv, blob, _, sz, fk, fp = _oracle.stream_inputs(rs, N, szlo, szhi, True)
    off64 = np.zeros(N, np.int64)
    off64[1:] = np.cumsum(sz[:-1], dtype=np.int64)      # the generator's u32 offsets wrap past 4 GB
    exp = np.zeros(N, np.int8)
    got = {name: np.zeros(N, np.int8) for _, name in MODES}
    chunks = {name: [0, 0, 0, 0] for _, name in MODES}
    t_tile = {name: 0.0 for _, name in MODES}
    t_cpu = 0.0
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
        t2 = time.time()
        exp[c0:c1] = _oracle.verify_batch(_golden.Batch(pub, sig, o, z, b))
        t_cpu += time.time() - t2
        for s0 in range(0, c1 - c0, SUB):
            s1 = min(c1 - c0, s0 + SUB)
            region, chunk, fsz = frames(pub[s0:s1], sig[s0:s1], o[s0:s1], z[s0:s1], b)
            for mode, name in MODES:
                t3 = time.time()
                if ZERO_COPY:   # one live tile per run: a region is registered (mapped into the GPU) by one tile
                    for t in tiles.values():
                        t.close()
                    tiles[name] = tango.VerifyTile(0, batch_max=16384, tcache_depth=0, chunk_mode=mode, **HELPER)
                log, diag = run_tile(tiles[name], region, chunk, fsz, ZERO_COPY)
                t_tile[name] += time.time() - t3
                got[name][c0 + s0:c0 + s1] = log
                chunks[name][0] += diag["gpu_chunk_lat_cnt"]
                chunks[name][1] += diag["gpu_chunk_thr_cnt"]
                chunks[name][2] += diag["gpu_chunk_quad_cnt"]
                chunks[name][3] += diag.get("quad_pair_cnt", 0)
        print("  stream %d: %d/%d" % (seed, c1, N), file=sys.stderr, flush=True)
    out = []
    for _, name in MODES:
        err = got[name]
        hist = tuple(int((err == -c).sum()) for c in range(4))
        bad = np.nonzero(err != exp)[0]
        out.append({"seed": seed, "szlo": szlo, "szhi": szhi, "signatures": N, "path": "k_tile_persist",
                    "staging": "zero_copy" if ZERO_COPY else ("copy+helper" if HELPER else "copy"),
                    "chunk_mode": name, "gpu_chunks": {"latency": chunks[name][0], "throughput": chunks[name][1],
                                                             "quad": chunks[name][2], "quad_pairs": chunks[name][3]},
                    "mismatches_vs_oracle": int(bad.size), "first_mismatches": [int(i) for i in bad[:5]],
                    "hist": hist, "hist_equals_reference": hist == ref_hist,
                    "false_rejects": int(((fk == 0) & (err == -3)).sum()),
                    "tile_s": round(t_tile[name], 1), "oracle_s": round(t_cpu, 1),
                    "total_s": round(time.time() - t0, 1)})
    return out


ZERO_COPY = "--zero-copy" in sys.argv

if __name__ == "__main__":
    ks = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or list(range(len(STREAMS)))
    tiles = {name: tango.VerifyTile(0, batch_max=16384, tcache_depth=0, chunk_mode=mode, **HELPER) for mode, name in MODES}
    fail = False
    try:
        for k in ks:
            for r in run(k, tiles):
                print(json.dumps(r), flush=True)
                fail |= bool(r["mismatches_vs_oracle"] or not r["hist_equals_reference"])
    finally:
        for t in tiles.values():
            t.close()
    sys.exit(1 if fail else 0)
