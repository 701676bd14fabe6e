"""Streaming verify tile (include/fd_tango_amd.h) on the GPU: frags
public_key | signature | message from an input mcache/dcache, HA dedup,
adaptive GPU batches, in-order publication of the passing frags with the
SHA-512-derived dedup tag, out of the tile's own output dcache.  Expected
behaviour is modelled frag by frag in Python: tcache window semantics of
FD_TCACHE_INSERT (src/tango/tcache/fd_tcache.h:372-403), verdicts from the
committed golden fixtures / the CPU oracle, tag = first 8 bytes of
SHA-512(R||A||M).  The producer-facing contract (a frag is released by
in_fseq only once the tile no longer reads it; a frag lapped before the
tile is done is dropped, never published) is checked with producers that
rewrite a small wrapping data region, with and without honouring the
credit (fd_verify_amd_bench_stream check mode)."""
import collections
import hashlib

import numpy as np
import pytest

import _golden
import _oracle

pytestmark = pytest.mark.gpu


def _feed(pub, sig, msgs, order, depth):
    """Publish frags `order` (indices into the pool) into a fresh
    mcache/dcache; returns (mcache, dcache, chunks, sizes, tsorig)."""
    from firedancer_amd import tango
    mtu = 96 + 1232
    chunk_mtu = ((mtu + 2 * 64 - 1) >> 7) << 1
    nchunk = chunk_mtu * (len(order) + 2)
    dcache = tango._aligned((64 * nchunk + 4095) & ~4095, 4096)   # page-aligned: can be GPU-mapped
    mc = tango.mcache_new(depth)
    chunk, chunks, sizes, ts = 0, [], [], []
    wmark = nchunk - chunk_mtu
    for seq, k in enumerate(order):
        m = msgs[k]
        sz = 96 + len(m)
        dcache[64 * chunk:64 * chunk + sz] = np.frombuffer(bytes(pub[k]) + bytes(sig[k]) + m, np.uint8)
        tso = (1000 + 7 * seq) & 0xFFFFFFFF
        tango.publish(mc, seq, 0, chunk, sz, 3, tso, 0)
        chunks.append(chunk); sizes.append(sz); ts.append(tso)
        chunk = tango.dcache_compact_next(chunk, sz, 0, wmark)
    return mc, dcache, chunks, sizes, ts


def _model(pub, sig, msgs, order, verdict, tc_depth):
    seen, q = set(), collections.deque()
    out, ha, sv = [], 0, 0
    for seq, k in enumerate(order):
        tag = int.from_bytes(bytes(sig[k][:8]), "little")
        if tc_depth and tag:
            if tag in seen:
                ha += 1
                continue
            seen.add(tag); q.append(tag)
            if len(q) > tc_depth:
                seen.discard(q.popleft())
        if verdict[k] != 0:
            sv += 1
            continue
        h = hashlib.sha512(bytes(sig[k][:32]) + bytes(pub[k]) + msgs[k]).digest()
        out.append((seq, int.from_bytes(h[:8], "little")))
    return out, ha, sv


def _pool(golden):
    pick = list(range(0, len(golden), 3))
    pub, sig = golden.pub[pick], golden.sig[pick]
    msgs = [golden.msg(i) for i in pick]
    return pub, sig, msgs, golden.expect[pick]


@pytest.mark.parametrize("batch_max,tc_depth,zero_copy", [(512, 1 << 12, False), (37, 8, False), (1, 0, False),
                                                         (512, 1 << 12, True), (37, 8, True)])
def test_tile_publishes_passing_frags_in_order(golden, batch_max, tc_depth, zero_copy):
    from firedancer_amd import tango
    pub, sig, msgs, verdict = _pool(golden)
    rng = np.random.default_rng(batch_max)
    n = 1500 if batch_max > 1 else 300
    order = rng.integers(0, len(msgs), n)           # repeats = HA duplicates
    mc_in, dc, chunks, sizes, ts = _feed(pub, sig, msgs, order, 2048)
    mc_out = tango.mcache_new(2048)
    tile = tango.VerifyTile(0, batch_max=batch_max, tcache_depth=tc_depth)
    if zero_copy:
        tile.register_dcache(dc)        # frags copied on the GPU from the mapped data region
    try:
        diag, lat = tile.run(mc_in, dc, 0, mc_out, 0, n, lat_max=n)
        exp, ha, sv = _model(pub, sig, msgs, order, verdict, tc_depth)
        assert diag["in_cnt"] == n and diag["ha_filt_cnt"] == ha and diag["sv_filt_cnt"] == sv
        assert diag["out_cnt"] == len(exp) and diag["ovrn_cnt"] == 0 and diag["bad_frag_cnt"] == 0
        assert tile.in_fseq == n                      # every input frag released
        for o, (seq_in, tag) in enumerate(exp):
            line = mc_out[o]
            k = order[seq_in]
            assert int(line["seq"]) == o
            assert int(line["sig"]) == tag
            assert (int(line["sz"]), int(line["ctl"]), int(line["tsorig"])) == (sizes[seq_in], 3, ts[seq_in])
            # published out of the tile's own dcache: the verified bytes
            assert tile.out_frame(line["chunk"], line["sz"]) == bytes(pub[k]) + bytes(sig[k]) + msgs[k]
        assert diag["batch_cnt"] >= 1 and diag["batch_sig_cnt"] == n - ha
        assert lat.size == len(exp)
    finally:
        tile.close()


def test_tile_fresh_signatures_vs_oracle():
    """Fresh seeded signatures with 10 % bit flips through the tile: the set
    of published frags equals the oracle's accepted set."""
    from firedancer_amd import ed25519, tango
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(4242, 2000, 0, 400, True)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    for i in np.nonzero(fk)[0]:
        byte, bit = divmod(int(fp[i]), 8)
        tgt = sig[i] if fk[i] == 1 else (blob[off[i]:] if fk[i] == 2 else pub[i])
        tgt[byte] ^= 1 << bit
    msgs = [bytes(blob[off[i]:off[i] + sz[i]]) for i in range(len(sz))]
    verdict = _oracle.verify_batch(_golden.Batch(pub, sig, off, sz, blob))
    order = np.arange(len(msgs))
    mc_in, dc, _, _, _ = _feed(pub, sig, msgs, order, 4096)
    mc_out = tango.mcache_new(4096)
    tile = tango.VerifyTile(0, batch_max=256, tcache_depth=1 << 12)
    try:
        diag, _ = tile.run(mc_in, dc, 0, mc_out, 0, len(order))
    finally:
        tile.close()
    exp, ha, sv = _model(pub, sig, msgs, order, verdict, 1 << 12)
    assert diag["out_cnt"] == len(exp) and diag["sv_filt_cnt"] == sv
    assert [int(mc_out[o]["sig"]) for o in range(len(exp))] == [t for _, t in exp]


def test_stream_bench_smoke():
    """Producer -> tile -> consumer threads with credit flow control."""
    from firedancer_amd import ed25519, tango
    n = 512
    rng = np.random.default_rng(3)
    prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    blob = rng.integers(0, 256, n * 200 + 1, dtype=np.uint8)
    off = (np.arange(n) * 200).astype(np.uint32)
    sz = np.full(n, 200, np.uint32)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    r = tango.bench_stream(0, 256, 0, pub, sig, off, sz, blob, 20000)
    assert r["published"] == 20000 and r["sv_filt"] == 0
    assert r["frags_per_s"] > 0 and 0 < r["p50_ns"] <= r["p99_ns"]
    r = tango.bench_stream(0, 256, 0, pub, sig, off, sz, blob, 5000, rate=50000.0)
    assert r["published"] == 5000 and r["p50_ns"] > 0
    r = tango.bench_stream(0, 1024, 0, pub, sig, off, sz, blob, 20000, zero_copy=True)
    assert r["published"] == 20000 and r["sv_filt"] == 0


def _stream_pool(seed, count, szhi=1232):
    """Fresh signatures, 10 % of them corrupted (bit flips in sig, msg or
    pub), with the oracle's verdicts and the expected dedup tags."""
    from firedancer_amd import ed25519
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(seed, count, 0, szhi, True)
    pub, sig = ed25519.sign_batch_gpu(prv, blob, off, sz)
    for i in np.nonzero(fk)[0]:
        byte, bit = divmod(int(fp[i]), 8)
        tgt = sig[i] if fk[i] == 1 else (blob[off[i]:] if fk[i] == 2 else pub[i])
        tgt[byte] ^= 1 << bit
    err = _oracle.verify_batch(_golden.Batch(pub, sig, off, sz, blob))
    tag = np.array([int.from_bytes(hashlib.sha512(bytes(sig[i][:32]) + bytes(pub[i]) +
                                                  bytes(blob[off[i]:off[i] + sz[i]])).digest()[:8], "little")
                    for i in range(count)], np.uint64)
    assert 0.05 < (err != 0).mean() < 0.15
    return pub, sig, off, sz, blob, err, tag


@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_producer_rewrites_wrapping_dcache(zero_copy):
    """A producer that writes every frame into a small wrapping data region
    (in_depth + 64 frames) as fast as the tile's in_fseq credit allows,
    at batch_max 256: every published frag's verdict, tag,
    bytes (in the tile's output dcache) and order equal the oracle's, none
    is missing, none overran."""
    from firedancer_amd import tango
    pub, sig, off, sz, blob, err, tag = _stream_pool(777 + zero_copy, 3000)
    nf = 60000
    r = tango.bench_stream(0, 256, 0, pub, sig, off, sz, blob, nf, zero_copy=zero_copy, writes=True,
                           expect_err=err, expect_tag=tag)
    want = int((err[np.arange(nf) % err.size] == 0).sum())
    assert r["mismatches"] == 0 and r["ovrn"] == 0
    assert r["checked"] == r["published"] == want and r["sv_filt"] == nf - want


@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_lapping_producer_never_publishes_rewritten_frags(zero_copy):
    """A producer that ignores the tile's credit and laps it: frags it
    rewrote before the tile was done are dropped as overrun; every frag
    that is published still carries exactly the bytes that were verified,
    with the oracle's verdict and tag, in input order."""
    from firedancer_amd import tango
    pub, sig, off, sz, blob, err, tag = _stream_pool(999 + zero_copy, 2000, 400)
    r = tango.bench_stream(0, 1024, 0, pub, sig, off, sz, blob, 400000, zero_copy=zero_copy, writes=True, lap=True,
                           expect_err=err, expect_tag=tag)
    assert r["mismatches"] == 0 and r["checked"] == r["published"] > 0
    assert r["published"] + r["sv_filt"] + r["ovrn"] <= 400000


@pytest.mark.parametrize("batch_max", [4096, 16384])
@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_large_batches_vs_oracle(batch_max, zero_copy):
    """Config 5 at its large batch caps: saturated stream of fresh
    signatures with 10 % corrupted frags through the persistent consumer;
    the published stream equals the oracle's accepted set, in order, with
    the right tags and bytes; every frag went through exactly one chunk of
    at most 8 (latency), 16 (quad) or 64 (throughput) frags."""
    from firedancer_amd import tango
    pub, sig, off, sz, blob, err, tag = _stream_pool(4096 + batch_max + zero_copy, 8192, 400)
    nf = 8 * batch_max + 12345
    r = tango.bench_stream(0, batch_max, 0, pub, sig, off, sz, blob, nf, zero_copy=zero_copy, expect_err=err,
                           expect_tag=tag)
    want = int((err[np.arange(nf) % err.size] == 0).sum())
    assert r["mismatches"] == 0 and r["ovrn"] == 0
    assert r["checked"] == r["published"] == want and r["sv_filt"] == nf - want
    assert r["gpu_frags_lat"] + r["gpu_frags_quad"] + r["gpu_frags_thr"] == nf
    assert r["gpu_frags_lat"] <= 8 * r["gpu_chunks_lat"] and r["gpu_frags_thr"] <= 64 * r["gpu_chunks_thr"]
    assert r["gpu_frags_quad"] <= 16 * r["gpu_chunks_quad"]


@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_auto_levels_vs_oracle(zero_copy):
    """The AUTO level rule end to end, every frag checked: a saturated
    stream ends up in throughput chunks (the window-full rule and the 2 ms
    episode of fd_verify_amd_tile_level_step), a stream paced at 20 M frags/s
    (above the latency chunks' capacity, well under the quad chunks') runs
    mostly in quad chunks; both publish exactly the oracle's accepted set."""
    from firedancer_amd import tango
    pub, sig, off, sz, blob, err, tag = _stream_pool(6060 + zero_copy, 8192, 400)
    for rate, nf in ((0.0, 1 << 20), (20e6, 1 << 20)):
        r = tango.bench_stream(0, 4096, 0, pub, sig, off, sz, blob, nf, rate=rate, zero_copy=zero_copy,
                               expect_err=err, expect_tag=tag)
        want = int((err[np.arange(nf) % err.size] == 0).sum())
        assert r["mismatches"] == 0 and r["ovrn"] == 0
        assert r["checked"] == r["published"] == want and r["sv_filt"] == nf - want
        assert r["gpu_frags_lat"] + r["gpu_frags_quad"] + r["gpu_frags_thr"] == nf
        if rate:
            assert r["gpu_frags_quad"] > nf // 2, r
        else:
            assert r["gpu_frags_thr"] > nf // 2, r


def test_tile_copy_without_helper_vs_oracle():
    """Copy mode with every copy on the stager (cfg.copy_cpu = COPY_INLINE;
    the bench's default gives copy mode a helper thread when the process has
    6 CPUs): the same exact published stream."""
    from firedancer_amd import tango
    batch_max = 16384
    pub, sig, off, sz, blob, err, tag = _stream_pool(4096 + batch_max, 8192, 400)
    nf = 4 * batch_max + 777
    r = tango.bench_stream(0, batch_max, 0, pub, sig, off, sz, blob, nf, expect_err=err, expect_tag=tag,
                           copy_inline=True)
    want = int((err[np.arange(nf) % err.size] == 0).sum())
    assert r["mismatches"] == 0 and r["ovrn"] == 0
    assert r["checked"] == r["published"] == want and r["sv_filt"] == nf - want


def test_tile_copy_helper_stalls_are_recopied_exactly():
    """Copy mode with the copy helper (the bench pins it when the process
    may use 6 CPUs) stalled 200 us before every 4th block it claims, under a
    producer that rewrites a small wrapping data region: the stager re-copies
    the stalled blocks into fresh frames (copy_steals > 0) while the late
    helper still writes the old ones, and every published frag's verdict,
    tag, bytes and order still equal the oracle's."""
    import os
    from firedancer_amd import tango
    if len(os.sched_getaffinity(0)) < 6:
        pytest.skip("the bench runs the copy helper only with 6 or more CPUs")
    pub, sig, off, sz, blob, err, tag = _stream_pool(5151, 4096, 400)
    nf = 200000
    r = tango.bench_stream(0, 4096, 0, pub, sig, off, sz, blob, nf, writes=True, expect_err=err, expect_tag=tag,
                           stall_helper=True)
    want = int((err[np.arange(nf) % err.size] == 0).sum())
    assert r["copy_steals"] > 0
    assert r["mismatches"] == 0 and r["ovrn"] == 0
    assert r["checked"] == r["published"] == want and r["sv_filt"] == nf - want


@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_txn_framing_vs_oracle(zero_copy):
    """Frags carrying wire transactions (multi-signer, legacy + v0, some
    corrupted, some duplicated): the tile publishes exactly the
    transactions the oracle accepts (fd_txn_parse + every signature), in
    order, tagged with the first signature's SHA-512 tag; drops count as
    SV_FILT / HA_FILT."""
    import hashlib
    import _txn
    from firedancer_amd import tango
    rng = np.random.default_rng(8)
    pays, nsig = _txn.build_txns(44, 200, nsig_hi=6)
    pays = [bytearray(p) for p in pays]
    for t in rng.choice(len(pays), 30, replace=False):
        pays[t][1 + int(rng.integers(0, 64))] ^= 0x08                      # a signature byte
    for t in rng.choice(len(pays), 10, replace=False):
        pays[t][1 + 64 * pays[t][0]] ^= 0x40                              # header -> parse failure
    pays = [bytes(p) for p in pays]
    order = list(range(len(pays))) + [3, 7, 11]                            # three HA duplicates
    depth = 1024
    mtu_chunks = ((1232 + 127) >> 7) << 1
    dcache = tango._aligned(64 * mtu_chunks * (len(order) + 2))
    mc_in, mc_out = tango.mcache_new(depth), tango.mcache_new(depth)
    chunk = 0
    chunks = []
    for seq, k in enumerate(order):
        p = pays[k]
        dcache[64 * chunk:64 * chunk + len(p)] = np.frombuffer(p, np.uint8)
        tango.publish(mc_in, seq, 0, chunk, len(p), 3, seq, 0)
        chunks.append(chunk)
        chunk += mtu_chunks
    blob, off, sz = _txn.pack(pays)
    eterr, _, _ = _oracle.txn_verify_batch(blob, off, sz)
    tile = tango.VerifyTile(0, batch_max=64, tcache_depth=4096, framing=tango.VerifyTile.FRAMING_TXN)
    if zero_copy:
        tile.register_dcache(dcache)    # transactions copied on the GPU from the mapped data region
    try:
        diag, _ = tile.run(mc_in, dcache, 0, mc_out, 0, len(order))
        frames = [tile.out_frame(mc_out[o]["chunk"], mc_out[o]["sz"]) for o in range(int(diag["out_cnt"]))]
    finally:
        tile.close()
    seen, exp = set(), []
    ha = sv = 0
    for seq, k in enumerate(order):
        p = pays[k]
        tag = int.from_bytes(p[1:9], "little") if 1 <= p[0] <= 127 and 64 * p[0] <= len(p) - 1 else 0
        if tag:
            if tag in seen:
                ha += 1
                continue
            seen.add(tag)
        if eterr[k]:
            sv += 1
            continue
        m = 1 + 64 * p[0]
        h = hashlib.sha512(p[1:33] + p[m + (1 if p[m] & 0x80 else 0) + 4: m + (1 if p[m] & 0x80 else 0) + 36] +
                           p[m:]).digest()
        exp.append((seq, int.from_bytes(h[:8], "little")))
    assert diag["ha_filt_cnt"] == ha == 3 and diag["sv_filt_cnt"] == sv and diag["out_cnt"] == len(exp)
    for o, (seq_in, tag) in enumerate(exp):
        assert frames[o] == pays[order[seq_in]] and int(mc_out[o]["tsorig"]) == seq_in
        assert int(mc_out[o]["sig"]) == tag


def _txn_through_tile(pays, chunk_mode=0, zero_copy=False, batch_max=4096, depth=1 << 16):
    """Wire transactions as frags (one per frame, in order) through a TXN
    tile with HA dedup off: (diag, verdict log, published frames, tags,
    published input seqs)."""
    from firedancer_amd import tango
    mtu_chunks = ((1232 + 127) >> 7) << 1
    n = len(pays)
    dcache = tango._aligned((64 * mtu_chunks * (n + 2) + 4095) & ~4095, 4096)
    mc_in, mc_out = tango.mcache_new(depth), tango.mcache_new(depth)
    for seq, p in enumerate(pays):
        c = seq * mtu_chunks
        if len(p):
            dcache[64 * c:64 * c + len(p)] = np.frombuffer(p, np.uint8)
        tango.publish(mc_in, seq, 0, c, len(p), 3, seq, 0)
    tile = tango.VerifyTile(0, batch_max=batch_max, tcache_depth=0, framing=tango.VerifyTile.FRAMING_TXN,
                            chunk_mode=chunk_mode)
    if zero_copy:
        tile.register_dcache(dcache)
    log = np.full(n, 99, np.int8)
    tile.set_verdict_log(log)
    try:
        diag, _ = tile.run(mc_in, dcache, 0, mc_out, 0, n)
        k = int(diag["out_cnt"])
        frames = [tile.out_frame(mc_out[o]["chunk"], mc_out[o]["sz"]) for o in range(k)]
        tags = [int(mc_out[o]["sig"]) for o in range(k)]
        seqs = [int(mc_out[o]["tsorig"]) for o in range(k)]
    finally:
        tile.close()
    return diag, log, frames, tags, seqs


def _txn_tag(p):
    """First signature's SHA-512 tag of a well-formed transaction (the
    synthetic and fixture ones have < 128 accounts: one-byte compact-u16)."""
    m = 1 + 64 * p[0]
    a = m + (1 if p[m] & 0x80 else 0) + 4
    return int.from_bytes(hashlib.sha512(p[1:33] + p[a:a + 32] + p[m:]).digest()[:8], "little")


@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_txn_reference_mutations_vs_oracle(zero_copy):
    """Every mutation of the reference's three fixture transactions
    (tests/golden/txn_mutations.bin: footprints from the COMPILED reference
    fd_txn_parse) as TXN frags through the persistent kernel: every frag's
    verdict equals the oracle's (-4 exactly where the reference's footprint
    is 0), and the published frags are the accepted ones, in order, with
    their bytes and first-signature tags."""
    import _txn
    for f in _txn.load_fixtures():
        allm = _txn.mutation_list(f.payload)
        keep = [i for i, m in enumerate(allm) if 1 <= len(m) <= 1232]   # an empty frag is a bad frag, not a txn
        muts = [allm[i] for i in keep]
        fps = f.footprint[keep]
        blob, off, sz = _txn.pack(muts)
        eterr, _, _ = _oracle.txn_verify_batch(blob, off, sz)
        assert np.array_equal(eterr == -4, fps == 0)
        diag, log, frames, tags, seqs = _txn_through_tile(muts, zero_copy=zero_copy)
        bad = np.nonzero(log != eterr)[0]
        assert bad.size == 0, [(int(i), int(log[i]), int(eterr[i])) for i in bad[:10]]
        acc = np.nonzero(eterr == 0)[0].tolist()
        assert seqs == acc and diag["out_cnt"] == len(acc) and diag["sv_filt_cnt"] == len(muts) - len(acc)
        assert all(frames[o] == muts[i] for o, i in enumerate(acc))
        assert tags == [_txn_tag(muts[i]) for i in acc]


# AUTO, LATENCY (8 slots; > 8 signers alone, 1 lane each), THROUGHPUT, QUAD (16 slots)
@pytest.mark.parametrize("chunk_mode", [0, 1, 2, 3])
def test_tile_txn_mixed_vs_oracle_per_chunk_mode(chunk_mode):
    """1500 multi-signer transactions (1..12 signers, 64..1232 B, legacy and
    v0) with corrupted signatures, signer keys, headers and truncations,
    through the persistent kernel with each chunk mode: every transaction's
    verdict equals the oracle's; accepted ones publish in order with their
    first signature's tag; slots are packed <= 64 (<= 8 in latency chunks,
    <= 16 in quad chunks)."""
    import test_txn_gpu
    pays = test_txn_gpu._mixed_batch(77 + chunk_mode, 1500)
    blob, off, sz = __import__("_txn").pack(pays)
    eterr, _, _ = _oracle.txn_verify_batch(blob, off, sz)
    diag, log, frames, tags, seqs = _txn_through_tile(pays, chunk_mode=chunk_mode, zero_copy=chunk_mode == 2)
    bad = np.nonzero(log != eterr)[0]
    assert bad.size == 0, [(int(i), int(log[i]), int(eterr[i])) for i in bad[:10]]
    acc = np.nonzero(eterr == 0)[0].tolist()
    assert seqs == acc and tags == [_txn_tag(pays[i]) for i in acc]
    assert set(np.unique(eterr).tolist()) >= {0, -3, -4}
    if chunk_mode == 2:
        assert diag["gpu_chunk_lat_cnt"] == 0 and diag["gpu_chunk_quad_cnt"] == 0
    if chunk_mode == 1:
        assert diag["gpu_chunk_lat_cnt"] > 0 and diag["gpu_chunk_quad_cnt"] == 0
    if chunk_mode == 3:
        assert diag["gpu_chunk_quad_cnt"] > 0 and diag["gpu_chunk_lat_cnt"] == 0
        assert diag["gpu_frag_quad_cnt"] <= 16 * diag["gpu_chunk_quad_cnt"]
        assert diag["quad_pair_cnt"] == 0          # pairs are PUB_SIG_MSG only


def test_tile_txn_many_signers_at_the_head_go_at_once():
    """Latency chunks hold 8 slots: a head transaction of 12 signers is a
    chunk of its own (1 lane per signature) and is handed over at once
    rather than waiting lat_fill_ns for more staged slots -- with the fill
    wait set to 2 s, every transaction of 9..12 signers still publishes
    within the run, each with the oracle's verdict."""
    import _txn
    pays, _ = _txn.build_txns(91, 40, nsig_lo=9, nsig_hi=12, msg_hi=600)
    blob, off, sz = _txn.pack(pays)
    eterr, _, _ = _oracle.txn_verify_batch(blob, off, sz)
    from firedancer_amd import tango
    mtu_chunks = ((1232 + 127) >> 7) << 1
    n = len(pays)
    dcache = tango._aligned((64 * mtu_chunks * (n + 2) + 4095) & ~4095, 4096)
    mc_in, mc_out = tango.mcache_new(1024), tango.mcache_new(1024)
    for seq, p in enumerate(pays):
        c = seq * mtu_chunks
        dcache[64 * c:64 * c + len(p)] = np.frombuffer(p, np.uint8)
        tango.publish(mc_in, seq, 0, c, len(p), 3, seq, 0)
    tile = tango.VerifyTile(0, batch_max=4096, tcache_depth=0, framing=tango.VerifyTile.FRAMING_TXN,
                            chunk_mode=tango.CHUNK_LATENCY, lat_fill_ns=2_000_000_000, lat_free_chunks=0)
    log = np.full(n, 99, np.int8)
    tile.set_verdict_log(log)
    # the run never sees the end of its input (frag_cnt 0): only the hand-off
    # rule can release the last staged transaction before the 2 s fill wait
    import ctypes
    import threading
    import time
    want = int((eterr == 0).sum())
    stop, seen = ctypes.c_int(0), []

    def watch():
        t0 = time.time()
        while time.time() - t0 < 1.5:
            if want == 0 or int(mc_out[(want - 1) % 1024]["seq"]) == want - 1:
                seen.append(time.time() - t0)
                break
            time.sleep(0.0005)
        stop.value = 1
    th = threading.Thread(target=watch)
    th.start()
    try:
        diag, _ = tile.run(mc_in, dcache, 0, mc_out, 0, 0, stop=stop)
    finally:
        th.join()
        tile.close()
    assert seen, "the last transactions waited for the 2 s fill"
    assert np.array_equal(log, eterr)
    assert diag["out_cnt"] == want and diag["gpu_chunk_lat_cnt"] == 0

def test_tile_txn_framing_needs_room_for_a_full_transaction():
    """TXN framing with batch_max < 19 could never stage a 19-signer
    transaction: refused up front instead of spinning."""
    from firedancer_amd import ed25519, tango
    with pytest.raises(ed25519.EngineError):
        tango.VerifyTile(0, batch_max=8, framing=tango.VerifyTile.FRAMING_TXN)
    t = tango.VerifyTile(0, batch_max=19, framing=tango.VerifyTile.FRAMING_TXN)
    t.close()


def test_two_tiles_share_one_gpu():
    """Two tiles created on one device before either runs split its wave
    slots (each run's persistent kernel takes 8 x CUs / 2 waves), so their
    runs proceed side by side from two threads; each publishes exactly the
    oracle's accepted set, in order, with the right tags."""
    import threading
    from firedancer_amd import ed25519, tango
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(5151, 6000, 0, 300, True)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    for i in np.nonzero(fk)[0]:
        byte, bit = divmod(int(fp[i]), 8)
        sig[i, byte % 64] ^= 1 << bit
    msgs = [bytes(blob[off[i]:off[i] + sz[i]]) for i in range(len(sz))]
    verdict = _oracle.verify_batch(_golden.Batch(pub, sig, off, sz, blob))
    halves = [np.arange(0, 3000), np.arange(3000, 6000)]
    feeds = [_feed(pub, sig, msgs, o, 4096) for o in halves]
    outs = [tango.mcache_new(4096) for _ in halves]
    tiles = [tango.VerifyTile(0, batch_max=1024, tcache_depth=1 << 12) for _ in halves]
    res = [None, None]

    def go(k):
        res[k] = tiles[k].run(feeds[k][0], feeds[k][1], 0, outs[k], 0, len(halves[k]))

    try:
        th = [threading.Thread(target=go, args=(k,)) for k in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th)
    finally:
        for t in tiles:
            t.close()
    for k, order in enumerate(halves):
        diag, _ = res[k]
        exp, ha, sv = _model(pub, sig, msgs, order, verdict, 1 << 12)
        assert diag["out_cnt"] == len(exp) and diag["sv_filt_cnt"] == sv and diag["ha_filt_cnt"] == ha
        assert [int(outs[k][o]["sig"]) for o in range(len(exp))] == [tg for _, tg in exp]


@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_runs_until_stop_and_continues(zero_copy):
    """The deployment shape: a run with frag_cnt 0 lasts until another
    thread raises *stop (the reference's cnc halt), publishing everything it
    took in; a second run on the same tile continues the input and output
    sequences (its kernel's tickets restart at the tile's descriptor count)
    and publishes the rest in order."""
    import ctypes
    import threading
    import time
    from firedancer_amd import ed25519, tango
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(6262, 3000, 0, 300, True)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    for i in np.nonzero(fk)[0]:
        byte, bit = divmod(int(fp[i]), 8)
        sig[i, byte % 64] ^= 1 << bit
    msgs = [bytes(blob[off[i]:off[i] + sz[i]]) for i in range(len(sz))]
    verdict = _oracle.verify_batch(_golden.Batch(pub, sig, off, sz, blob))
    order = np.arange(len(msgs))
    mc_in, dc, _, _, _ = _feed(pub, sig, msgs, order, 4096)
    mc_out = tango.mcache_new(4096)
    exp, ha, sv = _model(pub, sig, msgs, order, verdict, 0)
    first = 1800                                   # frags the first run takes in
    n_first = sum(1 for s_in, _ in exp if s_in < first)
    tile = tango.VerifyTile(0, batch_max=512, tcache_depth=0)
    if zero_copy:
        tile.register_dcache(dc)
    try:
        # run 1: only the first `first` frags are visible to it (the later
        # lines still read "never published"), stop once they are out
        mc_hide = tango.mcache_new(4096)
        mc_hide[:first] = mc_in[:first]
        stop = ctypes.c_int(0)

        def halt():
            t0 = time.time()
            while time.time() - t0 < 60:
                if int(mc_out[(n_first - 1) % 4096]["seq"]) == n_first - 1:
                    break
                time.sleep(0.001)
            stop.value = 1
        th = threading.Thread(target=halt)
        th.start()
        d1, _ = tile.run(mc_hide, dc, 0, mc_out, 0, 0, stop=stop)
        th.join()
        assert d1["in_cnt"] == first and d1["out_cnt"] == n_first
        # run 2: the rest, sequences continued
        d2, _ = tile.run(mc_in, dc, first, mc_out, n_first, len(order) - first)
        assert d2["out_cnt"] == len(exp) - n_first
    finally:
        tile.close()
    assert d1["sv_filt_cnt"] + d2["sv_filt_cnt"] == sv and tile.in_fseq == len(order)
    assert [int(mc_out[o]["seq"]) for o in range(len(exp))] == list(range(len(exp)))
    assert [int(mc_out[o]["sig"]) for o in range(len(exp))] == [t for _, t in exp]


@pytest.mark.parametrize("chunk_mode", [1, 2, 3])   # tango.CHUNK_LATENCY, CHUNK_THROUGHPUT, CHUNK_QUAD
@pytest.mark.parametrize("zero_copy", [False, True])
def test_tile_golden_codes_per_chunk_mode(monkeypatch, golden, chunk_mode, zero_copy):
    """Every golden vector (the reference's codes, the 156 limb-compare false
    rejects included) through k_tile_persist with every chunk forced to one
    mode: 8-lane latency chunks (k_dsm8's body), 64-frag throughput chunks
    (k_dsm's body) or 16-frag quad chunks (k_dsm4's body).  The tile's verdict log must equal the reference's code
    for every frag; the published set and the per-code SV_FILT counts follow."""
    from firedancer_amd import tango
    monkeypatch.setenv("FD_AMD_TILE_PAIRS", "1")      # quad chunks as pairs where 17+ frags are staged
    n = len(golden)
    idx = [i for i in range(n) if golden.msg_sz[i] <= 1232]
    assert len(idx) == n
    msgs = [golden.msg(i) for i in range(n)]
    order = np.arange(n)
    mc_in, dc, _, _, _ = _feed(golden.pub, golden.sig, msgs, order, 4096)
    mc_out = tango.mcache_new(4096)
    tile = tango.VerifyTile(0, batch_max=4096, tcache_depth=0, chunk_mode=chunk_mode)
    if zero_copy:
        tile.register_dcache(dc)
    log = np.full(n, 99, np.int8)
    tile.set_verdict_log(log)
    try:
        diag, _ = tile.run(mc_in, dc, 0, mc_out, 0, n)
    finally:
        tile.close()
    exp = golden.expect
    bad = np.nonzero(log != exp)[0]
    assert bad.size == 0, [(int(i), int(log[i]), int(exp[i])) for i in bad[:10]]
    assert diag["out_cnt"] == int((exp == 0).sum())
    assert [diag["sv_filt_sig_cnt"], diag["sv_filt_pubkey_cnt"], diag["sv_filt_msg_cnt"]] == \
        [int((exp == c).sum()) for c in (-1, -2, -3)]
    key = {1: "gpu_frag_lat_cnt", 2: "gpu_frag_thr_cnt", 3: "gpu_frag_quad_cnt"}[chunk_mode]
    assert diag[key] == n
    assert all(int(mc_out[o]["seq"]) == o for o in range(diag["out_cnt"]))
    if chunk_mode == 3:
        # the whole set is staged at once: quad chunks go as pairs (17..32 frags, one front pass)
        assert diag["quad_pair_cnt"] > 0 and 2 * diag["quad_pair_cnt"] <= diag["gpu_chunk_quad_cnt"]


@pytest.mark.parametrize("pairs", ["0", "1"])
def test_tile_quad_pairs_vs_oracle(monkeypatch, pairs):
    """Quad chunks with and without pairs (FD_AMD_TILE_PAIRS=1 opts in; 0,
    the default: no pair workspaces, every quad chunk runs its own front).  A pair's sub 1 waits
    for sub 0's front on another wave (often another XCD) and verifies
    entries 16..31 from sub 0's workspace: a stream of fresh signatures with
    10 % corrupted frags at a ragged length (pairs of 17..32, a lone quad
    chunk at the tail) publishes exactly the oracle's accepted set, in order,
    with the right tags, either way."""
    from firedancer_amd import tango
    monkeypatch.setenv("FD_AMD_TILE_PAIRS", pairs)
    pub, sig, off, sz, blob, err, tag = _stream_pool(9100 + int(pairs), 4096, 400)
    nf = 3 * 4096 + 17 * 29 + 5
    r = tango.bench_stream(0, 4096, 0, pub, sig, off, sz, blob, nf, zero_copy=pairs == "1", expect_err=err,
                           expect_tag=tag, chunk_mode=3)
    want = int((err[np.arange(nf) % err.size] == 0).sum())
    assert r["mismatches"] == 0 and r["ovrn"] == 0
    assert r["checked"] == r["published"] == want and r["sv_filt"] == nf - want
    assert r["gpu_frags_quad"] == nf and r["gpu_frags_quad"] <= 16 * r["gpu_chunks_quad"]
    if pairs == "1":
        assert r["quad_pairs"] > 0 and 2 * r["quad_pairs"] <= r["gpu_chunks_quad"]
    else:
        assert r["quad_pairs"] == 0


def _signed_feed(seed, count, depth):
    from firedancer_amd import ed25519
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(seed, count, 0, 300, False)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    msgs = [bytes(blob[off[i]:off[i] + sz[i]]) for i in range(len(sz))]
    return pub, sig, msgs, _feed(pub, sig, msgs, np.arange(count), depth)


def test_tile_halts_while_backpressured():
    """The consumer stops advancing out_fseq: the tile fills its output
    credit (out_depth frags) and is backpressured.  A raised *stop returns
    the run within 100 ms (the halt grace is 50 ms), the way the reference
    tile keeps its HALT check running while backpressured; the frags it
    could not publish are counted in halt_drop_cnt."""
    import ctypes
    import threading
    import time
    from firedancer_amd import tango
    n = 6000
    pub, sig, msgs, (mc_in, dc, _, _, _) = _signed_feed(3131, n, 8192)
    mc_out = tango.mcache_new(256)
    out_fseq = ctypes.c_ulong(0)                 # a consumer that never moves
    tile = tango.VerifyTile(0, batch_max=1024, tcache_depth=0)
    stop = ctypes.c_int(0)
    res = {}

    def go():
        try:
            res["r"] = tile.run(mc_in, dc, 0, mc_out, 0, 0, stop=stop, out_fseq=out_fseq)
        except Exception as e:   # noqa: BLE001
            res["e"] = e
        res["t"] = time.perf_counter()

    th = threading.Thread(target=go)
    th.start()
    try:
        t0 = time.time()
        while int(mc_out[255]["seq"]) != 255 and time.time() - t0 < 30:
            time.sleep(0.001)
        time.sleep(0.05)                            # the tile now spins backpressured
        assert th.is_alive()
        t_stop = time.perf_counter()
        stop.value = 1
        th.join(timeout=10)
        assert not th.is_alive()
    finally:
        stop.value = 1
        th.join(timeout=10)
        tile.close()
    assert "e" not in res, res.get("e")
    assert res["t"] - t_stop < 0.1
    diag, _ = res["r"]
    assert diag["out_cnt"] == 256 and diag["halt_drop_cnt"] > 0
    assert diag["out_cnt"] + diag["sv_filt_cnt"] + diag["halt_drop_cnt"] == diag["in_cnt"]


def test_tile_stop_drains_a_slow_share_without_drops():
    """*stop while the GPU is slow to drain (a 16-wave share, a full window)
    but the output is NOT backpressured (no out_fseq): the halt grace (here
    1 ms) never starts, the run publishes everything it took in, and
    halt_drop_cnt stays 0 (the grace runs only while
    backpressured)."""
    import ctypes
    import threading
    import time
    from firedancer_amd import tango
    n = 6000
    pub, sig, msgs, (mc_in, dc, _, _, _) = _signed_feed(3737, n, 8192)
    mc_out = tango.mcache_new(8192)
    tile = tango.VerifyTile(0, batch_max=1024, tcache_depth=0, waves=16, halt_grace_ns=1000000,
                            chunk_mode=tango.CHUNK_THROUGHPUT)
    stop = ctypes.c_int(0)
    res = {}

    def go():
        try:
            res["r"] = tile.run(mc_in, dc, 0, mc_out, 0, 0, stop=stop)
        except Exception as e:   # noqa: BLE001
            res["e"] = e

    th = threading.Thread(target=go)
    th.start()
    try:
        t0 = time.time()
        while int(mc_out[0]["seq"]) != 0 and time.time() - t0 < 30:
            time.sleep(0.0002)
        stop.value = 1                              # frags are still in flight on a slow share
        th.join(timeout=30)
        assert not th.is_alive()
    finally:
        stop.value = 1
        th.join(timeout=30)
        tile.close()
    assert "e" not in res, res.get("e")
    diag, _ = res["r"]
    assert diag["halt_drop_cnt"] == 0
    assert diag["out_cnt"] + diag["sv_filt_cnt"] == diag["in_cnt"] > 64
    assert all(int(mc_out[o]["seq"]) == o for o in range(int(diag["out_cnt"])))


def test_tiles_per_device_capped_at_hw_queues():
    """Each tile's run holds one hardware queue of the high-priority pool
    for its whole run; a process gets GPU_MAX_HW_QUEUES (4) per priority, so
    a fifth tile on one device is refused at creation instead of queueing
    its kernel behind another tile's run."""
    import os
    from firedancer_amd import ed25519, tango
    cap = int(os.environ.get("GPU_MAX_HW_QUEUES") or 4)
    tiles = []
    try:
        for _ in range(cap):
            tiles.append(tango.VerifyTile(0, batch_max=256, tcache_depth=0))
        with pytest.raises(ed25519.EngineError):
            tango.VerifyTile(0, batch_max=256, tcache_depth=0)
        tiles.pop().close()
        tiles.append(tango.VerifyTile(0, batch_max=256, tcache_depth=0))   # a freed queue is usable again
    finally:
        for t in tiles:
            t.close()


def test_engine_call_beside_a_tile_with_a_partial_share(golden, engine):
    """A tile whose run holds a quarter of the GPU's wave slots (cfg.waves)
    does not starve the device: an engine batch call on the same GPU
    completes while the run lasts, with the reference's codes."""
    import ctypes
    import threading
    import time
    from firedancer_amd import tango
    n = 500
    pub, sig, msgs, (mc_in, dc, _, _, _) = _signed_feed(4141, n, 1024)
    mc_out = tango.mcache_new(1024)
    tile = tango.VerifyTile(0, batch_max=1024, tcache_depth=0, waves=512)
    stop = ctypes.c_int(0)
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("r", tile.run(mc_in, dc, 0, mc_out, 0, 0, stop=stop)))
    th.start()
    try:
        t0 = time.time()
        while int(mc_out[n - 1]["seq"]) != n - 1 and time.time() - t0 < 30:
            time.sleep(0.001)
        assert th.is_alive() and int(mc_out[n - 1]["seq"]) == n - 1      # the tile's kernel is live
        out = {}
        eth = threading.Thread(target=lambda: out.setdefault("err", engine.verify_soa(
            golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)))
        eth.start()
        eth.join(timeout=60)
        assert not eth.is_alive()
        assert np.array_equal(out["err"], golden.expect)
        assert th.is_alive()
    finally:
        stop.value = 1
        th.join(timeout=30)
        tile.close()
    diag, _ = res["r"]
    assert diag["out_cnt"] == n


def test_tile_run_refuses_when_its_kernel_cannot_start():
    """A second tile created after a first tile's run took every wave slot:
    its kernel cannot start, so its run returns an error within ~2 s
    instead of spinning; the first run is unaffected."""
    import ctypes
    import threading
    import time
    from firedancer_amd import ed25519, tango
    n = 300
    pub, sig, msgs, (mc_in, dc, _, _, _) = _signed_feed(5151, n, 1024)
    mc_out = tango.mcache_new(1024)
    a = tango.VerifyTile(0, batch_max=1024, tcache_depth=0)          # the device's whole share
    stop = ctypes.c_int(0)
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("r", a.run(mc_in, dc, 0, mc_out, 0, 0, stop=stop)))
    th.start()
    b = None
    try:
        t0 = time.time()
        while int(mc_out[n - 1]["seq"]) != n - 1 and time.time() - t0 < 30:
            time.sleep(0.001)
        assert int(mc_out[n - 1]["seq"]) == n - 1
        b = tango.VerifyTile(0, batch_max=1024, tcache_depth=0, waves=1024)
        mc_out2 = tango.mcache_new(1024)
        t1 = time.perf_counter()
        try:
            d2, _ = b.run(mc_in, dc, 0, mc_out2, 0, n)
        except ed25519.EngineError:
            d2 = None
        # the run must not spin: it returns the error within ~2 s.  One box of
        # the pool ran the second kernel anyway (its scheduler time-sliced the
        # two queues: profiles/r06_gpu_tests_cannot_start_flake.txt): then the run
        # must have verified the whole feed like any other
        assert time.perf_counter() - t1 < 4.0
        if d2 is not None:
            assert d2["out_cnt"] == n and [int(mc_out2[o]["seq"]) for o in range(n)] == list(range(n))
        assert th.is_alive()
    finally:
        stop.value = 1
        th.join(timeout=30)
        if b is not None:
            b.close()                                # waits for its queued kernel, which exits at once
        a.close()
    diag, _ = res["r"]
    assert diag["out_cnt"] == n


def test_tile_trace_decomposes_latency():
    """fd_verify_amd_tile_set_trace: per published frag the cut wait, queue
    wait, service and publish wait; they sum to at most the frag's latency
    (the rest is the input wait), service is a chunk's GPU time (tens of
    us to a few ms), and latency chunks carry their flag."""
    from firedancer_amd import tango
    n = 3000
    pub, sig, msgs, (mc_in, dc, _, _, ts) = _signed_feed(6161, n, 4096)
    now = tango.tickcount()
    for s in range(n):                              # tsorig = now: latency from here
        mc_in[s]["tsorig"] = now
    mc_out = tango.mcache_new(4096)
    tile = tango.VerifyTile(0, batch_max=1024, tcache_depth=0, chunk_mode=tango.CHUNK_LATENCY)
    parts = np.zeros((n, 4), np.uint32)
    tile.set_trace(parts)
    try:
        diag, lat = tile.run(mc_in, dc, 0, mc_out, 0, n, lat_max=n)
    finally:
        tile.close()
    assert diag["out_cnt"] == n and lat.size == n
    svc = parts[:, 2] & 0x7FFFFFFF
    assert ((parts[:, 2] >> 31) == 1).all()          # every chunk a latency chunk
    assert (svc > 20_000).all() and (svc < 50_000_000).all()
    tot = parts[:, 0].astype(np.int64) + parts[:, 1] + svc + parts[:, 3]
    assert (tot <= lat.astype(np.int64) + 20_000).all()   # GPU clock mapping within 20 us
