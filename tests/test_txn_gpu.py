"""Transaction front end on the GPU (through the C-ABI, include/fd_txn_amd.h):
k_txn_parse vs the compiled reference parser's fixture, and the
multi-signer batch verdicts of fd_ed25519_amd_verify_txns vs the CPU oracle.
Bar: bit-exact footprints, descriptor bytes and codes.
"""
import numpy as np
import pytest

import _oracle
import _txn

pytestmark = pytest.mark.gpu

STRIDE = 3584   # >= FD_TXN_MAX_SZ, even


def _gpu_parse(payloads, want_desc=True):
    from firedancer_amd import ed25519, hip
    blob, off, sz = _txn.pack(payloads)
    n = len(payloads)
    d_blob, d_off, d_sz = (hip.DeviceBuffer.from_array(a) for a in (blob, off, sz))
    d_fp = hip.DeviceBuffer(4 * max(n, 1))
    d_out = hip.DeviceBuffer(STRIDE * max(n, 1)) if want_desc else None
    stream = hip.Stream()
    ed25519.txn_parse_dev(n, d_blob.ptr, d_off.ptr, d_sz.ptr, d_fp.ptr, d_out.ptr if want_desc else None,
                          STRIDE if want_desc else 0, stream.handle)
    stream.synchronize()
    fp = d_fp.to_array(np.uint32, n)
    out = d_out.to_array(np.uint8, STRIDE * n).reshape(n, STRIDE) if want_desc else None
    return fp, out


def test_gpu_parse_reference_mutations():
    """All mutations of the reference's three fixture transactions: the
    GPU footprint equals the reference's for every one, and the digest of
    the accepted descriptors equals the reference's."""
    for f in _txn.load_fixtures():
        muts = _txn.mutation_list(f.payload)
        fp, out = _gpu_parse(muts)
        bad = np.nonzero(fp != f.footprint)[0]
        assert bad.size == 0, [(int(i), int(fp[i]), int(f.footprint[i]), int(f.line[i])) for i in bad[:10]]
        d = _txn.FNV0
        for k in np.nonzero(fp)[0]:
            d = _txn.fnv(d, out[k, :fp[k]].tobytes())
        assert d == f.digest


def test_gpu_parse_synthetic_fuzz():
    """Random byte edits and truncations of synthetic legacy/v0 transactions:
    GPU footprint and descriptor bytes vs the oracle."""
    rng = np.random.default_rng(5)
    base, _ = _txn.build_txns(21, 40, nsig_hi=4, msg_hi=400)
    pays = []
    for p in base:
        pays.append(p)
        for _ in range(40):
            q = bytearray(p)
            for _ in range(int(rng.integers(1, 3))):
                q[int(rng.integers(0, len(q)))] = int(rng.integers(0, 256))
            if rng.random() < 0.2:
                q = q[:int(rng.integers(0, len(q) + 1))]
            pays.append(bytes(q))
    fp, out = _gpu_parse(pays)
    for k, p in enumerate(pays):
        efp, eout, _ = _oracle.txn_parse(p)
        assert int(fp[k]) == efp, k
        if efp:
            assert out[k, :efp].tobytes() == eout, k


def test_gpu_parse_edge_sizes():
    """Empty payload, a single byte, and a payload above USHORT_MAX."""
    fp, _ = _gpu_parse([b"", b"\x01", b"\x01" + b"\0" * 70000], want_desc=False)
    assert fp.tolist() == [0, 0, 0]


def test_verify_txns_reference_fixtures(engine):
    fx = _txn.load_fixtures()
    blob, off, sz = _txn.pack([f.payload for f in fx])
    terr, base, serr = engine.verify_txns(blob, off, sz, want_sigs=True)
    assert terr.tolist() == [0, 0, 0]
    assert base.tolist() == [0, 4, 5, 6] and serr.tolist() == [0] * 6


def _mixed_batch(seed, count):
    rng = np.random.default_rng(seed)
    pays, nsig = _txn.build_txns(seed, count)
    pays = [bytearray(p) for p in pays]
    for t in range(count):
        r = rng.random()
        n = int(nsig[t])
        m = 1 + 64 * n
        if r < 0.08:     # one signature bit
            pays[t][1 + int(rng.integers(0, 64 * n))] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.14:   # a signer's public key (inside the message)
            pays[t][m + (1 if pays[t][m] & 0x80 else 0) + 4 + int(rng.integers(0, 32 * n))] ^= 0x04
        elif r < 0.18:   # the header: parse failure
            pays[t][m + (1 if pays[t][m] & 0x80 else 0)] ^= 0x40
        elif r < 0.20:   # truncated
            pays[t] = pays[t][:int(rng.integers(0, len(pays[t])))]
    return [bytes(p) for p in pays]


def test_verify_txns_mixed_vs_oracle(engine):
    """600 synthetic multi-signer transactions (1..12 signers, 64..1232-B
    messages, legacy and v0) with corruptions: per-transaction verdicts,
    signature numbering and per-signature codes vs the oracle."""
    pays = _mixed_batch(31, 600)
    blob, off, sz = _txn.pack(pays)
    terr, base, serr = engine.verify_txns(blob, off, sz, want_sigs=True)
    eterr, ebase, eserr = _oracle.txn_verify_batch(blob, off, sz)
    assert np.array_equal(base, ebase)
    assert np.array_equal(serr, eserr), np.nonzero(serr != eserr)[0][:10]
    assert np.array_equal(terr, eterr)
    assert set(np.unique(terr).tolist()) >= {0, -4}


def test_verify_txns_chunked_small_engine():
    """An engine smaller than the batch: transactions are split into
    double-buffered chunks by count, payload bytes and signature slots."""
    from firedancer_amd import ed25519
    pays = _mixed_batch(32, 150)
    blob, off, sz = _txn.pack(pays)
    eng = ed25519.Engine(device=0, batch_max=40, blob_max=6000)
    try:
        terr, base, serr = eng.verify_txns(blob, off, sz, want_sigs=True)
    finally:
        eng.close()
    eterr, ebase, eserr = _oracle.txn_verify_batch(blob, off, sz)
    assert np.array_equal(terr, eterr) and np.array_equal(serr, eserr)


def test_verify_txns_empty_and_limits(engine):
    from firedancer_amd import ed25519
    t = engine.verify_txns(np.zeros(4, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    assert t.shape == (0,)
    with pytest.raises(ed25519.EngineError):
        engine.verify_txns(np.zeros(1300, np.uint8), np.zeros(1, np.uint32), np.full(1, 1233, np.uint32))


def test_synth_txn_workload_and_device_path(engine):
    """Config-4 workload (GPU-signed multi-signer transactions, 64..1232-B
    messages): every transaction parses and verifies; the device-resident
    entry point agrees with the host-staged one and with the oracle, also
    after corruptions."""
    from firedancer_amd import hip, workload
    payload, toff, tsz, tbase = workload.txn_batch(3000, 77)
    assert (tsz <= 1232).all() and int(tbase[-1]) > 2500
    rng = np.random.default_rng(1)
    bad = rng.choice(toff.size, 40, replace=False)
    for t in bad[:20]:
        payload[toff[t] + 1 + int(rng.integers(0, 64))] ^= 0x20         # a signature byte
    for t in bad[20:]:
        payload[toff[t] + tsz[t] - 1] ^= 0x01                           # last byte (data or LUT count)
    dev = workload.TxnDevice(payload, toff, tsz, tbase)
    st = hip.Stream()
    dev.run(st.handle)
    st.synchronize()
    terr, serr = dev.verdicts()
    eterr, ebase, eserr = _oracle.txn_verify_batch(payload, toff, tsz)
    assert np.array_equal(ebase, tbase)
    assert np.array_equal(terr, eterr) and np.array_equal(serr, eserr)
    h_terr, h_base, h_serr = engine.verify_txns(payload, toff, tsz, want_sigs=True)
    assert np.array_equal(h_terr, terr) and np.array_equal(h_serr, serr)
    ok = np.setdiff1d(np.arange(toff.size), bad)
    assert (terr[ok] == 0).all() and (terr[bad] != 0).all()


def test_config4_shard_full_size_properties():
    """configs[3] at the size of one GPU's shard of 2^24 signatures over 2
    GPUs: 2^23 signatures in multi-signer transactions (64..1232-B
    messages).  Every signature is valid: each rejected transaction must
    hold a limb-compare false reject, confirmed by the oracle."""
    from firedancer_amd import hip, workload
    payload, toff, tsz, tbase = workload.txn_batch(1 << 23, 424242)
    dev = workload.TxnDevice(payload, toff, tsz, tbase)
    st = hip.Stream()
    dev.run(st.handle)
    st.synchronize()
    terr, serr = dev.verdicts()
    assert dev.slot_cnt >= (1 << 23) * 0.99
    bad = np.nonzero(terr)[0]
    assert bad.size <= 40, bad.size
    if bad.size:
        eterr, _, _ = _oracle.txn_verify_batch(payload, toff[bad], tsz[bad])
        assert np.array_equal(eterr, terr[bad]) and (eterr == -3).all()
    assert (serr != 0).sum() == bad.size
