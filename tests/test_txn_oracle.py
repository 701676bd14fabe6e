"""Transaction front end, CPU side: the fd_txn_parse restatement
(oracle/fd_txn_oracle.c) against the committed fixture of the compiled
reference parser, the reference test's own fixture assertions
(src/ballet/txn/test_txn_parse.c:17-121), and the multi-signer verdict
rule on the reference's mainnet transactions and synthetic transactions.
"""
import struct

import numpy as np
import pytest

import _oracle
import _txn


@pytest.fixture(scope="module")
def fixtures():
    return _txn.load_fixtures()


def test_oracle_parse_matches_reference_on_mutations(fixtures):
    """Every mutation of the three reference fixtures: footprint and failing
    reference line equal, digest of the accepted descriptors equal."""
    for f in fixtures:
        muts = _txn.mutation_list(f.payload)
        assert len(muts) == f.footprint.size
        d = _txn.FNV0
        for k, m in enumerate(muts):
            fp, out, line = _oracle.txn_parse(m)
            assert (fp, line) == (int(f.footprint[k]), int(f.line[k])), k
            if fp:
                d = _txn.fnv(d, out)
        assert d == f.digest


def _desc(out):
    hdr = struct.unpack_from("<BBHHBBHHHBBBBH", out, 0)
    keys = ("ver nsig sig_off msg_off ro_s ro_u nacct acct_off bh_off nlut adtl_w adtl pad ninstr").split()
    d = dict(zip(keys, hdr))
    d["instr"] = [struct.unpack_from("<BBHHHH", out, 20 + 10 * j) for j in range(d["ninstr"])]
    d["lut"] = [struct.unpack_from("<HBBHH", out, 20 + 10 * d["ninstr"] + 8 * j) for j in range(d["nlut"])]
    return d


def test_reference_fixture_assertions(fixtures):
    """The values asserted by test_txn_parse.c txn1/txn2_correctness and
    the FD_TXN_MAX_SZ footprint of transaction3."""
    t1, t2, t3 = (f.payload for f in fixtures)
    fp, out, _ = _oracle.txn_parse(t1)
    d = _desc(out)
    assert fp and d["ver"] == 0xFF and d["nsig"] == 4
    assert [t1[d["sig_off"] + 64 * j] for j in range(4)] == [97, 189, 11, 108]
    assert d["msg_off"] == d["sig_off"] + 64 * 4
    assert (d["ro_s"], d["ro_u"], d["nacct"]) == (1, 11, 23)
    assert [t1[d["acct_off"] + 32 * j] for j in range(23)] == [220, 255, 85, 89, 201, 170, 194, 48, 228, 123, 151,
                                                               133, 6, 6, 203, 6, 11, 6, 0, 140, 3, 5, 168]
    assert t1[d["bh_off"]] == 155 and (d["nlut"], d["adtl_w"], d["adtl"]) == (0, 0, 0)
    assert d["ninstr"] == 7
    ix = d["instr"]
    assert ix[0][0] == 20 and ix[0][2] == 0 and ix[0][3] == 5 and t1[ix[0][5]:ix[0][5] + 5] == b"\x00\xE0\x93\x04\x00"
    assert ix[1][0] == 18 and ix[1][2] == 2 and ix[1][3] == 12 and t1[ix[1][4]] == 0 and t1[ix[1][5]] == 2
    assert ix[6][0] == 22 and ix[6][2] == 21 and ix[6][3] == 12 and t1[ix[6][4]] == 14 and t1[ix[6][5]] == 211

    fp, out, _ = _oracle.txn_parse(t2)
    d = _desc(out)
    assert fp and d["ver"] == 0 and d["nsig"] == 1 and t2[d["sig_off"]] == 184
    assert (d["ro_s"], d["ro_u"], d["nacct"]) == (0, 2, 6)
    assert [t2[d["acct_off"] + 32 * j] for j in range(6)] == [216, 176, 9, 213, 3, 4]
    assert t2[d["bh_off"]] == 148 and (d["nlut"], d["adtl_w"], d["adtl"]) == (3, 12, 21)
    assert d["ninstr"] == 2 and d["instr"][1][0] == 5 and d["instr"][1][2] == 39 and d["instr"][1][3] == 38
    l0 = d["lut"][0]
    assert t2[l0[0]] == 54 and l0[1:3] == (4, 4) and t2[l0[3]:l0[3] + 4] == bytes([142, 141, 143, 144])
    assert t2[l0[4] + 1] == 117
    assert [t2[x[0]] for x in d["lut"]] == [54, 34, 212]

    fp, _, _ = _oracle.txn_parse(t3)
    assert fp == 3570


def test_reference_mainnet_transactions_verify(fixtures):
    """All six signatures of the reference's fixtures are valid mainnet /
    flood-pcap signatures: the multi-signer rule accepts every transaction."""
    blob, off, sz = _txn.pack([f.payload for f in fixtures])
    terr, base, serr = _oracle.txn_verify_batch(blob, off, sz)
    assert terr.tolist() == [0, 0, 0]
    assert base.tolist() == [0, 4, 5, 6] and serr.tolist() == [0] * 6


def test_synthetic_multisigner_rule():
    """Synthetic legacy/v0 transactions with 1..12 signers parse and verify;
    corruptions give the per-signature code of the first bad signature, a
    header corruption gives FD_TXN_AMD_ERR_PARSE for the transaction and its
    reserved slots."""
    pays, nsig = _txn.build_txns(11, 60)
    pays = [bytearray(p) for p in pays]
    for p in pays:
        assert _oracle.txn_parse(bytes(p))[0] > 0
    # txn 0: flip a bit of its last signature's R; txn 1: change the message;
    # txn 2: break the header (signature count vs message header)
    n0 = nsig[0]
    pays[0][1 + 64 * (n0 - 1) + 5] ^= 0x10
    m1 = 1 + 64 * nsig[1]
    pays[1][m1 + (1 if pays[1][m1] & 0x80 else 0) + 4 + 32 * nsig[1] + 5] ^= 0x01   # a non-signer address
    pays[2][1 + 64 * nsig[2] + (1 if pays[2][1 + 64 * nsig[2]] & 0x80 else 0)] ^= 0x40
    blob, off, sz = _txn.pack([bytes(p) for p in pays])
    terr, base, serr = _oracle.txn_verify_batch(blob, off, sz)
    assert terr[3:].tolist() == [0] * 57
    assert terr[0] in (-1, -2, -3) and serr[base[0]:base[1]].tolist()[:-1] == [0] * (n0 - 1)
    assert terr[1] == -3 and all(e == -3 for e in serr[base[1]:base[2]])
    assert terr[2] == -4 and all(e == -4 for e in serr[base[2]:base[3]])
    assert base[-1] == nsig.sum()


def test_oracle_multisigner_rule_matches_compiled_reference():
    """oracle/ref_batch.c's ref_txn_verify_batch (the reference's own
    fd_txn_parse + fd_ed25519_verify, the CPU baseline and re-check of
    bench.py's transaction workload) gives the oracle's per-transaction
    verdicts on corrupted synthetic transactions."""
    import ctypes
    import os
    so = os.path.join(os.path.dirname(_oracle.REF_SO), "libfdref_batch.so")
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(12)
    pays, nsig = _txn.build_txns(12, 120)
    pays = [bytearray(p) for p in pays]
    for t in rng.choice(len(pays), 40, replace=False):
        pays[t][int(rng.integers(0, len(pays[t])))] ^= 1 << int(rng.integers(0, 8))
    blob, off, sz = _txn.pack([bytes(p) for p in pays])
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.ref_txn_verify_batch.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int]
    err = np.zeros(len(pays), np.int8)
    L.ref_txn_verify_batch(len(pays), blob.ctypes.data, off.ctypes.data, sz.ctypes.data, err.ctypes.data, 4)
    terr, _, _ = _oracle.txn_verify_batch(blob, off, sz)
    assert np.array_equal(err, terr)
    assert (err != 0).sum() >= 20
