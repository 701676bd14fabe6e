"""CPU tests of the checker itself: the clean-room oracle
(oracle/fd_ed25519_oracle.c) must reproduce the reference's verdicts on
every committed golden vector, its SHA-512 must equal hashlib's, its
reduction mod L must equal Python's, and seeded streams regenerated with the
product's host signer must hash to the digests pinned against the compiled
reference.  When oracle/_ref (the reference compiled from its own sources)
exists, it is checked against the fixtures too.
"""
import hashlib
import os
import random

import numpy as np
import pytest

import _golden
import _oracle
import _slide

L = _slide.L


def test_oracle_matches_reference_on_every_golden_vector(golden):
    got = _oracle.verify_batch(golden, nthread=8)
    bad = np.nonzero(got != golden.expect)[0]
    assert bad.size == 0, [(int(i), _golden.CLASSES[golden.cls[i]], int(golden.expect[i]), int(got[i])) for i in bad[:10]]


def test_golden_class_coverage(golden):
    for k, name in enumerate(_golden.CLASSES):
        assert (golden.cls == k).sum() > 0, name
    # every error code of the reference appears
    assert set(np.unique(golden.expect).tolist()) == {0, -1, -2, -3}
    # the AVX limb-compare false rejects are valid signatures rejected with -3
    fr = golden.cls == _golden.CLASSES.index("false_reject")
    assert fr.sum() >= 4 and (golden.expect[fr] == -3).all()
    # the reference's s-window bug (user.c:379) accepts every such vector
    sw = golden.cls == _golden.CLASSES.index("s_window")
    assert (golden.expect[sw] == 0).all()


def test_compiled_reference_matches_fixtures(golden):
    if _oracle.ref() is None:
        pytest.skip("oracle/_ref not built (no /root/reference on this host)")
    for i in range(0, len(golden), 3):
        assert _oracle.ref_verify(golden.msg(i), golden.sig[i], golden.pub[i]) == int(golden.expect[i])


def test_oracle_sha512_vs_hashlib():
    rng = random.Random(5)
    for n in list(range(0, 300)) + [1000, 1232, 1296, 4096]:
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert _oracle.sha512(d) == hashlib.sha512(d).digest(), n


def test_oracle_sc_reduce_vs_python():
    rng = random.Random(6)
    vals = [0, 1, L - 1, L, L + 1, 2 * L, 2**512 - 1, 2**252, 2**253 - 1]
    vals += [rng.getrandbits(512) for _ in range(2000)]
    for v in vals:
        out = _oracle.sc_reduce(v.to_bytes(64, "little"))
        assert int.from_bytes(out, "little") == v % L


def test_host_signer_rfc8032(golden):
    from firedancer_amd import ed25519
    secs = ["9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
            "4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
            "c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7"]
    idx = np.nonzero(golden.cls == _golden.CLASSES.index("rfc8032"))[0]
    assert len(idx) == 3
    for k, i in enumerate(idx):
        prv = bytes.fromhex(secs[k])
        pub = ed25519.public_from_private(prv)
        assert pub == bytes(golden.pub[i])
        assert ed25519.sign(golden.msg(i), pub, prv) == bytes(golden.sig[i])


def test_stream_regeneration_digest():
    """Stream 2 of tests/golden/ed25519_streams.jsonl (32768 signatures,
    64..1232-B messages, 10 % bit flips), regenerated with the product's host
    signer and checked by the oracle against the reference-pinned digest."""
    from firedancer_amd import ed25519
    s = _golden.load_streams()[2]
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(s["seed"], s["count"], s["szlo"], s["szhi"], s["mixed"])
    pub, sig = ed25519.sign_batch(prv, blob, off, sz, nthread=8)
    for i in np.nonzero(fk)[0]:
        byte, bit = divmod(int(fp[i]), 8)
        tgt = sig[i] if fk[i] == 1 else (blob[off[i]:] if fk[i] == 2 else pub[i])
        tgt[byte] ^= 1 << bit
    err = _oracle.verify_batch(_golden.Batch(pub, sig, off, sz, blob), nthread=8)
    assert [int((err == -k).sum()) for k in range(4)] == s["codes"]
    assert _golden.fnv1a64(err) == s["fnv1a64"]


def test_slide_restatement_properties():
    """The pure-Python slide used by the GPU digit test: digits are odd and in
    [-15, 15] and recombine to the scalar (value-preserving recoding)."""
    rng = random.Random(7)
    for _ in range(300):
        a = rng.randrange(L)
        r = _slide.slide(a)
        assert sum(d << i for i, d in enumerate(r)) == a
        assert all(d == 0 or (d % 2 == 1 and -15 <= d <= 15) for d in r)


def test_golden_fixtures_regenerate_identically():
    """Provenance: the committed fixtures are what the generators, linked
    against the compiled reference, write today (tests/golden/README.md)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not (os.path.isdir("/root/reference/src") and os.path.exists(os.path.join(root, "oracle", "_ref", "gen_golden"))):
        pytest.skip("needs /root/reference and oracle/_ref (build container)")
    r = subprocess.run([os.path.join(root, "tools", "regen_golden.sh")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("identical to the committed fixture") == 3
