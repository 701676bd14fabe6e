"""GPU keygen + sign (fd_ed25519_amd_sign_dev, k_sign): byte-identical to
the host signer, which test_oracle_golden pins to RFC 8032 s7.1 and to the
reference's own signer (fd_ed25519_user.c:279-343) through the golden
fixtures; and every GPU signature verifies."""
import numpy as np
import pytest

import _golden

pytestmark = pytest.mark.gpu

RFC_SECRETS = ["9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
               "4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
               "c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7"]


def test_gpu_signer_rfc8032(golden):
    from firedancer_amd import ed25519
    idx = np.nonzero(golden.cls == _golden.CLASSES.index("rfc8032"))[0]
    prv = np.frombuffer(b"".join(bytes.fromhex(s) for s in RFC_SECRETS), np.uint8).reshape(3, 32)
    msgs = [golden.msg(i) for i in idx]
    off = np.array([0, len(msgs[0]), len(msgs[0]) + len(msgs[1])], np.uint32)
    sz = np.array([len(m) for m in msgs], np.uint32)
    blob = np.frombuffer(b"".join(msgs) + b"\0" * 8, np.uint8)
    pub, sig = ed25519.sign_batch_gpu(prv, blob, off, sz)
    for k, i in enumerate(idx):
        assert bytes(pub[k]) == bytes(golden.pub[i])
        assert bytes(sig[k]) == bytes(golden.sig[i])


@pytest.mark.parametrize("seed,n,szhi", [(1, 4096, 1232), (2, 20000, 300)])
def test_gpu_signer_matches_host_signer(seed, n, szhi):
    from firedancer_amd import ed25519
    rng = np.random.default_rng(seed)
    prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    prv[:16] = 0xff                       # edge seeds
    prv[16:32] = 0x00
    sz = rng.integers(0, szhi + 1, n).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint32)
    blob = rng.integers(0, 256, int(sz.sum()) + 8, dtype=np.uint8)
    hp, hs = ed25519.sign_batch(prv, blob, off, sz)
    gp, gs = ed25519.sign_batch_gpu(prv, blob, off, sz)
    bad = np.nonzero((hp != gp).any(1) | (hs != gs).any(1))[0]
    assert bad.size == 0, bad[:10]


def test_gpu_signed_batch_verifies(engine):
    from firedancer_amd import ed25519
    n = 8192
    rng = np.random.default_rng(9)
    prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    off = (np.arange(n) * 200).astype(np.uint32)
    sz = np.full(n, 200, np.uint32)
    blob = rng.integers(0, 256, n * 200 + 1, dtype=np.uint8)
    pub, sig = ed25519.sign_batch_gpu(prv, blob, off, sz)
    err = engine.verify_soa(pub, sig, off, sz, blob)
    assert (err == 0).sum() >= n - 1           # an AVX limb false reject has probability ~1.6e-6
