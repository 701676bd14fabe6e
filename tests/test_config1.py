"""BASELINE configs[0] (SURVEY.md s8 d, "Config 1"): the reference's CPU
fd_ed25519_verify over 2^16 keypairs, 128-byte messages, all valid.

The workload is fixed by the survey: 32-byte secrets and the messages drawn
from splitmix64 seeded with 1234.  Expected verdicts: all 0 except the AVX
limb-compare false rejects (rate ~1.6e-6, so P(>=1) ~ 10 %),
each of which the compiled reference (oracle/_ref) must confirm when it is
present.  The CPU test is the plumbing run the config names; the GPU test
sends the same batch through the C-ABI engine and diffs it against the
oracle verdict for verdict.
"""
import numpy as np
import pytest

import _oracle

N = 1 << 16
MSG = 128


def splitmix64(seed, count):
    """splitmix64 stream (Steele et al.), vectorised: word k is the mix of
    seed + (k+1) * 0x9E3779B97F4A7C15."""
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + np.arange(1, count + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def test_splitmix64_known_answer():
    # first outputs of splitmix64 seeded with 0 (the published reference stream)
    got = splitmix64(0, 3)
    assert [int(v) for v in got] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


class _Batch:
    def __len__(self):
        return len(self.msg_sz)


@pytest.fixture(scope="module")
def config1():
    from firedancer_amd import ed25519
    words = splitmix64(1234, N * 4 + N * (MSG // 8))
    b = _Batch()
    prv = words[:N * 4].view(np.uint8).reshape(N, 32)
    b.blob = np.concatenate([words[N * 4:].view(np.uint8), np.zeros(1, np.uint8)])
    b.msg_off = (np.arange(N, dtype=np.uint32) * MSG).astype(np.uint32)
    b.msg_sz = np.full(N, MSG, np.uint32)
    b.pub, b.sig = ed25519.sign_batch(prv, b.blob, b.msg_off, b.msg_sz)
    return b


def test_config1_cpu_plumbing(config1):
    err = _oracle.verify_batch(config1)
    rej = np.nonzero(err != 0)[0]
    assert rej.size <= 3, rej.size
    assert (err[rej] == -3).all()
    if _oracle.ref() is not None:   # the reference compiled from its own sources: every verdict
        for i in range(N):
            m = bytes(config1.blob[config1.msg_off[i]:config1.msg_off[i] + MSG])
            assert _oracle.ref_verify(m, bytes(config1.sig[i]), bytes(config1.pub[i])) == int(err[i]), i


@pytest.mark.gpu
def test_config1_gpu_vs_oracle(engine, config1):
    err = engine.verify_soa(config1.pub, config1.sig, config1.msg_off, config1.msg_sz, config1.blob)
    exp = _oracle.verify_batch(config1)
    assert np.array_equal(err, exp), np.nonzero(err != exp)[0][:10]
