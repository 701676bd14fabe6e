"""Multi-device paths on the GPU (SURVEY.md s8 e: contiguous shards, no
collective).  On the single-GPU test box the native multi-device engine is
exercised with the same device listed twice (two engines, two host
threads, one GPU), and the one-process-per-GPU path with two ranks mapped
onto device 0 (FD_AMD_DEVICE_MAP=mod); both must give exactly the
single-engine / oracle verdicts."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import _golden
import _oracle
import _txn

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_multi_engine_soa_equals_single_and_oracle(engine, golden):
    from firedancer_amd import ed25519
    from test_gpu_parity import _sign_stream
    m = ed25519.MultiEngine([0, 0], batch_max=1 << 14, blob_max=(1 << 14) * 1232)
    try:
        assert m.ndev == 2
        assert np.array_equal(m.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob),
                              golden.expect)
        b = _sign_stream(2024, 1 << 16, 0, 1232, True)
        got = m.verify_soa(b.pub, b.sig, b.msg_off, b.msg_sz, b.blob)
        assert np.array_equal(got, engine.verify_soa(b.pub, b.sig, b.msg_off, b.msg_sz, b.blob))
        assert np.array_equal(got, _oracle.verify_batch(b))
        # uneven and degenerate shards
        for n in (0, 1, 7):
            e = m.verify_soa(golden.pub[:n], golden.sig[:n], golden.msg_off[:n], golden.msg_sz[:n], golden.blob)
            assert np.array_equal(e, golden.expect[:n])
    finally:
        m.close()


def test_multi_engine_txns_equal_oracle():
    from firedancer_amd import ed25519
    from test_txn_gpu import _mixed_batch
    pays = _mixed_batch(77, 700)
    blob, off, sz = _txn.pack(pays)
    m = ed25519.MultiEngine([0, 0, 0], batch_max=1 << 12, blob_max=(1 << 12) * 1232)
    try:
        terr, base, serr = m.verify_txns(blob, off, sz, want_sigs=True)
        assert m.verify_txns(blob, off[:0], sz[:0]).shape == (0,)
    finally:
        m.close()
    eterr, ebase, eserr = _oracle.txn_verify_batch(blob, off, sz)
    assert np.array_equal(base, ebase) and np.array_equal(serr, eserr) and np.array_equal(terr, eterr)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_run_the_engine_on_their_shards(golden):
    """bench.py's N-GPU shape on one GPU: two processes (rank -> device
    local % count), gloo for control only, each rank verifies its
    contiguous shard of the golden vectors with the engine; the union of
    the shards equals the reference's expected codes."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FD_AMD_DEVICE_MAP="mod")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_rank_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=110)
            assert p.returncode == 0, e[-2000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    outs.sort(key=lambda d: d["rank"])
    assert [d["lo"] for d in outs] == [0, outs[0]["hi"]] and outs[1]["hi"] == len(golden)
    allerr = np.array(outs[0]["err"] + outs[1]["err"], np.int8)
    assert np.array_equal(allerr, golden.expect)
    assert outs[0]["elapsed_max"] == outs[1]["elapsed_max"]
