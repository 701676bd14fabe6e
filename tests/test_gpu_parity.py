"""GPU parity: the HIP engine (through the C-ABI) vs the reference's verdicts.

Checkers, in order of authority:
  1. committed golden fixtures (tests/golden/), whose expected codes are the
     compiled reference's fd_ed25519_verify (src/ballet/ed25519/
     fd_ed25519_user.c:345-431) on the same bytes;
  2. seeded-stream digests pinned against the reference (same file);
  3. the CPU oracle (oracle/fd_ed25519_oracle.c) on fresh seeded inputs.

Bar: bit-exact verdict AND error code for every signature (integer work).
"""
import os

import numpy as np
import pytest

import _golden
import _oracle

pytestmark = pytest.mark.gpu


def _sign_stream(seed, count, szlo, szhi, mixed):
    from firedancer_amd import ed25519
    prv, blob, off, sz, fk, fp = _oracle.stream_inputs(seed, count, szlo, szhi, mixed)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    for i in np.nonzero(fk)[0]:
        byte, bit = divmod(int(fp[i]), 8)
        if fk[i] == 1:
            sig[i, byte] ^= 1 << bit
        elif fk[i] == 2:
            blob[off[i] + byte] ^= 1 << bit
        else:
            pub[i, byte] ^= 1 << bit
    return _golden.Batch(pub, sig, off, sz, blob)


def test_golden_vectors_soa(engine, golden):
    err = engine.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
    bad = np.nonzero(err != golden.expect)[0]
    detail = [(int(i), _golden.CLASSES[golden.cls[i]], int(golden.expect[i]), int(err[i])) for i in bad[:20]]
    assert bad.size == 0, "verdict mismatches (idx, class, expect, got): %s" % detail


def test_golden_vectors_every_class_present(golden):
    present = set(int(c) for c in golden.cls)
    for want in ("valid", "flip_sig", "flip_msg", "flip_pub", "s_window", "s_range", "malleate",
                 "offcurve_a", "offcurve_r", "small_order", "noncanon", "false_reject", "random",
                 "rfc8032", "mainnet", "zero_msg", "max_msg"):
        assert _golden.CLASSES.index(want) in present, want


def test_golden_vectors_pointer_array_api(engine, golden):
    n = len(golden)
    msgs = [golden.msg(i) for i in range(n)]
    err = engine.verify_batch(msgs, [bytes(golden.sig[i]) for i in range(n)], [bytes(golden.pub[i]) for i in range(n)])
    assert np.array_equal(err, golden.expect)


def test_dropin_fd_ed25519_verify(golden):
    """The reference's single-signature entry point, same codes."""
    from firedancer_amd import ed25519
    pick = list(range(0, len(golden), 37)) + list(np.nonzero(golden.cls == _golden.CLASSES.index("false_reject"))[0])
    for i in pick:
        got = ed25519.verify(golden.msg(i), bytes(golden.sig[i]), bytes(golden.pub[i]))
        assert got == int(golden.expect[i]), (i, _golden.CLASSES[golden.cls[i]], got, int(golden.expect[i]))


def test_small_engine_chunking(golden):
    """Batches larger than the engine capacity are split into double-buffered chunks."""
    from firedancer_amd import ed25519
    eng = ed25519.Engine(device=0, batch_max=100, blob_max=4096)
    try:
        err = eng.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
    finally:
        eng.close()
    assert np.array_equal(err, golden.expect)


@pytest.mark.parametrize("layout", ["permuted", "reversed", "sparse", "shared"])
@pytest.mark.parametrize("small", [False, True])
def test_soa_blob_layouts(engine, golden, layout, small):
    """verify_soa stages a chunk's message window as one block when it is
    dense (any order inside it) and gathers message by message otherwise;
    every layout must give the golden verdicts."""
    from firedancer_amd import ed25519
    n = len(golden)
    msgs = [golden.msg(i) for i in range(n)]
    rng = np.random.default_rng(5)
    if layout == "shared":   # duplicate messages share one copy in the blob
        uniq = {}
        parts, off, pos = [], np.zeros(n, np.uint32), 0
        for i, m in enumerate(msgs):
            if m not in uniq:
                uniq[m] = pos
                parts.append(m)
                pos += len(m)
            off[i] = uniq[m]
        blob = b"".join(parts)
    else:
        order = {"permuted": rng.permutation(n), "reversed": np.arange(n)[::-1], "sparse": np.arange(n)}[layout]
        gap = 3000 if layout == "sparse" else 0
        off, parts, pos = np.zeros(n, np.uint32), [], 0
        for j in order:
            off[j] = pos
            parts.append(msgs[j] + bytes(gap))
            pos += len(msgs[j]) + gap
        blob = b"".join(parts)
    blob = np.frombuffer(blob + b"\0", np.uint8)
    eng = ed25519.Engine(device=0, batch_max=100, blob_max=8192) if small else engine
    try:
        err = eng.verify_soa(golden.pub, golden.sig, off, golden.msg_sz, blob)
    finally:
        if small:
            eng.close()
    assert np.array_equal(err, golden.expect)


def test_empty_and_single(engine, golden):
    e0 = engine.verify_soa(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32),
                           np.zeros(0, np.uint32), np.zeros(1, np.uint8))
    assert e0.shape == (0,)
    for i in (0, len(golden) - 1):
        e1 = engine.verify_soa(golden.pub[i:i + 1], golden.sig[i:i + 1], np.zeros(1, np.uint32),
                               golden.msg_sz[i:i + 1], np.frombuffer(golden.msg(i) + b"\0", np.uint8))
        assert int(e1[0]) == int(golden.expect[i])


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_seeded_stream_digest(engine, idx):
    """Regenerate a stream pinned against the reference (65536 sigs) and
    compare the FNV-1a digest of the verdict array and the code histogram."""
    s = _golden.load_streams()[idx]
    b = _sign_stream(s["seed"], s["count"], s["szlo"], s["szhi"], s["mixed"])
    err = engine.verify_soa(b.pub, b.sig, b.msg_off, b.msg_sz, b.blob)
    hist = [int((err == -k).sum()) for k in range(4)]
    assert hist == s["codes"]
    assert _golden.fnv1a64(err) == s["fnv1a64"]


def test_random_mixed_vs_oracle(engine):
    """2^16 fresh mixed signatures (10 % bit flips), engine vs CPU oracle."""
    b = _sign_stream(777, 1 << 16, 0, 1232, True)
    err = engine.verify_soa(b.pub, b.sig, b.msg_off, b.msg_sz, b.blob)
    exp = _oracle.verify_batch(b)
    assert np.array_equal(err, exp), np.nonzero(err != exp)[0][:10]


def test_device_resident_path_and_stats():
    """fd_ed25519_amd_verify_dev on device buffers (the bench path), plus the
    work statistics against the oracle's instrumented counts."""
    from firedancer_amd import ed25519, hip
    b = _sign_stream(99, 4096, 200, 200, True)
    n = len(b)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in
         dict(pub=b.pub, sig=b.sig, off=b.msg_off, sz=b.msg_sz, blob=b.blob).items()}
    err = hip.DeviceBuffer(n)
    ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
    stats = hip.DeviceBuffer(4 * 3 * n)
    stream = hip.Stream()
    evs = [hip.Event() for _ in range(4)]
    ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr,
                          err.ptr, ws.ptr, stream.handle, evs)
    ed25519.work_stats_dev(n, ws.ptr, stats.ptr, stream.handle)
    stream.synchronize()
    assert all(evs[j].elapsed_ms(evs[j + 1]) > 0 for j in range(3))
    exp, st = _oracle.verify_batch(b, stats=True)
    assert np.array_equal(err.to_array(np.int8, n), exp)
    got = stats.to_array(np.uint32, 3 * n).reshape(3, n).T
    assert np.array_equal(got, st)


def test_large_batch_properties(engine):
    """2^18 valid 200-B signatures: every verdict must be 0 except the AVX
    limb-compare false rejects (rate ~1.6e-6), and every rejection must be
    confirmed by the oracle; resubmission is idempotent."""
    from firedancer_amd import ed25519
    n = 1 << 18
    rng = np.random.default_rng(2024)
    prv = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    blob = rng.integers(0, 256, n * 200 + 1, dtype=np.uint8)
    off = (np.arange(n, dtype=np.uint32) * 200).astype(np.uint32)
    sz = np.full(n, 200, np.uint32)
    pub, sig = ed25519.sign_batch(prv, blob, off, sz)
    err = engine.verify_soa(pub, sig, off, sz, blob)
    rej = np.nonzero(err != 0)[0]
    assert rej.size <= 8, rej.size
    for i in rej:
        assert _oracle.verify(bytes(blob[off[i]:off[i] + 200]), bytes(sig[i]), bytes(pub[i])) == int(err[i])
    err2 = engine.verify_soa(pub, sig, off, sz, blob)
    assert np.array_equal(err, err2)


def test_prep_digits_vs_python(golden):
    """k_prep output (the slide digits of h and s, and the top position) vs a
    pure-Python restatement with hashlib SHA-512, on the golden vectors that
    pass the s check."""
    import _slide
    from firedancer_amd import ed25519, hip
    sel = [i for i in range(len(golden)) if golden.expect[i] in (0, -3)][:300]
    b = _golden.Batch(golden.pub[sel], golden.sig[sel], None, golden.msg_sz[sel], None)
    msgs = [golden.msg(i) for i in sel]
    off = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint32)
    blob = np.frombuffer(b"".join(msgs) + b"\0" * 16, np.uint8)
    n = len(sel)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in
         dict(pub=b.pub, sig=b.sig, off=off, sz=b.msg_sz, blob=blob).items()}
    err = hip.DeviceBuffer(n)
    ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
    dig = hip.DeviceBuffer(512 * n)
    top = hip.DeviceBuffer(4 * n)
    stream = hip.Stream()
    ed25519.verify_dev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr, ws.ptr,
                       stream.handle)
    ed25519.debug_digits_dev(n, ws.ptr, dig.ptr, top.ptr, stream.handle)
    stream.synchronize()
    dg = dig.to_array(np.uint16, 256 * n).reshape(n, 256)
    tp = top.to_array(np.int32, n)
    for j in range(n):
        s = bytes(b.sig[j][32:])
        if s[31] == 0x10 and any(s[16:31]):
            continue                                   # decided by the s check, no digits
        h = _slide.h_scalar(b.sig[j], b.pub[j], msgs[j])
        ea = _slide.slide(h)
        eb = _slide.slide(int.from_bytes(s, "little"))
        ga = (dg[j] & 0xff).astype(np.uint8).view(np.int8).tolist()
        gb = (dg[j] >> 8).astype(np.uint8).view(np.int8).tolist()
        assert gb == eb, ("s digits", j)
        hv = sum(d << p for p, d in enumerate(ga))
        assert ga == ea, ("h digits", j, "gpu digits encode %x, want %x" % (hv, h))
        nz = [p for p in range(256) if ea[p] or eb[p]]
        assert tp[j] == (max(nz) if nz else -1)


@pytest.fixture(params=["k_dsm", "k_dsmp", "k_dsm4", "k_dsm8"])
def dsm_kernel(request):
    """Run a test once per double-scalar-mult kernel (throughput per-lane and
    pooled, 4-lane and 8-lane latency kernels), each forced for every batch
    size."""
    from firedancer_amd import ed25519
    ed25519.select_dsm_kernel(request.param)
    yield request.param
    ed25519.select_dsm_kernel("default")


def test_both_kernels_golden_and_mixed(engine, golden, dsm_kernel):
    """Golden fixtures and 2^15 fresh mixed signatures through each kernel."""
    err = engine.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
    assert np.array_equal(err, golden.expect), dsm_kernel
    b = _sign_stream(4321, 1 << 15, 0, 1232, True)
    err = engine.verify_soa(b.pub, b.sig, b.msg_off, b.msg_sz, b.blob)
    assert np.array_equal(err, _oracle.verify_batch(b)), dsm_kernel


def test_both_kernels_stats_and_false_rejects(dsm_kernel):
    """Work statistics (device path) and the limb-compare false rejects of
    the golden set through each kernel."""
    from firedancer_amd import ed25519, hip
    b = _sign_stream(98, 2048, 200, 200, True)
    n = len(b)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in
         dict(pub=b.pub, sig=b.sig, off=b.msg_off, sz=b.msg_sz, blob=b.blob).items()}
    err = hip.DeviceBuffer(n)
    ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
    stats = hip.DeviceBuffer(4 * 3 * n)
    stream = hip.Stream()
    ed25519.verify_dev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr, ws.ptr,
                       stream.handle)
    ed25519.work_stats_dev(n, ws.ptr, stats.ptr, stream.handle)
    stream.synchronize()
    exp, st = _oracle.verify_batch(b, stats=True)
    assert np.array_equal(err.to_array(np.int8, n), exp)
    assert np.array_equal(stats.to_array(np.uint32, 3 * n).reshape(3, n).T, st)


def test_config2_full_size_properties():
    """configs[1] at full size: 2^20 GPU-signed 200-B signatures through the
    device path.  Every signature is valid, so every rejection must be an
    AVX limb-compare false reject (rate ~1.6e-6) confirmed by the oracle;
    resubmission is idempotent."""
    from firedancer_amd import ed25519, hip, workload
    n = 1 << 20
    pub, sig, off, sz, blob = workload.sig_batch(n, 200, 20240)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
    err = hip.DeviceBuffer(n)
    ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
    st = hip.Stream()
    outs = []
    for _ in range(2):
        ed25519.verify_dev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr,
                           ws.ptr, st.handle)
        st.synchronize()
        outs.append(err.to_array(np.int8, n))
    assert np.array_equal(outs[0], outs[1])
    rej = np.nonzero(outs[0])[0]
    assert rej.size <= 12, rej.size
    for i in rej:
        assert _oracle.verify(bytes(blob[off[i]:off[i] + 200]), bytes(sig[i]), bytes(pub[i])) == int(outs[0][i]) == -3


def test_config2_full_size_mixed_vs_oracle():
    """configs[1]'s shape (2^20 x 200-B messages) with configs[2]'s 10 %
    corruption (one bit flipped in sig, message or pub), through the device
    path and its default kernel at this size (the pooled k_dsmp): every one
    of the 2^20 verdicts equals the CPU oracle's."""
    from firedancer_amd import ed25519, hip
    n = 1 << 20
    b = _sign_stream(20241, n, 200, 200, True)
    d = {k: hip.DeviceBuffer.from_array(v) for k, v in
         dict(pub=b.pub, sig=b.sig, off=b.msg_off, sz=b.msg_sz, blob=b.blob).items()}
    err = hip.DeviceBuffer(n)
    ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
    st = hip.Stream()
    ed25519.verify_dev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr,
                       ws.ptr, st.handle)
    st.synchronize()
    got = err.to_array(np.int8, n)
    exp = _oracle.verify_batch(b)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
    hist = [int((exp == -k).sum()) for k in range(4)]
    assert hist[0] > 0.85 * n and hist[2] > 0 and hist[3] > 0.05 * n, hist


def test_dropin_long_messages():
    """The reference verifies messages of any size; the drop-in entry point
    grows its staging (64 KB .. 1 MB messages, valid and corrupted)."""
    from firedancer_amd import ed25519
    rng = np.random.default_rng(12)
    for sz in (70000, 200001, 1 << 20):
        prv = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        msg = bytes(rng.integers(0, 256, sz, dtype=np.uint8))
        pub = ed25519.public_from_private(prv)
        sig = ed25519.sign(msg, pub, prv)
        assert ed25519.verify(msg, sig, pub) == 0 == _oracle.verify(msg, sig, pub)
        bad = bytearray(msg); bad[sz // 2] ^= 1
        assert ed25519.verify(bytes(bad), sig, pub) == _oracle.verify(bytes(bad), sig, pub) == -3


def test_pooled_kernel_ragged_batches(golden):
    """k_dsmp (pooled op classes) forced on ragged batch sizes: a single
    signature, partial waves, pools that never fill, sizes around 64 and the
    pool size (112), and the golden set; verdicts equal the reference's."""
    from firedancer_amd import ed25519
    ed25519.select_dsm_kernel("k_dsmp")
    eng = ed25519.Engine(device=0, batch_max=4096, blob_max=4096 * 1232)
    try:
        for n in (1, 2, 63, 64, 65, 111, 112, 113, 127, 129, 1000, len(golden)):
            n = min(n, len(golden))
            sel = np.arange(n)
            err = eng.verify_soa(golden.pub[sel], golden.sig[sel], golden.msg_off[sel], golden.msg_sz[sel],
                                 golden.blob)
            assert np.array_equal(err, golden.expect[sel]), n
    finally:
        eng.close()
        ed25519.select_dsm_kernel("default")
