"""Batch-engine API contracts on the GPU (include/fd_ed25519_amd.h,
fd_txn_amd.h): error paths leave nothing in flight, transactions that can
never be staged are refused instead of spinning, a device-side slot table
that does not match a transaction fails closed, and the zero-copy
(registered caller memory) batch path gives the same verdicts as the staged
one."""
import numpy as np
import pytest

import _golden
import _oracle
import _txn

pytestmark = pytest.mark.gpu


def test_oversized_message_after_first_chunk_is_refused_before_launch(golden):
    """A message larger than blob_max in a later chunk: the call fails with
    nothing launched, and the engine's next call (into a different output
    array) is exact -- no chunk of the failed call is left to write into
    the freed output array."""
    from firedancer_amd import ed25519
    eng = ed25519.Engine(device=0, batch_max=100, blob_max=4096)
    try:
        n = 300
        pub, sig = golden.pub[:n].copy(), golden.sig[:n].copy()
        off, sz = golden.msg_off[:n].copy(), golden.msg_sz[:n].copy()
        blob = np.concatenate([golden.blob, np.zeros(5000, np.uint8)])
        off[250], sz[250] = golden.blob.size, 5000
        with pytest.raises(ed25519.EngineError):
            eng.verify_soa(pub, sig, off, sz, blob)
        with pytest.raises(ed25519.EngineError):
            eng.verify_batch([bytes(5000)] + [golden.msg(i) for i in range(1, 150)],
                             [bytes(golden.sig[i]) for i in range(150)], [bytes(golden.pub[i]) for i in range(150)])
        err = eng.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
        assert np.array_equal(err, golden.expect)
    finally:
        eng.close()


def test_verify_txns_refuses_a_transaction_larger_than_batch_max():
    """batch_max 8 and a 12-signer transaction: ERR_INVAL up front (it used
    to loop forever launching empty chunks); smaller ones still verify."""
    from firedancer_amd import ed25519
    big, _ = _txn.build_txns(3, 1, nsig_lo=12, nsig_hi=12, msg_hi=600)
    small, _ = _txn.build_txns(4, 20, nsig_lo=1, nsig_hi=8, msg_hi=600)
    eng = ed25519.Engine(device=0, batch_max=8, blob_max=1 << 16)
    try:
        blob, off, sz = _txn.pack(small + big)
        with pytest.raises(ed25519.EngineError):
            eng.verify_txns(blob, off, sz)
        blob, off, sz = _txn.pack(small)
        assert eng.verify_txns(blob, off, sz).tolist() == [0] * 20
    finally:
        eng.close()


def test_verify_txns_dev_fails_closed_on_short_slot_table():
    """Device API: a tbase that reserves fewer slots than a transaction's
    signature count rejects that transaction (-4) instead of verifying a
    subset of its signatures; the others are unaffected."""
    from firedancer_amd import hip, workload
    payload, toff, tsz, tbase = workload.txn_batch(200, 91)
    assert tbase[1] - tbase[0] >= 1
    short = tbase.astype(np.int64)
    short[1:] -= 1
    dev = workload.TxnDevice(payload, toff, tsz, short.astype(np.uint32))
    st = hip.Stream()
    dev.run(st.handle)
    st.synchronize()
    terr, _ = dev.verdicts()
    eterr, _, _ = _oracle.txn_verify_batch(payload, toff, tsz)
    assert int(terr[0]) == -4
    assert np.array_equal(terr[1:], eterr[1:])


def _Registered(*arrays):
    from firedancer_amd import ed25519
    return ed25519.RegisteredPlanes(*arrays)


def test_registered_batches_equal_staged(engine, golden):
    """fd_ed25519_amd_verify_soa_registered on the golden vectors, on 2^16
    fresh mixed signatures (vs the oracle) and on a sparse layout that
    takes the gather fallback; unregistered planes are refused."""
    from firedancer_amd import ed25519
    r = _Registered(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
    try:
        err = engine.verify_soa_registered(r[0], r[1], r[2], r[3], r[4])
        assert np.array_equal(err, golden.expect)
    finally:
        r.close()
    from test_gpu_parity import _sign_stream
    b = _sign_stream(4711, 1 << 16, 0, 1232, True)
    small = ed25519.Engine(device=0, batch_max=1 << 13, blob_max=(1 << 13) * 1232)
    r = _Registered(b.pub, b.sig, b.msg_off, b.msg_sz, b.blob)
    try:
        err = small.verify_soa_registered(r[0], r[1], r[2], r[3], r[4])   # 8 chunks, 2 in flight
        assert np.array_equal(err, _oracle.verify_batch(b))
    finally:
        r.close()
        small.close()
    # sparse: 3000-byte gaps between messages -> gathered through the staging
    n = len(golden)
    off, parts, pos = np.zeros(n, np.uint32), [], 0
    for i in range(n):
        off[i] = pos
        parts.append(golden.msg(i) + bytes(3000))
        pos += int(golden.msg_sz[i]) + 3000
    blob = np.frombuffer(b"".join(parts) + b"\0", np.uint8)
    r = _Registered(golden.pub, golden.sig, off, golden.msg_sz, blob)
    try:
        assert np.array_equal(engine.verify_soa_registered(r[0], r[1], r[2], r[3], r[4]), golden.expect)
    finally:
        r.close()
    with pytest.raises(ed25519.EngineError):
        engine.verify_soa_registered(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)


def test_pooled_step_guard_is_reported_as_a_device_error(golden):
    """k_dsmp's hang guard (a bound on its step loop): capped through the
    debug entry point so that it trips, the batch call fails with
    FD_ED25519_AMD_ERR_DEVICE instead of returning verdicts computed from
    unfinished signatures, the device API sees FD_ED25519_AMD_VERDICT_DEVICE
    in every verdict, and with the cap lifted the same engine is exact."""
    from firedancer_amd import ed25519, hip
    eng = ed25519.Engine(device=0, batch_max=4096, blob_max=4096 * 1232)
    try:
        ed25519.select_dsm_kernel("k_dsmp")
        ed25519.debug_set_pool_iter_cap(10)
        with pytest.raises(ed25519.EngineError):
            eng.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
        n = len(golden)
        bufs = [hip.DeviceBuffer.from_array(a) for a in (golden.pub, golden.sig, golden.msg_off, golden.msg_sz,
                                                          golden.blob)]
        d_err, d_ws = hip.DeviceBuffer(n), hip.DeviceBuffer(ed25519.workspace_footprint(n))
        st = hip.Stream()
        ed25519.verify_dev(n, *[b.ptr for b in bufs], d_err.ptr, d_ws.ptr, st.handle)
        st.synchronize()
        assert (d_err.to_array(np.int8, n) == ed25519.VERDICT_DEVICE).all()
        ed25519.debug_set_pool_iter_cap(0)
        err = eng.verify_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob)
        assert np.array_equal(err, golden.expect)
    finally:
        ed25519.debug_set_pool_iter_cap(0)
        ed25519.select_dsm_kernel("default")
        eng.close()


def test_registered_plane_must_be_registered_to_its_end(golden):
    """A plane whose first page is registered but whose tail is not is
    refused (ERR_INVAL) before anything launches, instead of being read in
    place past the registered range by the latency path; the engine's next
    call is exact."""
    from firedancer_amd import ed25519
    n = 512
    raw = np.zeros(32 * n + 8192, np.uint8)
    o = (-raw.ctypes.data) % 4096
    pub = raw[o:o + 32 * n]                           # page-aligned, 4 pages
    pub[:] = golden.pub[:n].reshape(-1)
    ed25519.host_register(pub[:4096])                 # only its first page
    r = _Registered(golden.sig[:n], golden.msg_off[:n], golden.msg_sz[:n], golden.blob)
    eng = ed25519.Engine(device=0, batch_max=n, blob_max=n * 1232)
    try:
        with pytest.raises(ed25519.EngineError):
            eng.verify_soa_registered(pub.reshape(n, 32), r[0], r[1], r[2], r[3])
        p2 = _Registered(golden.pub[:n])
        try:
            err = eng.verify_soa_registered(p2[0], r[0], r[1], r[2], r[3])
            assert np.array_equal(err, golden.expect[:n])
        finally:
            p2.close()
    finally:
        eng.close()
        r.close()
        ed25519.host_unregister(pub[:4096])


def test_dropin_threads_route_to_their_devices(golden):
    """Drop-in callers on several threads, as the reference's verify tiles
    are threads of one process (fd_frank_main.c:118-143): each thread's
    fd_ed25519_amd_dropin_set_device holds for its own calls only (two
    threads set device 0 -- the one GPU of this box, listed twice as the
    multi-device tests do), a thread that set nothing takes the default
    (a valid device), and every verdict is the reference's."""
    import threading
    from firedancer_amd import ed25519, hip
    idx = [int(i) for i in np.arange(0, len(golden), 37)]
    out, errs = {}, []

    def tile(name, dev):
        try:
            if dev is not None:
                ed25519.dropin_set_device(dev)
            got = [ed25519.verify(golden.msg(i), bytes(golden.sig[i]), bytes(golden.pub[i])) for i in idx]
            out[name] = (ed25519.dropin_device(), got)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))

    ths = [threading.Thread(target=tile, args=a) for a in (("a", 0), ("b", 0), ("c", None))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    want = [int(golden.expect[i]) for i in idx]
    assert out["a"] == (0, want) and out["b"] == (0, want)
    assert 0 <= out["c"][0] < hip.device_count() and out["c"][1] == want
