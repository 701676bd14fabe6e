"""The streaming tile's hand-off, packing and chunk-level rules
(fd_verify_amd_tile_cut, _pack, _mode, _level: the pure functions
fd_verify_amd_tile_run applies to its staged frags; CPU only).  Whole chunks
go at once (8 frags in latency mode, 16 in quad mode, 64 in throughput
mode); a partial latency or quad chunk waits up to lat_fill_ns for company
unless the GPU has few chunks in flight; a partial throughput chunk waits up
to chunk_wait_ns; every flush condition hands over everything.  The level
follows the staging rate with hysteresis."""
import ctypes

import pytest

from firedancer_amd import ed25519, tango

BMAX, FILL, FREE, CHUNK_WAIT = 16384, 20000, 128, 50000


def cfg(**kw):
    c = tango.TileCfg()
    ed25519.lib().fd_verify_amd_tile_cfg_default(ctypes.byref(c))
    c.batch_max, c.lat_fill_ns, c.lat_free_chunks, c.chunk_wait_ns = BMAX, FILL, FREE, CHUNK_WAIT
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def cut(staged, handed, inflight=FREE, thr=False, waited=0, flush=False, **kw):
    c = cfg(**kw)
    return ed25519.lib().fd_verify_amd_tile_cut(ctypes.byref(c), staged, handed, inflight, int(thr), waited,
                                                int(flush))


def test_defaults():
    c = tango.TileCfg()
    ed25519.lib().fd_verify_amd_tile_cfg_default(ctypes.byref(c))
    assert (c.batch_max, c.lat_fill_ns, c.chunk_wait_ns, c.halt_grace_ns) == (4096, 20000, 50000, 50000000)
    assert (c.chunk_mode, c.publish_cpu, c.waves, c.window) == (tango.CHUNK_AUTO, tango.PUBLISH_AUTO, 0, 0)
    assert c.copy_cpu == tango.COPY_INLINE                # the copy helper is opt-in
    assert (c.quad_rate_hi, c.quad_rate_lo) == (0, 0)     # quad thresholds from the tile's capacity (the last fields)


def test_nothing_staged():
    assert cut(100, 100, flush=True) == 100


def test_latency_mode_whole_chunks_go_at_once():
    assert cut(100 + 19, 100) == 116                     # two whole 8-frag chunks, 3 wait for company
    assert cut(100 + 16, 100) == 116


def test_latency_mode_partial_chunk_waits_for_company():
    assert cut(100 + 3, 100) == 100                      # busy GPU: wait
    assert cut(100 + 3, 100, waited=FILL) == 103         # ... at most lat_fill_ns
    assert cut(100 + 3, 100, inflight=FREE - 1) == 103   # few chunks in flight: at once


def test_throughput_mode_hands_over_whole_chunks_only():
    assert cut(100 + 200, 100, thr=True) == 100 + 192
    assert cut(100 + 200, 100, thr=True, inflight=0) == 100 + 192   # an idle GPU does not flush
    assert cut(100 + 63, 100, thr=True, waited=FILL) == 100
    assert cut(100 + 63, 100, thr=True, waited=CHUNK_WAIT) == 163   # a remainder waited long enough


@pytest.mark.parametrize("thr", [False, True])
def test_flush_conditions_hand_over_everything(thr):
    assert cut(163, 100, thr=thr, flush=True) == 163
    assert cut(100 + 256, 100, thr=thr, batch_max=256) == 356     # batch_max staged
    assert cut(100 + 255, 100, thr=thr, batch_max=256) == 100 + (192 if thr else 248)
    assert cut(101, 100, thr=thr, batch_wait_ns=5000, waited=5000) == 101


def test_mode_hysteresis_and_fixed_modes():
    m = ed25519.lib().fd_verify_amd_tile_mode
    hi, lo = 10e6, 7e6
    assert m(tango.CHUNK_AUTO, 0, 9e6, hi, lo) == 0
    assert m(tango.CHUNK_AUTO, 0, 11e6, hi, lo) == 1
    assert m(tango.CHUNK_AUTO, 1, 8e6, hi, lo) == 1       # stays until below rate_lo
    assert m(tango.CHUNK_AUTO, 1, 6e6, hi, lo) == 0
    assert m(tango.CHUNK_LATENCY, 1, 50e6, hi, lo) == 0
    assert m(tango.CHUNK_THROUGHPUT, 0, 0.0, hi, lo) == 1


def test_quad_mode_cuts_16_slot_chunks_with_the_latency_fill_rule():
    q = tango.LVL_QUAD
    assert cut(100 + 40, 100, thr=q) == 132              # two whole 16-frag chunks, 8 wait
    assert cut(100 + 15, 100, thr=q) == 100              # busy GPU: a partial chunk waits for company
    assert cut(100 + 15, 100, thr=q, waited=FILL) == 115
    assert cut(100 + 15, 100, thr=q, inflight=FREE - 1) == 115
    assert cut(100 + 15, 100, thr=q, flush=True) == 115


def pack(slots, lvl):
    a = (ctypes.c_uint * max(len(slots), 1))(*slots)
    nsl = ctypes.c_ulong(0)
    n = ed25519.lib().fd_verify_amd_tile_pack(a, len(slots), lvl, ctypes.byref(nsl))
    return n, nsl.value


def test_pack_by_level():
    assert pack([1] * 100, tango.LVL_LAT) == (8, 8)
    assert pack([1] * 100, tango.LVL_QUAD) == (16, 16)
    assert pack([1] * 100, tango.LVL_THR) == (64, 64)
    assert pack([3, 5, 6, 2, 1], tango.LVL_QUAD) == (4, 16)    # whole frags up to 16 slots
    assert pack([3, 5, 6, 4], tango.LVL_QUAD) == (3, 14)       # 14 + 4 > 16: the 4 waits for the next chunk
    assert pack([12, 1, 1], tango.LVL_LAT) == (1, 12)          # more than 8: a chunk of its own (1 lane each)
    assert pack([12, 4, 1], tango.LVL_QUAD) == (2, 16)
    assert pack([19, 1], tango.LVL_QUAD) == (1, 19)
    assert pack([7] * 20, tango.LVL_THR) == (9, 63)


def level(mode, cur, rate, qhi=10e6, qlo=7e6, thi=30e6, tlo=24e6):
    return ed25519.lib().fd_verify_amd_tile_level(mode, cur, rate, qhi, qlo, thi, tlo)


def test_level_rule_three_way_hysteresis():
    L, Q, T = tango.LVL_LAT, tango.LVL_QUAD, tango.LVL_THR
    A = tango.CHUNK_AUTO
    assert level(A, L, 9e6) == L and level(A, L, 11e6) == Q and level(A, L, 31e6) == T   # a jump goes straight up
    assert level(A, Q, 8e6) == Q and level(A, Q, 6e6) == L                                # quad holds to quad_lo
    assert level(A, Q, 29e6) == Q and level(A, Q, 31e6) == T
    assert level(A, T, 25e6) == T and level(A, T, 20e6) == Q and level(A, T, 5e6) == L   # throughput holds to rate_lo
    # quad disabled (thresholds infinite): the two-level rule of fd_verify_amd_tile_mode
    inf = float("inf")
    for cur, rate in ((L, 9e6), (L, 31e6), (T, 25e6), (T, 20e6)):
        two = ed25519.lib().fd_verify_amd_tile_mode(A, int(cur == T), rate, 30e6, 24e6)
        assert level(A, cur, rate, inf, inf) == (T if two else L)
    assert level(tango.CHUNK_LATENCY, T, 50e6) == L
    assert level(tango.CHUNK_THROUGHPUT, L, 0.0) == T
    assert level(tango.CHUNK_QUAD, T, 0.0) == Q and level(tango.CHUNK_QUAD, L, 50e6) == Q


def test_level_step_holds():
    """fd_verify_amd_tile_level_step: a lower level only after an unbroken 2 ms
    ask; quad -> throughput once an episode of asks (gaps under 1 ms) has lasted
    2 ms; latency -> quad / throughput at once; quad -> throughput at once within
    5 holds of leaving throughput chunks."""
    import ctypes
    L, Q, T = tango.LVL_LAT, tango.LVL_QUAD, tango.LVL_THR
    st = (ctypes.c_ulong * 4)()
    step = ed25519.lib().fd_verify_amd_tile_level_step
    H, ms = 2_000_000, 1_000_000

    def s(lvl, want, now):
        return step(lvl, want, int(now), H, st)

    assert s(L, Q, 100) == Q and s(L, T, 100) == T        # up from latency chunks: at once
    assert s(Q, Q, 0) == Q
    # a stall's burst: the rule asks for throughput for 1 ms, then stops for 1 ms: the episode ends
    assert all(s(Q, T, t * ms) == Q for t in (1.0, 1.5, 2.0))
    assert s(Q, Q, 2.5 * ms) == Q and s(Q, Q, 3.0 * ms) == Q
    assert all(s(Q, T, t * ms) == Q for t in (3.1, 3.6, 4.1, 4.6, 5.0))   # a new episode from 3.1 ms
    assert s(Q, T, 5.1 * ms) == T
    # real overload with a dip: the dip (0.5 ms without an ask) does not restart the episode
    st[0] = st[1] = st[2] = st[3] = 0
    assert s(Q, T, 10 * ms) == Q and s(Q, Q, 10.5 * ms) == Q and s(Q, T, 11 * ms) == Q
    assert s(Q, T, 12 * ms) == T
    # down from throughput: only after an unbroken hold
    assert s(T, Q, 20 * ms) == T and s(T, T, 21 * ms) == T          # the ask broke: the hold restarts
    assert s(T, Q, 21.5 * ms) == T and s(T, Q, 23.4 * ms) == T and s(T, Q, 23.5 * ms) == Q
    # back up within 5 holds of leaving throughput chunks: at once
    assert s(Q, T, 24 * ms) == T
    assert s(T, Q, 25 * ms) == T and s(T, Q, 27 * ms) == Q          # left again at 27 ms
    assert s(Q, T, 37 * ms) == Q                                    # 5 holds later the hold applies again
    assert s(Q, L, 40 * ms) == Q and s(Q, L, 42 * ms) == L          # quad -> latency: the hold
    st[0] = st[1] = st[2] = st[3] = 0
    assert s(T, L, 0) == T and s(T, L, H) == L             # time 0 is a time like any other
    assert step(Q, T, 0, H, None) == T and step(T, L, 0, H, None) == L   # no state: no holds
