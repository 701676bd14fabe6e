"""The streaming tile's hand-off and chunk-mode rules
(fd_verify_amd_tile_cut, fd_verify_amd_tile_mode: the pure functions
fd_verify_amd_tile_run applies to its staged frags; CPU only).  Whole chunks
go at once (8 frags in latency mode, 64 in throughput mode); a partial
latency chunk waits up to lat_fill_ns for company unless the GPU has few
chunks in flight; a partial throughput chunk waits up to chunk_wait_ns;
every flush condition hands over everything.  The mode follows the
staging rate with hysteresis."""
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
    assert c.copy_cpu == tango.COPY_INLINE                # the copy helper is opt-in (the last field of the struct)


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
