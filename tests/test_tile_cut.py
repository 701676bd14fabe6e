"""The streaming tile's hand-off rule (fd_verify_amd_tile_cut, the pure
function fd_verify_amd_tile_run applies to its staged frags; CPU only):
latency mode hands everything over once the input drains, throughput mode
whole 64-frag chunks, and every flush condition hands over everything."""
import ctypes

import pytest

from firedancer_amd import ed25519

LIGHT, BMAX, WAIT, CHUNK_WAIT = 8192, 16384, 0, 50000


def cut(staged, handed, pubd, waited=0, idle_in=False, full=False, done_in=False, wait_ns=WAIT, bmax=BMAX):
    f = ed25519.lib().fd_verify_amd_tile_cut
    f.restype = ctypes.c_ulong
    f.argtypes = [ctypes.c_ulong] * 8 + [ctypes.c_int] * 3 + [ctypes.POINTER(ctypes.c_int)]
    m = ctypes.c_int(-1)
    up = f(staged, handed, pubd, LIGHT, bmax, waited, wait_ns, CHUNK_WAIT, int(idle_in), int(full), int(done_in),
           ctypes.byref(m))
    return up, m.value


def test_nothing_staged():
    assert cut(100, 100, 0, idle_in=True)[0] == 100


def test_latency_mode_waits_for_the_input_to_drain():
    assert cut(130, 100, 90) == (100, 1)                 # input still arriving: keep staging
    assert cut(130, 100, 90, idle_in=True) == (130, 1)   # drained: everything, latency chunks


def test_latency_mode_with_batch_wait_only_greedy_while_nothing_in_flight():
    assert cut(130, 100, 90, idle_in=True, wait_ns=10000)[0] == 100
    assert cut(130, 100, 100, idle_in=True, wait_ns=10000)[0] == 130
    assert cut(130, 100, 90, idle_in=True, wait_ns=10000, waited=10000)[0] == 130


def test_throughput_mode_hands_over_whole_chunks_only():
    pubd = 100 - LIGHT                                    # LIGHT frags in flight
    assert cut(100 + 200, 100, pubd) == (100 + 192, 0)
    assert cut(100 + 200, 100, pubd, idle_in=True) == (100 + 192, 0)   # drained input does not flush
    assert cut(100 + 63, 100, pubd)[0] == 100
    assert cut(100 + 63, 100, pubd, waited=CHUNK_WAIT)[0] == 163        # a remainder waited long enough


@pytest.mark.parametrize("kw", [dict(full=True), dict(done_in=True)])
def test_flush_conditions_hand_over_everything(kw):
    assert cut(163, 100, 100 - LIGHT, **kw)[0] == 163
    assert cut(163, 100, 90, **kw)[0] == 163


def test_batch_max_forces_a_hand_off():
    assert cut(100 + 256, 100, 90, bmax=256)[0] == 356
    assert cut(100 + 255, 100, 90, bmax=256)[0] == 100
