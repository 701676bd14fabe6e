"""CPU tests of the C-ABI boundary: the engine library loads without a GPU,
exports every symbol include/fd_ed25519_amd.h declares, and its host-side
(non-verify) entry points behave like the reference's.  No verify call is
made here -- those need a GPU and live in test_gpu_parity.py."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def declared_functions():
    """Every extern function declared by include/*.h (static inline helpers
    and macros excluded)."""
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"^#.*$", "", src, flags=re.M)
        src = re.sub(r"static inline[^{]*\{[^}]*\}", "", src)
        names.update(re.findall(r"\b(fd_\w+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    from firedancer_amd import ed25519
    L = ed25519.lib()
    names = declared_functions()
    assert "fd_ed25519_verify" in names and "fd_ed25519_amd_verify_dev" in names
    assert "fd_ed25519_amd_verify_txns" in names and "fd_txn_amd_parse_dev" in names
    assert "fd_txn_footprint" not in names
    for n in names:
        assert hasattr(L, n), n
    # and as real dynamic symbols (a C / Rust / Go caller links by name)
    out = subprocess.run(["nm", "-D", "--defined-only", ed25519.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [n for n in names if n not in exported]
    assert not missing, missing


def test_reference_codes_and_strerror():
    from firedancer_amd import ed25519
    assert (ed25519.FD_ED25519_SUCCESS, ed25519.FD_ED25519_ERR_SIG, ed25519.FD_ED25519_ERR_PUBKEY,
            ed25519.FD_ED25519_ERR_MSG) == (0, -1, -2, -3)
    # fd_ed25519_user.c:433-443
    assert ed25519.strerror(0) == "success"
    assert ed25519.strerror(-1) == "bad signature"
    assert ed25519.strerror(-2) == "bad public key"
    assert ed25519.strerror(-3) == "bad message"
    assert ed25519.strerror(7) == "unknown"
    hdr = open(os.path.join(ROOT, "include", "fd_ed25519_amd.h")).read()
    for name, val in (("FD_ED25519_SUCCESS", 0), ("FD_ED25519_ERR_SIG", -1), ("FD_ED25519_ERR_PUBKEY", -2),
                      ("FD_ED25519_ERR_MSG", -3)):
        assert re.search(r"#define %s\s+\(\s*%d\)" % (name, val), hdr), name


def test_workspace_footprint_monotone():
    from firedancer_amd import ed25519
    a, b, c = (ed25519.workspace_footprint(n) for n in (1, 64, 1 << 20))
    assert 0 < a <= b < c
    assert c >= (1 << 20) * 2000        # ~2 KB of scratch per signature
    assert c % 256 == 0


def test_tile_tickcount_tracks_monotonic_ns():
    """fd_verify_amd_tickcount (TSC-derived) stays on the CLOCK_MONOTONIC
    nanosecond scale: low 32 bits within 1 ms of time.monotonic_ns, and it
    advances at the monotonic rate over a 50 ms interval (1 %)."""
    import time
    from firedancer_amd import ed25519
    f = ed25519.lib().fd_verify_amd_tickcount
    f.restype = ctypes.c_uint
    f()                                               # one-time calibration
    d = (f() - (time.monotonic_ns() & 0xFFFFFFFF)) & 0xFFFFFFFF
    assert min(d, (1 << 32) - d) < 1_000_000
    a, ma = f(), time.monotonic_ns()
    time.sleep(0.05)
    b, mb = f(), time.monotonic_ns()
    assert abs(((b - a) & 0xFFFFFFFF) / (mb - ma) - 1.0) < 0.01


def test_engine_fails_loudly_without_device():
    """On a host without a HIP device the engine must refuse, not fall back."""
    from firedancer_amd import ed25519, hip
    if hip.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(ed25519.EngineError):
        ed25519.Engine(device=0)


def test_c_caller_compiles_against_header(tmp_path):
    """A plain C caller (the reference's own calling convention) compiles and
    links against the header + library."""
    from firedancer_amd import ed25519
    c = tmp_path / "caller.c"
    c.write_text('''
#include "fd_ed25519_amd.h"
#include "fd_txn_amd.h"
#include <stdio.h>
int main( void ) {
  if( sizeof(fd_txn_t)!=20UL || sizeof(fd_txn_instr_t)!=10UL || sizeof(fd_txn_acct_addr_lut_t)!=8UL ) return 1;
  if( fd_txn_footprint( 355UL, 0UL )!=FD_TXN_MAX_SZ ) return 1;   /* fd_txn.h:95 worst case */
  printf( "%s\\n", fd_ed25519_strerror( FD_ED25519_ERR_MSG ) );
  printf( "%lu\\n", fd_ed25519_amd_workspace_footprint( 64UL ) );
  return 0;
}
''')
    exe = tmp_path / "caller"
    libdir = os.path.dirname(ed25519.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c),
                           "-L", libdir, "-lfd_ed25519_amd", "-Wl,-rpath," + libdir, "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert out[0] == "bad" and out[1] == "message"


CLIENT = os.path.join(ROOT, "tests", "c", "dropin_client")


def _client():
    if not os.path.exists(CLIENT):          # built by __graft_entry__.build(); build it here if missing
        from firedancer_amd import build
        build.build_clients()
    return CLIENT


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU host: see the gpu test")
def test_plain_c_client_host_entry_points():
    """tests/c/dropin_client.c: a gcc-compiled C caller that includes only
    include/*.h and links the library by name, as a relinked Firedancer
    would.  Host mode: RFC 8032 test 1 bytes, strerror, the engine refusing
    to start without a device."""
    r = subprocess.run([_client(), "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "dropin_client cpu: OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_plain_c_client_on_gpu():
    """The same C caller on the GPU: fd_ed25519_verify codes, then 2000
    signatures (10 % corrupted) through verify_soa and verify_batch, every
    verdict equal to the drop-in call's."""
    r = subprocess.run([_client(), "gpu"], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "dropin_client gpu: OK" in r.stdout, r.stdout + r.stderr


def test_dropin_default_device_rule():
    """fd_ed25519_amd_dropin_pick: a drop-in thread that set no device gets
    a GPU of its own NUMA node, round robin by its ordinal among that node's
    threads (8 tiles on a 2-socket node with 4 GPUs per socket spread 1:1);
    all GPUs round robin when none is local or the node is unknown."""
    from firedancer_amd import ed25519
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    assert [ed25519.dropin_pick(nodes, 0, k) for k in range(5)] == [0, 1, 2, 3, 0]
    assert [ed25519.dropin_pick(nodes, 1, k) for k in range(5)] == [4, 5, 6, 7, 4]
    assert [ed25519.dropin_pick(nodes, -1, k) for k in range(9)] == [0, 1, 2, 3, 4, 5, 6, 7, 0]
    assert [ed25519.dropin_pick(nodes, 3, k) for k in range(3)] == [0, 1, 2]          # no GPU on node 3
    assert [ed25519.dropin_pick([1, 0, 1, 0], 1, k) for k in range(3)] == [0, 2, 0]   # interleaved enumeration
    assert [ed25519.dropin_pick([-1, -1], 0, k) for k in range(3)] == [0, 1, 0]       # nodes unknown
    assert ed25519.dropin_pick([], 0, 5) == 0


def test_dropin_set_device_refuses_bad_devices():
    """Out-of-range devices are refused; without a HIP device any explicit
    choice fails (no CPU fallback), the default is always accepted."""
    from firedancer_amd import ed25519, hip
    with pytest.raises(ed25519.EngineError):
        ed25519.dropin_set_device(-2)
    with pytest.raises(ed25519.EngineError):
        ed25519.dropin_set_device(1 << 20)
    ed25519.dropin_set_device(ed25519.DROPIN_AUTO)
    assert ed25519.dropin_device() == -1                 # no call made on this thread yet
    if hip.device_count() == 0:
        with pytest.raises(ed25519.EngineError):
            ed25519.dropin_set_device(0)
