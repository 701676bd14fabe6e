"""CPU tests of the build's k_tile_persist guard (firedancer_amd/build.py):
it inspects the compiled tile kernel for VGPR spills inside the persistent
loop (the builds that lost their scout wave, profiles/r05_scout_stop_cause.txt)
and fails closed when it cannot inspect."""
import os

import pytest

from firedancer_amd import build

OBJ = os.path.join(build.PKG, "_obj", "libfd_ed25519_amd", "fd_ed25519_kernels.hip.o")


@pytest.mark.skipif(not os.path.exists(OBJ), reason="engine objects not built here")
def test_shipped_tile_kernel_has_no_loop_spills():
    assert build.loop_spill_stores(OBJ, build.TILE_KERNEL) == 0


@pytest.mark.skipif(not os.path.exists(OBJ), reason="engine objects not built here")
def test_guard_cannot_locate_an_unknown_kernel():
    assert build.loop_spill_stores(OBJ, "_Z9no_kernelv") is None


def test_guard_fails_closed_without_llvm_tools(monkeypatch, tmp_path):
    """No disassembler -> loop_spill_stores is None -> build_engine refuses."""
    monkeypatch.setattr(build, "_device_object", lambda obj: None)
    assert build.loop_spill_stores(str(tmp_path / "x.o"), build.TILE_KERNEL) is None
    calls = []
    monkeypatch.setattr(build.subprocess, "check_call", lambda *a, **k: calls.append(a))
    with pytest.raises(RuntimeError, match="refusing the build"):
        build.build_engine(force=True, out=str(tmp_path / "lib.so"), defines=("FD_AMD_GUARD_TEST",))
    assert not any("-shared" in c[0] for c in calls)      # nothing was linked
