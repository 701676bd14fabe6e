"""NUMA placement of the engines' host side (firedancer_amd/csrc/fd_numa.cpp,
include/fd_ed25519_amd.h fd_ed25519_amd_sysfs_numa): the GPU's node comes
from sysfs (bus/pci/devices/<bdf>/numa_node) and the node's CPUs from
devices/system/node/node<N>/cpulist.  Checked here on synthetic sysfs trees,
no GPU needed.  The reference pins each tile to a core and keeps its input
link local (src/app/frank/fd_frank_main.c:118-143, fd_frank_init:67-80)."""
import ctypes
import os

import pytest

from firedancer_amd import ed25519


def _tree(tmp_path, bdf, node, cpulist):
    d = tmp_path / "bus" / "pci" / "devices" / bdf
    d.mkdir(parents=True)
    (d / "numa_node").write_text("%d\n" % node)
    if cpulist is not None:
        n = tmp_path / "devices" / "system" / "node" / ("node%d" % node)
        n.mkdir(parents=True)
        (n / "cpulist").write_text(cpulist + "\n")
    return str(tmp_path)


def _lookup(root, bdf, cpus_max=64):
    f = ed25519.lib().fd_ed25519_amd_sysfs_numa
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                  ctypes.c_int]
    f.restype = ctypes.c_int
    node = ctypes.c_int(-7)
    cpus = (ctypes.c_int * max(cpus_max, 1))()
    n = f(root.encode(), bdf.encode(), ctypes.byref(node), cpus, cpus_max)
    return n, node.value, list(cpus[:max(n, 0)])


@pytest.mark.parametrize("cpulist,want", [("8-11,20", [8, 9, 10, 11, 20]), ("0", [0]),
                                           ("0-3,64-67", [0, 1, 2, 3, 64, 65, 66, 67])])
def test_node_and_cpus_of_a_gpu(tmp_path, cpulist, want):
    root = _tree(tmp_path, "0000:0c:00.0", 1, cpulist)
    n, node, cpus = _lookup(root, "0000:0C:00.0")      # HIP may print hex digits in upper case
    assert node == 1 and n == len(want) and cpus == want


def test_cpu_list_is_capped(tmp_path):
    root = _tree(tmp_path, "0000:8a:00.0", 3, "0-127")
    n, node, cpus = _lookup(root, "0000:8a:00.0", cpus_max=16)
    assert node == 3 and n == 16 and cpus == list(range(16))


def test_unknown_node_and_missing_device(tmp_path):
    root = _tree(tmp_path, "0000:01:00.0", -1, None)
    n, node, _ = _lookup(root, "0000:01:00.0")
    assert n == 0 and node == -1                       # platform reports no node: nothing to bind
    n, node, _ = _lookup(root, "0000:02:00.0")
    assert n == -1 and node == -1                      # no such device
    bad = _tree(tmp_path / "b", "0000:03:00.0", 0, "1-x")
    n, node, _ = _lookup(bad, "0000:03:00.0")
    assert n == -1 and node == 0                       # malformed cpulist


def test_device_node_without_gpu_is_unknown():
    f = ed25519.lib().fd_ed25519_amd_device_numa_node
    f.restype = ctypes.c_int
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present")
    assert f(0) == -1


def test_python_cpulist_and_binding(tmp_path, monkeypatch):
    """shard.parse_cpulist (the bench ranks' binding) agrees with the native
    parser; bind_to_device_node leaves the affinity alone when the node is
    unknown (no GPU here)."""
    from firedancer_amd import shard
    assert shard.parse_cpulist("8-11,20\n") == [8, 9, 10, 11, 20]
    root = _tree(tmp_path, "0000:0c:00.0", 2, "0-3,64-67")
    assert _lookup(root, "0000:0c:00.0")[2] == shard.parse_cpulist("0-3,64-67")
    before = os.sched_getaffinity(0)
    monkeypatch.setattr(ed25519, "device_numa_node", lambda d: -1)
    assert shard.bind_to_device_node(0) == {"numa_node": -1, "cpus": 0}
    monkeypatch.setattr(ed25519, "device_numa_node", lambda d: 2)
    r = shard.bind_to_device_node(0, sysfs=root)       # node 2's CPUs that this process may use
    want = sorted({0, 1, 2, 3, 64, 65, 66, 67} & before)
    assert r == {"numa_node": 2, "cpus": len(want)}
    if want:
        assert sorted(os.sched_getaffinity(0)) == want
    os.sched_setaffinity(0, before)
