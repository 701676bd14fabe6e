"""Multi-GPU sharding of ed25519 batches (SURVEY.md s8 e).

Signatures are independent, so a batch shards across GPUs with no exchange
step: contiguous index ranges per device, one engine (own HIP streams,
pinned staging) per device, verdicts gathered by plain D2H copies.  No
collective touches the data path -- RCCL/xGMI are unused.

Two ways to run N GPUs:
  * one process per GPU (bench.py under torch.distributed.run): each rank
    verifies shard_range(n, rank, world); gloo carries only the start/stop
    barriers and the max-over-ranks of the elapsed time;
  * one process driving every local GPU: the native multi-device engine
    (fd_ed25519_amd_multi_*, ed25519.MultiEngine), one engine and one
    persistent host thread per device.
"""
import os

import numpy as np


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of n units for `rank` of `world` (sizes differ by
    <= 1): lo = n*rank//world, the split fd_ed25519_amd_shard_range uses."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world %r/%r" % (rank, world))
    return int(n) * rank // world, int(n) * (rank + 1) // world


def max_over_ranks(value):
    """Max of a float over all ranks of the default torch.distributed group
    (identity when not initialised).  Control plane only (gloo)."""
    try:
        import torch
        import torch.distributed as dist
    except ImportError:
        return float(value)
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _slice_soa(pub, sig, off, sz, blob, lo, hi):
    """Rebase a sub-range of an SoA batch onto its own compact blob."""
    if hi <= lo:
        return pub[lo:hi], sig[lo:hi], np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(1, np.uint8)
    o = off[lo:hi].astype(np.int64)
    s = sz[lo:hi].astype(np.int64)
    start, end = int(o.min()), int((o + s).max())
    return (pub[lo:hi], sig[lo:hi], (o - start).astype(np.uint32), sz[lo:hi],
            np.ascontiguousarray(blob[start:max(end, start + 1)]))


def parse_cpulist(text):
    """sysfs cpulist ("0-3,8,10-11") -> sorted list of CPU ids."""
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.extend(range(int(a), int(b or a) + 1))
    return cpus


def bind_to_device_node(device, sysfs="/sys"):
    """Pin this process to the CPUs of `device`'s NUMA node that it may use
    (the reference pins each tile to a core next to its link,
    src/app/frank/fd_frank_main.c:118-143).  Returns {"numa_node", "cpus"}
    (cpus: how many the process is now bound to, 0 = left unchanged).
    FD_ED25519_AMD_NUMA=0 leaves the affinity alone."""
    from . import ed25519
    node = int(ed25519.device_numa_node(device))
    out = {"numa_node": node, "cpus": 0}
    if node < 0 or os.environ.get("FD_ED25519_AMD_NUMA") == "0":
        return out
    try:
        cpus = parse_cpulist(open(os.path.join(sysfs, "devices/system/node/node%d/cpulist" % node)).read())
    except (OSError, ValueError):
        return out
    want = sorted(set(cpus) & os.sched_getaffinity(0))
    if want:
        os.sched_setaffinity(0, want)
        out["cpus"] = len(want)
    return out


def peer_slot(keys, rank):
    """Among the ranks whose key equals keys[rank] (e.g. the same NUMA node,
    or the same GPU): (this rank's index among them, how many there are)."""
    mine = keys[rank]
    same = [r for r, k in enumerate(keys) if k == mine]
    return same.index(rank), len(same)


def cpu_slice(cpus, k, n):
    """The k-th of n contiguous, disjoint slices of the sorted CPU list (the
    spinning threads of ranks that share a NUMA node must not share CPUs)."""
    cpus = sorted(cpus)
    if n < 1 or not (0 <= k < n):
        raise ValueError("bad slice %r of %r" % (k, n))
    per = len(cpus) // n
    return cpus[k * per:(k + 1) * per]
