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


# ---------------------------------------------------------------- node plan

FRAME_SZ = 1408                        # FD_VERIFY_AMD_FRAME_SZ
RING_ENTRY_BYTES = 16 + 16 + 24        # ring entry + chunk descriptor + 3 result words, per ring slot


def tile_window(batch_max, window=0):
    """The tile's default window (frags in flight), fd_verify_tile.cpp tile_window."""
    if window:
        return int(window)
    if batch_max >= 1 << 10:
        return 1 << 18
    return max(64 * batch_max, 1 << 16)


def tile_budget(batch_max, cpus, zero_copy=True, window=0, out_frame_cnt=0):
    """Host budget of ONE verify tile on the CPU slice `cpus` (sorted list):
    which spinning threads it runs on which CPU, and the pinned host memory
    it holds (fd_verify_amd_tile_new_cfg / _run).

    Threads, in the order they get a CPU of their own: the stager (the
    caller's thread, always), the publisher (cfg.publish_cpu; inline on the
    stager when the slice has one CPU), and, in copy mode only, the copy
    helper (cfg.copy_cpu; inline when the slice has fewer than 3 CPUs).
    Pinned memory: the output dcache ((4096 + batch_max + window) frames of
    1408 B), the ring / descriptors / results (a power of 2 >= the window,
    56 B per slot), 4 KB of control words."""
    cpus = sorted(cpus)
    if not cpus:
        raise ValueError("a tile needs at least one CPU")
    w = tile_window(batch_max, window)
    frames = int(out_frame_cnt) or 4096 + int(batch_max) + w
    ring = 1
    while ring < min(w, frames):
        ring <<= 1
    plan = {"stager_cpu": cpus[0],
            "publish_cpu": cpus[1] if len(cpus) >= 2 else None,
            "copy_cpu": cpus[2] if (not zero_copy and len(cpus) >= 3) else None}
    plan["spinning_threads"] = 1 + (plan["publish_cpu"] is not None) + (plan["copy_cpu"] is not None)
    plan["pinned_bytes"] = frames * FRAME_SZ + ring * RING_ENTRY_BYTES + 4096
    plan["window"] = w
    return plan


def node_plan(numa_of_rank, node_cpus, batch_max, zero_copy=True, cpu_quota=None):
    """The N-tile node (one tile per GPU, the reference's scaling unit,
    fd_frank_init:67-80, fd_frank_main.c:118-143): each rank gets a disjoint
    slice of its GPU's NUMA node's CPUs (ranks sharing a node split it,
    peer_slot / cpu_slice), capped so that all ranks together fit the
    process group's CPU quota (cgroup cpu.max, e.g. 16 on a one-GPU box's
    share), and a tile_budget on that slice.  Returns one plan per rank plus
    the node totals."""
    world = len(numa_of_rank)
    if cpu_quota:
        per = max(1, int(cpu_quota) // world)
    else:
        per = None
    plans = []
    for r in range(world):
        k, n = peer_slot(list(numa_of_rank), r)
        sl = cpu_slice(node_cpus[numa_of_rank[r]], k, n)
        if per is not None:
            sl = sl[:per]
        b = tile_budget(batch_max, sl, zero_copy=zero_copy)
        b.update(rank=r, numa_node=numa_of_rank[r], cpus=sl)
        plans.append(b)
    tot = {"ranks": world, "spinning_threads": sum(p["spinning_threads"] for p in plans),
           "pinned_bytes": sum(p["pinned_bytes"] for p in plans),
           "cpus_used": len({c for p in plans for c in p["cpus"][:p["spinning_threads"]]})}
    return plans, tot


def node_sum(per_rank, cols):
    """Rank 0's aggregation of the N-tile node rows (bench.py stream_node):
    per_rank[r] = list of floats in `cols` order; the node value of a rate
    column is the sum over ranks (every rank's tile ran at once, each on its
    own GPU, no data exchanged), latency columns stay per rank."""
    out = {c: sum(r[i] for r in per_rank) for i, c in enumerate(cols) if c.endswith("per_s")}
    out["per_rank"] = [dict(zip(cols, r)) for r in per_rank]
    return out
