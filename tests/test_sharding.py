"""Multi-rank path on CPU (gloo, world_size 2): every rank takes its
contiguous shard with no data-path collective, and the union of the shards'
verdicts equals the single-process result; the only collective is the
control-plane max of the elapsed time.  The per-shard verdicts come from the
oracle here (no GPU); the GPU engine runs the same shard_range split."""
import os
import socket

import numpy as np
import pytest

import _golden
import _oracle
from firedancer_amd.shard import _slice_soa, shard_range


def test_shard_range_partition():
    for n in (0, 1, 7, 64, 1000, (1 << 20) + 3):
        for world in (1, 2, 3, 4, 8):
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_shard_range_matches_native():
    """The Python split (bench ranks) and fd_ed25519_amd_shard_range (the
    native multi-device engine) give the same shards."""
    from firedancer_amd import ed25519
    for n in (0, 1, 7, 1000, (1 << 24) + 5):
        for world in (1, 2, 3, 8):
            for r in range(world):
                assert ed25519.shard_range(n, world, r) == shard_range(n, r, world)


def test_multi_engine_refuses_without_device():
    from firedancer_amd import ed25519, hip
    if hip.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(ed25519.EngineError):
        ed25519.MultiEngine([0, 0])


def test_slice_soa_rebases_messages(golden):
    lo, hi = 100, 180
    pub, sig, off, sz, blob = _slice_soa(golden.pub, golden.sig, golden.msg_off, golden.msg_sz, golden.blob, lo, hi)
    for j in range(hi - lo):
        assert bytes(blob[off[j]:off[j] + sz[j]]) == golden.msg(lo + j)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from firedancer_amd.shard import max_over_ranks
    g = _golden.load_vectors()
    lo, hi = shard_range(len(g), rank, world)
    pub, sig, off, sz, blob = _slice_soa(g.pub, g.sig, g.msg_off, g.msg_sz, g.blob, lo, hi)
    err = _oracle.verify_batch(_golden.Batch(pub, sig, off, sz, blob), nthread=2)
    elapsed = max_over_ranks(1.0 + rank)
    # test-only gather of the verdicts to check the union (the product path never does this)
    sizes = [shard_range(len(g), r, world)[1] - shard_range(len(g), r, world)[0] for r in range(world)]
    buf = [torch.zeros(s, dtype=torch.int8) for s in sizes]
    dist.all_gather(buf, torch.from_numpy(err.copy())) if len(set(sizes)) == 1 else None
    if len(set(sizes)) != 1:
        objs = [None] * world
        dist.all_gather_object(objs, err.tolist())
        allerr = np.concatenate([np.array(o, np.int8) for o in objs])
    else:
        allerr = torch.cat(buf).numpy()
    if rank == 0:
        q.put((elapsed, allerr.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_match_single_process():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    elapsed, allerr = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = _golden.load_vectors()
    assert elapsed == 2.0                      # max over ranks
    assert np.array_equal(np.array(allerr, np.int8), g.expect)


def test_peer_slot_and_cpu_slice():
    """Ranks that share a NUMA node (or a GPU) find their index among their
    peers, and split the node's CPUs into disjoint slices (the per-rank tile
    rows of bench.py pin each rank's spinning threads to its own slice)."""
    from firedancer_amd.shard import cpu_slice, peer_slot
    keys = [0, 0, 1, 1, 0, 1, 0, 1]                 # NUMA node per rank
    assert [peer_slot(keys, r) for r in range(8)] == [(0, 4), (1, 4), (0, 4), (1, 4), (2, 4), (2, 4), (3, 4),
                                                        (3, 4)]
    cpus = list(range(64, 96)) + list(range(0, 32))
    slices = [cpu_slice([c for c in cpus if c < 32], k, 4) for k in range(4)]
    assert slices == [list(range(8 * k, 8 * k + 8)) for k in range(4)]
    assert cpu_slice(range(10), 0, 1) == list(range(10))
    assert cpu_slice(range(10), 2, 3) == [6, 7, 8]
    with pytest.raises(ValueError):
        cpu_slice(range(10), 3, 3)


def _node_worker(rank, world, port, q):
    """One rank of an 8-tile node rehearsal on CPU: its config-4 shard, its
    CPU slice and host budget from the node plan, and the node-sum
    aggregation bench.py's stream_node performs (gloo, control plane only)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from firedancer_amd.shard import node_plan, node_sum, shard_range
    numa = [r // 4 for r in range(world)]                      # two NUMA nodes, four GPUs each
    node_cpus = {0: list(range(0, 64)), 1: list(range(64, 128))}
    plans, tot = node_plan(numa, node_cpus, 16384, zero_copy=True, cpu_quota=16)
    mine = plans[rank]
    lo, hi = shard_range(1 << 24, rank, world)
    rate = 1e6 * (rank + 1)                                    # a stand-in for the rank's measured tile rate
    cols = ["saturated_frags_per_s", "p50_us", "cpus"]
    t = torch.zeros(world * len(cols), dtype=torch.float64)
    t[rank * len(cols):(rank + 1) * len(cols)] = torch.tensor([rate, 1300.0 + rank, float(len(mine["cpus"]))],
                                                              dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    agg = node_sum(t.view(world, len(cols)).tolist(), cols)
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "lo": lo, "hi": hi, "cpus": mine["cpus"],
                                 "threads": mine["spinning_threads"], "pinned": mine["pinned_bytes"],
                                 "publish_cpu": mine["publish_cpu"], "copy_cpu": mine["copy_cpu"]})
    if rank == 0:
        q.put((got, agg, tot))
    dist.barrier()
    dist.destroy_process_group()


def test_eight_rank_node_plan_and_node_sum():
    """gloo world_size 8 (CPU; the 8-GPU node is unmeasured on hardware): the
    ranks' config-4 shards partition 2^24 signatures, each rank's tile gets a
    disjoint CPU slice on its own NUMA node within a 16-CPU quota (2 CPUs:
    stager + publisher, zero copy), eight tiles pin ~3.3 GB of host memory,
    and rank 0's node sum is the sum of the ranks' rates."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 8
    procs = [ctx.Process(target=_node_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, agg, tot = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = sorted(got, key=lambda x: x["rank"])
    assert got[0]["lo"] == 0 and got[-1]["hi"] == 1 << 24
    assert all(a["hi"] == b["lo"] for a, b in zip(got, got[1:]))
    flat = [c for g in got for c in g["cpus"]]
    assert len(flat) == len(set(flat)) == 16                    # disjoint, and the quota holds
    for g in got:
        node = g["rank"] // 4
        assert all(64 * node <= c < 64 * (node + 1) for c in g["cpus"])   # on the GPU's NUMA node
        assert g["threads"] == 2 and g["publish_cpu"] == g["cpus"][1] and g["copy_cpu"] is None
    assert tot["spinning_threads"] == 16 and tot["cpus_used"] == 16
    assert 3.0e9 < tot["pinned_bytes"] < 3.6e9
    assert agg["saturated_frags_per_s"] == sum(1e6 * (r + 1) for r in range(world))
    assert [round(r["p50_us"]) for r in agg["per_rank"]] == [1300 + r for r in range(world)]


def test_tile_budget_scarce_cpus():
    """One CPU: the publisher runs inline on the stager; copy mode gets its
    helper only from three CPUs."""
    from firedancer_amd.shard import tile_budget
    b = tile_budget(4096, [5])
    assert b["spinning_threads"] == 1 and b["publish_cpu"] is None
    b = tile_budget(4096, [5, 6, 7], zero_copy=False)
    assert b["spinning_threads"] == 3 and b["copy_cpu"] == 7
    b = tile_budget(1024, [5, 6], window=1 << 15)
    assert b["window"] == 1 << 15 and b["pinned_bytes"] < 60e6
