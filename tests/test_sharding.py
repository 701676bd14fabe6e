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
