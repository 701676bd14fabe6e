"""Multi-GPU sharding of ed25519 batches (SURVEY.md s8 e).

Signatures are independent, so a batch shards across GPUs with no exchange
step: contiguous index ranges per device, one engine (own HIP streams,
pinned staging) per device, verdicts gathered by plain D2H copies.  No
collective touches the data path -- RCCL/xGMI are unused.

Two ways to run N GPUs:
  * one process per GPU (bench.py under torch.distributed.run): each rank
    verifies shard_range(n, rank, world); gloo carries only the start/stop
    barriers and the max-over-ranks of the elapsed time;
  * one process driving every local GPU (MultiDeviceVerifier): one host
    thread per device, each feeding its own engine.
"""
import threading

import numpy as np


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of n units for `rank` of `world` (sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world %r/%r" % (rank, world))
    base, extra = divmod(int(n), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


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


class MultiDeviceVerifier:
    """Verify one SoA batch across `devices` (one engine + host thread each)."""

    def __init__(self, devices, batch_max=1 << 18, blob_max=None):
        from . import ed25519
        self.engines = [ed25519.Engine(device=d, batch_max=batch_max, blob_max=blob_max) for d in devices]

    def verify_soa(self, pub, sig, msg_off, msg_sz, blob):
        n = len(pub)
        err = np.zeros(n, np.int8)
        excs = []

        def work(k, eng):
            try:
                lo, hi = shard_range(n, k, len(self.engines))
                if hi > lo:
                    err[lo:hi] = eng.verify_soa(*_slice_soa(pub, sig, msg_off, msg_sz, blob, lo, hi))
            except Exception as e:  # surfaced below
                excs.append(e)

        th = [threading.Thread(target=work, args=(k, e)) for k, e in enumerate(self.engines)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if excs:
            raise excs[0]
        return err

    def close(self):
        for e in self.engines:
            e.close()
