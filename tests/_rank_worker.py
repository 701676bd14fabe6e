"""One rank of tests/test_multi_gpu.py::test_two_ranks_run_the_engine_on_their_shards
(started as its own process, before it touches the GPU): gloo for control,
the HIP engine for its shard of the golden vectors; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch.distributed as dist
    import _golden
    from firedancer_amd import ed25519, hip
    from firedancer_amd.shard import max_over_ranks, shard_range
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    local = int(os.environ["LOCAL_RANK"])
    ndev = hip.device_count()
    if os.environ.get("FD_AMD_DEVICE_MAP") == "mod":
        local %= ndev
    g = _golden.load_vectors()
    lo, hi = shard_range(len(g), rank, world)
    eng = ed25519.Engine(device=local, batch_max=4096, blob_max=4096 * 1232)
    try:
        dist.barrier()
        t0 = time.perf_counter()
        err = eng.verify_soa(g.pub[lo:hi], g.sig[lo:hi], g.msg_off[lo:hi], g.msg_sz[lo:hi], g.blob)
        elapsed = max_over_ranks(time.perf_counter() - t0)
    finally:
        eng.close()
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps({"rank": rank, "lo": lo, "hi": hi, "err": err.tolist(), "elapsed_max": elapsed}))


if __name__ == "__main__":
    main()
