#!/usr/bin/env python3
"""bench.py -- ed25519 verifies/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n SIGS] [--msg-sz B]

A "step" is one pass of the verify pipeline (k_prep -> k_decomp -> k_dsm)
over one batch of n synthetic signatures (BASELINE.json configs[1]:
2^20 single-signer signatures, 200-byte Solana-txn-sized messages, fresh
random keypairs), with the inputs already resident in HBM when the timed
region starts.  For N > 1 (launched by torch.distributed.run) every rank
verifies its own shard of n signatures on its own GPU -- signatures are
independent, so there is no data-path collective (weak scaling); gloo is
used only for the start/stop barriers and the max-over-ranks of the time.

Rank 0 prints ONE JSON line: value = signatures verified by all ranks / max
elapsed, plus "roofline" (k_dsm vs the measured integer-multiply issue
peak), "cpu_baseline" (the reference's own fd_ed25519_verify compiled from
its sources, oracle/_ref, timed on this host on a bounded sample of the same
workload) and the end-to-end p50/p99 latency of a 4096-signature host batch.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

# The streaming tile keeps 4 GPU batches in flight on 4 HIP streams; with
# HIP's default of 4 hardware queues per process only 2 of them run
# concurrently (measured in round 1 with a concurrency probe), so give the process 8
# (read at HIP runtime init, before any device call; well under the pool's
# limit of 32).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# k_dsm algorithmic work: one field mul = 109 signed
# 32x32->64 multiply-accumulates (100 products + 9 x19 pre-multiplies), one
# square = 60.  Per signature, over the ref10 op flow's useful lanes:
#   N_sq  = 4 (2A) + 4 I                      (I = loop iterations)
#   N_mul = 68 (Ai table) + 3 I + 8 n_h + 7 n_s + 2 (final compare)
MAC_MUL, MAC_SQ = 109, 60
# Decompression (k_decomp), per point: 255 squares + ~19.5 muls.
DECOMP_MAC_PER_SIG = 2 * (255 * MAC_SQ + 19.5 * MAC_MUL)
# Peak: gfx950 issues v_mad_i64_i32 at half rate = 64 lane-ops/clk/CU
# (tools/ubench_valu: 55.3/clk/CU sustained with 16 chains), 256 CUs,
# 2.4 GHz max clock (MI355X_MICROARCH.md chip table).
PEAK_TMAC = 64 * 256 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sigs", "--n", dest="n", type=int, default=1 << 20, help="signatures per GPU per step")
    ap.add_argument("--msg-sz", type=int, default=200)
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="repeat passes over the CPU sample until this much wall time is spent")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-stream", action="store_true", help="skip the streaming-tile sweep (config 5)")
    ap.add_argument("--workload", choices=("sigs", "txn"), default="sigs",
                    help="sigs: configs[1] (default bench line); txn: configs[3] multi-signer transactions")
    ap.add_argument("--stream-frags", type=int, default=1 << 20, help="frags per streaming-tile run")
    return ap.parse_args()


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` at batch n, from the PMC summary
    committed under profiles/ (tools/prof_pmc.sh + tools/pmc_summary.py on
    the same build), scaled linearly from the profiled batch size."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_latest.json")
    try:
        d = json.load(open(path))
        b = d[kernel]["derived"]["hbm_bytes_per_launch"]
        return b * n / d.get("_sigs_per_launch", 262144)
    except (OSError, KeyError, ValueError):
        return None


def make_workload(n, msg_sz, seed):
    """configs[1]: n fresh keypairs, random msg_sz-byte messages, signed on
    the GPU (k_sign, byte-identical to the host / reference signer)."""
    from firedancer_amd import workload
    return workload.sig_batch(n, msg_sz, seed)


def run_txn(args, rank, world, local, dist):
    """configs[3]: GPU-signed multi-signer transactions (1..12 signers,
    64..1232-B messages, legacy + v0), device resident, parsed + verified +
    reduced per transaction on the GPU; weak scaling (each rank its own
    shard of args.n signatures)."""
    from firedancer_amd import hip, workload
    t0 = time.perf_counter()
    payload, toff, tsz, tbase = workload.txn_batch(args.n, 5000 + rank)
    gen_s = time.perf_counter() - t0
    dev = workload.TxnDevice(payload, toff, tsz, tbase)
    stream = hip.Stream()
    for _ in range(args.warmup):
        dev.run(stream.handle)
    stream.synchronize()
    e0, e1 = hip.Event(), hip.Event()
    if dist:
        dist.barrier()
    stream.synchronize()
    t0 = time.perf_counter()
    e0.record(stream.handle)
    for _ in range(args.steps):
        dev.run(stream.handle)
    e1.record(stream.handle)
    stream.synchronize()
    elapsed = time.perf_counter() - t0
    gpu_ms = e0.elapsed_ms(e1) / args.steps
    if dist:
        from firedancer_amd.shard import max_over_ranks
        elapsed = max_over_ranks(elapsed)
        dist.barrier()
    terr, _ = dev.verdicts()
    if rank != 0:
        return
    slots = dev.slot_cnt * args.steps * world
    out = {
        "metric": "ed25519 verifies/sec (node, 1/2/4/8 GPUs); p50 latency @4096-sig batch",
        "value": slots / elapsed, "unit": "verifies/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32x32->int64 (field limbs), u64 (SHA-512)",
        "data": "synthetic: GPU-signed multi-signer transactions, resident in HBM",
        "config": {"workload": "configs[3]: multi-signer txns (1..12 signers, 64..1232-B messages, legacy+v0), "
                               "%d signatures per GPU" % dev.slot_cnt,
                   "txns_per_gpu": dev.txn_cnt, "sigs_per_gpu": dev.slot_cnt, "parallelism": "shard%d" % world},
        "txns_per_s": dev.txn_cnt * args.steps * world / elapsed,
        "gpu_ms_per_step": gpu_ms,
        "verdicts": {"ok": int((terr == 0).sum()), "rejected": int((terr != 0).sum())},
        "mean_payload_sz": float(tsz.mean()), "workload_gen_s": gen_s,
    }
    print(json.dumps(out))


def cpu_baseline(pub, sig, off, sz, blob, sample, threads, gpu_err, seconds):
    """The reference's fd_ed25519_verify (oracle/_ref, compiled from its own
    sources) on `threads` host threads; falls back to the clean-room port.
    Bounded sample: passes over the first `sample` signatures of the bench
    batch until `seconds` of wall time are spent (about 10 s by default)."""
    import ctypes
    n = min(sample, pub.shape[0])
    err = np.zeros(n, np.int8)
    vp = ctypes.c_void_p
    args = [ctypes.c_uint64(n), pub.ctypes.data_as(vp), sig.ctypes.data_as(vp), off.ctypes.data_as(vp),
            sz.ctypes.data_as(vp), blob.ctypes.data_as(vp), err.ctypes.data_as(vp)]
    refso = os.path.join(ROOT, "oracle", "_ref", "libfdref_batch.so")
    if os.path.exists(refso):
        L = ctypes.CDLL(refso)
        fn, kind = L.ref_ed25519_verify_batch, "reference"
        fn.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        call = lambda: fn(*args, threads)  # noqa: E731
    else:
        L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        fn, kind = L.oracle_ed25519_verify_batch, "port"
        fn.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        call = lambda: fn(*args, None, threads)  # noqa: E731
    t0 = time.perf_counter()
    passes = 0
    while True:
        call()
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": passes * n / dt, "unit": "verifies/s", "cores": threads, "kind": kind,
            "sample": "%d passes over %d of the bench batch's %d-B signatures, %d threads, %.1f s wall"
                      % (passes, n, int(sz[0]), threads, dt),
            "verdicts_equal_gpu": bool(np.array_equal(err, gpu_err[:n]))}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from firedancer_amd import ed25519, hip

    ndev = hip.device_count()
    if os.environ.get("FD_AMD_DEVICE_MAP") == "mod" and ndev:   # rehearsal: more ranks than GPUs
        local = local % ndev
    if ndev <= local:
        raise SystemExit("bench.py: no HIP device %d visible" % local)
    hip.set_device(local)

    if args.workload == "txn":
        return run_txn(args, rank, world, local, dist)

    n = args.n
    t0 = time.perf_counter()
    pub, sig, off, sz, blob = make_workload(n, args.msg_sz, 1000 + rank)
    gen_s = time.perf_counter() - t0

    d = {k: hip.DeviceBuffer.from_array(v) for k, v in
         dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
    d_err = hip.DeviceBuffer(n)
    d_ws = hip.DeviceBuffer(ed25519.workspace_footprint(n))
    d_stats = hip.DeviceBuffer(4 * 3 * n)
    stream = hip.Stream()
    run = lambda ev=None: ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr,  # noqa: E731
                                                 d["blob"].ptr, d_err.ptr, d_ws.ptr, stream.handle, ev)

    for _ in range(args.warmup):
        run()
    stream.synchronize()

    evs = [[hip.Event() for _ in range(4)] for _ in range(args.steps)]
    if dist:
        dist.barrier()
    stream.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        run(evs[k])
    stream.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()

    stage_ms = np.zeros(3)
    for ev in evs:
        for j in range(3):
            stage_ms[j] += ev[j].elapsed_ms(ev[j + 1])
    stage_ms /= args.steps

    err = d_err.to_array(np.int8, n)
    ed25519.work_stats_dev(n, d_ws.ptr, d_stats.ptr, stream.handle)
    stream.synchronize()
    st = d_stats.to_array(np.uint32, 3 * n).reshape(3, n).astype(np.float64)
    I, nh, ns = st[0].sum(), st[1].sum(), st[2].sum()
    live = float((st[0] > 0).sum())
    dsm_mac = MAC_MUL * (68 * live + 3 * I + 8 * nh + 7 * ns + 2 * live) + MAC_SQ * (4 * live + 4 * I)
    achieved = dsm_mac / (stage_ms[2] * 1e-3) / 1e12
    traffic = pmc_traffic("k_dsm", n)

    if rank != 0:
        return
    total = n * args.steps * world
    out = {
        "metric": "ed25519 verifies/sec (node, 1/2/4/8 GPUs); p50 latency @4096-sig batch",
        "value": total / elapsed,
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32x32->int64 (field limbs), u64 (SHA-512)",
        "data": "synthetic: fresh random keypairs and messages, signed on the GPU (k_sign), inputs resident in HBM",
        "config": {"workload": "configs[1]: 1xMI355X batch of 2^20 single-signer sigs, 200-byte messages",
                   "sigs_per_gpu_per_step": n, "msg_sz": args.msg_sz, "parallelism": "shard%d" % world},
        "stage_ms": {"k_prep": stage_ms[0], "k_decomp": stage_ms[1], "k_dsm": stage_ms[2]},
        "verdicts": {"ok": int((err == 0).sum()), "rejected": int((err != 0).sum())},
        "roofline": {"bound": "valu-imad64", "kernel": "k_dsm", "achieved": achieved, "peak": PEAK_TMAC,
                     "unit": "TMAC/s", "frac": achieved / PEAK_TMAC, "traffic": traffic,
                     "traffic_note": "HBM bytes per launch from the committed PMC pass (profiles/r01_pmc_latest.json: "
                                     "2*FETCH_SIZE+WRITE_SIZE KB, gfx950 correction), scaled to this batch",
                     "mac_per_sig": dsm_mac / max(live, 1.0)},
        "workload_gen_s": gen_s,
    }
    if not args.no_latency:
        lat = []
        eng = ed25519.Engine(device=local, batch_max=4096, blob_max=4096 * args.msg_sz)
        m = 4096
        b_off = (np.arange(m, dtype=np.uint32) * args.msg_sz).astype(np.uint32)
        for r in range(30):
            lo = (r * m) % max(1, n - m)
            sub_blob = blob[off[lo]:off[lo] + m * args.msg_sz]
            t1 = time.perf_counter()
            eng.verify_soa(pub[lo:lo + m], sig[lo:lo + m], b_off, sz[lo:lo + m], sub_blob)
            lat.append((time.perf_counter() - t1) * 1e3)
        eng.close()
        lat = np.array(lat[3:])
        out["latency_ms_4096"] = {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                                  "path": "host SoA -> pinned staging -> H2D -> 3 kernels -> D2H"}
    if not args.no_latency:
        # PCIe-inclusive rate: the same 2^20 batch handed over as host SoA
        # buffers (pinned double-buffered staging, chunks of 2^17), priced
        # against the measured pinned H2D ceiling.  Never the headline value.
        chunk = 1 << 17
        eng = ed25519.Engine(device=local, batch_max=chunk, blob_max=chunk * args.msg_sz)
        eng.verify_soa(pub[:chunk], sig[:chunk], off[:chunk], sz[:chunk], blob)
        reps, t1 = 3, time.perf_counter()
        for _ in range(reps):
            herr = eng.verify_soa(pub, sig, off, sz, blob)
        dt = (time.perf_counter() - t1) / reps
        eng.close()
        h2d_gbs = hip.h2d_bandwidth()
        per_sig = 104 + args.msg_sz
        out["host_soa"] = {"verifies_per_s": n / dt, "chunk": chunk, "h2d_bytes_per_sig": per_sig,
                           "h2d_gb_per_s": n * per_sig / dt / 1e9, "pinned_h2d_peak_gb_per_s": h2d_gbs,
                           "pcie_bound_verifies_per_s": h2d_gbs * 1e9 / per_sig,
                           "verdicts_match_resident": bool((herr == err).all()),
                           "path": "host SoA -> pinned packed staging (2 chunks in flight) -> H2D -> kernels -> D2H"}
    if world == 1 and not args.no_stream:
        # config 5: tango mcache/dcache feed -> verify tile -> consumer, per batch cap
        from firedancer_amd import tango
        m = min(n, 1 << 16)
        rows = []
        for bmax in (256, 1024, 4096, 16384):
            row = {"batch_max": bmax}
            for zc in (False, True):
                key = "zero_copy" if zc else "copy"
                sat = tango.bench_stream(local, bmax, 0, pub[:m], sig[:m], off[:m], sz[:m], blob, args.stream_frags,
                                         zero_copy=zc)
                rr = {"saturated_frags_per_s": sat["frags_per_s"], "saturated_mean_batch": sat["mean_batch"]}
                for load in (0.5, 0.8):
                    rate = load * sat["frags_per_s"]
                    nf = int(min(args.stream_frags, max(20000, rate * 1.0)))
                    r = tango.bench_stream(local, bmax, 0, pub[:m], sig[:m], off[:m], sz[:m], blob, nf, rate=rate,
                                           zero_copy=zc)
                    rr["at_%d%%" % int(load * 100)] = {"offered_frags_per_s": rate, "frags_per_s": r["frags_per_s"],
                                                        "p50_us": r["p50_ns"] / 1e3, "p99_us": r["p99_ns"] / 1e3,
                                                        "mean_batch": r["mean_batch"]}
                row[key] = rr
            rows.append(row)
        out["stream_tile"] = {"path": "producer (metadata only; frames pre-placed in the data region as a NIC would) "
                                      "-> in mcache/dcache -> verify tile (adaptive GPU batches, 4 in flight; copy: "
                                      "host staging, zero_copy: GPU-mapped data region) -> out mcache -> consumer; "
                                      "latency = scheduled send to tile publish",
                              "frags_per_run": args.stream_frags, "rows": rows}
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(pub, sig, off, sz, blob, args.cpu_sample, args.cpu_threads, err,
                                           args.cpu_seconds)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
