#!/usr/bin/env python3
"""bench.py -- ed25519 verifies/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n SIGS] [--msg-sz B]
    python bench.py --workload txn [--total-sigs 16777216]

Default (configs[1]): a "step" is one pass of the verify pipeline (k_prep ->
k_decomp -> the double-scalar multiply: k_ai + k_dsmp + k_fin at this size)
over one batch of n synthetic signatures (2^20 single-signer signatures,
200-byte Solana-txn-sized messages, fresh random keypairs), with the inputs
already resident in HBM when the timed region starts.  Consecutive steps
alternate between --streams (default 4) stream/workspace sets: four
batches in flight (the runtime maps them onto two of its hardware queues;
GPU_MAX_HW_QUEUES=8 did not help, profiles/r05_ab_hwq.txt; three measured +2 % over two:
a batch's multiply starts in the previous one's drain and the fronts queue
behind fewer multiplies, profiles/r02_k_dsmp_pool_ab.txt; four +1.0 % over
three and six -0.5 %, interleaved on one box, profiles/r05_ab_streams.txt).  For N > 1 (launched by torch.distributed.run) every rank verifies
its own batch of n signatures on its own GPU -- signatures are independent,
so there is no data-path collective (weak scaling); gloo is used only for
the start/stop barriers and the max-over-ranks of the time.

--workload txn (configs[3]): 2^24 signatures in multi-signer transactions
(1..12 signers, 64..1232-B messages, legacy + v0), split across the ranks
by contiguous shards (strong scaling: the total is fixed); a step parses,
verifies and reduces every transaction of the rank's shard on its GPU.

Rank 0 prints ONE JSON line: value = signatures verified by all ranks / max
elapsed, plus "roofline" (the double-scalar-multiply stage of one batch
alone vs the integer-multiply issue peak), "cpu_baseline" (the reference's own fd_ed25519_verify compiled from
its sources, oracle/_ref, timed on every host core of this box on a
bounded sample of the same workload), the end-to-end p50/p99 latency of a
4096-signature host batch, the drop-in single-call latency, the
PCIe-inclusive host paths and the streaming tile sweep (config 5).
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

import numpy as np

# HIP's hardware-queue count is left as the process finds it (the box
# default is 4, HIP's own): the streaming tile runs one persistent kernel on
# one stream, and the resident batches use --streams (4) streams.  The value
# in effect is reported in the JSON line (config.hip_hw_queues).
HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES", "default (4)")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ed25519 verifies/sec (node, 1/2/4/8 GPUs); p50 latency @4096-sig batch"
DTYPE = "int32x32->int64 (field limbs), u64 (SHA-512)"
# k_dsm algorithmic work: one field mul = 109 signed
# 32x32->64 multiply-accumulates (100 products + 9 x19 pre-multiplies), one
# square = 60.  Per signature, over the ref10 op flow's useful lanes:
#   N_sq  = 4 (2A) + 4 I                      (I = loop iterations)
#   N_mul = 68 (Ai table) + 3 I + 8 n_h + 7 n_s + 2 (final compare)
MAC_MUL, MAC_SQ = 109, 60
# Peak: gfx950 issues v_mad_i64_i32 at half rate = 64 lane-ops/clk/CU
# (tools/ubench_valu: 55.3/clk/CU sustained with 16 chains), 256 CUs,
# 2.4 GHz max clock (MI355X_MICROARCH.md chip table).
PEAK_TMAC = 64 * 256 * 2.4e9 / 1e12
# the reference's single-thread fd_ed25519_verify at 200-B messages on the
# build container
REF_US_PER_CALL_SURVEY = 53.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sigs", "--n", dest="n", type=int, default=1 << 20, help="signatures per GPU per step")
    ap.add_argument("--msg-sz", type=int, default=200)
    ap.add_argument("--dsm-kernel", choices=("default", "k_dsm", "k_dsmp"), default="default",
                    help="throughput double-scalar-mult kernel (A/B; default: the library's size rule)")
    ap.add_argument("--streams", type=int, default=4,
                    help="batches in flight (consecutive steps alternate streams / workspaces)")
    ap.add_argument("--total-sigs", type=int, default=1 << 24,
                    help="txn workload: signatures over all ranks (strong scaling)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="repeat passes over the CPU sample until this much wall time is spent")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-stream", action="store_true", help="skip the streaming-tile sweep (config 5)")
    ap.add_argument("--workload", choices=("sigs", "txn"), default="sigs",
                    help="sigs: configs[1] (default bench line); txn: configs[3] multi-signer transactions")
    ap.add_argument("--stream-frags", type=int, default=1 << 25,
                    help="frags per saturated streaming-tile run (2^25: ~0.6 s at saturation, so the run's ramp "
                         "and drain -- ~5 ms in all -- weigh under 1 %% of the whole-run rate, as for a tile that "
                         "runs continuously; 2^23 gave whole-run rates ~4 %% under the steady ones)")
    ap.add_argument("--paced-seconds", type=float, default=0.5,
                    help="length of a paced streaming-tile run (latency over its steady state: after its first 20 ms)")
    ap.add_argument("--txn-full-check", action="store_true",
                    help="--workload txn: re-verify every transaction with the compiled reference (slow)")
    ap.add_argument("--no-host-fed", action="store_true",
                    help="skip the all-rank registered-host-memory pass (host_fed_node)")
    ap.add_argument("--multi-engine", action="store_true",
                    help="one process drives --gpus devices through the native multi-device engine "
                         "(fd_ed25519_amd_multi_verify_soa) on host buffers; prints its own JSON line")
    ap.add_argument("--detail", default=None,
                    help="where rank 0 writes the full record (default gpurun_out/bench_detail_*.json); stdout "
                         "carries only the compact line")
    return ap.parse_args()


# ---------------------------------------------------------------- host facts

def cgroup_throttle():
    """(nr_throttled, throttled_usec) of this process's cgroup (v2 cpu.stat),
    or None: a paced tile run that the CPU quota throttled shows its stalls
    here, not in the tile."""
    try:
        st = dict(ln.split() for ln in open("/sys/fs/cgroup/cpu.stat") if ln.strip())
        return int(st.get("nr_throttled", 0)), int(st.get("throttled_usec", 0))
    except (OSError, ValueError):
        return None


def host_cores():
    """Cores this process may use: the affinity set, capped by a cgroup CPU
    quota and by the host share the pool grants a one-GPU box
    (OMP_NUM_THREADS, set to it there) -- the machine itself may show many
    more CPUs than the box owns."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    share = None
    try:
        share = int(os.environ["OMP_NUM_THREADS"])
    except (KeyError, ValueError):
        pass
    cap = min(x for x in (aff, quota, share) if x)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return cap, aff, {"cgroup_quota": quota, "omp_num_threads": share, "machine_cpus": os.cpu_count()}, model


def ref_batch_lib():
    """The reference's own verify (oracle/_ref, compiled from its sources in
    the build container).  The CPU baseline is the reference itself: no
    silent fallback to the port."""
    import ctypes
    path = os.path.join(ROOT, "oracle", "_ref", "libfdref_batch.so")
    if not os.path.exists(path):
        raise SystemExit("bench.py: %s missing -- build it with __graft_entry__.build() in a container that has "
                         "/root/reference (or pass --no-cpu)" % path)
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.ref_ed25519_verify_batch.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, vp, vp, ctypes.c_int]
    L.ref_txn_verify_batch.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int]
    return L


def _vp(a):
    import ctypes
    return ctypes.c_void_p(a.ctypes.data)


def timed_passes(call, seconds):
    t0 = time.perf_counter()
    passes = 0
    while True:
        call()
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return passes, dt


def cpu_baseline(pub, sig, off, sz, blob, sample, threads, gpu_err, seconds):
    """The reference's fd_ed25519_verify (oracle/_ref) on every host core,
    then on one core.  Bounded sample: passes over the first `sample`
    signatures of the bench batch until `seconds` of wall time are spent."""
    L = ref_batch_lib()
    cores, aff, quota, model = host_cores()
    nt = threads or cores
    n = min(sample, pub.shape[0])
    err = np.zeros(n, np.int8)
    args = [n, _vp(pub), _vp(sig), _vp(off), _vp(sz), _vp(blob), _vp(err)]
    passes, dt = timed_passes(lambda: L.ref_ed25519_verify_batch(*args, nt), seconds)
    n1 = min(n, 1 << 15)
    args1 = [n1] + args[1:]
    p1, dt1 = timed_passes(lambda: L.ref_ed25519_verify_batch(*args1, 1), min(3.0, seconds))
    per_core = p1 * n1 / dt1
    return {"value": passes * n / dt, "unit": "verifies/s", "cores": nt, "kind": "reference",
            "sample": "%d passes over %d of the bench batch's %d-B signatures on %d threads, %.1f s wall; "
                      "single-thread: %d passes over %d" % (passes, n, int(sz[0]), nt, dt, p1, n1),
            "per_core_verifies_per_s": per_core, "us_per_call_1_thread": 1e6 / per_core,
            "host": {"cpu_model": model, "usable_cores": cores, "affinity_cpus": aff, "limits": quota},
            "verdicts_equal_gpu": bool(np.array_equal(err, gpu_err[:n]))}


# ---------------------------------------------------------------- workloads

def make_workload(n, msg_sz, seed):
    """configs[1]: n fresh keypairs, random msg_sz-byte messages, signed on
    the GPU (k_sign, byte-identical to the host / reference signer)."""
    from firedancer_amd import workload
    return workload.sig_batch(n, msg_sz, seed)


def dsm_kernels(n, choice):
    """The double-scalar-mult launches a resident batch of n runs: the pooled
    k_ai + k_dsmp + k_fin from the library's pool threshold up, else k_dsm."""
    from firedancer_amd import ed25519
    pooled = choice == "k_dsmp" or (choice == "default" and n >= ed25519.POOL_BATCH_MIN_DEFAULT)
    return ["k_ai", "k_dsmp", "k_fin"] if pooled else ["k_dsm"]


def dsm_roofline(st, kernel_ms, n, kernel="k_dsm", note=None):
    """Algorithmic double-scalar-mult multiply-accumulates (from the kernels'
    own work statistics) per launch / the DSM stage's time, against the
    integer-multiply peak.  kernel: '+'-joined launch names of the stage."""
    st = st.astype(np.float64)
    I, nh, ns = st[0].sum(), st[1].sum(), st[2].sum()
    live = float((st[0] > 0).sum())
    mac = MAC_MUL * (68 * live + 3 * I + 8 * nh + 7 * ns + 2 * live) + MAC_SQ * (4 * live + 4 * I)
    achieved = mac / (kernel_ms * 1e-3) / 1e12
    names = kernel.split("+") if "(" not in kernel else []
    traffic = [pmc_traffic(k, n) for k in names] or [None]
    raw = [pmc_traffic(k, n, corrected=False) for k in names] or [None]
    r = {"bound": "valu-imad64", "kernel": kernel, "achieved": achieved, "peak": PEAK_TMAC, "unit": "TMAC/s",
         "frac": achieved / PEAK_TMAC, "traffic": None if None in traffic else sum(traffic),
         "traffic_raw": None if None in raw else sum(raw),
         "traffic_note": "HBM bytes per launch from the committed PMC pass (profiles/%s), scaled to this batch: "
                         "traffic = 2*FETCH_SIZE+WRITE_SIZE (the guide's gfx950 FETCH correction, stated for wide "
                         "coalesced reads), traffic_raw = FETCH_SIZE+WRITE_SIZE (k_dsmp's reads are 16-B row "
                         "gathers and one-word event pops, so the truth may lie nearer the raw figure)"
                         % os.path.basename(pmc_summary_path() or "none"),
         "mac_per_sig": mac / max(live, 1.0)}
    # the same MACs over the committed rocprofv3 kernel durations of the stage (a profiler-timed figure beside
    # the HIP-event one), and against the clock the chip held under the kernel (GRBM_GUI_ACTIVE / 8 XCDs over
    # the kernel's duration) instead of the 2.4 GHz the peak assumes
    rp = rocprof_stage_ms(names) if names else None
    if rp:
        ms, src = rp
        r["rocprof_stage_ms"] = ms
        r["frac_rocprof"] = mac / (ms * 1e-3) / 1e12 / PEAK_TMAC
        r["rocprof_source"] = "profiles/" + os.path.basename(src)
        clk = held_clock_ghz("k_dsmp" if "k_dsmp" in names else names[-1])
        if clk:
            r["held_clock_ghz"] = clk
            r["frac_at_held_clock"] = achieved / (64 * 256 * clk * 1e9 / 1e12)
    if note:
        r["note"] = note
    return r


def dsm_in_pipeline(st, ms_per_step, stage_ms, n):
    """Derived, not an event timing: the step time of the timed region minus
    the lone-batch k_prep and k_decomp times, i.e. what the double-scalar
    multiply adds per batch when batches overlap, and the MAC rate that
    implies against the same peak."""
    ms = ms_per_step - stage_ms[0] - stage_ms[1]
    r = dsm_roofline(st, ms, n, kernel="pipeline")
    return {"dsm_ms": ms, "achieved": r["achieved"], "frac": r["frac"], "unit": "TMAC/s",
            "note": "ms_per_step - k_prep - k_decomp (lone-batch event times); a derived share, not a kernel "
                    "duration"}


def pmc_summary_path():
    """The newest round's committed PMC summary (profiles/rNN_pmc_latest.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_latest.json")))
    return paths[-1] if paths else None


def pmc_traffic(kernel, n, corrected=True):
    """HBM bytes per launch of `kernel` at batch n, from the PMC summary
    committed under profiles/ (tools/prof_pmc.sh + tools/pmc_summary.py on
    the same build), scaled linearly from the profiled batch size.
    corrected: 2*FETCH_SIZE+WRITE_SIZE (the guide's gfx950 correction), else
    FETCH_SIZE+WRITE_SIZE as counted."""
    path = pmc_summary_path()
    try:
        d = json.load(open(path or ""))
        der = d[kernel]["derived"]
        b = der["hbm_bytes_per_launch"] if corrected else (der["fetch_kb_raw"] + der["write_kb_raw"]) * 1024
        return b * n / d.get("_sigs_per_launch", 262144)
    except (OSError, KeyError, ValueError):
        return None


def rocprof_stats_path():
    """The newest round's committed rocprofv3 --stats summary of the headline
    kernels (profiles/rNN_rocprof_kernel_stats.csv, tools/final_measure.sh)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_rocprof_kernel_stats.csv")))
    return paths[-1] if paths else None


def rocprof_stage_ms(names):
    """Sum of the rocprofv3 average durations of the launches `names`, ms, and the file; None if missing."""
    import csv
    path = rocprof_stats_path()
    try:
        rows = list(csv.DictReader(open(path or "")))
        avg = {r["Name"].split("(")[0]: float(r["AverageNs"]) for r in rows}
        return sum(avg[k] for k in names) / 1e6, path
    except (OSError, KeyError, ValueError):
        return None


def held_clock_ghz(kernel):
    """The clock the chip held under `kernel`: GRBM_GUI_ACTIVE of the committed PMC pass / 8 XCDs over the
    kernel's committed rocprofv3 average duration (GHz), or None."""
    try:
        d = json.load(open(pmc_summary_path() or ""))
        busy = d[kernel]["counters"]["GRBM_GUI_ACTIVE"] / 8.0
        ms, _ = rocprof_stage_ms([kernel])
        return busy / (ms * 1e-3) / 1e9
    except (OSError, KeyError, ValueError, TypeError):
        return None


LINE_MAX = 6000   # the driver parses the final stdout line; round 4's 38 KB line did not parse


def write_detail(out, args):
    """The whole record (every paced run, decompositions, stall clocks) goes
    to a side file; stdout carries only the compact line."""
    path = args.detail or os.path.join(ROOT, "gpurun_out", "bench_detail_%s_n%d_%d.json"
                                       % (out.get("mode", args.workload), out["n_gpus"], int(time.time())))
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    except OSError as e:
        return "unwritten (%s)" % e
    return os.path.relpath(path, ROOT)


def _r(x, nd=4):
    """Round for the compact line: 4 significant digits."""
    if isinstance(x, float):
        return float("%.*g" % (nd, x))
    return x


def _pick(d, keys):
    return {k: _r(d[k]) for k in keys if d is not None and k in d}


# a paced run whose harness threads stalled: the producer (the NIC's stand-in) ran late by more than its longest
# wait for input credit (that wait is the tile holding its input, never excused), or the consumer (the dedup
# tile's stand-in) stopped polling for this long; the tile's own threads' stalls are not excused
HARNESS_STALL_US = {"producer_late_max": 1000.0, "consumer_gap_max": 2000.0}


def harness_stalled(run):
    st = run.get("stalls_us", {})
    late = st.get("producer_late_max", 0.0) - st.get("producer_credit_wait_max", 0.0)
    return late > HARNESS_STALL_US["producer_late_max"] or \
        st.get("consumer_gap_max", 0.0) > HARNESS_STALL_US["consumer_gap_max"]


def worst_of(rs):
    """The worst run's p99 / p50 over all runs, and over the runs whose harness threads did not stall
    (None when every run stalled); both are reported, the first is the row check."""
    worst = max(rs, key=lambda x: x["p99_over_p50"])
    clean = [x for x in rs if not harness_stalled(x)]
    return worst, (max(x["p99_over_p50"] for x in clean) if clean else None), len(rs) - len(clean)


TOPUP_MAX = 3   # extra paced runs per load, only while fewer than three runs are free of harness stalls


def top_up(rs, run):
    """Run more paced runs (run() -> one run) while fewer than three of rs are free of harness stalls,
    at most TOPUP_MAX of them: a producer descheduled for 0.1-0.3 s (seen on busy boxes) otherwise decides
    the row's median p50 when it hits two of three runs.  Every run, extra ones included, stays in rs and
    in the all-runs tail check."""
    extra = 0
    while sum(not harness_stalled(x) for x in rs) < 3 and extra < TOPUP_MAX:
        rs.append(run())
        extra += 1
    return extra


def p50_run(rs):
    """The run whose p50 is the row's: the median over the runs free of harness stalls (all runs when
    none is)."""
    clean = [x for x in rs if not harness_stalled(x)] or rs
    return sorted(clean, key=lambda x: x["p50_us"])[len(clean) // 2]


def unstalled_ok(loads):
    """Every load's stall-free runs within 2.5 x p50; a load whose every run had a harness stall vouches for
    nothing, so it fails the check (VERDICT/ADVICE r05: it used to pass)."""
    return all(x["worst_p99_over_p50_unstalled"] is not None and x["worst_p99_over_p50_unstalled"] <= 2.5
               for x in loads)


def tile_summary(st):
    """One entry per streaming-tile row: saturated whole-run / steady rate,
    roofline frac, median p50 and the WORST run's p99 / p50 at each load."""
    rows = []
    for row in st["rows"]:
        for key in ("copy", "zero_copy"):
            if key not in row:
                continue
            r = row[key]
            e = {"bmax": row["batch_max"], "mode": key, "sat": _r(r["saturated_frags_per_s"]),
                 "steady": _r(r["saturated_steady_frags_per_s"]), "ok": r["check_mismatches"] == 0}
            if "roofline" in r:
                e["frac"] = _r(r["roofline"]["frac"], 3)
                e["frac_steady"] = _r(r["roofline"]["frac_steady"], 3)
            for load in ("50", "80"):
                a = r["at_%s%%" % load]
                e["p50_us_" + load] = _r(a["p50_us"])
                e["worst_p99_us_" + load] = _r(a["worst_p99_us"])
                e["worst_x_" + load] = _r(a["worst_p99_over_p50"], 3)
                if a.get("harness_stalled_runs"):
                    e["stalled_runs_" + load] = a["harness_stalled_runs"]
                    e["worst_x_unstalled_" + load] = _r(a["worst_p99_over_p50_unstalled"], 3)
            rows.append(e)
    s = {"all_checks_pass": st["all_checks_pass"],
         "every_row_worst_p99_within_2_5x_p50": st["every_row_p99_within_2_5x_p50"],
         "every_row_worst_p99_within_2_5x_p50_runs_without_harness_stalls":
             st["every_row_p99_within_2_5x_p50_unstalled"],
         "every_row_p50_nondecreasing_with_load": st["every_row_p50_nondecreasing_with_load"],
         "min_p50_ratio_80_over_50": _r(min(r["at_80%"]["p50_us"] / max(r["at_50%"]["p50_us"], 1e-3)
                                            for row in st["rows"] for k, r in row.items() if k in ("copy", "zero_copy")), 4),
         "frags_per_run": st["frags_per_run"], "rows": rows}
    fx = st.get("fixed_1M_frags_per_s_batch_max_4096")
    if fx:
        s["fixed_1M_4096"] = {k: {"p50_us": _r(v["p50_us"]), "p99_us": _r(v["p99_us"])} for k, v in fx.items()}
    tx = st.get("txn_framing")
    if tx:
        s["txn_framing"] = []
        for r in tx["rows"]:
            e = {"bmax": r["batch_max"], "txns_per_s": _r(r["saturated_txns_per_s"]),
                 "verifies_per_s": _r(r["saturated_verifies_per_s"]),
                 "steady_verifies_per_s": _r(r["saturated_steady_verifies_per_s"]), "ok": r["check_mismatches"] == 0}
            for ld in ("50", "80"):
                a = r["at_%s%%" % ld]
                e["p50_us_" + ld] = _r(a["p50_us"])
                e["worst_p99_us_" + ld] = _r(a["worst_p99_us"])
                e["worst_x_" + ld] = _r(a["worst_p99_over_p50"], 3)
                if a.get("harness_stalled_runs"):
                    e["stalled_runs_" + ld] = a["harness_stalled_runs"]
                    e["worst_x_unstalled_" + ld] = _r(a["worst_p99_over_p50_unstalled"], 3)
            s["txn_framing"].append(e)
        s["every_row_worst_p99_within_2_5x_p50"] = s["every_row_worst_p99_within_2_5x_p50"] and \
            all(r["p99_within_2_5x_p50"] for r in tx["rows"])
        s["every_row_worst_p99_within_2_5x_p50_runs_without_harness_stalls"] = \
            s["every_row_worst_p99_within_2_5x_p50_runs_without_harness_stalls"] and \
            all(r["p99_within_2_5x_p50_unstalled"] for r in tx["rows"])
        s["all_checks_pass"] = s["all_checks_pass"] and all(r["check_mismatches"] == 0 for r in tx["rows"])
    return s


def node_summary(nt):
    return {"ranks": nt["ranks"], "saturated_frags_per_s_node": _r(nt["saturated_frags_per_s_node"]),
            "at_50%_frags_per_s_node": _r(nt["at_50%_frags_per_s_node"]),
            "per_rank": [[_r(p["saturated_frags_per_s"]), _r(p["at_50%"]["p50_us"]), _r(p["at_50%"]["p99_us"]),
                          p["cpus"], p["device"]] for p in nt["per_rank"]],
            "per_rank_cols": ["saturated_frags_per_s", "p50_us@50%", "p99_us@50%", "cpus", "device"]}


def compact_line(out, detail):
    """The driver's line: the mandated keys, roofline, cpu_baseline,
    latency_ms_4096 and per-row tile summaries; everything else is in the
    side file `detail`."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "mode", "txns_per_s")
    line = {k: _r(out[k], 6) if k in ("value", "ms_per_step") else out[k] for k in keep if k in out}
    line["config"] = out["config"]
    if out.get("roofline"):
        line["roofline"] = _pick(out["roofline"], ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                                                   "traffic_raw", "mac_per_sig", "frac_rocprof", "rocprof_source",
                                                   "held_clock_ghz", "frac_at_held_clock"))
        line["roofline"]["traffic_unit"] = "bytes per launch (PMC)"
    if out.get("cpu_baseline"):
        cb = out["cpu_baseline"]
        line["cpu_baseline"] = _pick(cb, ("value", "unit", "cores", "kind", "sample", "verdicts_equal_gpu",
                                          "us_per_call_1_thread"))
        line["cpu_baseline"]["cpu_model"] = cb.get("host", {}).get("cpu_model")
    for k in ("latency_ms_4096", "latency_ms_4096_registered"):
        if k in out:
            line[k] = _pick(out[k], ("p50", "p99"))
    if "dropin_call_us" in out:
        line["dropin_call_us"] = _pick(out["dropin_call_us"], ("p50", "p99", "reference_us_per_call_this_host"))
    if "stage_ms" in out:
        line["stage_ms"] = _pick(out["stage_ms"], ("k_prep", "k_decomp", "k_dsm"))
    if out.get("dsm_in_pipeline"):
        line["dsm_in_pipeline_frac"] = _r(out["dsm_in_pipeline"]["frac"])
    for k in ("host_soa", "host_fed_node"):
        if out.get(k):
            line[k + "_verifies_per_s"] = _r(out[k]["verifies_per_s"])
    if "verdicts" in out:
        line["verdicts"] = {k: v for k, v in out["verdicts"].items() if not isinstance(v, dict)}
    # the summaries never cost the line: a summary that fails says so (the detail file has the record)
    if "stream_tile" in out:
        try:
            line["stream_tile"] = tile_summary(out["stream_tile"])
        except (KeyError, TypeError, ValueError, ZeroDivisionError) as e:
            line["stream_tile"] = {"summary_error": repr(e)[:200]}
    if out.get("stream_tile_node"):
        try:
            line["stream_tile_node"] = node_summary(out["stream_tile_node"])
        except (KeyError, TypeError, ValueError, ZeroDivisionError) as e:
            line["stream_tile_node"] = {"summary_error": repr(e)[:200]}
    line["detail"] = detail
    s = json.dumps(line, separators=(",", ":"))
    if len(s) > LINE_MAX:   # never let the line outgrow the driver's parser: drop the bulkiest parts first
        for k in ("stream_tile_node", "stream_tile"):
            if k in line and len(s) > LINE_MAX:
                line[k] = {"dropped": "line over %d B; see detail" % LINE_MAX}
                s = json.dumps(line, separators=(",", ":"))
    return s


def emit(out, args):
    print(compact_line(out, write_detail(out, args)), flush=True)


def gather_sum(dist, values):
    if not dist:
        return values
    import torch
    t = torch.tensor(values, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


# ---------------------------------------------------------------- configs[3]

def run_txn(args, rank, world, dist):
    """configs[3]: GPU-signed multi-signer transactions (1..12 signers,
    64..1232-B messages, legacy + v0), device resident; args.total_sigs
    signatures split across the ranks (strong scaling), each rank parsing,
    verifying and reducing its shard on its GPU."""
    from firedancer_amd import ed25519, hip, workload
    from firedancer_amd.shard import max_over_ranks, shard_range
    lo, hi = shard_range(args.total_sigs, rank, world)
    t0 = time.perf_counter()
    payload, toff, tsz, tbase = workload.txn_batch(hi - lo, 5000 + rank)
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
    elapsed = max_over_ranks(elapsed)
    terr, _ = dev.verdicts()
    d_stats = hip.DeviceBuffer(4 * 3 * max(dev.slot_cnt, 1))
    ed25519.work_stats_dev(dev.slot_cnt, dev.d_ws.ptr, d_stats.ptr, stream.handle)
    stream.synchronize()
    st = d_stats.to_array(np.uint32, 3 * dev.slot_cnt).reshape(3, dev.slot_cnt)
    rej = np.nonzero(terr)[0]
    slots, txns, nrej = gather_sum(dist, [float(dev.slot_cnt), float(dev.txn_cnt), float(rej.size)])
    if dist:
        dist.barrier()
    if rank != 0:
        return
    out = {
        "metric": METRIC, "value": slots * args.steps / elapsed, "unit": "verifies/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": DTYPE,
        "data": "synthetic: GPU-signed multi-signer transactions, resident in HBM",
        "config": {"workload": "configs[3]: %d signatures in multi-signer txns (1..12 signers, 64..1232-B messages, "
                               "legacy+v0), contiguous shards over %d GPU(s)" % (int(slots), world),
                   "total_sigs": int(slots), "total_txns": int(txns), "sigs_rank0": dev.slot_cnt,
                   "parallelism": "shard%d" % world},
        "txns_per_s": txns * args.steps / elapsed,
        "gpu_ms_per_step_rank0": gpu_ms,
        "roofline": dsm_roofline(st, gpu_ms, dev.slot_cnt, kernel="txn pass (parse+k_prep+k_decomp+k_dsm+reduce)",
                                 note="whole-pass GPU time in the denominator: a lower bound on k_dsm's fraction"),
        "verdicts": {"ok_txns": int(txns - nrej), "rejected_txns": int(nrej)},
        "mean_payload_sz": float(tsz.mean()), "workload_gen_s_rank0": gen_s,
    }
    if world == 1 and not args.no_cpu:
        # CPU baseline: the reference's fd_txn_parse + fd_ed25519_verify on
        # every core over a bounded sample of the same transactions; and the
        # re-check of every rejected transaction by the reference itself
        L = ref_batch_lib()
        cores, aff, quota, model = host_cores()
        nt = args.cpu_threads or cores
        k = min(toff.size, 1 << 17)
        err = np.zeros(k, np.int8)
        passes, dt = timed_passes(lambda: L.ref_txn_verify_batch(k, _vp(payload), _vp(toff), _vp(tsz), _vp(err), nt),
                                  args.cpu_seconds)
        sig_k = int(tbase[k])
        out["cpu_baseline"] = {"value": passes * sig_k / dt, "unit": "verifies/s", "cores": nt, "kind": "reference",
                               "sample": "%d passes over the first %d transactions (%d signatures) on %d threads, "
                                         "%.1f s wall" % (passes, k, sig_k, nt, dt),
                               "host": {"cpu_model": model, "usable_cores": cores, "affinity_cpus": aff,
                                        "limits": quota},
                               "verdicts_equal_gpu": bool(np.array_equal(err, terr[:k]))}
        if rej.size:
            r_off = np.ascontiguousarray(toff[rej])
            r_sz = np.ascontiguousarray(tsz[rej])
            r_err = np.zeros(rej.size, np.int8)
            L.ref_txn_verify_batch(rej.size, _vp(payload), _vp(r_off), _vp(r_sz), _vp(r_err), nt)
            out["verdicts"]["rejected_rechecked_by_reference"] = bool(np.array_equal(r_err, terr[rej]))
            out["verdicts"]["rejected_codes"] = sorted(set(int(c) for c in terr[rej]))
        if args.txn_full_check:
            # every transaction of the run re-verified by the compiled
            # reference, acceptances included (outside the timed region)
            t1 = time.perf_counter()
            f_err = np.zeros(toff.size, np.int8)
            L.ref_txn_verify_batch(toff.size, _vp(payload), _vp(toff), _vp(tsz), _vp(f_err), nt)
            out["verdicts"]["all_txns_rechecked_by_reference"] = {
                "txns": int(toff.size), "signatures": int(tbase[-1]), "equal": bool(np.array_equal(f_err, terr)),
                "mismatches": int((f_err != terr).sum()), "threads": nt, "seconds": time.perf_counter() - t1}
    emit(out, args)


# ---------------------------------------------------------------- configs[4]

# decompression work per signature (k_decomp's bodies: two points, each
# pow22523 = 250 squares + 11 muls, plus ~9 more muls and 4 squares), in the
# same MAC units as the double-scalar multiply
MAC_DECOMP = 2 * (254 * MAC_SQ + 20 * MAC_MUL)


def _lat_parts(r):
    """The tile's per-frag latency decomposition (fd_verify_amd_tile_set_trace), us."""
    us = lambda k: r[k] / 1e3  # noqa: E731
    return {"cut_wait": [us("cut_p50_ns"), us("cut_p99_ns")], "queue_wait": [us("queue_p50_ns"), us("queue_p99_ns")],
            "service": [us("service_p50_ns"), us("service_p99_ns")],
            "publish_wait": [us("publish_p50_ns"), us("publish_p99_ns")],
            "input_wait": [us("input_p50_ns"), us("input_p99_ns")],
            "service_p50_latency_chunks": us("service_lat_chunk_p50_ns"),   # latency and quad chunks
            "service_p50_throughput_chunks": us("service_thr_chunk_p50_ns"),
            "chunks": {"latency": int(r["gpu_chunks_lat"]), "quad": int(r["gpu_chunks_quad"]),
                       "throughput": int(r["gpu_chunks_thr"])},
            "mode_switches": int(r["mode_switches"]),
            "note": "[p50, p99] us per published frag: staged -> handed over (cut), -> a wave claimed the chunk "
                    "(queue), -> results stored (service, GPU clock mapped onto the host's), -> published "
                    "(in-order wait + poll); input = producer publish -> staged; steady state (frags scheduled 20 ms "
                    "or more after the run's start)"}


def stream_rows(local, pub, sig, off, sz, blob, args, mac_per_sig=None, world=1, dist=None):
    """config 5: tango mcache/dcache feed -> verify tile -> consumer, per
    batch cap, copy and zero-copy staging.  The pool carries 10 % corrupted
    frags (one message bit each: full verify cost, verdict -3); saturated
    runs check every published frag against the batch engine's verdicts and
    the SHA-512 tags (verdict, tag and order of every frag; the bytes in the
    tile's output dcache of every 16th); paced runs (50 % / 80 % of the
    row's saturated rate, three interleaved runs each: median p50, worst run's
    p99 / p50; and
    a fixed 1 M frags/s) measure latency and its decomposition."""
    from firedancer_amd import ed25519, tango
    m = min(pub.shape[0], 1 << 16)
    p_pub, p_sig, p_sz = pub[:m], sig[:m], sz[:m]
    p_off = (off[:m] - off[0]).astype(np.uint32)
    p_blob = blob[off[0]:off[0] + int(p_off[-1]) + int(p_sz[-1])].copy()
    rng = np.random.default_rng(55)
    bad = rng.choice(m, m // 10, replace=False)
    for i in bad:
        p_blob[p_off[i] + int(rng.integers(0, max(int(p_sz[i]), 1)))] ^= 1 << int(rng.integers(0, 8))
    eng = ed25519.Engine(device=local, batch_max=m, blob_max=p_blob.size + 64)
    p_err = eng.verify_soa(p_pub, p_sig, p_off, p_sz, p_blob)
    eng.close()
    p_tag = np.array([int.from_bytes(hashlib.sha512(bytes(p_sig[i][:32]) + bytes(p_pub[i]) +
                                                    bytes(p_blob[p_off[i]:p_off[i] + p_sz[i]])).digest()[:8],
                                     "little") for i in range(m)], np.uint64)
    pool = (p_pub, p_sig, p_off, p_sz, p_blob)

    def paced(bmax, zc, rate):
        nf = int(max(50000, rate * args.paced_seconds))
        th0 = cgroup_throttle()
        r = tango.bench_stream(local, bmax, 0, *pool, nf, rate=rate, zero_copy=zc)
        th1 = cgroup_throttle()
        return {"offered_frags_per_s": rate, "frags_per_s": r["frags_per_s"], "frags": nf,
                "cgroup_throttled": None if th0 is None or th1 is None else
                {"periods": th1[0] - th0[0], "us": th1[1] - th0[1]},
                "p50_us": r["p50_ns"] / 1e3, "p99_us": r["p99_ns"] / 1e3,
                "p99_over_p50": r["p99_ns"] / max(r["p50_ns"], 1.0),
                "all_frags": {"p50_us": r["all_p50_ns"] / 1e3, "p99_us": r["all_p99_ns"] / 1e3,
                              "note": "every frag, the run's first 20 ms included"},
                "mean_chunk": r["mean_batch"], "sv_filt": int(r["sv_filt"]),
                "decomposition": _lat_parts(r),
                "stalls_us": {"producer_late_max": r["producer_late_max_ns"] / 1e3,
                              "producer_credit_wait_max": r["producer_credit_wait_max_ns"] / 1e3,
                              "tile_pass_max": r["tile_pass_max_ns"] / 1e3,
                              "consumer_gap_max": r["consumer_gap_max_ns"] / 1e3},
                "copy_steals": int(r["copy_steals"]),
                "loop": {k: int(r[k]) for k in ("passes", "hand_offs", "stop_window", "stop_frames", "stop_batch_max",
                                                "stop_pass_bound")}}

    rows = []
    bmaxes = (256, 1024, 4096, 16384) if world == 1 else (16384,)
    for bmax in bmaxes:
        row = {"batch_max": bmax}
        for zc in (False, True) if world == 1 else (True,):
            key = "zero_copy" if zc else "copy"
            sat = tango.bench_stream(local, bmax, 0, *pool, args.stream_frags, zero_copy=zc, expect_err=p_err,
                                     expect_tag=p_tag, sample_bytes=True)
            rr = {"saturated_frags_per_s": sat["frags_per_s"],
                  "saturated_steady_frags_per_s": sat["steady_frags_per_s"],
                  "saturated_mean_hand_off": sat["mean_batch"],
                  "published": int(sat["published"]), "sv_filt": int(sat["sv_filt"]), "ovrn": int(sat["ovrn"]),
                  "check_mismatches": int(sat["mismatches"]), "checked": int(sat["checked"]),
                  "saturated_loop": {k: int(sat[k]) for k in ("passes", "hand_offs", "stop_window", "stop_frames",
                                                                "stop_batch_max", "stop_pass_bound", "gpu_chunks_lat",
                                                                "gpu_chunks_thr", "gpu_frags_lat", "gpu_frags_thr",
                                                                "gpu_chunks_quad", "gpu_frags_quad",
                                                                "mode_switches", "copy_steals")},
                  "saturated_stager_ns_per_frag": {k: _r(sat["stager_%s_ns" % k]) for k in ("list", "copy", "stage",
                                                                                             "hand")},
                  "saturated_stalls_us": {"producer_late_max": sat["producer_late_max_ns"] / 1e3,
                                          "tile_pass_max": sat["tile_pass_max_ns"] / 1e3,
                                          "consumer_gap_max": sat["consumer_gap_max_ns"] / 1e3}}
            if mac_per_sig:
                a = sat["frags_per_s"] * (mac_per_sig + MAC_DECOMP) / 1e12
                a_st = sat["steady_frags_per_s"] * (mac_per_sig + MAC_DECOMP) / 1e12
                rr["roofline"] = {"achieved": a, "peak": PEAK_TMAC, "unit": "TMAC/s", "frac": a / PEAK_TMAC,
                                  "frac_steady": a_st / PEAK_TMAC,
                                  "mac_per_frag": mac_per_sig + MAC_DECOMP,
                                  "note": "saturated frags/s x (DSM MACs per signature of the resident batch + "
                                          "decompression's %d) vs the integer-multiply peak; frac over the whole run (its ramp and "
                                          "drain included), frac_steady over the input's 10-90 %% span" % MAC_DECOMP}
            # three interleaved rounds of the two loads (a single run's p50 moved by up to 2 %
            # between back-to-back runs on one box)
            runs = {0.5: [], 0.8: []}
            for _ in range(3):
                for load in (0.5, 0.8):
                    runs[load].append(paced(bmax, zc, load * sat["frags_per_s"]))
            for load, rs in runs.items():
                # p50 is the median of the runs' p50 (over the runs free of harness stalls, topped up to
                # three when a stall hit some); the tail is the WORST run's p99 / p50 over every run (a
                # single bad run must fail the row: VERDICT r04 weak 2, 9); every run is kept whole
                extra = top_up(rs, lambda: paced(bmax, zc, load * sat["frags_per_s"]))
                med = p50_run(rs)
                worst, worst_clean, nstall = worst_of(rs)
                r = {"p50_us": med["p50_us"], "frags_per_s": med["frags_per_s"],
                     "offered_frags_per_s": med["offered_frags_per_s"],
                     "worst_p99_us": worst["p99_us"], "worst_p99_over_p50": worst["p99_over_p50"],
                     "worst_run": rs.index(worst), "harness_stalled_runs": nstall, "extra_runs": extra,
                     "worst_p99_over_p50_unstalled": worst_clean, "runs": rs}
                rr["at_%d%%" % int(load * 100)] = r
            lo, hi = rr["at_50%"], rr["at_80%"]
            # medians of three runs; the only slack is the spread of the 50 % runs' own p50s (the
            # measured run-to-run noise: copy-mode p50s barely move with load, 0.1-0.2 % either way)
            lo_clean = [x for x in lo["runs"] if not harness_stalled(x)] or lo["runs"]
            sp = max(x["p50_us"] for x in lo_clean) - min(x["p50_us"] for x in lo_clean)
            rr["p50_spread_us_50"] = sp
            rr["p50_nondecreasing_with_load"] = hi["p50_us"] >= lo["p50_us"] - sp
            rr["p99_within_2_5x_p50"] = max(lo["worst_p99_over_p50"], hi["worst_p99_over_p50"]) <= 2.5
            rr["p99_within_2_5x_p50_unstalled"] = unstalled_ok((lo, hi))
            row[key] = rr
        rows.append(row)
    fixed = {}
    if world == 1:
        for zc in (False, True):
            fixed["zero_copy" if zc else "copy"] = paced(4096, zc, 1e6)
    allr = [r[k] for r in rows for k in ("copy", "zero_copy") if k in r]
    for k, r in fixed.items():
        r["p99_within_2_5x_p50"] = r["p99_over_p50"] <= 2.5
    out = {"path": "producer (metadata only; frames pre-placed in the data region as a NIC would) -> in "
                   "mcache/dcache -> verify tile (one persistent GPU kernel fed through mapped ring/descriptor "
                   "memory; by the staging rate: latency chunks of 8 frags (8 lanes each), quad chunks of 16 (4 lanes each), "
                   "64-frag throughput chunks (1 lane each); copy: frag copied "
                   "into the tile's output dcache and released; zero_copy: GPU copies from the mapped input region, "
                   "input released when the frag is published; a second host thread publishes) -> out mcache + "
                   "tile-owned out dcache -> consumer (saturated runs check verdict, tag and order of every frag, "
                   "bytes of every 16th); latency = scheduled send to tile publish",
           "pool": "%d signatures of %d B, %d with one message bit flipped" % (m, int(p_sz[0]), bad.size),
           "frags_per_run": args.stream_frags,
           "all_checks_pass": all(r["check_mismatches"] == 0 for r in allr),
           "every_row_p99_within_2_5x_p50": all(r["p99_within_2_5x_p50"] for r in allr),
           "every_row_p99_within_2_5x_p50_unstalled": all(r["p99_within_2_5x_p50_unstalled"] for r in allr),
           "harness_stall_rule_us": HARNESS_STALL_US,
           "every_row_p50_nondecreasing_with_load": all(r["p50_nondecreasing_with_load"] for r in allr),
           "p50_rule": "median p50 at 80 % >= median p50 at 50 % minus the spread of the 50 % runs' p50s; medians over the runs free of harness stalls (topped up to three, at most 3 extra runs)",
           "rows": rows}
    if fixed:
        out["fixed_1M_frags_per_s_batch_max_4096"] = fixed
    return out


def _txn_first_tag(p):
    """SHA-512 tag of a wire transaction's first signature: R = signature 0,
    A = account address 0, M = the message (fd_txn.h layout; the synthetic
    transactions have < 128 accounts, so every compact-u16 is one byte)."""
    m = 1 + 64 * int(p[0])
    a = m + (1 if int(p[m]) & 0x80 else 0) + 4
    return int.from_bytes(hashlib.sha512(bytes(p[1:33]) + bytes(p[a:a + 32]) + bytes(p[m:])).digest()[:8], "little")


def txn_stream_row(local, args):
    """configs[3]'s frames through the tile's persistent kernel (TXN
    framing): GPU-signed multi-signer transactions, 10 % with a corrupted
    signature byte, saturated (every published transaction checked: verdict,
    first signature's tag, bytes of every 16th, order) and paced at 50 % /
    80 % of that rate (three interleaved runs each: median p50, worst run's
    p99 / p50)."""
    from firedancer_amd import ed25519, tango, workload
    payload, toff, tsz, _ = workload.txn_batch(1 << 17, 777)
    payload = payload.copy()
    rng = np.random.default_rng(56)
    bad = rng.choice(toff.size, toff.size // 10, replace=False)
    for t in bad:
        payload[int(toff[t]) + 1 + int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
    eng = ed25519.Engine(device=local, batch_max=1 << 16, blob_max=payload.size + 64)
    terr = eng.verify_txns(payload, toff, tsz)
    eng.close()
    tag = np.array([_txn_first_tag(payload[int(o):int(o) + int(z)]) for o, z in zip(toff, tsz)], np.uint64)
    zpub, zsig = np.zeros((toff.size, 32), np.uint8), np.zeros((toff.size, 64), np.uint8)
    pool = (zpub, zsig, toff, tsz, payload)
    nf = min(args.stream_frags // 4, 1 << 21)   # transactions per saturated TXN run
    sigs_per_txn = float(ed25519.txn_slots(payload, toff, tsz)[1]) / toff.size

    def paced(bmax, rate):
        r = tango.bench_stream(local, bmax, 0, *pool, int(min(nf, max(20000, rate * args.paced_seconds))), rate=rate,
                               zero_copy=True, txn=True)
        return {"offered_txns_per_s": rate, "txns_per_s": r["frags_per_s"], "p50_us": r["p50_ns"] / 1e3,
                "p99_us": r["p99_ns"] / 1e3, "p99_over_p50": r["p99_ns"] / max(r["p50_ns"], 1.0),
                "decomposition": _lat_parts(r),
                "stalls_us": {"producer_late_max": r["producer_late_max_ns"] / 1e3,
                              "producer_credit_wait_max": r["producer_credit_wait_max_ns"] / 1e3,
                              "tile_pass_max": r["tile_pass_max_ns"] / 1e3,
                              "consumer_gap_max": r["consumer_gap_max_ns"] / 1e3}}

    def row(bmax):
        sat = tango.bench_stream(local, bmax, 0, *pool, nf, zero_copy=True, txn=True, expect_err=terr, expect_tag=tag,
                                 sample_bytes=True)
        out = {"batch_max": bmax, "saturated_txns_per_s": sat["frags_per_s"],
               "saturated_verifies_per_s": sat["frags_per_s"] * sigs_per_txn,
               "saturated_steady_verifies_per_s": sat["steady_frags_per_s"] * sigs_per_txn,
               "check_mismatches": int(sat["mismatches"]), "checked": int(sat["checked"]),
               "published": int(sat["published"]), "sv_filt": int(sat["sv_filt"]),
               "gpu_chunks": {"latency": int(sat["gpu_chunks_lat"]), "quad": int(sat["gpu_chunks_quad"]),
                              "throughput": int(sat["gpu_chunks_thr"])}}
        runs = {0.5: [], 0.8: []}
        for _ in range(3):
            for load in (0.5, 0.8):
                runs[load].append(paced(bmax, load * sat["frags_per_s"]))
        for load, rs in runs.items():
            extra = top_up(rs, lambda: paced(bmax, load * sat["frags_per_s"]))
            med = p50_run(rs)
            worst, worst_clean, nstall = worst_of(rs)
            out["at_%d%%" % int(load * 100)] = {"p50_us": med["p50_us"], "txns_per_s": med["txns_per_s"],
                                                "worst_p99_us": worst["p99_us"],
                                                "worst_p99_over_p50": worst["p99_over_p50"],
                                                "harness_stalled_runs": nstall, "extra_runs": extra,
                                                "worst_p99_over_p50_unstalled": worst_clean, "runs": rs}
        out["p99_within_2_5x_p50"] = max(out["at_50%"]["worst_p99_over_p50"],
                                         out["at_80%"]["worst_p99_over_p50"]) <= 2.5
        out["p99_within_2_5x_p50_unstalled"] = unstalled_ok((out["at_50%"], out["at_80%"]))
        return out

    rows = [row(4096), row(16384)]
    return {"path": "TXN framing (wire transactions, multi-signer) on the tile's persistent kernel: the host reads each "
                    "transaction's signature count, chunks are packed by signature slots (<= 64), a chunk's lanes "
                    "parse its transactions, verify every signature and reduce per transaction; zero copy",
            "pool": "%d transactions, %.2f signatures each, %d with a flipped signature bit" % (toff.size, sigs_per_txn,
                                                                                             bad.size),
            "rows": rows}


def stream_node(local, pub, sig, off, sz, blob, args, rank, world, dist):
    """N GPUs, the reference's scaling unit (N verify tiles, one per
    input link: fd_frank_init:67-80, fd_frank_main.c:118-143): every rank
    runs its own tile on its own GPU at batch_max 16384, zero copy, all at
    once -- saturated, then at half its own saturated rate -- with its
    host threads on its GPU's NUMA node (ranks that share a node split its
    CPUs).  Rank 0 reports the node sum."""
    import torch
    from firedancer_amd import hip, tango
    from firedancer_amd.shard import max_over_ranks, node_plan, node_sum, peer_slot
    from firedancer_amd import ed25519
    ndev = max(1, hip.device_count())
    keys = [None] * world
    saved = os.sched_getaffinity(0)
    dist.all_gather_object(keys, {"numa": ed25519.device_numa_node(local), "dev": local % ndev,
                                  "cpus": sorted(saved), "quota": host_cores()[2]["cgroup_quota"]})
    # every rank's CPU slice and host budget from one node plan (ranks on a NUMA node split its CPUs; the
    # processes' shared cgroup quota, if any, caps the sum)
    numa = [x["numa"] for x in keys]
    node_cpus = {}
    for x in keys:
        node_cpus[x["numa"]] = sorted(set(node_cpus.get(x["numa"], [])) | set(x["cpus"]))
    plans, plan_tot = node_plan(numa, node_cpus, 16384, zero_copy=True, cpu_quota=keys[0]["quota"])
    cpus = plans[rank]["cpus"]
    # the rank's threads stay inside its slice: with 5 or more CPUs the tile
    # bench pins its spinning threads there; below that (8 ranks in a 16-CPU
    # quota get 2 each) they share the slice unpinned, publishing inline,
    # rather than every rank picking the same quiet CPUs of the whole machine
    if cpus:
        os.sched_setaffinity(0, cpus)
    _, share = peer_slot([x["dev"] for x in keys], rank)
    waves = 0
    if share > 1:   # rehearsal: ranks mapped onto one GPU split its wave slots
        cus = ctypes_cus(local)
        waves = 8 * cus // share
    m = min(pub.shape[0], 1 << 16)
    p_off = (off[:m] - off[0]).astype(np.uint32)
    pool = (pub[:m], sig[:m], p_off, sz[:m], blob[off[0]:off[0] + int(p_off[-1]) + int(sz[m - 1])].copy())
    nf = args.stream_frags
    res = []
    try:
        dist.barrier()
        t0 = time.perf_counter()
        sat = tango.bench_stream(local, 16384, 0, *pool, nf, zero_copy=True, waves=waves)
        span_sat = max_over_ranks(time.perf_counter() - t0)
        dist.barrier()
        rate = 0.5 * sat["frags_per_s"]
        half = tango.bench_stream(local, 16384, 0, *pool, int(min(nf, max(20000, rate))), rate=rate, zero_copy=True,
                                  waves=waves)
        res = [sat["frags_per_s"], half["frags_per_s"], half["p50_ns"] / 1e3, half["p99_ns"] / 1e3, float(len(cpus)),
               float(waves)]
    finally:
        os.sched_setaffinity(0, saved)
    cols = ["saturated_frags_per_s", "half_frags_per_s", "p50_us", "p99_us", "cpus", "waves"]
    t = torch.zeros(world * len(cols), dtype=torch.float64)
    if res:
        t[rank * len(cols):(rank + 1) * len(cols)] = torch.tensor(res, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    agg = node_sum(t.view(world, len(cols)).tolist(), cols)
    return {"ranks": world, "batch_max": 16384, "staging": "zero_copy",
            "saturated_frags_per_s_node": agg["saturated_frags_per_s"],
            "saturated_run_span_s_max": span_sat,
            "at_50%_frags_per_s_node": agg["half_frags_per_s"],
            "per_rank": [{"saturated_frags_per_s": r["saturated_frags_per_s"],
                          "at_50%": {"frags_per_s": r["half_frags_per_s"], "p50_us": r["p50_us"], "p99_us": r["p99_us"]},
                          "cpus": int(r["cpus"]), "waves": int(r["waves"]), "numa_node": keys[i]["numa"],
                          "device": keys[i]["dev"]} for i, r in enumerate(agg["per_rank"])],
            "host_budget": plan_tot,
            "note": "every rank's tile runs at once (barrier before each run); node value = sum of the ranks' rates"}


def ctypes_cus(device):
    import ctypes
    from firedancer_amd import hip
    v = ctypes.c_int(0)
    H = hip.hip()
    if H.hipDeviceGetAttribute(ctypes.byref(v), 63, int(device)) != 0 or v.value <= 0:   # MultiprocessorCount
        return 256
    return v.value


# ---------------------------------------------------------------- multi-engine

def run_multi_engine(args):
    """One process, --gpus devices, the native multi-device engine
    (fd_ed25519_amd_multi_*): one engine and one NUMA-bound host thread per
    device, a host SoA batch of gpus x n signatures split into contiguous
    shards per step (weak scaling: n per device).  PCIe-inclusive by
    construction -- the shape of a host that feeds every GPU of the node from
    one process.  FD_AMD_DEVICE_MAP=mod maps more engines than GPUs onto the
    visible ones (rehearsal on a one-GPU box)."""
    from firedancer_amd import ed25519, hip
    ndev = hip.device_count()
    if not ndev:
        raise SystemExit("bench.py: no HIP device")
    g = args.gpus
    if g > ndev and os.environ.get("FD_AMD_DEVICE_MAP") != "mod":
        raise SystemExit("bench.py --multi-engine: %d GPUs asked, %d visible" % (g, ndev))
    devices = [d % ndev for d in range(g)]
    n = args.n
    pub1, sig1, off1, sz1, blob1 = make_workload(n, args.msg_sz, 1000)
    ref = ed25519.Engine(device=0, batch_max=1 << 17, blob_max=(1 << 17) * args.msg_sz)
    err1 = ref.verify_soa(pub1, sig1, off1, sz1, blob1)
    ref.close()
    pub = np.concatenate([pub1] * g)
    sig = np.concatenate([sig1] * g)
    sz = np.concatenate([sz1] * g)
    off = np.concatenate([off1.astype(np.int64) + k * blob1.size for k in range(g)]).astype(np.uint32)
    blob = np.concatenate([blob1] * g)
    chunk = 1 << 17
    m = ed25519.MultiEngine(devices, batch_max=chunk, blob_max=chunk * args.msg_sz)
    try:
        for _ in range(max(1, args.warmup)):
            err = m.verify_soa(pub, sig, off, sz, blob)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            err = m.verify_soa(pub, sig, off, sz, blob)
        dt = time.perf_counter() - t0
    finally:
        m.close()
    nodes = [ed25519.device_numa_node(d) for d in sorted(set(devices))]
    emit({
        "metric": METRIC, "value": g * n * args.steps / dt, "unit": "verifies/s", "n_gpus": g,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": DTYPE,
        "data": "synthetic: fresh random keypairs and messages (one 2^20 batch repeated per device), host SoA buffers",
        "mode": "multi_engine",
        "config": {"workload": "configs[1] shape, %d x %d signatures from host memory per step" % (g, n),
                   "devices": devices, "sigs_per_gpu_per_step": n, "msg_sz": args.msg_sz, "chunk": chunk,
                   "parallelism": "multi-engine %d" % g, "hip_hw_queues": HW_QUEUES,
                   "device_map": os.environ.get("FD_AMD_DEVICE_MAP", "identity")},
        "numa_nodes": nodes,
        "verdicts_match_single_engine": bool(all(np.array_equal(err[k * n:(k + 1) * n], err1) for k in range(g))),
        "path": "host SoA -> fd_ed25519_amd_multi_verify_soa: per device one NUMA-bound thread, pinned staging (2 "
                "chunks in flight) -> H2D -> kernels -> mapped verdicts",
    }, args)


# ---------------------------------------------------------------- configs[1]

def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # gloo prints its connection report on stdout from C++; keep stdout
        # for rank 0's one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)

    from firedancer_amd import ed25519, hip
    from firedancer_amd.shard import bind_to_device_node

    if args.multi_engine:
        return run_multi_engine(args)
    ndev = hip.device_count()
    if os.environ.get("FD_AMD_DEVICE_MAP") == "mod" and ndev:   # rehearsal: more ranks than GPUs
        local = local % ndev
    if ndev <= local:
        raise SystemExit("bench.py: no HIP device %d visible" % local)
    hip.set_device(local)
    # this rank's host thread(s) on its GPU's NUMA node, as the reference
    # pins each verify tile to a core next to its input link
    numa = bind_to_device_node(local)

    if args.workload == "txn":
        return run_txn(args, rank, world, dist)

    n = args.n
    if args.dsm_kernel != "default":
        ed25519.select_dsm_kernel(args.dsm_kernel)
    t0 = time.perf_counter()
    pub, sig, off, sz, blob = make_workload(n, args.msg_sz, 1000 + rank)
    gen_s = time.perf_counter() - t0

    d = {k: hip.DeviceBuffer.from_array(v) for k, v in
         dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
    # consecutive steps alternate between `streams` (stream, verdicts,
    # workspace) sets, batches in flight: one batch's hashing/decompression
    # and the start of its multiply fill the SIMDs the previous batch's last
    # double-scalar-mult waves leave idle
    ns = max(1, args.streams)
    sets = [(hip.Stream(), hip.DeviceBuffer(n), hip.DeviceBuffer(ed25519.workspace_footprint(n))) for _ in range(ns)]
    d_stats = hip.DeviceBuffer(4 * 3 * n)
    stream, d_err, d_ws = sets[0]

    def run(k, ev=None):
        st_, er_, ws_ = sets[k % ns]
        ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, er_.ptr,
                              ws_.ptr, st_.handle, ev)

    def sync_all():
        for st_, _, _ in sets:
            st_.synchronize()

    for k in range(max(args.warmup, ns)):
        run(k)
    sync_all()

    if dist:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for k in range(args.steps):
        run(k)
    sync_all()
    elapsed = time.perf_counter() - t0
    if dist:
        from firedancer_amd.shard import max_over_ranks
        elapsed = max_over_ranks(elapsed)
        dist.barrier()

    # per-kernel times (and the roofline) from HIP events on one stream with
    # nothing else running, after the timed region
    nev = 3
    evs = [[hip.Event() for _ in range(4)] for _ in range(nev)]
    for k in range(nev):
        run(0, evs[k])
    sync_all()
    stage_ms = np.zeros(3)
    for ev in evs:
        for j in range(3):
            stage_ms[j] += ev[j].elapsed_ms(ev[j + 1])
    stage_ms /= nev

    err = d_err.to_array(np.int8, n)
    for _, er_, _ in sets[1:]:
        assert np.array_equal(er_.to_array(np.int8, n), err)
    ed25519.work_stats_dev(n, d_ws.ptr, d_stats.ptr, stream.handle)
    stream.synchronize()
    st = d_stats.to_array(np.uint32, 3 * n).reshape(3, n)

    # host-fed node throughput: every rank at once verifies its batch from
    # registered host memory (fd_ed25519_amd_verify_soa_registered: each
    # chunk's planes and message window DMA'd, no host copy), the shape of a
    # node whose GPUs are fed from host memory, PCIe included; max-over-ranks
    # time.  Never the headline value.
    host_fed = None
    if not args.no_host_fed:
        chunk, reps = 1 << 17, 3
        eng = ed25519.Engine(device=local, batch_max=chunk, blob_max=chunk * args.msg_sz)
        reg = ed25519.RegisteredPlanes(pub, sig, off, sz, blob)
        rerr = np.zeros(n, np.int8)
        eng.verify_soa_registered(reg[0], reg[1], reg[2], reg[3], reg[4], rerr)
        if dist:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(reps):
            eng.verify_soa_registered(reg[0], reg[1], reg[2], reg[3], reg[4], rerr)
        dt_rank = time.perf_counter() - t1
        reg.close()
        eng.close()
        ok = float(np.array_equal(rerr, err))
        if dist:
            from firedancer_amd.shard import max_over_ranks
            dt_max = max_over_ranks(dt_rank)
        else:
            dt_max = dt_rank
        ok_all, sum_rate = gather_sum(dist, [ok, n * reps / dt_rank])
        host_fed = {"verifies_per_s": world * n * reps / dt_max, "sum_of_rank_rates": sum_rate,
                    "per_rank_sigs": n, "chunk": chunk, "passes": reps,
                    "h2d_gb_per_s_node": world * n * reps * (104 + args.msg_sz) / dt_max / 1e9,
                    "verdicts_match_resident": ok_all == world,
                    "path": "every rank at once: registered caller SoA (fd_ed25519_amd_host_register once) -> DMA "
                            "of each chunk's planes and message window, no host copy -> kernels; rank bound to its "
                            "GPU's NUMA node; value = all ranks' signatures / max-over-ranks time"}

    node_tile = None
    if world > 1 and not args.no_stream:
        node_tile = stream_node(local, pub, sig, off, sz, blob, args, rank, world, dist)

    if rank != 0:
        return
    total = n * args.steps * world
    out = {
        "metric": METRIC,
        "value": total / elapsed,
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPE,
        "data": "synthetic: fresh random keypairs and messages, signed on the GPU (k_sign), inputs resident in HBM",
        "config": {"workload": "configs[1]: 1xMI355X batch of 2^20 single-signer sigs, 200-byte messages",
                   "sigs_per_gpu_per_step": n, "msg_sz": args.msg_sz, "parallelism": "shard%d" % world,
                   "streams": ns, "hip_hw_queues": HW_QUEUES,
                   "device_map": os.environ.get("FD_AMD_DEVICE_MAP", "identity")},
        "numa_rank0": numa,
        "host_fed_node": host_fed,
        "stage_ms": {"k_prep": stage_ms[0], "k_decomp": stage_ms[1], "k_dsm": stage_ms[2],
                     "note": "one batch alone on one stream (HIP events), after the timed region"},
        "verdicts": {"ok": int((err == 0).sum()), "rejected": int((err != 0).sum())},
        "roofline": dsm_roofline(st, stage_ms[2], n, kernel="+".join(dsm_kernels(n, args.dsm_kernel)),
                                 note="DSM stage of one batch alone on one stream (HIP events); with %d "
                                      "streams in the timed region the next batch's k_prep/k_decomp also fill "
                                      "the SIMDs its last waves leave idle" % ns),
        "dsm_in_pipeline": dsm_in_pipeline(st, elapsed / args.steps * 1e3, stage_ms, n) if ns > 1 else None,
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
        lat = np.array(lat[3:])
        out["latency_ms_4096"] = {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                                  "path": "host SoA -> packed pinned staging (read in place by k_front) -> k_front -> "
                                          "k_dsm8 -> verdicts through mapped memory"}
        # the same batches from registered caller memory: k_front reads the
        # caller's planes in place, no copy on either side
        reg = ed25519.RegisteredPlanes(pub, sig, off, sz, blob)
        lat, rerr = [], np.zeros(m, np.int8)
        for r in range(30):
            lo = (r * m) % max(1, n - m)
            t1 = time.perf_counter()
            eng.verify_soa_registered(reg[0][lo:lo + m], reg[1][lo:lo + m], reg[2][lo:lo + m], reg[3][lo:lo + m],
                                      reg[4], rerr)
            lat.append((time.perf_counter() - t1) * 1e3)
            assert np.array_equal(rerr, err[lo:lo + m])
        reg.close()
        eng.close()
        lat = np.array(lat[3:])
        out["latency_ms_4096_registered"] = {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                                             "path": "registered caller SoA (fd_ed25519_amd_verify_soa_registered) read "
                                                     "in place by k_front -> k_dsm8 -> verdicts through mapped memory"}
        # the reference's drop-in entry point, one signature per call (the
        # verify tile's calling pattern, fd_frank_verify_synth_load.c:380)
        calls = []
        for r in range(220):
            i = (r * 7919) % n
            msg = bytes(blob[off[i]:off[i] + sz[i]])
            t1 = time.perf_counter()
            rc = ed25519.verify(msg, bytes(sig[i]), bytes(pub[i]))
            calls.append((time.perf_counter() - t1) * 1e6)
            assert rc == int(err[i])
        calls = np.array(calls[20:])
        out["dropin_call_us"] = {"p50": float(np.percentile(calls, 50)), "p99": float(np.percentile(calls, 99)),
                                 "reference_us_per_call_survey": REF_US_PER_CALL_SURVEY,
                                 "path": "fd_ed25519_verify: one signature per call, a GPU batch of one "
                                         "(packed staging -> k_front -> k_dsm8 -> mapped result)"}
        # PCIe-inclusive rates: the same 2^20 batch handed over as host SoA
        # buffers, chunks of 2^17 with 2 in flight, priced against the
        # measured pinned H2D ceiling.  Never the headline value.
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
        if host_fed:
            out["host_soa_registered"] = {"verifies_per_s": host_fed["verifies_per_s"] / world,
                                          "note": "rank 0's share of host_fed_node (every rank ran it at once)"}
    if world == 1 and not args.no_stream:
        out["stream_tile"] = stream_rows(local, pub, sig, off, sz, blob, args, mac_per_sig=out["roofline"]["mac_per_sig"])
        out["stream_tile"]["txn_framing"] = txn_stream_row(local, args)
    if node_tile:
        out["stream_tile_node"] = node_tile
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(pub, sig, off, sz, blob, args.cpu_sample, args.cpu_threads, err,
                                           args.cpu_seconds)
        if "dropin_call_us" in out:
            out["dropin_call_us"]["reference_us_per_call_this_host"] = out["cpu_baseline"]["us_per_call_1_thread"]
    emit(out, args)


if __name__ == "__main__":
    main()
