"""Python mirror of the tango pieces the streaming verify tile speaks
(include/fd_tango_amd.h; reference src/tango/fd_tango_base.h:146-203,
src/tango/mcache/fd_mcache.h:299-322, src/tango/dcache/fd_dcache.h:211-269)
and a handle on the tile itself (fd_verify_amd_tile_*).  The tile's run
loop is native (firedancer_amd/csrc/fd_verify_tile.cpp); this module only
lays out memory and calls it."""
import ctypes

import numpy as np

from . import ed25519

FRAG_META = np.dtype([("seq", "<u8"), ("sig", "<u8"), ("chunk", "<u4"), ("sz", "<u2"), ("ctl", "<u2"),
                      ("tsorig", "<u4"), ("tspub", "<u4")])
assert FRAG_META.itemsize == 32
CHUNK_LG_SZ = 6
CHUNK_SZ = 64
DIAG_FIELDS = ("in_cnt", "ha_filt_cnt", "ha_filt_sz", "sv_filt_cnt", "sv_filt_sz", "out_cnt", "out_sz",
               "ovrn_cnt", "backp_cnt", "batch_cnt", "batch_sig_cnt", "bad_frag_cnt", "gpu_chunk_lat_cnt",
               "gpu_chunk_thr_cnt", "gpu_frag_lat_cnt", "gpu_frag_thr_cnt", "sv_filt_sig_cnt", "sv_filt_pubkey_cnt",
               "sv_filt_msg_cnt", "halt_drop_cnt", "mode_switch_cnt", "gpu_chunk_quad_cnt", "gpu_frag_quad_cnt",
               "quad_pair_cnt")
CHUNK_AUTO, CHUNK_LATENCY, CHUNK_THROUGHPUT, CHUNK_QUAD = 0, 1, 2, 3
LVL_LAT, LVL_THR, LVL_QUAD = 0, 1, 2
PUBLISH_AUTO, PUBLISH_INLINE = -2, -1
COPY_INLINE = -1


class TileCfg(ctypes.Structure):
    """fd_verify_amd_tile_cfg_t (include/fd_tango_amd.h)."""
    _fields_ = [("device", ctypes.c_int), ("framing", ctypes.c_int), ("batch_max", ctypes.c_ulong),
                ("batch_wait_ns", ctypes.c_ulong), ("tcache_depth", ctypes.c_ulong), ("out_frame_cnt", ctypes.c_ulong),
                ("waves", ctypes.c_ulong), ("chunk_mode", ctypes.c_int), ("publish_cpu", ctypes.c_int),
                ("window", ctypes.c_ulong), ("lat_fill_ns", ctypes.c_ulong), ("lat_free_chunks", ctypes.c_ulong),
                ("chunk_wait_ns", ctypes.c_ulong), ("thr_rate_hi", ctypes.c_ulong), ("thr_rate_lo", ctypes.c_ulong),
                ("halt_grace_ns", ctypes.c_ulong),
                ("copy_cpu", ctypes.c_int), ("quad_rate_hi", ctypes.c_ulong), ("quad_rate_lo", ctypes.c_ulong)]

    @classmethod
    def default(cls, **kw):
        c = cls()
        ed25519.lib().fd_verify_amd_tile_cfg_default(ctypes.byref(c))
        for k, v in kw.items():
            setattr(c, k, v)
        return c


def _aligned(nbytes, align=64):
    raw = np.zeros(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def mcache_new(depth):
    """An mcache ring of `depth` (power of 2) frag metadata, every line
    marked "not yet published" for the first lap (seq = line - depth)."""
    assert depth and not depth & (depth - 1)
    m = _aligned(32 * depth).view(FRAG_META)
    m["seq"] = (np.arange(depth, dtype=np.int64) - depth).astype(np.uint64)
    return m


def publish(mcache, seq, sig, chunk, sz, ctl, tsorig, tspub):
    """fd_mcache_publish (fd_mcache.h:299-322) from Python (single-threaded use)."""
    line = mcache[seq & (mcache.size - 1)]
    line["seq"] = (seq - 1) & 0xFFFFFFFFFFFFFFFF
    line["sig"], line["chunk"], line["sz"], line["ctl"] = sig, chunk, sz, ctl
    line["tsorig"], line["tspub"] = tsorig, tspub
    line["seq"] = seq


def dcache_compact_next(chunk, sz, chunk0, wmark):
    """fd_dcache_compact_next (fd_dcache.h:263-269)."""
    chunk += ((sz + (2 * CHUNK_SZ - 1)) >> (1 + CHUNK_LG_SZ)) << 1
    return chunk0 if chunk > wmark else chunk


def tickcount():
    return int(ed25519.lib().fd_verify_amd_tickcount())


class VerifyTile:
    """fd_verify_amd_tile_t: adaptive-batching GPU verify tile that publishes
    out of its own output dcache."""

    FRAMING_PUB_SIG_MSG = 0
    FRAMING_TXN = 1
    FRAME_SZ = 1408

    def __init__(self, device=0, batch_max=4096, batch_wait_ns=0, tcache_depth=1 << 16, framing=0, out_frame_cnt=0,
                 **cfg):
        """cfg: further fd_verify_amd_tile_cfg_t fields (waves, chunk_mode, publish_cpu, window, lat_fill_ns,
        lat_free_chunks, chunk_wait_ns, thr_rate_hi, thr_rate_lo, halt_grace_ns, copy_cpu)."""
        L = ed25519.lib()
        self._h = None
        c = TileCfg.default(device=int(device), batch_max=int(batch_max), batch_wait_ns=int(batch_wait_ns),
                            tcache_depth=int(tcache_depth), out_frame_cnt=int(out_frame_cnt), framing=int(framing),
                            **cfg)
        self._h = L.fd_verify_amd_tile_new_cfg(ctypes.byref(c))
        if not self._h:
            raise ed25519.EngineError("fd_verify_amd_tile_new_cfg failed (bad configuration -- framing %r, "
                                      "batch_max %d -- or no HIP device)" % (framing, batch_max))
        base = L.fd_verify_amd_tile_out_chunk0(self._h)
        nbytes = int(L.fd_verify_amd_tile_out_data_sz(self._h))
        self.out_region = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(base))

    def close(self):
        if self._h:
            self.out_region = None
            ed25519.lib().fd_verify_amd_tile_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def out_frame(self, chunk, sz):
        """Bytes of a published frag (fd_chunk_to_laddr(out_chunk0, chunk))."""
        return bytes(self.out_region[CHUNK_SZ * int(chunk):CHUNK_SZ * int(chunk) + int(sz)])

    def register_dcache(self, region):
        """Map the numpy data region into the GPU (zero-copy staging).  The
        previous region stays referenced until the tile has unregistered it."""
        rc = ed25519.lib().fd_verify_amd_tile_register_dcache(self._h, ctypes.c_void_p(region.ctypes.data),
                                                             region.nbytes)
        if rc:
            raise ed25519.EngineError("fd_verify_amd_tile_register_dcache rc=%d" % rc)
        self._region = region

    def set_trace(self, parts):
        """Per-frag latency decomposition of the next runs into parts (uint32 [n][4], or None)."""
        self._trace = parts
        ed25519.lib().fd_verify_amd_tile_set_trace(self._h, ctypes.c_void_p(parts.ctypes.data) if parts is not None
                                                   else None, 0 if parts is None else parts.shape[0])

    def set_verdict_log(self, log):
        """Verdicts of the frags the next runs verify: log[seq - in_seq0] (int8 array, or None)."""
        self._vlog = log
        ed25519.lib().fd_verify_amd_tile_set_verdict_log(self._h, ctypes.c_void_p(log.ctypes.data) if log is not None
                                                         else None, 0 if log is None else log.size)

    def run(self, in_mcache, in_chunk0, in_seq0, out_mcache, out_seq0, frag_cnt, lat_max=0, stop=None,
            out_fseq=None, in_fseq=None):
        """Consume frag_cnt input frags (frag_cnt 0: until stop, a ctypes.c_int
        another thread sets nonzero); returns (diag dict, latency samples).
        self.in_fseq holds the tile's final producer credit.  out_fseq: a
        ctypes.c_ulong the consumer advances (None: no output flow control);
        in_fseq: a ctypes.c_ulong for the producer credit (None: a private one)."""
        diag = (ctypes.c_ulong * len(DIAG_FIELDS))()
        lat = np.zeros(max(lat_max, 1), np.uint32)
        fseq = in_fseq if in_fseq is not None else ctypes.c_ulong(0)
        vp = ctypes.c_void_p
        rc = ed25519.lib().fd_verify_amd_tile_run(
            self._h, vp(in_mcache.ctypes.data), in_mcache.size, vp(in_chunk0.ctypes.data), int(in_seq0),
            ctypes.byref(fseq), vp(out_mcache.ctypes.data), out_mcache.size, int(out_seq0),
            ctypes.byref(out_fseq) if out_fseq is not None else None, int(frag_cnt),
            ctypes.byref(stop) if stop is not None else None,
            ctypes.byref(diag), vp(lat.ctypes.data) if lat_max else None, int(lat_max))
        if rc:
            raise ed25519.EngineError("fd_verify_amd_tile_run rc=%d" % rc)
        self.in_fseq = fseq.value
        d = dict(zip(DIAG_FIELDS, list(diag)))
        return d, lat[:min(lat_max, d["out_cnt"])]


BENCH_ZERO_COPY, BENCH_WRITE, BENCH_LAP, BENCH_SAMPLE_BYTES = 1, 2, 4, 8
BENCH_CHUNK_LAT, BENCH_CHUNK_THR, BENCH_PUB_INLINE, BENCH_TXN, BENCH_COPY_INLINE = 16, 32, 64, 128, 256
BENCH_STALL_HELPER, BENCH_CHUNK_QUAD = 512, 1024


def bench_stream(device, batch_max, batch_wait_ns, pub, sig, msg_off, msg_sz, blob, frag_cnt, rate=0.0,
                 zero_copy=False, writes=False, lap=False, dcache_frames=0, expect_err=None, expect_tag=None,
                 sample_bytes=False, chunk_mode=0, pub_inline=False, txn=False, waves=0, copy_inline=False,
                 stall_helper=False):
    """fd_verify_amd_bench_stream: producer (rate frags/s, 0 = saturate) -> tile -> consumer; returns
    dict(frags_per_s, p50_ns, p99_ns, p999_ns, mean_batch, published, sv_filt, ovrn, mismatches, checked).
    With expect_err/expect_tag (per pool entry) the consumer checks every published frag."""
    out = (ctypes.c_double * 49)()
    p = [np.ascontiguousarray(a) for a in (pub, sig, msg_off, msg_sz, blob)]
    ee = np.ascontiguousarray(expect_err, np.int8) if expect_err is not None else None
    et = np.ascontiguousarray(expect_tag, np.uint64) if expect_tag is not None else None
    flags = (BENCH_ZERO_COPY if zero_copy else 0) | (BENCH_WRITE if writes else 0) | (BENCH_LAP if lap else 0) | \
        (BENCH_SAMPLE_BYTES if sample_bytes else 0) | {0: 0, 1: BENCH_CHUNK_LAT, 2: BENCH_CHUNK_THR, 3: BENCH_CHUNK_QUAD}[chunk_mode] | \
        (BENCH_PUB_INLINE if pub_inline else 0) | (BENCH_TXN if txn else 0) | (BENCH_COPY_INLINE if copy_inline else 0) | \
        (BENCH_STALL_HELPER if stall_helper else 0)
    vp = ctypes.c_void_p
    rc = ed25519.lib().fd_verify_amd_bench_stream(int(device), int(batch_max), int(batch_wait_ns), float(rate), flags,
                                                  int(dcache_frames), p[2].shape[0],
                                                  *[vp(a.ctypes.data) for a in p],
                                                  vp(ee.ctypes.data) if ee is not None else None,
                                                  vp(et.ctypes.data) if et is not None else None,
                                                  int(frag_cnt), int(waves), out)
    if rc:
        raise ed25519.EngineError("fd_verify_amd_bench_stream rc=%d" % rc)
    keys = ("frags_per_s", "p50_ns", "p99_ns", "p999_ns", "mean_batch", "published", "sv_filt", "ovrn", "mismatches",
            "checked", "gpu_chunks_lat", "gpu_chunks_thr", "gpu_frags_lat", "gpu_frags_thr", "producer_late_max_ns",
            "tile_pass_max_ns", "consumer_gap_max_ns", "cut_p50_ns", "cut_p99_ns", "queue_p50_ns", "queue_p99_ns",
            "service_p50_ns", "service_p99_ns", "publish_p50_ns", "publish_p99_ns", "input_p50_ns", "input_p99_ns",
            "service_lat_chunk_p50_ns", "service_thr_chunk_p50_ns", "mode_switches", "traced", "producer_credit_wait_max_ns", "passes",
            "hand_offs", "stop_window", "stop_frames", "stop_batch_max", "stop_pass_bound", "all_p50_ns", "all_p99_ns", "steady_frags_per_s", "copy_steals",
            "gpu_chunks_quad", "gpu_frags_quad", "stager_list_ns", "stager_copy_ns", "stager_stage_ns",
            "stager_hand_ns", "quad_pairs")
    return dict(zip(keys, list(out)))
