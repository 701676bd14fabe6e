#ifndef HEADER_fd_tango_amd_h
#define HEADER_fd_tango_amd_h

/* Tango-compatible streaming verify tile on the MI355X engine (SURVEY.md
 * s8 f2, config 5).
 *
 * Part 1 reproduces the tango ABI the tile speaks: the 32-byte fragment
 * metadata (src/tango/fd_tango_base.h:146-203), 64-byte chunk addressing
 * (:123-126, :239-263), the mcache publish protocol
 * (src/tango/mcache/fd_mcache.h:299-322: seq-1 first, fields, then seq)
 * and the compact dcache chunk advance (src/tango/dcache/fd_dcache.h:
 * 211-269).  When the reference's own tango headers were included first
 * their definitions are used.
 *
 * Part 2 is the tile: it consumes frags public_key(32) | signature(64) |
 * message from an input mcache/dcache (the framing of the reference verify
 * tile, src/app/frank/load/fd_frank_verify_synth_load.c:340-347), drops HA
 * duplicates with a tag cache before verification (:351-370; tag = the
 * first 8 signature bytes), verifies in adaptive GPU batches, and publishes
 * the passing frags in arrival order to an output mcache (:404-411) with
 * the metadata `sig` field set to the dedup tag produced by the verify
 * itself (the first 8 bytes of SHA-512(R||A||M), app/frank/README.md:
 * 107-110; consumed by the dedup tile, disco/dedup/fd_dedup.h:247).
 * Drops are counted like the reference's cnc diagnostics
 * (app/frank/fd_frank.h:23-28: HA_FILT_{CNT,SZ}, SV_FILT_{CNT,SZ}).
 */

#include "fd_ed25519_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ===== Part 1: tango ABI ===== */

#ifndef HEADER_fd_src_tango_fd_tango_base_h

typedef unsigned short ushort;

#define FD_CHUNK_LG_SZ      (6)
#define FD_CHUNK_SZ         (64UL)
#define FD_FRAG_META_ALIGN  (32UL)

struct __attribute__((aligned(32))) fd_frag_meta {
  ulong  seq;     /* frag sequence number, written last by the publisher */
  ulong  sig;     /* application signature: here the dedup tag */
  uint   chunk;   /* compressed location of the frag in the data region */
  ushort sz;      /* frag size in bytes */
  ushort ctl;     /* SOM/EOM/ERR + origin */
  uint   tsorig;  /* compressed timestamps */
  uint   tspub;
};
typedef struct fd_frag_meta fd_frag_meta_t;

static inline void *
fd_chunk_to_laddr( void * chunk0, ulong chunk ) { return (void *)((ulong)chunk0 + (chunk << FD_CHUNK_LG_SZ)); }

static inline void const *
fd_chunk_to_laddr_const( void const * chunk0, ulong chunk ) { return (void const *)((ulong)chunk0 + (chunk << FD_CHUNK_LG_SZ)); }

#endif /* HEADER_fd_src_tango_fd_tango_base_h */

#ifndef HEADER_fd_src_tango_mcache_fd_mcache_h
/* fd_mcache.h:299-322 semantics: a consumer polling line seq&(depth-1)
   never sees a torn record it would accept as frag seq. */
static inline void
fd_mcache_publish( fd_frag_meta_t * mcache, ulong depth, ulong seq, ulong sig, ulong chunk, ulong sz, ulong ctl,
                   ulong tsorig, ulong tspub ) {
  fd_frag_meta_t * m = mcache + (seq & (depth-1UL));
  __atomic_store_n( &m->seq, seq - 1UL, __ATOMIC_RELEASE );
  __atomic_thread_fence( __ATOMIC_RELEASE );
  m->sig = sig; m->chunk = (uint)chunk; m->sz = (ushort)sz; m->ctl = (ushort)ctl;
  m->tsorig = (uint)tsorig; m->tspub = (uint)tspub;
  __atomic_store_n( &m->seq, seq, __ATOMIC_RELEASE );
}
#endif

#ifndef HEADER_fd_src_tango_dcache_fd_dcache_h
/* fd_dcache.h:263-269: advance to the next chunk pair, wrap at wmark */
static inline ulong
fd_dcache_compact_next( ulong chunk, ulong sz, ulong chunk0, ulong wmark ) {
  chunk += ((sz + (2UL*FD_CHUNK_SZ - 1UL)) >> (1 + FD_CHUNK_LG_SZ)) << 1;
  return chunk > wmark ? chunk0 : chunk;
}
#endif

/* ===== Part 2: the verify tile ===== */

/* diagnostics (fd_frank.h:23-28 names, plus engine-side counts) */
typedef struct {
  ulong in_cnt;        /* input frags read (staged, filtered or rejected) */
  ulong ha_filt_cnt;   /* dropped as HA duplicates before verify */
  ulong ha_filt_sz;
  ulong sv_filt_cnt;   /* dropped by signature verification */
  ulong sv_filt_sz;
  ulong out_cnt;       /* frags published */
  ulong out_sz;
  ulong ovrn_cnt;      /* input frags lost to producer overrun (skipped, or lapped before the tile was done) */
  ulong backp_cnt;     /* times the output was backpressured */
  ulong batch_cnt;     /* hand-offs to the GPU */
  ulong batch_sig_cnt; /* signature slots handed over (PUB_SIG_MSG: frags; TXN: the transactions' signatures) */
  ulong bad_frag_cnt;  /* frags too short / too long to carry a signature, or (zero copy) reaching past the mapped region */
  ulong gpu_chunk_lat_cnt;   /* chunks the GPU verified 8 lanes per signature (latency mode) */
  ulong gpu_chunk_thr_cnt;   /* ... 1 lane per signature (throughput mode) */
  ulong gpu_frag_lat_cnt;    /* frags in those chunks */
  ulong gpu_frag_thr_cnt;
  ulong sv_filt_code_cnt[3]; /* SV_FILT by verdict: FD_ED25519_ERR_SIG, _PUBKEY, _MSG (a TXN parse failure,
                                FD_TXN_AMD_ERR_PARSE, counts in sv_filt_cnt only) */
  ulong halt_drop_cnt;       /* frags taken in but neither published nor filtered: the run halted (*stop) while
                                its output stayed backpressured past the halt grace */
  ulong mode_switch_cnt;     /* switches between chunk levels (latency / quad / throughput) */
  ulong gpu_chunk_quad_cnt;  /* chunks the GPU verified 4 lanes per signature (quad chunks) */
  ulong gpu_frag_quad_cnt;   /* frags in those chunks */
  ulong quad_pair_cnt;       /* quad chunk pairs handed over: two quad chunks over 17..32 frags sharing one front
                                pass (hash + decompression); each counts as two quad chunks above */
} fd_verify_amd_diag_t;

typedef struct fd_verify_amd_tile fd_verify_amd_tile_t;

/* Tile configuration (fd_verify_amd_tile_new_cfg).  Fill it with
   fd_verify_amd_tile_cfg_default, then change what differs.

   GPU side (both framings): ONE persistent kernel per run
   (k_tile_persist) holds `waves` wave slots of the GPU while the run lasts
   (0: 8 x CUs divided by the tiles that exist on the device -- create a
   GPU's tiles before running any; tiles in different processes set their
   share here) and verifies what the tile's host side hands over through
   mapped host memory -- ring entries (frag chunk, output frame, size,
   signature slots) and chunk descriptors -- on one high-priority stream,
   so it needs one hardware queue and the GPU never drains between
   hand-offs.  A process gets GPU_MAX_HW_QUEUES (default 4) such queues:
   creating more tiles than that on one device fails (NULL).  Its share
   must be free when the run starts: a run whose kernel does not start
   within 2 s (another kernel holds the slots) or stops making progress
   returns FD_ED25519_AMD_ERR_DEVICE instead of waiting.

   Chunks.  A chunk takes one wave whatever its size and holds whole frags.
   Three chunk levels: latency chunks hold up to 8 signature slots verified
   8 lanes per signature (~0.45 ms on a SIMD of its own); quad chunks up to
   16 slots, 4 lanes per signature (~0.6 ms alone, ~0.97 ms with every wave
   slot busy); throughput chunks up to 64 slots, 1 lane per signature (~1.2
   ms alone, ~2.2 ms with every wave slot busy), 3-4x the latency chunks'
   signatures per wave-ms.  A PUB_SIG_MSG frag is one slot; a TXN frag takes
   as many slots as its signature count (its first byte), and one of more
   slots than its level's chunk holds makes a 1-lane chunk of its own, handed
   over at once.  All rates and counts below are in slots.
   chunk_mode AUTO picks the level by the staging rate (EWMA over ~0.8 ms;
   fd_verify_amd_tile_level; a higher level at once, except quad to
   throughput, and a lower one only after the rule asked for it for 2 ms,
   fd_verify_amd_tile_level_step): quad chunks above quad_rate_hi, latency chunks
   again below quad_rate_lo (0: 55 % / 40 % of the latency chunks' capacity,
   min(min(waves, 4 x CUs) x 8 / 0.45 ms, window / 0.55 ms)); throughput
   chunks above thr_rate_hi, back below thr_rate_lo (0: 92 % / 90 % of the
   quad chunks' capacity, min(min(waves, 8 x CUs) x 16 / 0.97 ms, window /
   1.1 ms), x 0.75 in TXN framing, whose whole transactions fill ~3/4 of a
   quad chunk's slots).  Quad chunks are skipped (quad thresholds infinite, the
   throughput ones 55 % / 40 % of the latency capacity) when their capacity
   is under 1.25 x the latency chunks'; never throughput chunks when the
   window caps them below the level under them, window / 2 ms.  Whole chunks
   go at once; a partial latency or quad chunk goes once its oldest frag
   waited lat_fill_ns, or at once while fewer than lat_free_chunks chunks are
   in flight; a partial throughput chunk once its oldest waited
   chunk_wait_ns.  Everything staged goes at
   batch_max staged frags, when the window or the output frames run out,
   at the end of the input, and (batch_wait_ns != 0) once the oldest waited
   batch_wait_ns.  At most `window` frags are in flight (handed over, not
   yet published; 0: 2^18 from batch_max 1024, else
   64 x batch_max, >= 2^16).
   Host side.  The caller's thread polls, dedups and stages; publishing
   runs on a second host thread when publish_cpu >= 0 (pinned there) or,
   with FD_VERIFY_AMD_PUBLISH_AUTO, when the caller's CPU set holds another
   CPU (the thread gets that set minus the caller's current CPU);
   FD_VERIFY_AMD_PUBLISH_INLINE keeps both on the caller's thread.  In copy
   mode a third thread, pinned to copy_cpu (>= 0), copies blocks of each
   staging pass's frags beside the caller's thread (passes of 32 frags or
   more; FD_VERIFY_AMD_COPY_INLINE, the default: the caller copies all); a
   block the helper has not finished 30 us after the caller ran out of
   blocks is copied again by the caller into fresh frames, so a descheduled
   helper never stalls the tile.  After *stop the run publishes everything
   it took in; only while its output is backpressured does a grace of
   halt_grace_ns run, after which it returns (halt_drop_cnt).

   Output data region.  Like the reference verify tile, which publishes
   frags out of a dcache it owns (fd_frank_verify_synth_load.c:324,409-411),
   the tile owns its output dcache: out_frame_cnt frames of
   FD_VERIFY_AMD_FRAME_SZ bytes (0: 4096 + batch_max + the window; pinned
   host memory, ~370 MB at the 2^18 window).  Every
   published frag's chunk is relative to fd_verify_amd_tile_out_chunk0 and
   its bytes are the bytes that were verified.  A frame is reused only once
   the consumer's out_fseq has passed the frag it last carried
   (backpressure otherwise), so the output never changes under a consumer
   that honours flow control. */
#define FD_VERIFY_AMD_FRAME_SZ (1408UL)   /* 22 chunks >= 96 + FD_ED25519_AMD_MSG_MAX */

#define FD_VERIFY_AMD_CHUNK_AUTO       (0)
#define FD_VERIFY_AMD_CHUNK_LATENCY    (1)   /* every chunk a latency chunk */
#define FD_VERIFY_AMD_CHUNK_THROUGHPUT (2)   /* every chunk a throughput chunk */
#define FD_VERIFY_AMD_CHUNK_QUAD       (3)   /* every chunk a quad chunk */
/* Quad pairs (environment FD_AMD_TILE_PAIRS=1 when the tile first runs; off
   by default): PUB_SIG_MSG quad chunks are handed over as pairs of two over
   17..32 frags that share one front pass (hash, decompression) on the first
   chunk's wave; the second waits for it.  Exact either way; measured to
   move capacity < 2 %, so opt-in.  diag quad_pair_cnt. */
/* chunk levels (fd_verify_amd_tile_level, the thr argument of _cut / _pack) */
#define FD_VERIFY_AMD_LVL_LAT  (0)           /* 8 slots, 8 lanes per signature */
#define FD_VERIFY_AMD_LVL_THR  (1)           /* 64 slots, 1 lane per signature */
#define FD_VERIFY_AMD_LVL_QUAD (2)           /* 16 slots, 4 lanes per signature */
#define FD_VERIFY_AMD_PUBLISH_AUTO   (-2)
#define FD_VERIFY_AMD_PUBLISH_INLINE (-1)
#define FD_VERIFY_AMD_COPY_INLINE    (-1)

typedef struct {
  int   device;           /* HIP device */
  int   framing;          /* FD_VERIFY_AMD_FRAMING_* (below) */
  ulong batch_max;        /* 1 .. 2^20 */
  ulong batch_wait_ns;
  ulong tcache_depth;     /* HA dedup window (tags remembered, 0 disables) */
  ulong out_frame_cnt;    /* 0: default */
  ulong waves;            /* 0: the device's share */
  int   chunk_mode;       /* FD_VERIFY_AMD_CHUNK_* */
  int   publish_cpu;      /* FD_VERIFY_AMD_PUBLISH_AUTO / _INLINE, or a CPU */
  ulong window;           /* frags in flight; 0: 2^18 from batch_max 1024,
                             else max( 64 x batch_max, 2^16 ) */
  ulong lat_fill_ns;
  ulong lat_free_chunks;
  ulong chunk_wait_ns;
  ulong thr_rate_hi;      /* frags/s, 0: default */
  ulong thr_rate_lo;
  ulong halt_grace_ns;
  int   copy_cpu;         /* FD_VERIFY_AMD_COPY_INLINE, or a CPU for the copy helper */
  ulong quad_rate_hi;     /* slots/s, 0: default (~0UL: never quad chunks in AUTO) */
  ulong quad_rate_lo;
} fd_verify_amd_tile_cfg_t;

/* Defaults: device 0, PUB_SIG_MSG, batch_max 4096, batch_wait_ns 0,
   tcache_depth 2^16, out_frame_cnt 0, waves 0, AUTO chunks, AUTO
   publisher, window 0, lat_fill_ns 20 us, lat_free_chunks CUs / 2,
   chunk_wait_ns 50 us, thr rates 0, halt_grace_ns 50 ms, copy inline,
   quad rates 0. */
void
fd_verify_amd_tile_cfg_default( fd_verify_amd_tile_cfg_t * cfg );

/* NULL on failure (bad configuration, no device, out of memory). */
fd_verify_amd_tile_t *
fd_verify_amd_tile_new_cfg( fd_verify_amd_tile_cfg_t const * cfg );

/* The defaults with these five fields. */
fd_verify_amd_tile_t *
fd_verify_amd_tile_new( int device, ulong batch_max, ulong batch_wait_ns, ulong tcache_depth, ulong out_frame_cnt );

void
fd_verify_amd_tile_delete( fd_verify_amd_tile_t * tile );

/* Local address of chunk 0 of the tile's output data region (published
   chunk c lives at fd_chunk_to_laddr( out_chunk0, c )), and its size. */
void *
fd_verify_amd_tile_out_chunk0( fd_verify_amd_tile_t * tile );

ulong
fd_verify_amd_tile_out_data_sz( fd_verify_amd_tile_t * tile );

/* Frag framing.  PUB_SIG_MSG (default): public_key(32) | signature(64) |
   message, one signature per frag (fd_frank_verify_synth_load.c:340-347).
   TXN: the frag is a wire-format Solana transaction (fd_txn.h); the tile
   parses it on the GPU (fd_txn_parse semantics), verifies every signature
   against its account address (multi-signer) and publishes the transaction
   iff it parses and all its signatures pass; HA dedup uses its first
   signature, the published tag is that signature's SHA-512 tag.  A frag
   that fails to parse counts as SV_FILT (its verdict is
   FD_TXN_AMD_ERR_PARSE); an empty or over-MTU frag is a bad frag.  The
   same persistent kernel verifies both framings (the host reads each
   transaction's signature count; a chunk's lanes parse its transactions,
   verify their signatures and reduce per transaction).  TXN needs
   batch_max >= 19 (the most signatures a 1232-B transaction can carry),
   else ERR_INVAL. */
#define FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG (0)
#define FD_VERIFY_AMD_FRAMING_TXN         (1)
int
fd_verify_amd_tile_set_framing( fd_verify_amd_tile_t * tile, int framing );

/* Input staging.
   Copy mode (default): the tile copies each input frag into its own output
   frame, re-checks the frag's mcache line afterwards (a frag lapped during
   the copy is counted as overrun and dropped), and releases the frag to
   the producer right away (in_fseq advances at staging).  The GPU reads the
   frames from the mapped output region.
   Zero-copy mode: fd_verify_amd_tile_register_dcache maps the host data
   region [base, base+sz) holding the input frags into the GPU
   (hipHostRegister).  When a run's in_chunk0 lies inside it, the tile hands
   the GPU only (chunk, size) per frag; the GPU copies each frag from the
   input region into the device and into the tile's output frame.  The
   input frags of a batch are released (in_fseq) only when that batch has
   retired, and a frag whose mcache line was lapped by then is dropped as
   overrun instead of published. */
int
fd_verify_amd_tile_register_dcache( fd_verify_amd_tile_t * tile, void * base, ulong sz );

/* Run the tile until `frag_cnt` input sequence numbers were consumed (0:
   until *stop != 0) and every accepted frag is published.  A raised *stop
   (stop may be NULL when frag_cnt != 0) also ends a frag_cnt run; the run
   then publishes what it took in, and returns at the latest halt_grace_ns
   after the stop was seen even if the output is backpressured (the rest is
   counted in halt_drop_cnt), the way the reference tile keeps its HALT
   check running while backpressured (fd_frank_verify_synth_load.c:
   223-274).  Input:
   in_mcache (depth in_depth, power of 2), in_chunk0 = local address of
   chunk 0 of the input data region (fd_chunk_to_laddr), first sequence
   number in_seq0.  in_fseq (NULL = none) receives the tile's flow-control
   sequence for the producer (the reference's fseq, fd_fseq_update): every
   input frag below it is no longer read by the tile, so the producer may
   reuse its mcache line and its data.  Output: out_mcache (depth
   out_depth), first sequence out_seq0, frags in the tile's output data
   region; out_fseq (NULL = no flow control) is the slowest consumer's next
   expected sequence number.  Latency samples (tspub - tsorig, in the
   caller's timestamp units) of up to lat_max published frags go to lat
   (NULL to skip).  Returns FD_ED25519_AMD_OK or a negative
   FD_ED25519_AMD_ERR_*. */
int
fd_verify_amd_tile_run( fd_verify_amd_tile_t *  tile,
                        fd_frag_meta_t const *  in_mcache,
                        ulong                   in_depth,
                        void const *            in_chunk0,
                        ulong                   in_seq0,
                        ulong *                 in_fseq,
                        fd_frag_meta_t *        out_mcache,
                        ulong                   out_depth,
                        ulong                   out_seq0,
                        ulong const *           out_fseq,
                        ulong                   frag_cnt,
                        int const *             stop,
                        fd_verify_amd_diag_t *  diag,
                        uint *                  lat,
                        ulong                   lat_max );

/* The tile's timestamp clock (tsorig/tspub units): nanoseconds on the
   CLOCK_MONOTONIC scale, low 32 bits (fd_frag_meta_ts_comp-style
   compression), read from the invariant TSC calibrated once against
   CLOCK_MONOTONIC (the reference stamps frags with fd_tickcount). */
uint
fd_verify_amd_tickcount( void );

/* Per-frag latency decomposition of the next runs (persistent path):
   parts[4 i .. 4 i + 3] for the i-th published frag (the same frags, in
   the same order, as the run's lat samples), in ns: cut wait (staged ->
   handed over), queue wait (handed over -> a wave claimed its chunk),
   service (claimed -> results stored; bit 31 set for a latency chunk),
   publish wait (results stored -> published: the in-order wait behind
   older frags plus the host's poll).  GPU times are mapped onto the host
   clock through the scout's clock word.  parts NULL stops tracing. */
void
fd_verify_amd_tile_set_trace( fd_verify_amd_tile_t * tile, uint * parts, ulong parts_max );

/* Verdict log of the next runs (PUB_SIG_MSG framing): log[seq - in_seq0]
   = the verdict (FD_ED25519_SUCCESS / ERR_*) of every input frag the GPU
   verified whose run-relative sequence is below log_max; frags dropped
   before verification (HA duplicates, bad frags, overruns) leave their
   entry untouched.  log NULL stops logging. */
void
fd_verify_amd_tile_set_verdict_log( fd_verify_amd_tile_t * tile, schar * log, ulong log_max );

/* The hand-off rule (pure; what fd_verify_amd_tile_run applies to its
   staged signature slots [handed, staged)): returns how far to hand over
   now (the run then hands over the whole frags below that).  thr: the
   chunk level, FD_VERIFY_AMD_LVL_THR (64 slots), _QUAD (16) or _LAT (8).
   Whole chunks go at once; a partial latency or quad chunk once waited_ns
   (its oldest frag's wait) >= lat_fill_ns or while chunks_in_flight <
   lat_free_chunks; a partial throughput chunk once waited_ns >=
   chunk_wait_ns; everything at batch_max staged, on flush (end of input,
   or the window / frames ran out while nothing handed over is still
   unpublished) or waited_ns >= batch_wait_ns != 0. */
ulong
fd_verify_amd_tile_cut( fd_verify_amd_tile_cfg_t const * cfg, ulong staged, ulong handed, ulong chunks_in_flight,
                        int thr, ulong waited_ns, int flush );

/* The persistent path's chunk-mode rule (pure): 1 = throughput chunks.
   AUTO: from latency chunks to throughput chunks when rate > rate_hi,
   back when rate < rate_lo; the other modes are fixed. */
int
fd_verify_amd_tile_mode( int chunk_mode, int thr, double rate, double rate_hi, double rate_lo );

/* The persistent path's chunk-level rule (pure): the next level
   (FD_VERIFY_AMD_LVL_*) from the current one.  AUTO: a latency level moves
   to throughput above rate_hi, else to quad above quad_hi; quad moves to
   throughput above rate_hi and back to latency below quad_lo; throughput
   moves down below rate_lo, to quad unless the rate is also below quad_lo.
   The fixed modes return their level. */
int
fd_verify_amd_tile_level( int chunk_mode, int lvl, double rate, double quad_hi, double quad_lo, double rate_hi,
                          double rate_lo );

/* The level step with its holds (pure): the level to run next when the rule
   above asks for `want` at level lvl at time now_ns.  A lower level only once
   the rule has asked for it for hold_ns without a break; throughput chunks in
   place of quad chunks once an episode of asking for them (asks less than
   hold_ns / 2 apart) has lasted hold_ns -- at once within 5 x hold_ns of
   leaving throughput chunks; every other move at once.  st: 4 words of state
   the caller zeroes at the start of a run (NULL: no holds, want is returned). */
int
fd_verify_amd_tile_level_step( int lvl, int want, ulong now_ns, ulong hold_ns, ulong * st );

/* The chunk packing rule (pure): of cnt staged frags carrying slots[i]
   signature slots each, the next chunk takes the first n (returned; *nsl =
   their slots): at most 64 frags and the level's slots (thr:
   FD_VERIFY_AMD_LVL_*, 64 / 16 / 8), whole frags only, so a frag of more
   slots than that is a chunk of its own (verified 1 lane per signature). */
ulong
fd_verify_amd_tile_pack( uint const * slots, ulong cnt, int thr, ulong * nsl );

/* Streaming benchmark and end-to-end check (config 5): a producer thread
   publishes frags public_key | signature | message cyclically from the
   given pool (SoA layout of fd_ed25519_amd_verify_soa; frag s carries pool
   entry s % pool_n) into a private mcache/dcache -- at `rate` frags/s (open
   loop; tsorig = scheduled send time) or, with rate 0, as fast as the tile
   accepts (credit-based flow control on the tile's in_fseq) -- the tile
   runs on `device`, and a consumer drains the
   output.  Runs until frag_cnt input frags were consumed.

   flags: FD_VERIFY_AMD_BENCH_ZERO_COPY maps the input data region into the
   GPU (fd_verify_amd_tile_register_dcache).  FD_VERIFY_AMD_BENCH_WRITE:
   the producer writes every frame into a wrapping data region of
   dcache_frames MTU frames (0: in_depth + 64) before publishing it, as a
   NIC would (otherwise every pool frame is pre-placed once and only
   metadata is published).  FD_VERIFY_AMD_BENCH_LAP: the producer ignores
   the tile's credit (only with WRITE; overrun test).
   FD_VERIFY_AMD_BENCH_SAMPLE_BYTES: the consumer compares the bytes of
   every 16th published frag only (verdict, tag and order of every one), so
   the check does not limit the saturated rate.

   expect_err / expect_tag (pool_n each, NULL = no check): the consumer
   checks every published frag against them -- the frag's verdict must be
   0, its tag (meta sig) must equal expect_tag, its bytes in the tile's
   output region must equal the pool frame, and publication must follow
   input order; in check mode tsorig = the input sequence number (not a
   time), so latency is not measured.  The producer input sequence is
   deterministic, so with no overrun the published set is exactly the pool
   entries with expect_err == 0 in input order.

   out[0] = frags/s through the tile, out[1..3] = p50 / p99 / p999 latency
   in ns (producer publish -> tile publish), out[4] = mean GPU batch size,
   out[5] = frags published, out[6] = frags dropped by verification
   (SV_FILT), out[7] = overrun frags, out[8] = check mismatches (published
   frags that fail a check, plus frags that should have been published and
   were not, overrun ones excepted), out[9] = frags checked, out[10..13] =
   the GPU chunks in latency / throughput mode and the frags in each,
   out[14] = the paced producer's
   largest lateness behind its schedule (ns; its stalls count as latency),
   out[15] = the tile thread's longest pass of its run loop (ns; a stall of
   the host thread shows here), out[16] = the consumer's longest gap between
   two frags it saw.  Latency decomposition (fd_verify_amd_tile_set_trace,
   every published frag, ns; not in check mode): out[17..26] = p50, p99 of
   the cut wait, queue wait, service, publish wait and input wait (latency
   minus the other four: producer publish -> staged), out[27] / out[28] =
   p50 service of latency / throughput chunks, out[29] = chunk-mode
   switches, out[30] = frags traced, out[31] = the producer's longest wait for
   input credit (ns: the tile holding its input, not a producer stall); out[32..37] = the run
   loop's passes, hand-offs, and passes whose staging stopped at the
   window, the output frames, batch_max staged frags and the per-pass
   bound.  Paced runs start once the tile's kernel runs (+2 ms): a run's
   kernel launch is not part of the stream; their latency percentiles
   (out[1..3], out[17..28]) cover the steady state, the frags scheduled
   20 ms or more after the start, and out[38] / out[39] = p50 / p99 of every
   frag.  out[40] (check mode) = the steady-state rate: input frags between
   10 % and 90 % of the run over the time the consumer took from one to the
   other (out[0] includes the run's ramp and drain); out[41] = copy blocks
   the tile's stager re-copied because its helper had stalled; out[42] /
   out[43] = the GPU's quad chunks and the frags in them; out[44..47] =
   the tile thread's time per staged frag (ns, over its passes that staged
   something): listing the pass's frags, copying them (copy mode),
   re-checking and staging them, handing chunks over; out[48] = the quad
   chunk pairs handed over (diag quad_pair_cnt).  out holds 49 doubles.
   Threads: producer, tile, the tile's publisher and consumer each pinned
   to a CPU of their own when the process may use 5 or more (else unpinned,
   publisher inline); copy mode adds the tile's copy helper on a fifth CPU
   when there are 6 or more (FD_VERIFY_AMD_BENCH_COPY_INLINE: none).  waves: the tile's cfg.waves (0: the device's share;
   ranks that share a GPU in separate processes each pass theirs).  Returns
   0 or an error code. */
#define FD_VERIFY_AMD_BENCH_ZERO_COPY (1)
#define FD_VERIFY_AMD_BENCH_WRITE     (2)
#define FD_VERIFY_AMD_BENCH_LAP       (4)
#define FD_VERIFY_AMD_BENCH_SAMPLE_BYTES (8)
#define FD_VERIFY_AMD_BENCH_CHUNK_LAT (16)   /* chunk_mode LATENCY */
#define FD_VERIFY_AMD_BENCH_CHUNK_THR (32)   /* chunk_mode THROUGHPUT */
#define FD_VERIFY_AMD_BENCH_PUB_INLINE (64)  /* publish on the tile's thread */
#define FD_VERIFY_AMD_BENCH_TXN        (128) /* TXN framing: pool entry k is the wire transaction
                                                blob[msg_off[k], +msg_sz[k]) (pub, sig unused); expect_err /
                                                expect_tag per transaction (verdict, first signature's tag) */
#define FD_VERIFY_AMD_BENCH_COPY_INLINE (256) /* copy mode: no copy helper thread */
#define FD_VERIFY_AMD_BENCH_CHUNK_QUAD   (1024) /* chunk_mode QUAD */
#define FD_VERIFY_AMD_BENCH_STALL_HELPER (512) /* test hook: the copy helper spins 200 us before every 4th
                                                 block it claims, so the stager re-copies blocks (out[41]) */

int
fd_verify_amd_bench_stream( int           device,
                            ulong         batch_max,
                            ulong         batch_wait_ns,
                            double        rate,
                            int           flags,
                            ulong         dcache_frames,
                            ulong         pool_n,
                            uchar const * pub,
                            uchar const * sig,
                            uint const *  msg_off,
                            uint const *  msg_sz,
                            uchar const * blob,
                            schar const * expect_err,
                            ulong const * expect_tag,
                            ulong         frag_cnt,
                            ulong         waves,
                            double *      out );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_tango_amd_h */
