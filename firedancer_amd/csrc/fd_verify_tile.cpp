/* firedancer_amd/csrc/fd_verify_tile.cpp
 *
 * Tango-compatible streaming verify tile on the MI355X engine
 * (include/fd_tango_amd.h).
 *
 * The reference verify tile (src/app/frank/load/fd_frank_verify_synth_load.c:
 * 219-437) verifies one frag per fd_ed25519_verify call.  Here the run loop
 * is split into a host side that never blocks on the GPU and ONE persistent
 * GPU kernel per run (k_tile_persist) that verifies whole chunks of frags:
 *
 *   poll    -- read the next input frag metadata (seq-checked, overrun-aware)
 *   dedup   -- HA tag cache (tag = first 8 signature bytes), FD_TCACHE_INSERT
 *              semantics (src/tango/tcache/fd_tcache.h:372-403): a tag is a
 *              duplicate iff it is one of the last `depth` distinct tags
 *   stage   -- reserve a frame of the tile-owned output dcache; copy mode:
 *              copy the frag into it, re-check the mcache line, release the
 *              input frag; zero-copy: hand the GPU (chunk, size) only
 *   hand    -- cut staged frags into chunks for the persistent kernel by the
 *              load.  PUB_SIG_MSG framing: a frag is one signature slot;
 *              TXN framing: a frag is a wire transaction whose signature
 *              count the host reads from its first byte, chunks are packed
 *              by signature slots and the GPU parses, verifies every
 *              signature and reduces per transaction
 *   publish -- in arrival order (fd_mcache_publish protocol) out of the
 *              output dcache, with the GPU's SHA-512-derived dedup tag as
 *              meta.sig; failures count SV_FILT; zero-copy releases input
 *              frags only now.  Publishing runs on a second host thread when
 *              the tile has a CPU for it.
 *
 * The output data region follows the reference tile's ownership model: the
 * tile publishes frags from a dcache it owns (fd_frank_verify_synth_load.c:
 * 324,409-411) and takes output credit from its consumers' fseq
 * (fd_frank_verify.c:85-92,167).
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <dirent.h>
#include <unistd.h>
#include <sys/syscall.h>
#include <x86intrin.h>
#include <thread>
#include <sched.h>
#include <pthread.h>
#include <vector>
#include <atomic>
#include <mutex>
#include <algorithm>

#include "../../include/fd_ed25519_amd.h"
#include "../../include/fd_txn_amd.h"
#include "../../include/fd_tango_amd.h"
#include "fd_ed25519_engine.h"
#include "fd_ed25519_kernels.h"

/* ------------------------------------------------------------------ */
/* HA tag cache: ring of the last `depth` distinct tags + open-addressed
   set (linear probing, backward-shift delete), map_cnt a power of 2 >=
   2*depth+2 so probes stay short. */

namespace {

struct tcache_t {
  ulong depth, map_cnt, oldest; int sh;
  std::vector<ulong> ring, map;
  void init( ulong d ) {
    depth = d; oldest = 0;
    map_cnt = 4; sh = 62; while( map_cnt < 2UL*d + 2UL ) { map_cnt <<= 1; sh--; }
    ring.assign( d ? d : 1, 0UL ); map.assign( map_cnt, 0UL );
  }
  ulong slot( ulong tag ) const { return (tag * 0x9E3779B97F4A7C15UL) >> sh; }   /* Fibonacci hashing */
  bool find( ulong tag, ulong * at ) const {
    ulong i = slot( tag );
    for( ;; ) {
      ulong v = map[i];
      if( v == tag ) { *at = i; return true; }
      if( !v ) { *at = i; return false; }
      i = (i + 1UL) & (map_cnt - 1UL);
    }
  }
  void remove( ulong tag ) {
    ulong i;
    if( !tag || !find( tag, &i ) ) return;
    /* backward-shift deletion keeps every probe chain contiguous */
    ulong j = i;
    for( ;; ) {
      j = (j + 1UL) & (map_cnt - 1UL);
      ulong v = map[j];
      if( !v ) break;
      ulong h = slot( v );
      /* can v move to the hole at i?  yes iff h is not cyclically in (i, j] */
      bool in = (i <= j) ? (h > i && h <= j) : (h > i || h <= j);
      if( !in ) { map[i] = v; i = j; }
    }
    map[i] = 0UL;
  }
  /* FD_TCACHE_INSERT: returns 1 if tag is a duplicate, else inserts it
     (evicting the oldest tag once the window is full) and returns 0 */
  int insert( ulong tag ) {
    if( !depth || !tag ) return 0;          /* FD_TCACHE_TAG_NULL is never inserted */
    ulong at;
    if( find( tag, &at ) ) return 1;
    map[at] = tag;
    ulong old = ring[oldest];
    ring[oldest] = tag;
    if( ++oldest >= depth ) oldest = 0;
    remove( old );
    return 0;
  }
};

struct pending_t {            /* one staged / in-flight frag (ring entry) */
  ulong  seq;                 /* input sequence number */
  ushort sz, ctl;
  uint   tsorig;
  uint   fidx;                /* its output frame */
  uint   t_stage;             /* host clock (low 32 bits of ns) when staged */
  uint   t_hand;              /* ... when its chunk was handed over (bit 0: latency chunk) */
  uint   sl_end;              /* signature slots staged up to and including this entry (mod 2^32) */
  uint   slots;               /* its signature slots (PUB_SIG_MSG: 1; TXN: fd_amd_txn_slots1) */
  uint   pad;
};

inline ulong mono_ns( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (ulong)ts.tv_sec * 1000000000UL + (ulong)ts.tv_nsec;
}

/* CLOCK_MONOTONIC nanoseconds read from the invariant TSC (as the
   reference stamps frags with fd_tickcount, not a syscall-class clock):
   clock_gettime costs ~20 ns, a per-frag cost on both sides of the tile at
   ~20 M frags/s.  Calibrated once against CLOCK_MONOTONIC over 20 ms. */
struct tsc_clock_t {
  ulong  ns0, tsc0;
  double ns_per_tick;
  tsc_clock_t() {
    ulong a_ns = mono_ns(), a_t = __rdtsc();
    while( mono_ns() - a_ns < 20000000UL ) { /* spin */ }
    ulong b_ns = mono_ns(), b_t = __rdtsc();
    ns_per_tick = (double)(b_ns - a_ns) / (double)(b_t - a_t);
    ns0 = b_ns; tsc0 = b_t;
  }
};

inline tsc_clock_t const & tsc_clock( void ) {
  static tsc_clock_t const c;   /* thread-safe one-time init */
  return c;
}

inline ulong now_ns( void ) {
  tsc_clock_t const & c = tsc_clock();
  return c.ns0 + (ulong)((double)(long)(__rdtsc() - c.tsc0) * c.ns_per_tick);
}

} /* namespace */

#define FRAME_CHUNKS ((uint)(FD_VERIFY_AMD_FRAME_SZ >> FD_CHUNK_LG_SZ))
#define FRAME_FREE   (~0UL)
#define TXN_SIG_MAX_AT_MTU (19UL)   /* most signatures fd_amd_txn_slots1 reserves for a 1232-B payload */
#define STAGE_PASS   (256UL)        /* frags staged per pass of the run loop before it hands over */
#define CHUNK_SLOTS  (64UL)         /* signature slots of a throughput chunk (one lane each) */
#define LAT_SLOTS    (8UL)          /* ... of a latency chunk (8 lanes each) */
#define QUAD_SLOTS   (16UL)         /* ... of a quad chunk (4 lanes each) */
/* a quad chunk's service with every wave slot busy (0.97 ms measured:
   2047 waves x 16 frags saturate at 33 M frags/s, profiles/
   r06_quad_probe_a.jsonl), and a frag's time in flight in quad mode (the
   quad capacity and the window it needs) */
#define QUAD_SVC_S    (0.97e-3)
#define QUAD_FLIGHT_S (1.1e-3)

/* a lower chunk level is taken only once the rule asked for it this long,
   and throughput chunks instead of quad chunks too (fd_verify_amd_tile_level_step) */
#define LVL_HOLD_NS (2000000UL)

/* order of the chunk levels by capacity: latency < quad < throughput */
static inline int lvl_rank( int lvl ) {
  return lvl == FD_VERIFY_AMD_LVL_THR ? 2 : lvl == FD_VERIFY_AMD_LVL_QUAD ? 1 : 0;
}

/* slots of a chunk of chunk level lvl (FD_VERIFY_AMD_LVL_*) */
static inline ulong lvl_slots( int lvl ) {
  return lvl == FD_VERIFY_AMD_LVL_THR ? CHUNK_SLOTS : lvl == FD_VERIFY_AMD_LVL_QUAD ? QUAD_SLOTS : LAT_SLOTS;
}

/* Copy mode's helper protocol (below) */
#define CP_NB       (2UL)                    /* copy blocks per pass: the two halves (one CAS each: finer blocks cost
                                                more in cache-line round trips than they balance) */
#define CP_NJ       (4UL)                    /* job arrays in the helper's ring */
#define CP_STEAL_NS (30000UL)                /* a helper block still unfinished this long after the stager ran out of
                                                blocks is re-copied by the stager into fresh frames */
#define COPY_SPLIT_MIN (32UL)                /* passes of fewer frags are copied on the stager alone */

/* Copy mode's staging copy: whole 16-B words (a frag's chunks are 64-B
   granular, so the rounded-up tail stays inside its own chunks) with
   non-temporal stores -- the frame is read next by the GPU over PCIe, not by
   this CPU, so it skips the read-for-ownership of every destination line and
   stays out of the cache.  Weakly ordered: the stager fences (sfence) before
   it publishes the head that hands the frames over. */
/* the same in whole 64-B lines with AVX-512 (frames and frags are 64-B
   aligned and 64-B granular): a quarter of the store instructions */
__attribute__((target("avx512f"))) static void
stage_copy_nt512( uchar * dst, uchar const * src, ulong sz ) {
  ulong const n = (sz + 63UL) >> 6;
  __m512i const * s = (__m512i const *)src;
  __m512i * d = (__m512i *)dst;
  ulong k = 0;
  for( ; k + 2UL <= n; k += 2UL ) {
    __m512i const a = _mm512_load_si512( s + k ), b = _mm512_load_si512( s + k + 1 );
    _mm512_stream_si512( d + k, a ); _mm512_stream_si512( d + k + 1, b );
  }
  for( ; k < n; k++ ) _mm512_stream_si512( d + k, _mm512_load_si512( s + k ) );
}

static bool const g_avx512 = __builtin_cpu_supports( "avx512f" );

static inline void
stage_copy_nt( uchar * dst, uchar const * src, ulong sz ) {
  if( g_avx512 && !(((ulong)dst | (ulong)src) & 63UL) ) { stage_copy_nt512( dst, src, sz ); return; }
  ulong const n = (sz + 15UL) >> 4;
  __m128i const * s = (__m128i const *)src;
  __m128i * d = (__m128i *)dst;
  ulong k = 0;
  for( ; k + 4UL <= n; k += 4UL ) {
    __m128i const a = _mm_loadu_si128( s + k ), b = _mm_loadu_si128( s + k + 1 );
    __m128i const c = _mm_loadu_si128( s + k + 2 ), e = _mm_loadu_si128( s + k + 3 );
    _mm_stream_si128( d + k, a ); _mm_stream_si128( d + k + 1, b );
    _mm_stream_si128( d + k + 2, c ); _mm_stream_si128( d + k + 3, e );
  }
  for( ; k < n; k++ ) _mm_stream_si128( d + k, _mm_loadu_si128( s + k ) );
}

/* Copy mode's deferred staging: a pass first reserves a frame per frag and
   lists the copies, then copies them, and only then re-checks each frag's
   mcache line and stages it (a frag lapped during its copy leaves its frame
   unused). */
struct copy_job_t {
  uchar *                dst;
  uchar const *          src;
  fd_frag_meta_t const * m;
  ulong                  seq, sz, tag;   /* tag: the HA dedup tag, read from the source before the copy */
  uint                   f, tsorig, slots;
  ushort                 ctl;
};

static void
copy_jobs( copy_job_t const * j, ulong lo, ulong hi ) {
  for( ulong k=lo; k<hi; k++ ) {
    if( k + 2UL < hi ) for( ulong o = 0; o < j[k+2].sz; o += 64UL ) __builtin_prefetch( j[k+2].src + o );
    stage_copy_nt( j[k].dst, j[k].src, j[k].sz );
  }
}

/* The copy helper (cfg.copy_cpu).  A pass posts its job list as a
   generation g into job array g % CP_NJ; the stager and the helper both
   claim its two halves by CAS on `claim` (g << 16 | next block),
   and the helper marks each block it copied in done[g % CP_NJ][b] = g.
   The stager never waits on a helper that stopped running (a descheduled
   pinned thread held a pass for up to 9 ms, profiles/r05_bench_a_detail.json):
   a helper block still unfinished CP_STEAL_NS after the stager ran out of
   blocks is copied again by the stager into FRESH frames, and the frames the
   helper may still write stay reserved ("orphaned") until its done mark
   shows up -- nothing ever reads them, so a late helper write (its source
   possibly rewritten by then) cannot reach a published frag.  The stager
   never rewrites a posted job record (the helper may still be reading it):
   the fresh frames of a re-copied block live in the stager's own frame
   list.  A job array is reused only when none of its blocks is orphaned. */
struct copier_t {
  alignas(64) std::atomic<ulong> claim;
  alignas(64) std::atomic<int>   quit;
  alignas(64) std::atomic<ulong> done[CP_NJ][CP_NB];
  std::atomic<ulong>             nj[CP_NJ], bsz[CP_NJ];   /* a pass's frags and its block size (half, rounded up) */
  copy_job_t                     jobs[CP_NJ][STAGE_PASS];
};

/* Test hook (FD_VERIFY_AMD_BENCH_STALL_HELPER): the helper spins this long
   before every 4th block it claims, so the stager's re-copy path runs */
static std::atomic<ulong> copier_stall_ns( 0UL );

static void
copier_loop( copier_t * cp, int cpu ) {
  cpu_set_t one; CPU_ZERO( &one ); CPU_SET( cpu, &one );
  (void)pthread_setaffinity_np( pthread_self(), sizeof one, &one );
  ulong const stall = copier_stall_ns.load( std::memory_order_relaxed );
  ulong nclaim = 0UL;
  for( ;; ) {
    ulong c = cp->claim.load( std::memory_order_acquire );
    ulong const g = c >> 16, b = c & 0xffffUL;
    if( g ) {
      ulong const s = g % CP_NJ, nj = cp->nj[s].load( std::memory_order_relaxed ), bz = cp->bsz[s].load( std::memory_order_relaxed );
      if( b < CP_NB && b * bz < nj ) {
        if( cp->claim.compare_exchange_weak( c, c + 1UL, std::memory_order_acq_rel ) ) {
          if( stall && !(nclaim++ & 3UL) ) { ulong const t0 = now_ns(); while( now_ns() - t0 < stall ) _mm_pause(); }
          copy_jobs( cp->jobs[s], b * bz, std::min( nj, (b + 1UL) * bz ) );
          _mm_sfence();   /* the copies before the done mark */
          cp->done[s][b].store( g, std::memory_order_release );
        }
        continue;
      }
    }
    if( cp->quit.load( std::memory_order_acquire ) ) break;
    _mm_pause();
  }
}

struct orphan_t { ulong g, s, b; std::vector<uint> frames; };

/* The window rule: frags handed over and not yet published */
static ulong
tile_window( fd_verify_amd_tile_cfg_t const * c ) {
  if( c->window ) return c->window;
  /* in flight = rate x latency: ~1.3-2.2 ms at up to ~60 M frags/s under
     load, plus a hand-off's worth of head-of-line wait (a window that binds
     at 80 % load shows up as input wait in the tail: 2^17 did at batch_max
     1024 on a 60 M frags/s box, profiles/r05_bench_tile_window1024.json) */
  if( c->batch_max >= (1UL << 10) ) return 1UL << 18;
  /* small batch caps: quad chunks carry ~26 M frags/s at 80 % load for
     ~0.7 ms each; a 2^15 window bound them there (input wait p99 ~1 ms,
     p99 3 x p50; profiles/r06_bench_quad_b_detail.json) */
  return std::max( 64UL * c->batch_max, 1UL << 16 );
}

struct fd_verify_amd_tile {
  fd_verify_amd_tile_cfg_t cfg;
  int                device;
  ulong              batch_max;
  tcache_t           tc;
  int                framing;   /* FD_VERIFY_AMD_FRAMING_* */
  int                cus;
  uint8_t *          reg_base;  /* host data region mapped into the GPU (zero copy) */
  ulong              reg_sz;
  uint8_t *          reg_dev;
  /* the tile-owned output dcache: frame_cnt frames, pinned and mapped */
  uint8_t *          out_base;
  uint8_t *          out_dev;
  ulong              frame_cnt;
  std::vector<ulong> frame_pub;  /* out seq of the frag a frame last carried (FRAME_FREE: none) */
  uint8_t *          frame_busy; /* 1 while a frame is staged, in flight, or orphaned (stager sets, publisher clears) */
  ulong              frame_next_idx;   /* next frame to reserve (cyclic) */
  ulong              out_seq_end;   /* out seq after the last run's last publish (a run continuing it keeps frame_pub) */
  /* persistent consumer (k_tile_persist) */
  bool                 persist_ok;  /* its resources are allocated */
  hipStream_t          pst;
  hipEvent_t           pdone;
  bool                 pending;     /* a kernel of an earlier run had not finished when that run returned */
  fd_amd_tile_hctl_t * hctl;  void * hctl_dev;
  fd_amd_tile_ent_t *  ring;  void * ring_dev;
  fd_amd_tile_desc_t * desc;  void * desc_dev;   /* chunk descriptors (same size as the ring) */
  uint64_t *           res;   void * res_dev;   /* results: R tags, R verdict words, R time stamps */
  fd_amd_tile_dctl_t * dctl;
  fd_amd_tile_dctl_t   d0;          /* its seed (host copy, alive while the copy is queued) */
  uint8_t *            scratch;
  /* quad pairs (FD_AMD_TILE_PAIR): pair_cnt shared workspaces + flags, the
     next pair's sequence number, and per workspace the ring index after the
     frags of the pair that last used it (free once published) */
  uint8_t *            pair_ws;
  uint32_t *           pair_flag;
  ulong                pair_cnt, pair_seq;
  std::vector<ulong>   pair_end;
  std::vector<uint32_t> pair_zero;  /* the flags' seed (alive while its copy is queued) */
  ulong                n_pair;     /* the last run's pairs */
  ulong                R;          /* ring size (power of 2) */
  ulong                window;     /* frags in flight at most (handed to the GPU, not yet published) */
  uint32_t             waves;      /* grid of a run (the share), fixed at the first run */
  double               rate_hi, rate_lo;     /* throughput chunks above / below (slots/s) */
  double               quad_hi, quad_lo;     /* quad chunks (instead of latency chunks) above / below */
  bool                 counted;       /* in the per-device tile count */
  ulong                desc_seq;      /* descriptors published, monotonic over the tile's life */
  std::vector<pending_t> ppend;    /* per ring slot */
  std::vector<ulong>   desc_end;   /* per descriptor: ring index after its last frag */
  ulong                ring_seq;   /* ring index of the next frag, monotonic over the tile's life */
  ulong                pass_max_ns;   /* longest pass of the last run's loop (stall diagnosis) */
  uint *               trace;  ulong trace_max;
  schar *              vlog;   ulong vlog_max;
  /* the last run's loop: passes, hand-offs, and the passes whose staging
     stopped at the window, the output frames, batch_max staged, or the
     STAGE_PASS bound; copy blocks the stager re-copied (helper stalls) */
  ulong                n_pass, n_hand, n_stop_window, n_stop_frames, n_stop_bmax, n_stop_pass, n_steal;
  /* the last run's stager time (TSC ticks) in passes that staged something:
     listing, copying (copy mode), re-check + staging, hand-off; and the
     frags those passes staged */
  ulong                ph_tick[4], ph_frags;
  volatile int         started;    /* the current run's kernel wrote its first clock word */
};

extern "C" void
fd_verify_amd_tile_cfg_default( fd_verify_amd_tile_cfg_t * c ) {
  if( !c ) return;
  memset( c, 0, sizeof *c );
  c->device = 0;
  c->framing = FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG;
  c->batch_max = 4096UL;
  c->tcache_depth = 1UL << 16;
  c->chunk_mode = FD_VERIFY_AMD_CHUNK_AUTO;
  c->publish_cpu = FD_VERIFY_AMD_PUBLISH_AUTO;
  c->lat_fill_ns = 20000UL;
  c->lat_free_chunks = 0UL;         /* resolved to CUs / 2 at creation */
  c->chunk_wait_ns = 50000UL;
  c->halt_grace_ns = 50000000UL;
  c->copy_cpu = FD_VERIFY_AMD_COPY_INLINE;
}

extern "C" int
fd_verify_amd_tile_register_dcache( fd_verify_amd_tile_t * t, void * base, ulong sz ) {
  if( !t || !base || !sz ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( t->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  /* an unregister that fails (the range was unregistered elsewhere) must not
     leave its error pending for the next launch check (hipGetLastError) */
  if( t->reg_base ) {
    if( hipHostUnregister( t->reg_base ) != hipSuccess ) (void)hipGetLastError();
    t->reg_base = NULL; t->reg_dev = NULL; t->reg_sz = 0;
  }
  uintptr_t lo = (uintptr_t)base & ~(uintptr_t)4095, hi = ((uintptr_t)base + sz + 4095) & ~(uintptr_t)4095;
  if( hipHostRegister( (void *)lo, hi - lo, hipHostRegisterMapped ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  void * dev = NULL;
  if( hipHostGetDevicePointer( &dev, (void *)lo, 0 ) != hipSuccess ) {
    if( hipHostUnregister( (void *)lo ) != hipSuccess ) (void)hipGetLastError();
    return FD_ED25519_AMD_ERR_DEVICE;
  }
  t->reg_base = (uint8_t *)lo; t->reg_sz = hi - lo; t->reg_dev = (uint8_t *)dev;
  return FD_ED25519_AMD_OK;
}

/* Live tiles per device (process-wide).  A run's persistent kernel takes
   8 x CUs / (tiles on its device) wave slots unless cfg.waves fixes its
   share.  Each tile's kernel occupies a hardware queue of the high-priority
   pool for the whole run, and HIP shares GPU_MAX_HW_QUEUES queues per
   priority among a process's streams: a tile beyond that count would queue
   its kernel behind another tile's until that run ends, so creation refuses
   it (tile_queue_max). */
namespace {
std::mutex g_tile_mu;
int        g_tile_cnt[64];
}

static int
tile_queue_max( void ) {
  char const * e = getenv( "GPU_MAX_HW_QUEUES" );
  int v = e && *e ? atoi( e ) : 0;
  return v > 0 ? v : 4;   /* HIP's default */
}

static bool
tile_count( fd_verify_amd_tile_t * t, bool in ) {
  int device = t->device;
  if( device < 0 || device >= 64 || t->counted == in ) return true;
  std::lock_guard<std::mutex> g( g_tile_mu );
  if( in && g_tile_cnt[device] >= tile_queue_max() ) return false;
  g_tile_cnt[device] += in ? 1 : -1;
  t->counted = in;
  return true;
}

static uint32_t
tile_share( fd_verify_amd_tile_t const * t ) {
  if( t->cfg.waves ) return (uint32_t)t->cfg.waves;
  int n = 1;
  if( t->device >= 0 && t->device < 64 ) {
    std::lock_guard<std::mutex> g( g_tile_mu );
    n = std::max( 1, g_tile_cnt[t->device] );
  }
  return std::max( 2u, (uint32_t)(8 * t->cus) / (uint32_t)n );
}

extern "C" int
fd_verify_amd_tile_set_framing( fd_verify_amd_tile_t * t, int framing ) {
  if( !t || (framing != FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG && framing != FD_VERIFY_AMD_FRAMING_TXN) )
    return FD_ED25519_AMD_ERR_INVAL;
  /* every transaction must fit one hand-off */
  if( framing == FD_VERIFY_AMD_FRAMING_TXN && t->batch_max < TXN_SIG_MAX_AT_MTU ) return FD_ED25519_AMD_ERR_INVAL;
  t->framing = framing;
  return FD_ED25519_AMD_OK;
}

extern "C" void *
fd_verify_amd_tile_out_chunk0( fd_verify_amd_tile_t * t ) {
  return t ? t->out_base : NULL;
}

extern "C" ulong
fd_verify_amd_tile_out_data_sz( fd_verify_amd_tile_t * t ) {
  return t ? t->frame_cnt * FD_VERIFY_AMD_FRAME_SZ : 0UL;
}

extern "C" void
fd_verify_amd_tile_set_trace( fd_verify_amd_tile_t * t, uint * parts, ulong parts_max ) {
  if( !t ) return;
  t->trace = parts; t->trace_max = parts ? parts_max : 0UL;
}

extern "C" void
fd_verify_amd_tile_set_verdict_log( fd_verify_amd_tile_t * t, schar * log, ulong log_max ) {
  if( !t ) return;
  t->vlog = log; t->vlog_max = log ? log_max : 0UL;
}

extern "C" uint
fd_verify_amd_tickcount( void ) {
  return (uint)now_ns();
}

/* The kernel of an earlier run that returned an error before it finished
   (a run never waits for it unboundedly): 0 once it is done. */
static int
tile_kernel_busy( fd_verify_amd_tile_t * t ) {
  if( !t->pending ) return 0;
  if( hipEventQuery( t->pdone ) == hipErrorNotReady ) return 1;
  t->pending = false;
  return 0;
}

/* Free the persistent consumer's resources (all of them, or what a failed
   allocation got): a later run allocates them afresh. */
static void
tile_persist_free( fd_verify_amd_tile_t * t ) {
  if( t->pst )     (void)hipStreamDestroy( t->pst );
  if( t->pdone )   (void)hipEventDestroy( t->pdone );
  if( t->hctl )    (void)hipHostFree( t->hctl );
  if( t->ring )    (void)hipHostFree( t->ring );
  if( t->desc )    (void)hipHostFree( t->desc );
  if( t->res )     (void)hipHostFree( t->res );
  if( t->dctl )    (void)hipFree( t->dctl );
  if( t->scratch ) (void)hipFree( t->scratch );
  if( t->pair_ws ) (void)hipFree( t->pair_ws );
  if( t->pair_flag ) (void)hipFree( t->pair_flag );
  t->pst = NULL; t->pdone = NULL; t->hctl = NULL; t->ring = NULL; t->desc = NULL; t->res = NULL;
  t->dctl = NULL; t->scratch = NULL; t->pair_ws = NULL; t->pair_flag = NULL; t->pair_cnt = 0UL;
  t->persist_ok = false;
}

extern "C" void
fd_verify_amd_tile_delete( fd_verify_amd_tile_t * t ) {
  if( !t ) return;
  (void)tile_count( t, false );
  (void)hipSetDevice( t->device );
  if( t->pending && t->hctl ) {   /* an abandoned kernel: ask it to exit, then wait for it */
    __atomic_store_n( &t->hctl->stop, 1u, __ATOMIC_RELEASE );
    (void)hipEventSynchronize( t->pdone );
  }
  if( t->pst ) (void)hipStreamSynchronize( t->pst );
  if( t->reg_base ) (void)hipHostUnregister( t->reg_base );
  if( t->out_base ) (void)hipHostFree( t->out_base );
  tile_persist_free( t );
  free( t->frame_busy );
  delete t;
}

/* The chunk levels' rate thresholds (slots/s) for the tile's share and
   window, at the start of every run (the framing may change between runs).
   TXN chunks hold whole transactions, so a quad chunk's 16 slots are ~3/4
   filled on a mix of 1..12 signers: its capacity in slots is taken at
   0.75 x (at 92 % of the full figure, TXN quad chunks queued for ms at 28 M
   slots/s, profiles/r06_bench_quad_c_detail.json). */
static void
tile_set_levels( fd_verify_amd_tile_t * t ) {
  /* latency chunks' capacity: one 8-slot chunk per SIMD at ~0.45 ms, and
     the window over their ~0.55 ms in flight.  Throughput chunks keep a frag
     in flight 1.3-2.2 ms, so a small window caps them at W / 2 ms: when that
     is below the latency chunks' capacity the tile stays in latency chunks
     (batch_max 256: 8 M vs 18 M frags/s).  Rates are signature slots/s. */
  double const cap  = std::min( (double)std::min( (ulong)t->waves - 1UL, 4UL * (ulong)t->cus ) * 8.0 / 450e-6,
                                (double)t->window / 550e-6 );
  /* quad chunks (16 slots, 4 lanes each): two per SIMD at ~0.9 ms, a frag
     ~1.1 ms in flight; used between the two when they carry well above the
     latency chunks' capacity */
  double const qpack = t->framing == FD_VERIFY_AMD_FRAMING_TXN ? 0.75 : 1.0;
  double const qcap = qpack * std::min( (double)std::min( (ulong)t->waves - 1UL, 8UL * (ulong)t->cus ) * (double)QUAD_SLOTS / QUAD_SVC_S,
                                (double)t->window / QUAD_FLIGHT_S );
  bool const   quad_ok = qcap > 1.25 * cap;
  double const below = quad_ok ? qcap : cap;   /* the capacity under throughput chunks */
  bool const   thr_ok = (double)t->window / 2e-3 > below;
  t->quad_hi = t->cfg.quad_rate_hi ? (double)t->cfg.quad_rate_hi : quad_ok ? 0.55 * cap : HUGE_VAL;
  t->quad_lo = t->cfg.quad_rate_lo ? (double)t->cfg.quad_rate_lo : quad_ok ? 0.40 * cap : HUGE_VAL;
  if( t->quad_lo > t->quad_hi ) t->quad_lo = t->quad_hi;
  /* quad chunks serve up to ~90 % of their capacity at p50 ~0.8 ms (0.80 ms
     at 30 M frags/s, against 1.28 ms in throughput chunks; 0.67 ms at 25 M),
     so they hold until 92 % of it, and are taken back below 90 % (was 80 %:
     half load on a 55 M frags/s box, 27.9 M, sat inside that band, so one
     stall's burst left it in throughput chunks for good); the holds of
     fd_verify_amd_tile_level_step damp the narrow band */
  t->rate_hi = t->cfg.thr_rate_hi ? (double)t->cfg.thr_rate_hi : thr_ok ? (quad_ok ? 0.92 : 0.55) * below : HUGE_VAL;
  t->rate_lo = t->cfg.thr_rate_lo ? (double)t->cfg.thr_rate_lo : thr_ok ? (quad_ok ? 0.90 : 0.40) * below : HUGE_VAL;
  if( t->rate_lo > t->rate_hi ) t->rate_lo = t->rate_hi;
}

/* The persistent consumer's resources (allocated at the first run):
   control words, ring, descriptors and results in mapped coherent host
   memory, the device control block, per-wave scratch.  A failure frees
   what was allocated (ERR_DEVICE), so a retry starts clean. */
static int
tile_persist_alloc( fd_verify_amd_tile_t * t ) {
  if( t->persist_ok ) return FD_ED25519_AMD_OK;
  ulong W = std::min( tile_window( &t->cfg ), t->frame_cnt );
  if( !W ) return FD_ED25519_AMD_ERR_INVAL;
  ulong R = 1UL; while( R < W ) R <<= 1;
  uint32_t waves = tile_share( t );
  if( waves < 2u || waves > 65536u ) return FD_ED25519_AMD_ERR_INVAL;
  t->window = W; t->R = R; t->waves = waves;
  tile_set_levels( t );
  unsigned const hf = hipHostMallocMapped | hipHostMallocCoherent;
  /* The run's kernel occupies its hardware queue for the whole run, and HIP
     multiplexes streams onto a few hardware queues per priority
     (GPU_MAX_HW_QUEUES, 4 by default): a normal stream that landed on the
     same queue would wait behind the persistent kernel until the run ends.
     A high-priority stream comes from the other pool, so engine calls never
     queue behind it (tiles themselves are capped per device: tile_count). */
  int prio_lo = 0, prio_hi = 0;
  if( hipDeviceGetStreamPriorityRange( &prio_lo, &prio_hi ) != hipSuccess ) prio_hi = 0;
  if( hipStreamCreateWithPriority( &t->pst, hipStreamNonBlocking, prio_hi ) != hipSuccess ||
      hipEventCreateWithFlags( &t->pdone, hipEventDisableTiming ) != hipSuccess ||
      hipHostMalloc( (void **)&t->hctl, sizeof(fd_amd_tile_hctl_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->hctl_dev, t->hctl, 0 ) != hipSuccess ||
      hipHostMalloc( (void **)&t->ring, R * sizeof(fd_amd_tile_ent_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->ring_dev, t->ring, 0 ) != hipSuccess ||
      hipHostMalloc( (void **)&t->desc, R * sizeof(fd_amd_tile_desc_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->desc_dev, t->desc, 0 ) != hipSuccess ||
      hipHostMalloc( (void **)&t->res, 3UL * R * sizeof(uint64_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->res_dev, t->res, 0 ) != hipSuccess ||
      hipMalloc( (void **)&t->dctl, sizeof(fd_amd_tile_dctl_t) ) != hipSuccess ||
      hipMalloc( (void **)&t->scratch, waves * fd_amd_tile_scratch_stride() ) != hipSuccess ) {
    (void)hipGetLastError();
    tile_persist_free( t );
    return FD_ED25519_AMD_ERR_DEVICE;
  }
  memset( t->hctl, 0, sizeof(fd_amd_tile_hctl_t) );
  memset( t->ring, 0, R * sizeof(fd_amd_tile_ent_t) );
  memset( t->desc, 0, R * sizeof(fd_amd_tile_desc_t) );
  memset( t->res,  0, 3UL * R * sizeof(uint64_t) );   /* word 0 never matches an index + 1 */
  /* quad pairs: as many workspaces as half the waves could run at once
     (each pair is two quad chunks).  Opt-in (FD_AMD_TILE_PAIRS=1): sub 1's
     wave sleeps through sub 0's front, so a pair frees SIMD issue slots but
     not wave slots, and measured it moved quad capacity by < 2 % and p50 at
     30 M frags/s by -6 %, p99 at 20 M auto +60 % through extra level
     switches (profiles/r06_quad_pairs_ab.txt) -- not worth its default. */
  {
    char const * e = getenv( "FD_AMD_TILE_PAIRS" );
    ulong pc = 64UL; while( pc < (ulong)waves / 2UL ) pc <<= 1;
    if( e && *e == '1' &&
        hipMalloc( (void **)&t->pair_ws, pc * fd_amd_tile_scratch_stride() ) == hipSuccess &&
        hipMalloc( (void **)&t->pair_flag, pc * sizeof(uint32_t) ) == hipSuccess &&
        /* zeroed by a copy queued ahead of the first kernel on the tile's
           stream (no device-wide sync: another tile's kernel may be running) */
        ( t->pair_zero.assign( pc, 0u ),
          hipMemcpyAsync( t->pair_flag, t->pair_zero.data(), pc * sizeof(uint32_t), hipMemcpyHostToDevice, t->pst ) == hipSuccess ) ) {
      t->pair_cnt = pc;
    } else {
      (void)hipGetLastError();
      if( t->pair_ws ) (void)hipFree( t->pair_ws );
      if( t->pair_flag ) (void)hipFree( t->pair_flag );
      t->pair_ws = NULL; t->pair_flag = NULL; t->pair_cnt = 0UL;
    }
    t->pair_seq = 0UL;
    t->pair_end.assign( t->pair_cnt, 0UL );
  }
  t->desc_seq = 0UL;
  t->ppend.assign( R, pending_t{} );
  t->desc_end.assign( R, 0UL );
  t->ring_seq = 0UL;
  t->persist_ok = true;
  return FD_ED25519_AMD_OK;
}

extern "C" fd_verify_amd_tile_t *
fd_verify_amd_tile_new_cfg( fd_verify_amd_tile_cfg_t const * cfg ) {
  if( !cfg ) return NULL;
  fd_verify_amd_tile_cfg_t c = *cfg;
  if( !c.batch_max || c.batch_max > (1UL<<20) ) return NULL;
  if( c.framing != FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG && c.framing != FD_VERIFY_AMD_FRAMING_TXN ) return NULL;
  if( c.framing == FD_VERIFY_AMD_FRAMING_TXN && c.batch_max < TXN_SIG_MAX_AT_MTU ) return NULL;
  if( c.chunk_mode < FD_VERIFY_AMD_CHUNK_AUTO || c.chunk_mode > FD_VERIFY_AMD_CHUNK_QUAD ) return NULL;
  if( c.publish_cpu < FD_VERIFY_AMD_PUBLISH_AUTO || c.publish_cpu >= CPU_SETSIZE ) return NULL;
  if( c.copy_cpu < FD_VERIFY_AMD_COPY_INLINE || c.copy_cpu >= CPU_SETSIZE ) return NULL;
  if( c.waves == 1UL || c.waves > 65536UL ) return NULL;
  int cnt = 0, cus = 0;
  if( hipGetDeviceCount( &cnt ) != hipSuccess || c.device < 0 || c.device >= cnt ) return NULL;
  if( hipSetDevice( c.device ) != hipSuccess ) return NULL;
  if( hipDeviceGetAttribute( &cus, hipDeviceAttributeMultiprocessorCount, c.device ) != hipSuccess || cus <= 0 ) return NULL;
  if( !c.lat_free_chunks ) c.lat_free_chunks = (ulong)cus / 2UL;
  if( !c.out_frame_cnt ) c.out_frame_cnt = 4096UL + c.batch_max + tile_window( &c );   /* in flight + a pass + the consumer's lag */
  if( c.out_frame_cnt > (0xFFFFFFFFUL / FRAME_CHUNKS) ) return NULL;   /* chunk indices are 32-bit */
  fd_verify_amd_tile_t * t = new fd_verify_amd_tile_t();
  t->cfg = c; t->device = c.device; t->batch_max = c.batch_max;
  t->framing = c.framing; t->cus = cus;
  t->tc.init( c.tcache_depth );
  bool ok = hipHostMalloc( (void **)&t->out_base, c.out_frame_cnt * FD_VERIFY_AMD_FRAME_SZ, hipHostMallocMapped ) == hipSuccess &&
            hipHostGetDevicePointer( (void **)&t->out_dev, t->out_base, 0 ) == hipSuccess;
  t->frame_cnt = c.out_frame_cnt;
  t->frame_pub.assign( c.out_frame_cnt, FRAME_FREE );
  t->frame_busy = (uint8_t *)calloc( c.out_frame_cnt, 1 );
  t->out_seq_end = ~0UL;
  if( !ok || !t->frame_busy || !tile_count( t, true ) ) {
    if( ok && t->frame_busy ) fprintf( stderr, "fd_verify_amd_tile_new: device %d already runs %d tiles in this process "
                                       "(one hardware queue each, GPU_MAX_HW_QUEUES)\n", c.device, tile_queue_max() );
    fd_verify_amd_tile_delete( t );
    return NULL;
  }
  return t;
}

extern "C" fd_verify_amd_tile_t *
fd_verify_amd_tile_new( int device, ulong batch_max, ulong batch_wait_ns, ulong tcache_depth, ulong out_frame_cnt ) {
  fd_verify_amd_tile_cfg_t c;
  fd_verify_amd_tile_cfg_default( &c );
  c.device = device; c.batch_max = batch_max; c.batch_wait_ns = batch_wait_ns;
  c.tcache_depth = tcache_depth; c.out_frame_cnt = out_frame_cnt;
  return fd_verify_amd_tile_new_cfg( &c );
}

/* ------------------------------------------------------------------ */
/* the run: stager (the caller's thread), publisher, persistent kernel  */

/* The hand-off rule (header).  Pure; the CPU tests call it.  Units:
   signature slots (PUB_SIG_MSG: frags). */
extern "C" ulong
fd_verify_amd_tile_cut( fd_verify_amd_tile_cfg_t const * c, ulong staged, ulong handed, ulong chunks_in_flight,
                        int thr, ulong waited_ns, int flush ) {
  if( staged == handed ) return handed;
  ulong const n = staged - handed, K = lvl_slots( thr );
  if( flush || n >= c->batch_max || (c->batch_wait_ns && waited_ns >= c->batch_wait_ns) ) return staged;
  bool const rest = thr == FD_VERIFY_AMD_LVL_THR ? waited_ns >= c->chunk_wait_ns
                        : ( waited_ns >= c->lat_fill_ns || chunks_in_flight < c->lat_free_chunks );
  return rest ? staged : handed + (n & ~(K - 1UL));
}

extern "C" int
fd_verify_amd_tile_mode( int chunk_mode, int thr, double rate, double rate_hi, double rate_lo ) {
  if( chunk_mode == FD_VERIFY_AMD_CHUNK_LATENCY ) return 0;
  if( chunk_mode == FD_VERIFY_AMD_CHUNK_THROUGHPUT ) return 1;
  return thr ? rate >= rate_lo : rate > rate_hi;
}

extern "C" int
fd_verify_amd_tile_level( int chunk_mode, int lvl, double rate, double quad_hi, double quad_lo, double rate_hi,
                          double rate_lo ) {
  if( chunk_mode == FD_VERIFY_AMD_CHUNK_LATENCY )    return FD_VERIFY_AMD_LVL_LAT;
  if( chunk_mode == FD_VERIFY_AMD_CHUNK_THROUGHPUT ) return FD_VERIFY_AMD_LVL_THR;
  if( chunk_mode == FD_VERIFY_AMD_CHUNK_QUAD )       return FD_VERIFY_AMD_LVL_QUAD;
  if( lvl == FD_VERIFY_AMD_LVL_THR ) {
    if( rate >= rate_lo ) return FD_VERIFY_AMD_LVL_THR;
    return rate >= quad_lo ? FD_VERIFY_AMD_LVL_QUAD : FD_VERIFY_AMD_LVL_LAT;
  }
  if( rate > rate_hi ) return FD_VERIFY_AMD_LVL_THR;
  if( lvl == FD_VERIFY_AMD_LVL_QUAD ) return rate >= quad_lo ? FD_VERIFY_AMD_LVL_QUAD : FD_VERIFY_AMD_LVL_LAT;
  return rate > quad_hi ? FD_VERIFY_AMD_LVL_QUAD : FD_VERIFY_AMD_LVL_LAT;
}

/* The level step with its holds (pure; the CPU tests call it).  A lower
   level, and throughput chunks in place of quad chunks, only once the rule
   has asked for it for hold_ns: a host stall of a few hundred us dips the
   rate EWMA (the way down), and the burst that stages its backlog afterwards
   lifts it over rate_hi for ~1 ms (the way up) -- at half load on a 55 M
   frags/s box such a burst moved quad chunks (p50 ~0.7 ms) to throughput
   chunks (p50 1.26 ms) for the rest of the run.  Latency to quad (and
   latency to throughput) stays immediate: the lower level has a third of the
   capacity; so does quad back to throughput within 5 hold times of leaving
   throughput chunks (a dip at 80 % load is undone at once, not after
   another hold's backlog).  The way up counts an episode of asking, not one
   unbroken ask: the episode ends only after hold_ns / 2 without an ask, since
   a stall under real overload dips the EWMA under rate_hi for a few hundred
   us too, and restarting the hold at every dip kept 80 % load in quad chunks
   for 6-7 ms, a backlog that took the rest of the run to drain (p50 8-11 ms
   in 2 of 18 runs, profiles/r06_level_hold_ab.txt).  st (zeroed at the start
   of a run): [0] 1 + since when the rule has asked for a lower level (0: it
   has not), [1] 1 + when the current episode of asking for throughput from
   quad began (0: none), [2] 1 + when the tile last left throughput chunks
   (0: never), [3] 1 + when the rule last asked for throughput from quad. */
extern "C" int
fd_verify_amd_tile_level_step( int lvl, int want, ulong now_ns, ulong hold_ns, ulong * st ) {
  if( !st ) return want;   /* no state: no holds */
  ulong const now1 = now_ns + 1UL;
  bool const down = lvl_rank( want ) < lvl_rank( lvl );
  bool const up   = lvl == FD_VERIFY_AMD_LVL_QUAD && want == FD_VERIFY_AMD_LVL_THR;
  bool const fast = st[2] && now1 - st[2] < 5UL * hold_ns;      /* left throughput chunks just now */
  if( !down ) st[0] = 0UL;
  if( lvl != FD_VERIFY_AMD_LVL_QUAD || ( !up && st[3] && now1 - st[3] >= hold_ns / 2UL ) ) st[1] = st[3] = 0UL;
  if( down ) {
    if( !st[0] ) st[0] = now1;
    if( now1 - st[0] < hold_ns ) return lvl;
    st[0] = 0UL;
  } else if( up && !fast ) {
    if( !st[1] ) st[1] = now1;
    st[3] = now1;
    if( now1 - st[1] < hold_ns ) return lvl;
    st[1] = st[3] = 0UL;
  }
  if( lvl == FD_VERIFY_AMD_LVL_THR && want != lvl ) st[2] = now1;
  return want;
}

/* Chunk packing (pure; the CPU tests call it): from ring entries with
   slots[0..cnt) signature slots each, the next chunk starting at entry 0:
   returns its entry count and sets *nsl to its slots.  Up to 64 entries
   and K slots (64, or 8 for a latency chunk); an entry is never split, so
   an entry of more than K slots (a transaction of > 8 signatures in latency
   mode) makes a chunk of its own -- the caller verifies that one 1 lane per
   signature (slots > 8). */
extern "C" ulong
fd_verify_amd_tile_pack( uint const * slots, ulong cnt, int thr, ulong * nsl ) {
  ulong const K = lvl_slots( thr );
  ulong n = 0UL, s = 0UL;
  while( n < cnt && n < 64UL ) {
    ulong const k = slots[n];
    if( n && s + k > K ) break;
    s += k; n++;
    if( s >= K ) break;
  }
  *nsl = s;
  return n;
}

namespace {

/* One run, shared by the stager (the caller's thread) and the publisher (a
   second thread, or the stager itself between passes).  Each atomic on its
   own line: the two threads exchange ring positions only. */
struct prun_t {
  fd_verify_amd_tile_t * t;
  fd_frag_meta_t const * in_mcache; ulong in_depth, in_seq0;
  fd_frag_meta_t *       out_mcache; ulong out_depth;
  ulong const *          out_fseq;
  int const *            stop;
  bool                   zc;
  uint *                 lat; ulong lat_max;
  ulong                  mask, R;
  fd_amd_tile_hctl_t *   H;
  /* publisher-owned */
  ulong pubd, out_seq, lat_n, out_cr, t_halt;
  long  g_off;                   /* host ns - GPU ticks x 10 (the best sample of the current window) */
  long  g_off_cur; ulong g_win;  /* the window being sampled, and its start */
  ulong g_last;                  /* latest full GPU clock sample */
  bool  g_ok;
  fd_verify_amd_diag_t d;        /* publisher's counters (out, sv_filt, ovrn, backp) */
  alignas(64) std::atomic<ulong> handed;    /* stager -> publisher: ring indices [.., handed) were handed over */
  alignas(64) std::atomic<ulong> pubd_a;    /* publisher -> stager: [.., pubd) are published or dropped */
  alignas(64) std::atomic<ulong> end;       /* stager -> publisher: the final ring index (~0 while staging) */
  alignas(64) std::atomic<int>   quit;      /* stager -> publisher: stop now (error, or halted) */
  alignas(64) std::atomic<int>   halt;      /* publisher -> stager: *stop was raised and the output stayed
                                               backpressured for halt_grace_ns: give up the rest */
};

inline void beat( fd_amd_tile_hctl_t * H ) { __atomic_fetch_add( &H->beat, 1UL, __ATOMIC_RELAXED ); }

/* The GPU clock (s_memrealtime, 100 MHz) on the host's: sample the scout's
   clock word, keep the smallest (host - GPU) offset of each 20 ms window
   (the sample read soonest after its store), use the last full window's. */
void
gclock_sample( prun_t & r, ulong tn ) {
  ulong g = __atomic_load_n( &r.H->gclock, __ATOMIC_ACQUIRE );
  if( !g ) return;
  r.g_last = g;
  long off = (long)tn - (long)(g * 10UL);
  if( !r.g_ok ) { r.g_off = r.g_off_cur = off; r.g_win = tn; r.g_ok = true; return; }
  if( off < r.g_off_cur ) r.g_off_cur = off;
  if( off < r.g_off ) r.g_off = off;   /* a better sample now beats the last window's */
  if( tn - r.g_win >= 20000000UL ) { r.g_off = r.g_off_cur; r.g_off_cur = off; r.g_win = tn; }
}

inline ulong
gclock_ns( prun_t const & r, uint ticks32 ) {   /* low 32 bits of a recent GPU clock -> host ns */
  ulong g = r.g_last + (ulong)(long)(int)(ticks32 - (uint)r.g_last);
  return (ulong)((long)(g * 10UL) + r.g_off);
}

/* Publish what has come back, in ring order: count the results that are
   in, then (zero copy) check once that the oldest of them was not lapped --
   lapping goes in sequence order, so if its mcache line is intact now,
   after the GPU read every frag of the pass, so are the newer ones' --
   then publish them with one timestamp.  Every published or dropped frag
   frees its output frame.  Returns whether anything moved; returns early
   (leaving the rest) when quit is raised or, after *stop, the output stayed
   backpressured for halt_grace_ns (then raises r.halt). */
bool
publish_pass( prun_t & r ) {
  fd_verify_amd_tile_t * t = r.t;
  ulong const mask = r.mask, h = r.handed.load( std::memory_order_acquire );
  uint64_t const * rw = t->res + r.R;
  ulong ready = 0UL;
  while( r.pubd + ready != h && ready < 4096UL ) {
    ulong w = __atomic_load_n( rw + ((r.pubd + ready) & mask), __ATOMIC_ACQUIRE );
    if( (w >> 8) != r.pubd + ready + 1UL ) break;
    ready++;
  }
  if( !ready ) return false;
  ulong const tn = now_ns();
  uint  const tspub = (uint)tn;
  if( t->trace ) gclock_sample( r, tn );
  bool lap_ok = true;
  if( r.zc ) {
    ulong const s0 = t->ppend[r.pubd & mask].seq;
    lap_ok = __atomic_load_n( &r.in_mcache[ s0 & (r.in_depth-1UL) ].seq, __ATOMIC_ACQUIRE ) == s0;
  }
  bool ok = true;
  for( ulong end = r.pubd + ready; r.pubd != end; ) {
    ulong const j = r.pubd & mask;
    ulong const w = rw[j];
    pending_t const & m = t->ppend[j];
    /* zero copy: the GPU read the frag some time before now; if its mcache
       line has been lapped since, the producer may have rewritten it */
    if( !lap_ok && __atomic_load_n( &r.in_mcache[ m.seq & (r.in_depth-1UL) ].seq, __ATOMIC_ACQUIRE ) != m.seq ) {
      r.d.ovrn_cnt++;
      __atomic_store_n( &t->frame_busy[m.fidx], (uint8_t)0, __ATOMIC_RELEASE );
      r.pubd++;
      continue;
    }
    schar const v = (schar)(uchar)(w & 0xffUL);
    ulong const rs = m.seq - r.in_seq0;
    if( t->vlog && rs < t->vlog_max ) t->vlog[rs] = v;
    if( v ) {
      r.d.sv_filt_cnt++; r.d.sv_filt_sz += m.sz;
      if( v >= -3 && v <= -1 ) r.d.sv_filt_code_cnt[-v - 1]++;   /* TXN parse failures (-4) count SV_FILT only */
      __atomic_store_n( &t->frame_busy[m.fidx], (uint8_t)0, __ATOMIC_RELEASE );
      r.pubd++;
      continue;
    }
    if( r.out_fseq && (long)(r.out_seq - r.out_cr) >= 0 ) {   /* credit check against the slowest consumer */
      r.out_cr = __atomic_load_n( r.out_fseq, __ATOMIC_ACQUIRE ) + r.out_depth;
      if( (long)(r.out_seq - r.out_cr) >= 0 ) {
        r.d.backp_cnt++;
        /* backpressured: keep the heartbeat and the halt check running, as
           the reference tile keeps its housekeeping (fd_frank_verify_synth_load.c:
           223-274); let the stager see what was published so far */
        r.pubd_a.store( r.pubd, std::memory_order_release );
        ulong spin = 0;
        for( ;; ) {
          r.out_cr = __atomic_load_n( r.out_fseq, __ATOMIC_ACQUIRE ) + r.out_depth;
          if( (long)(r.out_seq - r.out_cr) < 0 ) break;
          if( !(++spin & 1023UL) ) {
            beat( r.H );
            if( r.quit.load( std::memory_order_acquire ) ) { ok = false; break; }
            if( r.stop && __atomic_load_n( r.stop, __ATOMIC_ACQUIRE ) ) {
              /* the halt grace runs only while backpressured (it restarts
                 with every new backpressure episode) */
              ulong const t2 = now_ns();
              if( !r.t_halt ) r.t_halt = t2;
              if( t2 - r.t_halt > t->cfg.halt_grace_ns ) { r.halt.store( 1, std::memory_order_release ); ok = false; break; }
            }
          }
          _mm_pause();
        }
        r.t_halt = 0UL;
        if( !ok ) break;
      }
    }
    ulong const f = m.fidx;
    t->frame_pub[f] = r.out_seq;
    fd_mcache_publish( r.out_mcache, r.out_depth, r.out_seq, t->res[j], f * FRAME_CHUNKS, m.sz, m.ctl, m.tsorig, tspub );
    __atomic_store_n( &t->frame_busy[f], (uint8_t)0, __ATOMIC_RELEASE );
    if( r.lat_n < r.lat_max ) {
      if( r.lat ) r.lat[r.lat_n] = tspub - m.tsorig;
      if( t->trace && r.lat_n < t->trace_max ) {
        uint * p = t->trace + 4UL * r.lat_n;
        ulong const tm = t->res[2UL * r.R + j];
        ulong const c_ns = gclock_ns( r, (uint)tm ), d_ns = gclock_ns( r, (uint)(tm >> 32) );
        uint const hand = m.t_hand, c32 = (uint)c_ns, d32 = (uint)d_ns;
        auto clamp = []( uint a, uint b ) -> uint { int x = (int)(a - b); return x > 0 ? (uint)x : 0u; };
        p[0] = clamp( hand, m.t_stage );
        p[1] = clamp( c32, hand );
        p[2] = std::min( clamp( d32, c32 ), 0x7fffffffu ) | (m.t_hand & 1u ? 0x80000000u : 0u);
        p[3] = clamp( tspub, d32 );
      }
      r.lat_n++;
    }
    r.out_seq++; r.d.out_cnt++; r.d.out_sz += m.sz;
    r.pubd++;
  }
  r.pubd_a.store( r.pubd, std::memory_order_release );
  return true;
}

} /* namespace */

static int
tile_run_persist( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth, void const * in_chunk0,
                  ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache, ulong out_depth, ulong out_seq0,
                  ulong const * out_fseq, ulong frag_cnt, int const * stop, fd_verify_amd_diag_t * diag, uint * lat,
                  ulong lat_max, uint8_t const * zc_dev, ulong zc_lim ) {
  int rc = tile_persist_alloc( t );
  if( rc ) { fprintf( stderr, "fd_verify_amd_tile_run: allocating the persistent consumer failed (%d)\n", rc ); return rc; }
  tile_set_levels( t );   /* this run's framing */
  if( tile_kernel_busy( t ) ) {
    fprintf( stderr, "fd_verify_amd_tile_run: the kernel of an earlier run of this tile has not finished\n" );
    return FD_ED25519_AMD_ERR_DEVICE;
  }
  bool const txn = t->framing == FD_VERIFY_AMD_FRAMING_TXN;
  ulong const F = t->frame_cnt, mask = t->R - 1UL, W = t->window, base = t->ring_seq;
  fd_amd_tile_hctl_t * H = t->hctl;

  /* seed the control words, then launch: the kernel's ticket counter and
     the mirrors start at this run's first descriptor */
  ulong const dbase = t->desc_seq;
  __atomic_store_n( &H->head, dbase, __ATOMIC_RELAXED );
  __atomic_store_n( &H->stop, 0u, __ATOMIC_RELAXED );
  __atomic_store_n( &H->kerr, 0u, __ATOMIC_RELAXED );
  __atomic_store_n( &H->gclock, 0UL, __ATOMIC_RELAXED );
  __atomic_store_n( &H->gdone, 0UL, __ATOMIC_RELAXED );
  /* the device control block, seeded in stream order before the kernel
     (no host wait: a kernel that cannot start must not block the caller) */
  memset( &t->d0, 0, sizeof t->d0 );
  t->d0.ticket = dbase;
  for( int x=0; x<FD_AMD_TILE_MIRRORS; x++ ) t->d0.mw[x].w = dbase;
  if( hipMemcpyAsync( t->dctl, &t->d0, sizeof t->d0, hipMemcpyHostToDevice, t->pst ) != hipSuccess )
    return FD_ED25519_AMD_ERR_DEVICE;
  fd_amd_tile_args_t A;
  memset( &A, 0, sizeof A );
  A.hctl = (fd_amd_tile_hctl_t *)t->hctl_dev;
  A.ent  = (fd_amd_tile_ent_t const *)t->ring_dev;
  A.desc = (fd_amd_tile_desc_t const *)t->desc_dev;
  A.res_tag  = (uint64_t *)t->res_dev;
  A.res_word = (uint64_t *)t->res_dev + t->R;
  A.res_time = t->trace ? (uint64_t *)t->res_dev + 2UL * t->R : NULL;
  A.mask = mask;
  A.src  = zc_dev ? zc_dev : t->out_dev;
  A.out  = zc_dev ? t->out_dev : NULL;
  A.dctl = t->dctl;
  A.scratch = t->scratch;
  A.watchdog = 500000000UL;   /* 5 s of s_memrealtime (100 MHz) without a heartbeat */
  A.txn = txn ? 1u : 0u;
  A.pair_ws = t->pair_ws; A.pair_flag = t->pair_flag; A.pair_mask = t->pair_cnt ? (uint32_t)(t->pair_cnt - 1UL) : 0u;
  t->n_pair = 0UL;
#ifdef FD_AMD_DIAG
  { char const * e = getenv( "FD_AMD_TILE_PROF" ); A.prof = e && *e && *e != '0'; }   /* diagnostics build only */
#endif
  int const lrc = fd_amd_launch_tile_persist( &A, t->waves, t->pst );
  if( lrc || hipEventRecord( t->pdone, t->pst ) != hipSuccess ) {
    fprintf( stderr, "fd_verify_amd_tile_run: launching the tile kernel failed (%d: %s; %u waves)\n", lrc,
             lrc > 0 ? hipGetErrorString( (hipError_t)lrc ) : "-", (unsigned)t->waves );
    (void)hipStreamSynchronize( t->pst );
    return FD_ED25519_AMD_ERR_DEVICE;
  }
  ulong const t_launch = now_ns();

  prun_t r;
  r.t = t; r.in_mcache = in_mcache; r.in_depth = in_depth; r.in_seq0 = in_seq0;
  r.out_mcache = out_mcache; r.out_depth = out_depth; r.out_fseq = out_fseq; r.stop = stop;
  r.zc = zc_dev != NULL; r.lat = lat; r.lat_max = (lat || t->trace) ? std::max( lat ? lat_max : 0UL, t->trace_max ) : 0UL;
  if( lat && t->trace ) r.lat_max = std::min( lat_max, t->trace_max );
  r.mask = mask; r.R = t->R; r.H = H;
  r.pubd = base; r.out_seq = out_seq0; r.lat_n = 0UL; r.out_cr = 0UL; r.t_halt = 0UL;
  r.g_off = r.g_off_cur = 0L; r.g_win = 0UL; r.g_last = 0UL; r.g_ok = false;
  memset( &r.d, 0, sizeof r.d );
  r.handed.store( base ); r.pubd_a.store( base ); r.end.store( ~0UL ); r.quit.store( 0 ); r.halt.store( 0 );

  /* the publisher: a thread of its own when the tile has a CPU for it */
  std::thread pub;
  {
    cpu_set_t cs; CPU_ZERO( &cs );
    bool two = false;
    if( t->cfg.publish_cpu >= 0 ) { CPU_SET( t->cfg.publish_cpu, &cs ); two = true; }
    else if( t->cfg.publish_cpu == FD_VERIFY_AMD_PUBLISH_AUTO &&
             !pthread_getaffinity_np( pthread_self(), sizeof cs, &cs ) && CPU_COUNT( &cs ) >= 2 ) {
      int me = sched_getcpu();
      if( me >= 0 && me < CPU_SETSIZE ) CPU_CLR( me, &cs );
      two = CPU_COUNT( &cs ) >= 1;
    }
    if( two ) {
      try {
        pub = std::thread( [&r, cs]() {
          (void)pthread_setaffinity_np( pthread_self(), sizeof cs, &cs );
          for( ;; ) {
            bool any = publish_pass( r );
            if( r.quit.load( std::memory_order_acquire ) || r.halt.load( std::memory_order_acquire ) ) break;
            if( r.pubd == r.end.load( std::memory_order_acquire ) ) break;
            if( !any ) _mm_pause();
          }
        } );
      } catch( ... ) { two = false; }
    }
  }
  bool const inline_pub = !pub.joinable();

  /* copy mode's helper: a thread of its own when cfg.copy_cpu names a CPU */
  copier_t * cp = NULL;
  std::thread cth;
  if( !zc_dev && t->cfg.copy_cpu >= 0 ) {
    cp = new (std::nothrow) copier_t();
    if( cp ) {
      cp->claim.store( 0UL ); cp->quit.store( 0 );
      for( ulong s=0; s<CP_NJ; s++ ) { cp->nj[s].store( 0UL ); cp->bsz[s].store( 1UL ); for( ulong b=0; b<CP_NB; b++ ) cp->done[s][b].store( 0UL ); }
      try { cth = std::thread( copier_loop, cp, t->cfg.copy_cpu ); } catch( ... ) { delete cp; cp = NULL; }
    }
  }
  ulong cgen = 0UL;                       /* the helper's last posted generation */
  std::vector<orphan_t> orphans;
  ulong orphan_cnt[CP_NJ] = { 0, 0, 0, 0 };
  std::vector<copy_job_t> ljobs( zc_dev ? 0UL : STAGE_PASS );   /* a pass copied without the helper */
  std::vector<uint>       jfr( zc_dev ? 0UL : STAGE_PASS );     /* the frame each listed frag is staged from (a
                                                                  re-copied block's fresh frames: never written
                                                                  into the posted jobs, which the helper reads) */
  /* copy mode with the helper is pipelined: a pass posted to the helper is
     copied while the stager lists the next one, and staged (in input order,
     before that next pass) once its blocks are done -- the stager copies
     what the helper has not claimed by then */
  struct { bool on; ulong g, s, nj, sl, seq0; std::vector<uint> jf; } pend = { false, 0UL, 0UL, 0UL, 0UL, 0UL, {} };
  if( !zc_dev ) pend.jf.resize( STAGE_PASS );

  ulong in_seq = in_seq0, staged = base, handed = base;
  ulong staged_sl = 0UL, handed_sl = 0UL;   /* signature slots staged / handed over in this run */
  ulong in_cnt = diag->in_cnt, cons = out_seq0, fseq_pub = ~0UL;
  ulong ovrn = 0, bad = 0, ha = 0, ha_sz = 0, backp = 0, nbatch = 0, nsig = 0, switches = 0;
  ulong cdone = dbase;                   /* first descriptor not known to be finished */
  ulong n_pass = 0, n_hand = 0, n_stop_window = 0, n_stop_frames = 0, n_stop_bmax = 0, n_stop_pass = 0, n_steal = 0;
  ulong ph_tick[4] = { 0, 0, 0, 0 }, ph_frags = 0;
  t->started = 0;
  ulong iter = 0UL, pass_t = now_ns(), pass_max = 0UL;
  ulong t_chk = pass_t, g_seen = 0UL, t_prog = pass_t, gc_first = 0UL, gc_last = 0UL, gc_host = 0UL;
  ulong r_t0 = pass_t, r_n0 = 0UL;
  bool  r_blk = false;                   /* staging stopped on the window / frames / credit this interval */
  bool  r_win = false;                   /* ... on the window or the frames (the GPU's chunks do not keep up) */
  double rate = 0.0;
  int thr = fd_verify_amd_tile_level( t->cfg.chunk_mode, FD_VERIFY_AMD_LVL_LAT, 0.0, t->quad_hi, t->quad_lo, t->rate_hi,
                                      t->rate_lo );   /* chunk level, FD_VERIFY_AMD_LVL_* */
  ulong lvl_st[4] = { 0UL, 0UL, 0UL, 0UL };   /* the level holds' state (fd_verify_amd_tile_level_step) */
  bool halted = false;
  uchar const * in_chunk0b = (uchar const *)in_chunk0;
  fd_verify_amd_tile_cfg_t cc = t->cfg;   /* the cut rule's parameters */
  std::vector<uint> pk_slots( 64 );
  /* listing prefetch distances (frags ahead): mcache lines, and the frag
     bytes the copy / HA tag / TXN count read next.  32 / 24 (were 16 / 8):
     copy mode +8-15 % interleaved in two A/Bs, equal within noise in a third
     on the same kind of noisy box; zero copy unchanged
     (profiles/r06_listing_prefetch_ab_a/b/c.jsonl).
     FD_AMD_TILE_PF="mc,data" overrides them (A/B only) */
  ulong pf_mc = 32UL, pf_dt = 24UL;
  {
    char const * e = getenv( "FD_AMD_TILE_PF" );
    if( e && *e ) {
      char * q = NULL; ulong a = strtoul( e, &q, 0 ), b = (q && *q == ',') ? strtoul( q + 1, NULL, 0 ) : pf_dt;
      if( a >= 1UL && a <= 256UL ) pf_mc = a;
      if( b >= 1UL && b <= 256UL ) pf_dt = b;
    }
  }

  /* reserve the next output frame (cyclic): free -- not staged, in flight
     or orphaned -- and no longer read by a consumer that honours flow
     control.  false (and why) when there is none. */
  auto reserve = [&]( uint * fo, bool * credit ) -> bool {
    ulong const f = t->frame_next_idx;
    *credit = false;
    if( __atomic_load_n( &t->frame_busy[f], __ATOMIC_ACQUIRE ) ) return false;
    if( out_fseq && t->frame_pub[f] != FRAME_FREE && (long)(t->frame_pub[f] - cons) >= 0 ) {
      cons = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE );
      if( (long)(t->frame_pub[f] - cons) >= 0 ) { *credit = true; return false; }
    }
    t->frame_busy[f] = 1u;
    t->frame_pub[f] = FRAME_FREE;
    if( ++t->frame_next_idx == F ) t->frame_next_idx = 0UL;
    *fo = (uint)f;
    return true;
  };
  auto unreserve = [&]( uint f ) { __atomic_store_n( &t->frame_busy[f], (uint8_t)0, __ATOMIC_RELEASE ); };
  /* copy mode's producer credit: everything copied -- but never past a frag
     whose source an orphaned helper block may still be reading */
  auto copy_rel = [&]() -> ulong {
    ulong rel = pend.on ? pend.seq0 : in_seq;   /* a posted pass is not copied yet */
    for( orphan_t const & o : orphans ) rel = std::min( rel, cp->jobs[o.s][o.b * cp->bsz[o.s].load( std::memory_order_relaxed )].seq );
    return rel;
  };
  /* re-check each copied frag's mcache line and stage it, in input order */
  auto stage_jobs = [&]( copy_job_t const * js, uint const * jf_, ulong n, uint ts ) {
    __atomic_thread_fence( __ATOMIC_ACQUIRE );
    for( ulong k=0; k<n; k++ ) {
      copy_job_t const & j = js[k];
      uint const jf = jf_[k];
      /* a frag lapped while it was copied is dropped (speculative read,
         then seq re-check); its frame is free again */
      if( __atomic_load_n( &j.m->seq, __ATOMIC_ACQUIRE ) != j.seq ) { ovrn++; unreserve( jf ); continue; }
      in_cnt++;
      if( t->tc.depth && t->tc.insert( j.tag ) ) { ha++; ha_sz += j.sz; unreserve( jf ); continue; }
      fd_amd_tile_ent_t * en = t->ring + (staged & mask);
      en->src_chunk = (uint32_t)(jf * FRAME_CHUNKS);
      en->out_chunk = (uint32_t)(jf * FRAME_CHUNKS);
      en->sz        = (uint32_t)j.sz;
      en->slots     = j.slots;
      staged_sl += j.slots;
      t->ppend[staged & mask] = pending_t{ j.seq, (ushort)j.sz, j.ctl, j.tsorig, jf, ts, 0u, (uint)staged_sl, j.slots, 0u };
      staged++;
    }
  };
  /* the posted pass: claim the blocks the helper has not, wait a little for
     the helper's own, re-copy what is still missing into fresh frames (the
     old ones become orphans), then stage it */
  auto finish_pend = [&]( uint ts ) {
    ulong const tA = __rdtsc();
    ulong const g = pend.g, s = pend.s, nj_ = pend.nj, bz = cp->bsz[s].load( std::memory_order_relaxed ), nb = CP_NB;
    copy_job_t const * js = cp->jobs[s];
    ulong mine = 0UL;   /* bit b: the stager copied block b */
    for( ;; ) {
      ulong c = cp->claim.load( std::memory_order_acquire );
      ulong const b = c & 0xffffUL;
      if( (c >> 16) != g || b >= nb ) break;
      if( cp->claim.compare_exchange_weak( c, c + 1UL, std::memory_order_acq_rel ) ) {
        copy_jobs( js, b * bz, std::min( nj_, (b + 1UL) * bz ) );
        mine |= 1UL << b;
      }
    }
    ulong const tw = now_ns();
    for( ulong b = 0; b < nb && b * bz < nj_; b++ ) {
      if( mine >> b & 1UL ) continue;
      while( cp->done[s][b].load( std::memory_order_acquire ) != g && now_ns() - tw < CP_STEAL_NS ) _mm_pause();
      if( cp->done[s][b].load( std::memory_order_acquire ) == g ) continue;
      orphan_t o; o.g = g; o.s = s; o.b = b;
      ulong const lo = b * bz, hi = std::min( nj_, lo + bz );
      bool okb = true;
      std::vector<uint> fresh;
      for( ulong k = lo; k < hi && okb; k++ ) {
        uint f2; bool credit;
        okb = reserve( &f2, &credit );
        if( okb ) fresh.push_back( f2 );
      }
      if( !okb ) {   /* no frames to re-copy into: wait for the helper after all */
        for( uint f2 : fresh ) unreserve( f2 );
        while( cp->done[s][b].load( std::memory_order_acquire ) != g ) _mm_pause();
        continue;
      }
      for( ulong k = lo; k < hi; k++ ) {
        o.frames.push_back( js[k].f );
        pend.jf[k] = fresh[k - lo];
        stage_copy_nt( t->out_base + (ulong)pend.jf[k] * FD_VERIFY_AMD_FRAME_SZ, js[k].src, js[k].sz );
      }
      orphan_cnt[s]++;
      orphans.push_back( std::move( o ) );
      n_steal++;
    }
    ulong const tB = __rdtsc();
    stage_jobs( js, pend.jf.data(), nj_, ts );
    pend.on = false;
    ph_tick[1] += tB - tA; ph_tick[2] += __rdtsc() - tB;
  };

  for( ;; ) {
    /* the kernel's watchdog needs a heartbeat now and then, not every
       pass: each store after a GPU read of the line is a cache-line
       ownership round trip */
    if( !(++iter & 63UL) ) beat( H );
    if( !gc_first && (gc_first = __atomic_load_n( &H->gclock, __ATOMIC_ACQUIRE )) ) t->started = 1;
    ulong const tn = now_ns();
    pass_max = std::max( pass_max, tn - pass_t ); pass_t = tn;

    /* 1. publish (inline), then the publisher's progress */
    if( inline_pub ) (void)publish_pass( r );
    ulong const pubd = r.pubd_a.load( std::memory_order_acquire );
    /* orphaned copy blocks the helper has finished since: their frames are free */
    for( ulong k = 0; k < orphans.size(); ) {
      orphan_t & o = orphans[k];
      if( cp->done[o.s][o.b].load( std::memory_order_acquire ) == o.g ) {
        for( uint f : o.frames ) unreserve( f );
        orphan_cnt[o.s]--;
        orphans[k] = std::move( orphans.back() ); orphans.pop_back();
      } else k++;
    }
    /* producer credit: copy mode is done with a frag once it is copied,
       zero copy once it is published (or dropped) */
    if( in_fseq ) {
      ulong rel = !zc_dev ? copy_rel() : pubd == staged ? in_seq : t->ppend[pubd & mask].seq;
      if( rel != fseq_pub ) { __atomic_store_n( in_fseq, rel, __ATOMIC_RELEASE ); fseq_pub = rel; }
    }
    /* after *stop: drain what was taken in; give up only if the publisher
       reports the output backpressured past the halt grace */
    bool const stopping = stop && __atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0;
    bool done_in = (frag_cnt && in_seq - in_seq0 >= frag_cnt) || stopping;
    if( done_in && pubd == staged && !pend.on ) break;
    if( r.halt.load( std::memory_order_acquire ) ) { halted = true; break; }

    /* 2. stage (at most STAGE_PASS frags, so hand-offs keep flowing).  Copy
          mode lists the pass's copies first (a frame reserved per frag),
          copies them -- with the helper when there is one -- and then
          re-checks and stages each frag in input order */
    bool full = false, wfull = false;
    ulong const stage_end = staged + STAGE_PASS;
    ulong const staged_a = staged, pt0 = __rdtsc();
    ulong pt1 = 0UL, pt2 = 0UL;
    n_pass++;
    uint const ts32 = (uint)tn;
    ulong nj = 0UL;
    /* the helper's next job array, when it is free of orphans */
    ulong const gnext = cgen + 1UL, snext = gnext % CP_NJ;
    copy_job_t * jobs = ( cp && !orphan_cnt[snext] ) ? cp->jobs[snext] : ljobs.data();
    ulong sl_pass = 0UL;                   /* slots listed in this pass (copy mode) */
    ulong const pnj = pend.on ? pend.nj : 0UL, psl = pend.on ? pend.sl : 0UL;   /* the posted pass, not staged yet */
    while( !done_in && staged_sl + psl + sl_pass - handed_sl < t->batch_max && staged + nj != stage_end ) {
      if( frag_cnt && in_seq - in_seq0 >= frag_cnt ) break;
      if( staged + pnj + nj - pubd >= W ) { full = wfull = true; n_stop_window++; break; }
      fd_frag_meta_t const * m = in_mcache + (in_seq & (in_depth-1UL));
      __builtin_prefetch( in_mcache + ((in_seq + pf_mc) & (in_depth-1UL)) );
      ulong seq_found = __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE );
      long  d = (long)(seq_found - in_seq);
      if( d < 0 ) break;                                                  /* not yet published */
      if( d > 0 ) { ovrn += (ulong)d; in_seq = seq_found; continue; }     /* overrun: resync */
      ulong chunk = m->chunk, sz = m->sz, ctl = m->ctl, tsorig = m->tsorig;
      __atomic_thread_fence( __ATOMIC_ACQUIRE );
      if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != in_seq ) { ovrn++; in_seq++; continue; }
      bool const sz_ok = txn ? ( sz >= 1UL && sz <= FD_TXN_AMD_MTU ) : ( sz >= 96UL && sz - 96UL <= FD_ED25519_AMD_MSG_MAX );
      if( !sz_ok || (zc_dev && (chunk << FD_CHUNK_LG_SZ) + ((sz + 63UL) & ~63UL) > zc_lim) ) {
        bad++; in_seq++; in_cnt++; continue;
      }
      uchar const * p = (uchar const *)fd_chunk_to_laddr_const( in_chunk0b, chunk );
      if( !zc_dev || t->tc.depth || txn ) {
        /* the frag pf_dt ahead: its bytes are read next (copy; the HA tag; TXN's signature count).
           Kept for the copy helper's passes too: without it the helper's copy took 11-12 ns per
           frag instead of 2-5 and copy mode fell from 52-58 to 40-43 M frags/s
           (profiles/r06_copy_prefetch_ab.jsonl) */
        fd_frag_meta_t const * m8 = in_mcache + ((in_seq + pf_dt) & (in_depth-1UL));
        uchar const * p8 = (uchar const *)fd_chunk_to_laddr_const( in_chunk0b, __atomic_load_n( &m8->chunk, __ATOMIC_RELAXED ) );
        ulong const n8 = zc_dev ? 1UL : std::min( (ulong)__atomic_load_n( &m8->sz, __ATOMIC_RELAXED ), (ulong)FD_VERIFY_AMD_FRAME_SZ );
        for( ulong o = 0; o < n8; o += 64UL ) __builtin_prefetch( p8 + o );
      }
      /* read from the source before any copy (the seq re-check after the
         copy, or at publish in zero copy, covers them): the signature
         slots (TXN: fd_amd_txn_slots1 on the first byte) and the HA tag
         (the first 8 bytes of the first signature) */
      ulong const k2 = txn ? fd_amd_txn_slots1( p, sz ) : 1UL;
      ulong tag = 0UL;
      if( t->tc.depth && k2 ) memcpy( &tag, p + (txn ? 1UL : 32UL), 8 );
      uint f; bool credit;
      if( !reserve( &f, &credit ) ) { full = true; if( credit ) backp++; else { wfull = true; n_stop_frames++; } break; }
      if( !zc_dev ) {
        /* copy mode: the frame is the tile's copy */
        jobs[nj++] = copy_job_t{ t->out_base + (ulong)f * FD_VERIFY_AMD_FRAME_SZ, p, m, in_seq, sz, tag, f, (uint)tsorig,
                                 (uint)k2, (ushort)ctl };
        sl_pass += k2;
        in_seq++;
        continue;
      }
      in_seq++; in_cnt++;
      if( t->tc.depth && t->tc.insert( tag ) ) { ha++; ha_sz += sz; unreserve( f ); continue; }
      fd_amd_tile_ent_t * en = t->ring + (staged & mask);
      en->src_chunk = (uint32_t)chunk;
      en->out_chunk = (uint32_t)(f * FRAME_CHUNKS);
      en->sz        = (uint32_t)sz;
      en->slots     = (uint32_t)k2;
      staged_sl += k2;
      t->ppend[staged & mask] = pending_t{ in_seq - 1UL, (ushort)sz, (ushort)ctl, (uint)tsorig, f, ts32, 0u, (uint)staged_sl,
                                           (uint)k2, 0u };
      staged++;
    }
    pt1 = __rdtsc();
    /* copy mode: first the posted pass (its frags precede this pass's) */
    if( pend.on ) finish_pend( ts32 );
    if( nj ) {
      for( ulong k=0; k<nj; k++ ) jfr[k] = jobs[k].f;
      if( jobs != ljobs.data() && nj >= COPY_SPLIT_MIN ) {
        /* post the pass to the helper; it is staged after the next pass's listing */
        ulong const g = gnext, s = snext, bz = (nj + 1UL) / 2UL;
        cgen = g;
        cp->nj[s].store( nj, std::memory_order_relaxed );
        cp->bsz[s].store( bz, std::memory_order_relaxed );
        cp->claim.store( g << 16, std::memory_order_release );
        pend.on = true; pend.g = g; pend.s = s; pend.nj = nj; pend.sl = sl_pass; pend.seq0 = jobs[0].seq;
        std::swap( pend.jf, jfr );
        if( jfr.size() < STAGE_PASS ) jfr.resize( STAGE_PASS );
      } else {
        ulong const c0 = __rdtsc();
        copy_jobs( jobs, 0UL, nj );
        pt2 = __rdtsc();
        stage_jobs( jobs, jfr.data(), nj, ts32 );
        ph_tick[1] += pt2 - c0; ph_tick[2] += __rdtsc() - pt2;
      }
    }
    if( staged != staged_a || nj ) {   /* listing (zero copy: listing and staging); copy mode timed its copy and stage above */
      ph_tick[0] += pt1 - pt0;
      ph_frags += staged - staged_a;
    }
    r_blk = r_blk || full;
    r_win = r_win || wfull;
    n_stop_bmax += staged_sl - handed_sl >= t->batch_max;
    n_stop_pass += staged == stage_end || nj == STAGE_PASS;
    __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
    /* copy mode releases what it copied -- but never past a frag whose copy
       an orphaned helper block may still be reading */
    if( in_fseq && !zc_dev ) {
      ulong const rel = copy_rel();
      if( rel != fseq_pub ) { __atomic_store_n( in_fseq, rel, __ATOMIC_RELEASE ); fseq_pub = rel; }
    }
    done_in = done_in || (frag_cnt && in_seq - in_seq0 >= frag_cnt);

    /* 3. chunk mode by the staging rate (slots/s, mean over ~0.4 ms) */
    ulong const t3 = now_ns();
    if( t3 - r_t0 >= 200000UL ) {
      double inst = (double)(staged_sl - r_n0) * 1e9 / (double)(t3 - r_t0);
      /* staging that stopped at the window, the frames or the consumer's
         credit measures the tile's own completions, not the offered load:
         such an interval never lowers the rate (else a full window reads as
         light load, the tile drops to latency chunks -- a third of the
         capacity -- and the backlog grows) */
      if( r_blk ) inst = std::max( inst, rate );
      rate = rate > 0.0 ? 0.75 * rate + 0.25 * inst : inst;   /* ~0.8 ms memory: a burst does not flip the mode */
      int nthr = fd_verify_amd_tile_level( t->cfg.chunk_mode, thr, rate, t->quad_hi, t->quad_lo, t->rate_hi, t->rate_lo );
      /* staging that stopped on the window or the frames in quad chunks: they
         do not keep up, whatever the rate says -- it then measures their
         completions, which on a slow or busy box stay under rate_hi (a
         saturated run on such a box stayed in quad chunks at 17-25 M frags/s,
         profiles/r06_level_hold_ab.txt) */
      if( thr == FD_VERIFY_AMD_LVL_QUAD && r_win && t->cfg.chunk_mode == FD_VERIFY_AMD_CHUNK_AUTO && t->rate_hi < HUGE_VAL )
        nthr = FD_VERIFY_AMD_LVL_THR;
      r_t0 = t3; r_n0 = staged_sl; r_blk = false; r_win = false;
      /* down, and quad -> throughput, only after the rule asked for it for
         LVL_HOLD_NS: a producer stall of a few hundred us dips the EWMA below
         the lower threshold, and a dip from throughput into quad chunks at 80 %
         load left a backlog that flipped the level dozens of times per run
         (p99 5.8 ms; profiles/r06_bench_quad_a_detail.json); the burst after a
         stall lifted half load into throughput chunks for good (p50 1.26 ms,
         profiles/r06_level_hold_ab.txt) */
      nthr = fd_verify_amd_tile_level_step( thr, nthr, t3, LVL_HOLD_NS, lvl_st );
      switches += nthr != thr;
      thr = nthr;
    }

    /* 4. hand over: cut staged slots into chunks (whole entries, packed by
          slots) and publish their descriptors (x86 stores are ordered:
          entries and descriptors are visible before the head) */
    if( staged != handed ) {
      while( cdone != t->desc_seq && t->desc_end[cdone & mask] <= pubd ) cdone++;
      ulong const waited = (ulong)(uint)((uint)t3 - t->ppend[handed & mask].t_stage);
      /* a full window (or no free frame) flushes only when nothing handed
         over is still unpublished: otherwise the chunks in flight free room,
         and flushing each pass's few freed frags cut the saturated stream
         into part-filled chunks (47 frags per 64-lane chunk at 16384 zero
         copy, profiles/r05_tile_cut_full_ab.txt) */
      bool const flush = done_in || (full && handed == pubd);
      ulong upto_sl = fd_verify_amd_tile_cut( &cc, staged_sl, handed_sl, t->desc_seq - cdone, thr, waited, flush );
      /* quad pairs: the cut's whole quad chunks go as whole pairs (32 frags;
         the 16 held back wait at most ~16 frags' arrival, or the cut's
         lat_fill_ns, then go with the rest) */
      if( thr == FD_VERIFY_AMD_LVL_QUAD && !txn && t->pair_cnt && upto_sl != staged_sl )
        upto_sl = handed_sl + ((upto_sl - handed_sl) & ~(2UL * QUAD_SLOTS - 1UL));
      /* whole entries up to that slot count (PUB_SIG_MSG: one slot per entry) */
      ulong upto = handed;
      if( upto_sl == staged_sl ) upto = staged;
      else if( !txn ) upto = handed + (upto_sl - handed_sl);
      else while( upto != staged && (uint)(t->ppend[upto & mask].sl_end - (uint)handed_sl) <= (uint)(upto_sl - handed_sl) ) upto++;
      /* TXN: a head transaction that fills a chunk's slots on its own (more
         signatures than a latency / quad chunk holds) is a chunk of its own
         (fd_verify_amd_tile_pack) -- it goes at once instead of waiting for
         the cut's whole chunks behind it */
      if( txn && upto == handed && t->ppend[handed & mask].slots >= lvl_slots( thr ) ) upto = handed + 1UL;
      if( upto != handed ) {
        ulong const ph0 = __rdtsc();
        ulong ds = t->desc_seq;
        uint const th = (uint)t3 & ~1u;
        for( ulong c = handed; c < upto; ) {
          ulong const avail = std::min( 64UL, upto - c );
          ulong nsl = 0UL, cnt;
          if( txn ) {
            for( ulong q = 0; q < avail; q++ ) pk_slots[q] = t->ppend[(c + q) & mask].slots;
            cnt = fd_verify_amd_tile_pack( pk_slots.data(), avail, thr, &nsl );
          } else {
            cnt = nsl = std::min( avail, lvl_slots( thr ) );   /* the same rule, one slot per frag */
          }
          /* a chunk of more slots than its level's lanes allow (a TXN frag of
             many signatures) runs 1 lane per signature */
          bool const lat_chunk  = thr == FD_VERIFY_AMD_LVL_LAT  && nsl <= LAT_SLOTS;
          bool const quad_chunk = thr == FD_VERIFY_AMD_LVL_QUAD && nsl <= QUAD_SLOTS;
          /* quad pair: 17..32 frags as two quad chunks on one front pass
             (sub 0 hashes and decompresses all of them) when a pair
             workspace is free (its last pair's frags all published) */
          if( quad_chunk && !txn && t->pair_cnt && avail > QUAD_SLOTS &&
              t->pair_end[t->pair_seq & (t->pair_cnt - 1UL)] <= pubd ) {
            ulong const pn = std::min( avail, 2UL * QUAD_SLOTS ), sq = t->pair_seq++;
            t->pair_end[sq & (t->pair_cnt - 1UL)] = c + pn;
            for( uint32_t sub = 0u; sub < 2u; sub++ ) {
              fd_amd_tile_desc_t * pd = t->desc + (ds & mask);
              pd->first = c;
              pd->count = (uint32_t)pn | FD_AMD_TILE_QUAD | FD_AMD_TILE_PAIR;
              pd->pad   = sub | (uint32_t)((sq & 0x3fffffffUL) << 1);   /* the kernel's flag value: seq + 1 (30 bits) */
              t->desc_end[ds & mask] = c + pn;
              ds++;
            }
            for( ulong q = 0; q < pn; q++ ) t->ppend[(c + q) & mask].t_hand = th | 1u;
            c += pn; t->n_pair++;
            continue;
          }
          fd_amd_tile_desc_t * dd = t->desc + (ds & mask);
          dd->pad = 0u;
          dd->first = c;
          dd->count = (uint32_t)cnt | (lat_chunk ? FD_AMD_TILE_LAT : 0u) | (quad_chunk ? FD_AMD_TILE_QUAD : 0u);
          t->desc_end[ds & mask] = c + cnt;
          /* bit 0: a latency or quad chunk (the trace's service split) */
          for( ulong q = 0; q < cnt; q++ ) t->ppend[(c + q) & mask].t_hand = th | ((lat_chunk || quad_chunk) ? 1u : 0u);
          c += cnt; ds++;
        }
        t->desc_seq = ds;
        nbatch++; nsig += (ulong)(uint)(t->ppend[(upto - 1UL) & mask].sl_end - (uint)handed_sl); n_hand++;
        handed_sl += (ulong)(uint)(t->ppend[(upto - 1UL) & mask].sl_end - (uint)handed_sl);
        handed = upto;
        r.handed.store( handed, std::memory_order_release );
        if( !zc_dev ) _mm_sfence();   /* the staged copies (non-temporal stores) before the head */
        __atomic_store_n( &H->head, ds, __ATOMIC_RELEASE );
        ph_tick[3] += __rdtsc() - ph0;
      }
    }

    /* 5. every ~1 ms: the kernel started, is alive and makes progress.
          Read from the scout's words only: its clock advances every
          ~10 us while the kernel lives (HIP is asked about the kernel only
          once that clock has stood still for 100 ms), and gdone counts the
          chunks finished. */
    if( t3 - t_chk >= 1000000UL ) {
      t_chk = t3;
      ulong const g  = __atomic_load_n( &H->gdone,  __ATOMIC_ACQUIRE );
      ulong const gc = __atomic_load_n( &H->gclock, __ATOMIC_ACQUIRE );
      if( gc != gc_last ) { gc_last = gc; gc_host = t3; }
      if( g != g_seen || t->desc_seq - dbase == g ) { g_seen = g; t_prog = t3; }
      char const * why = NULL;
      hipError_t q = hipSuccess;
      if( !gc ) {
        if( t3 - t_launch > 2000000000UL ) why = "the tile kernel did not start within 2 s (its wave slots are held by another kernel?)";
      } else if( gc && t3 - gc_host > 100000000UL ) {
        q = hipEventQuery( t->pdone );
        why = q != hipErrorNotReady ? "the tile kernel exited early" : "the tile kernel's scout stopped (its clock stood still for 100 ms)";
      } else if( gc && t3 - t_prog > 2000000000UL ) why = "the tile kernel made no progress for 2 s";
      if( why ) {
        fprintf( stderr, "fd_verify_amd_tile_run: %s (%s, watchdog %u; chunks done %lu of %lu, staged %lu handed %lu "
                 "published %lu)\n", why, hipGetErrorString( q ), __atomic_load_n( &H->kerr, __ATOMIC_ACQUIRE ),
                 g, t->desc_seq - dbase, staged - base, handed - base, pubd - base );
        rc = FD_ED25519_AMD_ERR_DEVICE;
        break;
      }
    }
  }

  /* end: stop the publisher, the helper, then the kernel (its waves exit
     once nothing is left to claim; chunks already claimed finish) */
  r.end.store( staged, std::memory_order_release );
  if( rc || halted ) r.quit.store( 1, std::memory_order_release );
  if( pub.joinable() ) pub.join();
  if( cp ) {
    cp->quit.store( 1, std::memory_order_release );
    if( cth.joinable() ) cth.join();   /* it finishes the block it holds first */
    for( orphan_t const & o : orphans ) for( uint f : o.frames ) unreserve( f );
    orphans.clear();
    /* a posted pass never staged (halted, or an error): its frames are free */
    if( pend.on ) { for( ulong k=0; k<pend.nj; k++ ) unreserve( pend.jf[k] ); pend.on = false; }
    delete cp;
  }
  __atomic_store_n( &H->stop, 1u, __ATOMIC_RELEASE );
  {
    /* a kernel that never started is not waited for (it exits at once
       when it does start: stop is raised) */
    ulong const t0 = now_ns(), lim = __atomic_load_n( &H->gclock, __ATOMIC_ACQUIRE ) ? 5000000000UL : 0UL;
    hipError_t q;
    while( (q = hipEventQuery( t->pdone )) == hipErrorNotReady && now_ns() - t0 < lim ) {
      beat( H );
      std::this_thread::yield();
    }
    if( q == hipErrorNotReady ) { t->pending = true; rc = FD_ED25519_AMD_ERR_DEVICE; }
    else if( q != hipSuccess ) rc = FD_ED25519_AMD_ERR_DEVICE;
    if( q != hipSuccess )
      fprintf( stderr, "fd_verify_amd_tile_run: the tile kernel %s after the stop (%s; scout clock ran %.3f ms, last change "
               "%.3f ms before the stop, chunks done %lu of %lu, kerr %u)\n", q == hipErrorNotReady ? "did not exit" : "failed",
               hipGetErrorString( q ), gc_first ? 1e-5 * (double)(__atomic_load_n( &H->gclock, __ATOMIC_ACQUIRE ) - gc_first) : -1.0,
               gc_host ? 1e-6 * (double)(t0 - gc_host) : -1.0, (ulong)__atomic_load_n( &H->gdone, __ATOMIC_ACQUIRE ),
               t->desc_seq - dbase, __atomic_load_n( &H->kerr, __ATOMIC_ACQUIRE ) );
  }
  ulong st[6] = { 0, 0, 0, 0, 0, 0 };
  if( !t->pending && ( hipMemcpyAsync( st, t->dctl->stat, sizeof st, hipMemcpyDeviceToHost, t->pst ) != hipSuccess ||
                       hipStreamSynchronize( t->pst ) != hipSuccess ) ) rc = FD_ED25519_AMD_ERR_DEVICE;
  if( __atomic_load_n( &H->kerr, __ATOMIC_ACQUIRE ) ) {
    fprintf( stderr, "fd_verify_amd_tile_run: the tile kernel's watchdog fired (no host heartbeat for 5 s)\n" );
    rc = FD_ED25519_AMD_ERR_DEVICE;
  }
  /* frags staged or in flight that were neither published nor filtered
     (halted, or an error): their frames are free for the next run */
  for( ulong q = r.pubd; q != staged; q++ ) unreserve( t->ppend[q & mask].fidx );
  diag->gpu_chunk_lat_cnt += st[0]; diag->gpu_chunk_thr_cnt += st[1];
  diag->gpu_frag_lat_cnt  += st[2]; diag->gpu_frag_thr_cnt  += st[3];
  diag->gpu_chunk_quad_cnt += st[4]; diag->gpu_frag_quad_cnt += st[5];
  diag->quad_pair_cnt += t->n_pair;
  diag->ovrn_cnt += ovrn + r.d.ovrn_cnt; diag->bad_frag_cnt += bad;
  diag->ha_filt_cnt += ha; diag->ha_filt_sz += ha_sz;
  diag->sv_filt_cnt += r.d.sv_filt_cnt; diag->sv_filt_sz += r.d.sv_filt_sz;
  for( int k=0; k<3; k++ ) diag->sv_filt_code_cnt[k] += r.d.sv_filt_code_cnt[k];
  diag->out_cnt += r.d.out_cnt; diag->out_sz += r.d.out_sz;
  diag->backp_cnt += backp + r.d.backp_cnt;
  diag->batch_cnt += nbatch; diag->batch_sig_cnt += nsig;
  diag->mode_switch_cnt += switches;
  if( halted || rc ) diag->halt_drop_cnt += staged - r.pubd;
  t->ring_seq = staged;
  t->pass_max_ns = pass_max;
  t->n_pass = n_pass; t->n_hand = n_hand; t->n_stop_window = n_stop_window; t->n_stop_frames = n_stop_frames;
  t->n_stop_bmax = n_stop_bmax; t->n_stop_pass = n_stop_pass; t->n_steal = n_steal;
  for( int k=0; k<4; k++ ) t->ph_tick[k] = ph_tick[k];
  t->ph_frags = ph_frags;
  __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
  if( in_fseq ) __atomic_store_n( in_fseq, in_seq, __ATOMIC_RELEASE );
  t->out_seq_end = r.out_seq;
  return rc;
}

extern "C" int
fd_verify_amd_tile_run( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth,
                        void const * in_chunk0, ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache,
                        ulong out_depth, ulong out_seq0, ulong const * out_fseq, ulong frag_cnt, int const * stop,
                        fd_verify_amd_diag_t * diag, uint * lat, ulong lat_max ) {
  if( !t || !in_mcache || !in_depth || (in_depth & (in_depth-1UL)) || !in_chunk0 || !out_mcache || !out_depth ||
      (out_depth & (out_depth-1UL)) || !diag || (!frag_cnt && !stop) ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( t->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;

  /* Output session.  A run whose out_seq0 continues the previous run's
     output keeps the frames' publication record, so a frame a lagging
     consumer may still read is not reused before out_fseq passes it; any
     other out_seq0 starts a new session (a new consumer), with every frame
     free. */
  if( out_seq0 != t->out_seq_end ) std::fill( t->frame_pub.begin(), t->frame_pub.end(), FRAME_FREE );
  t->frame_next_idx = 0UL;

  /* zero copy: the input data region is mapped into the GPU; frags are
     handed over as (chunk, size) and copied on the device.  zc_lim: bytes
     of the mapped region from in_chunk0 on (a frag reaching past it is
     refused as a bad frag, never read by the GPU). */
  uint8_t const * zc_dev = NULL;
  ulong zc_lim = 0UL;
  if( t->reg_base && (uint8_t const *)in_chunk0 >= t->reg_base &&
      (uint8_t const *)in_chunk0 < t->reg_base + t->reg_sz &&
      t->reg_sz - (ulong)((uint8_t const *)in_chunk0 - t->reg_base) <= (1UL << 38) ) {
    zc_dev = t->reg_dev + ((uint8_t const *)in_chunk0 - t->reg_base);
    zc_lim = t->reg_sz - (ulong)((uint8_t const *)in_chunk0 - t->reg_base);
  }
  return tile_run_persist( t, in_mcache, in_depth, in_chunk0, in_seq0, in_fseq, out_mcache, out_depth, out_seq0, out_fseq,
                           frag_cnt, stop, diag, lat, lat_max, zc_dev, zc_lim );
}

/* ------------------------------------------------------------------ */
/* streaming benchmark and end-to-end check: producer -> tile -> consumer */

/* The `want` quietest CPUs of `allowed` (CPU 0 excluded: it takes most
   of the machine's interrupts): per-CPU busy time from /proc/stat over
   ~30 ms, then one CPU per physical core while there are enough.  The
   bench box is one cgroup on a shared machine, so the spinning threads
   would otherwise land on CPUs other tenants keep busy, and a thread
   preempted for 1-2 ms shows up as a latency tail (profiles/
   r05_bench_*: producer_late_max 1.7 ms in one paced run).  Falls back to
   the highest-numbered CPUs when /proc/stat is unreadable.  Returns the
   number of CPUs written to out. */
static int
tile_quiet_cpus( cpu_set_t const * allowed, int want, int * out ) {
  auto snap = []( std::vector<unsigned long long> & busy, std::vector<unsigned long long> & tot ) -> bool {
    FILE * f = fopen( "/proc/stat", "r" );
    if( !f ) return false;
    char line[512];
    while( fgets( line, sizeof line, f ) ) {
      int c; unsigned long long v[8] = { 0 };
      if( strncmp( line, "cpu", 3 ) || line[3] < '0' || line[3] > '9' ) continue;
      if( sscanf( line + 3, "%d %llu %llu %llu %llu %llu %llu %llu %llu", &c, v, v+1, v+2, v+3, v+4, v+5, v+6, v+7 ) < 5 ) continue;
      if( c < 0 || c >= CPU_SETSIZE ) continue;
      if( (size_t)c >= busy.size() ) { busy.resize( (size_t)c + 1, 0ULL ); tot.resize( (size_t)c + 1, 0ULL ); }
      unsigned long long t = 0; for( int k=0; k<8; k++ ) t += v[k];
      tot[c] = t; busy[c] = t - v[3] - v[4];   /* all but idle and iowait */
    }
    fclose( f );
    return true;
  };
  std::vector<unsigned long long> b0, t0, b1, t1;
  bool ok = snap( b0, t0 );
  if( ok ) { struct timespec ts = { 0, 30000000L }; nanosleep( &ts, NULL ); ok = snap( b1, t1 ); }
  std::vector<std::pair<double, int>> cand;
  for( int c=CPU_SETSIZE-1; c>0; c-- ) {
    if( !CPU_ISSET( c, allowed ) ) continue;
    double load = 0.0;
    if( ok && (size_t)c < b1.size() && (size_t)c < b0.size() && t1[c] > t0[c] )
      load = (double)(b1[c] - b0[c]) / (double)(t1[c] - t0[c]);
    cand.emplace_back( load, c );
  }
  std::stable_sort( cand.begin(), cand.end(), []( std::pair<double, int> const & a, std::pair<double, int> const & b ) {
    return a.first < b.first; } );   /* stable: ties keep the highest-numbered first */
  auto core = []( int c ) -> int {   /* the first CPU listed as c's SMT sibling (its core), or c */
    char pth[128]; snprintf( pth, sizeof pth, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c );
    FILE * f = fopen( pth, "r" ); int k = c;
    if( f ) { if( fscanf( f, "%d", &k ) != 1 ) k = c; fclose( f ); }
    return k;
  };
  int n = 0;
  std::vector<int> cores;
  for( int pass=0; pass<2 && n<want; pass++ ) {   /* pass 0: one CPU per core; pass 1: fill with siblings */
    for( auto const & x : cand ) {
      if( n >= want ) break;
      int const c = x.second, k = core( c );
      bool used = false;
      for( int q=0; q<n; q++ ) if( out[q] == c ) used = true;
      if( used ) continue;
      if( !pass && std::find( cores.begin(), cores.end(), k ) != cores.end() ) continue;
      out[n++] = c; cores.push_back( k );
    }
  }
  return n;
}

/* Move every other thread of this process off the given CPUs (those
   whose mask would not become empty); returns the threads moved and their
   old masks. */
static std::vector<std::pair<pid_t, cpu_set_t>>
tile_isolate_cpus( int const * cpus, int n ) {
  std::vector<std::pair<pid_t, cpu_set_t>> moved;
  pid_t const me = (pid_t)syscall( SYS_gettid );
  DIR * d = opendir( "/proc/self/task" );
  if( !d ) return moved;
  for( struct dirent * e; (e = readdir( d )); ) {
    pid_t const tid = (pid_t)atoi( e->d_name );
    if( tid <= 0 || tid == me ) continue;
    cpu_set_t old, nw; CPU_ZERO( &old );
    if( sched_getaffinity( tid, sizeof old, &old ) ) continue;
    nw = old;
    for( int k=0; k<n; k++ ) if( cpus[k] >= 0 ) CPU_CLR( cpus[k], &nw );
    if( !CPU_COUNT( &nw ) || CPU_EQUAL( &nw, &old ) ) continue;
    if( !sched_setaffinity( tid, sizeof nw, &nw ) ) moved.emplace_back( tid, old );
  }
  closedir( d );
  return moved;
}

extern "C" int
fd_verify_amd_bench_stream( int device, ulong batch_max, ulong batch_wait_ns, double rate, int flags,
                            ulong dcache_frames, ulong pool_n, uchar const * pub, uchar const * sig,
                            uint const * msg_off, uint const * msg_sz, uchar const * blob, schar const * expect_err,
                            ulong const * expect_tag, ulong frag_cnt, ulong waves, double * out ) {
  if( !pool_n || !frag_cnt || !out || frag_cnt > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  bool const txn = !!(flags & FD_VERIFY_AMD_BENCH_TXN);
  for( ulong k=0; k<pool_n; k++ )
    if( txn ? (!msg_sz[k] || msg_sz[k] > FD_ED25519_AMD_MSG_MAX) : msg_sz[k] > FD_ED25519_AMD_MSG_MAX ) return FD_ED25519_AMD_ERR_INVAL;
  bool zero_copy = !!(flags & FD_VERIFY_AMD_BENCH_ZERO_COPY);
  bool writes    = !!(flags & FD_VERIFY_AMD_BENCH_WRITE);
  bool lap       = writes && (flags & FD_VERIFY_AMD_BENCH_LAP);
  bool check     = expect_err && expect_tag;
  ulong byte_mask = (flags & FD_VERIFY_AMD_BENCH_SAMPLE_BYTES) ? 15UL : 0UL;   /* compare bytes of every 16th frag */
  /* input depth > the frags the tile holds (zero copy releases a frag to the
     producer only once published: a depth under the tile's window would
     bound the stream instead of the tile); the rewriting modes keep 8
     batches (their dcache is sized past the depth) */
  ulong depth_min = 8UL*batch_max + 1024UL;
  ulong window = 0UL;                                          /* A/B: the tile's window (0 = tile_window's rule) */
  { char const * w = getenv( "FD_AMD_BENCH_WINDOW" ); if( w && *w ) window = strtoul( w, NULL, 0 ); }
  if( !writes ) {
    fd_verify_amd_tile_cfg_t wc; fd_verify_amd_tile_cfg_default( &wc ); wc.batch_max = batch_max; wc.window = window;
    depth_min = std::max( depth_min, tile_window( &wc ) + 4096UL );
  }
  ulong depth = 1UL; while( depth < depth_min ) depth <<= 1;
  /* output depth: 2^17 frags, ~2.5 ms of the saturated rate, so that a
     consumer descheduled for that long does not backpressure the tile (a
     2.5 ms consumer gap behind the reference's 16384-deep verify -> dedup
     link, receive_buffer_size, fdctl/config/default.toml:241, frank.rs:88,
     filled it and then the tile's window: profiles/r05_bench_final_f2_detail.json,
     4096 zero copy at 80 %); two batches when larger */
  ulong out_depth = 1UL; while( out_depth < std::max( 2UL*batch_max + 1024UL, 1UL << 17 ) ) out_depth <<= 1;
  ulong const frame = FD_VERIFY_AMD_FRAME_SZ, frame_c = FRAME_CHUNKS;
  /* Data region: either every pool frame once (what a NIC would have
     DMA'd; the producer publishes metadata only, so the bench measures the
     tile, not a producer-side memcpy), or a wrapping region of D frames the
     producer writes before publishing (D > depth: a frame is rewritten only
     after the mcache line of its previous frag was lapped, the tango sizing
     that makes the consumer's seq re-check sufficient). */
  ulong D = writes ? (dcache_frames ? dcache_frames : depth + 64UL) : pool_n;
  if( writes && D <= depth ) return FD_ED25519_AMD_ERR_INVAL;
  ulong region = (D * frame + 4095UL) & ~4095UL;
  std::vector<fd_frag_meta_t> in_mc( depth ), out_mc( out_depth );
  for( ulong i=0; i<depth; i++ )     in_mc[i].seq  = i - depth;       /* "never published" */
  for( ulong i=0; i<out_depth; i++ ) out_mc[i].seq = i - out_depth;
  uchar * dcache = (uchar *)aligned_alloc( 4096, region );
  if( !dcache ) return FD_ED25519_AMD_ERR_INVAL;
  memset( dcache, 0, region );
  /* frag k of the pool: pub | sig | msg, or (TXN) the wire transaction blob[msg_off, +msg_sz) */
  auto put_frame = [&]( uchar * p, ulong k ) {
    if( txn ) { memcpy( p, blob + msg_off[k], msg_sz[k] ); return; }
    memcpy( p, pub + 32UL*k, 32 ); memcpy( p + 32, sig + 64UL*k, 64 ); memcpy( p + 96, blob + msg_off[k], msg_sz[k] );
  };
  auto frag_sz = [&]( ulong k ) -> ulong { return (txn ? 0UL : 96UL) + msg_sz[k]; };
  if( !writes ) for( ulong k=0; k<pool_n; k++ ) put_frame( dcache + k * frame, k );

  /* the four spinning threads (producer, tile, its publisher, consumer)
     each get a CPU of their own from the process's allowed set, so the
     scheduler does not stack them (the saturated rate otherwise varies run
     to run): the quietest allowed CPUs, one per core, away from CPU 0,
     which takes most of the machine's interrupts (tile passes of 1-5 ms
     and p99 spikes were seen with the tile thread on CPU 0) */
  cpu_set_t allowed, saved; CPU_ZERO( &allowed ); CPU_ZERO( &saved );
  int cpus[5] = { -1, -1, -1, -1, -1 }, ncpu = 0;
  bool pin = !sched_getaffinity( 0, sizeof allowed, &allowed ) && CPU_COUNT( &allowed ) >= 5;
  if( pin ) {
    saved = allowed;
    int const want = CPU_COUNT( &allowed ) >= 6 ? 5 : 4;   /* the fifth: copy mode's helper */
    char const * pk = getenv( "FD_AMD_BENCH_CPU_PICK" );      /* A/B: "top" = the round-4 rule */
    if( pk && !strcmp( pk, "top" ) ) { for( int c=CPU_SETSIZE-1; c>0 && ncpu<want; c-- ) if( CPU_ISSET( c, &allowed ) ) cpus[ncpu++] = c; }
    else ncpu = tile_quiet_cpus( &allowed, want, cpus );
    pin = ncpu >= 4;
    static int said = 0;
    if( !said ) { said = 1; fprintf( stderr, "fd_verify_amd_bench_stream: spinning threads on CPUs %d %d %d %d %d\n",
                                     cpus[0], cpus[1], cpus[2], cpus[3], cpus[4] ); }
  }
  auto pin_to = [&]( int k ) {
    if( !pin ) return;
    cpu_set_t one; CPU_ZERO( &one ); CPU_SET( cpus[k], &one );
    (void)pthread_setaffinity_np( pthread_self(), sizeof one, &one );
  };
  /* the process's other threads (HIP runtime, interpreter) stay off the
     spinning threads' CPUs while the run lasts (as a deployed tile owns its
     cores); their masks are restored afterwards */
  std::vector<std::pair<pid_t, cpu_set_t>> moved;
  if( pin ) moved = tile_isolate_cpus( cpus, ncpu );

  fd_verify_amd_tile_cfg_t cfg;
  fd_verify_amd_tile_cfg_default( &cfg );
  cfg.device = device; cfg.batch_max = batch_max; cfg.batch_wait_ns = batch_wait_ns; cfg.tcache_depth = 0UL;
  cfg.waves = waves; cfg.window = window;
  /* output frames: the frags in flight, a pass, and a consumer that lags by
     up to the output depth (a frame is reused once out_fseq passed it) */
  cfg.out_frame_cnt = tile_window( &cfg ) + out_depth + batch_max + 4096UL;
  cfg.framing = txn ? FD_VERIFY_AMD_FRAMING_TXN : FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG;
  cfg.chunk_mode = (flags & FD_VERIFY_AMD_BENCH_CHUNK_LAT) ? FD_VERIFY_AMD_CHUNK_LATENCY
                 : (flags & FD_VERIFY_AMD_BENCH_CHUNK_THR) ? FD_VERIFY_AMD_CHUNK_THROUGHPUT
                 : (flags & FD_VERIFY_AMD_BENCH_CHUNK_QUAD) ? FD_VERIFY_AMD_CHUNK_QUAD : FD_VERIFY_AMD_CHUNK_AUTO;
  { /* A/B: "quad_hi,quad_lo,thr_hi,thr_lo" in slots/s (0 = the default) */
    char const * q = getenv( "FD_AMD_BENCH_LEVELS" );
    if( q && *q ) {
      ulong v[4] = { 0, 0, 0, 0 }; char * e = (char *)q;
      for( int k=0; k<4 && *e; k++ ) { v[k] = strtoul( e, &e, 0 ); if( *e == ',' ) e++; }
      cfg.quad_rate_hi = v[0]; cfg.quad_rate_lo = v[1]; cfg.thr_rate_hi = v[2]; cfg.thr_rate_lo = v[3];
    }
  }
  cfg.publish_cpu = (flags & FD_VERIFY_AMD_BENCH_PUB_INLINE) || !pin ? FD_VERIFY_AMD_PUBLISH_INLINE : cpus[3];
  cfg.copy_cpu    = zero_copy || (flags & FD_VERIFY_AMD_BENCH_COPY_INLINE) || !pin || cpus[4] < 0 ? FD_VERIFY_AMD_COPY_INLINE
                                                                                               : cpus[4];
  copier_stall_ns.store( (flags & FD_VERIFY_AMD_BENCH_STALL_HELPER) ? 200000UL : 0UL, std::memory_order_relaxed );
  fd_verify_amd_tile_t * tile = fd_verify_amd_tile_new_cfg( &cfg );
  if( !tile ) { free( dcache ); return FD_ED25519_AMD_ERR_DEVICE; }
  if( zero_copy && fd_verify_amd_tile_register_dcache( tile, dcache, region ) ) {
    fd_verify_amd_tile_delete( tile ); free( dcache ); return FD_ED25519_AMD_ERR_DEVICE;
  }
  uchar const * out_chunk0 = (uchar const *)fd_verify_amd_tile_out_chunk0( tile );
  std::vector<uint> parts;
  if( !check ) { parts.resize( 4UL * frag_cnt ); fd_verify_amd_tile_set_trace( tile, parts.data(), frag_cnt ); }

  ulong in_fseq = 0UL;                                   /* the tile's credit to the producer */
  std::atomic<ulong> out_fseq( 0UL );                    /* consumer progress (the tile's output credit) */
  std::vector<uint> lat( frag_cnt );
  /* steady state: published frags scheduled 20 ms or more after the
     producer's start (paced runs; the consumer marks them from tsorig) */
  std::vector<uchar> steady( check ? 0UL : frag_cnt, (uchar)0 );
  ulong const warm_ns = 20000000UL;
  fd_verify_amd_diag_t diag; memset( &diag, 0, sizeof diag );
  int tile_rc = 0;
  ulong mism = 0, checked = 0, late_max = 0, gap_max = 0, credit_max = 0;
  ulong t0 = now_ns(), t_prod0 = 0UL;   /* the rate is timed from the producer's start */

  std::thread prod( [&]() {
    pin_to( 1 );
    /* start once the tile's kernel runs (+2 ms): the launch of a run's
       persistent kernel is not part of the stream's latency (a deployed
       tile runs until halted) */
    {
      ulong const w0 = now_ns();
      while( !tile->started && !__atomic_load_n( &tile_rc, __ATOMIC_ACQUIRE ) && now_ns() - w0 < 5000000000UL ) { /* spin */ }
      ulong const w1 = now_ns(); while( now_ns() - w1 < 2000000UL ) { /* spin */ }
    }
    ulong p0 = now_ns(), cr = 0;   /* cr: first seq not covered by the cached credit */
    __atomic_store_n( &t_prod0, p0, __ATOMIC_RELEASE );
    uint  tnow = 0;                /* saturated: one timestamp per 32 frags (the producer must outrun the tile) */
    ulong lim = writes ? std::min( depth, D ) : depth;
    ulong k = 0, fw = 0;           /* seq % pool_n, seq % D, kept incrementally (no division per frag) */
    for( ulong seq=0; seq<frag_cnt; seq++, k = (k + 1UL == pool_n) ? 0UL : k + 1UL, fw = (fw + 1UL == D) ? 0UL : fw + 1UL ) {
      ulong due = rate > 0.0 ? p0 + (ulong)((double)seq * 1e9 / rate) : 0UL;   /* paced: open loop */
      if( due ) {
        ulong tn;
        while( (tn = now_ns()) < due ) { /* spin */ }
        late_max = std::max( late_max, tn - due );
      }
      /* credit: neither the mcache line nor (when writing) the data frame
         of a frag the tile still reads is reused; refreshed only when the
         cached credit runs out */
      if( !lap && seq >= cr ) {   /* out of credit: the tile holds the input (its wait is timed apart from lateness) */
        ulong const c0 = now_ns();
        while( seq >= cr ) cr = __atomic_load_n( &in_fseq, __ATOMIC_ACQUIRE ) + lim;
        credit_max = std::max( credit_max, now_ns() - c0 );
      }
      ulong sz = frag_sz( k );
      ulong fr = writes ? fw : k;
      if( writes ) put_frame( dcache + fr * frame, k );
      /* tsorig = the scheduled send time when paced, so producer stalls
         count as latency; the input seq when lapping (the check needs it) */
      if( !due && !(seq & 31UL) ) tnow = fd_verify_amd_tickcount();
      uint tso = lap ? (uint)seq : due ? (uint)due : tnow;
      fd_mcache_publish( in_mc.data(), depth, seq, 0UL, fr * frame_c, sz, 3UL, tso, 0UL );
    }
  } );
  ulong t10 = 0, t90 = 0, s10 = 0, s90 = 0;   /* check mode: when the consumer reached 10 % / 90 % of the input */
  std::thread cons( [&]() {
    pin_to( 2 );
    ulong seq = 0, fseq = 0;   /* fseq: last value published to out_fseq (every 64 frags, or when idle) */
    ulong exp_s = 0, exp_k = 0; /* check: next input seq that should be published, and seq % pool_n */
    long  last = -1;
    ulong tl = 0;              /* when the previous frag was seen */
    for( ;; ) {
      fd_frag_meta_t const * m = &out_mc[ seq & (out_depth-1UL) ];
      if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) == seq ) {
        if( !(seq & 15UL) ) { ulong tn = now_ns(); if( tl ) gap_max = std::max( gap_max, tn - tl ); tl = tn; }
        if( !check && seq < frag_cnt && rate > 0.0 ) {
          ulong const p0 = __atomic_load_n( &t_prod0, __ATOMIC_ACQUIRE );
          steady[seq] = (uchar)((int)((uint)m->tsorig - (uint)(p0 + warm_ns)) >= 0);
        }
        if( check ) {
          ulong tag = m->sig, chunk = m->chunk, sz = m->sz, s_in, k;
          if( lap ) {
            s_in = m->tsorig;
            if( (long)s_in <= last ) mism++;
            k = s_in % pool_n;
          } else {
            while( exp_s < frag_cnt && expect_err[exp_k] ) { exp_s++; exp_k = (exp_k + 1UL == pool_n) ? 0UL : exp_k + 1UL; }
            s_in = exp_s++; k = exp_k;
            exp_k = (exp_k + 1UL == pool_n) ? 0UL : exp_k + 1UL;
          }
          last = (long)s_in;
          /* the steady-state rate: input frags between 10 % and 90 % of the run */
          if( !t10 && s_in >= frag_cnt / 10UL ) { t10 = now_ns(); s10 = s_in; }
          if( !t90 && s_in >= 9UL * (frag_cnt / 10UL) ) { t90 = now_ns(); s90 = s_in; }
          uchar const * q = out_chunk0 + (chunk << FD_CHUNK_LG_SZ);
          bool ok = s_in < frag_cnt && !expect_err[k] && tag == expect_tag[k] && sz == frag_sz( k );
          if( ok && !(checked & byte_mask) )
            ok = txn ? !memcmp( q, blob + msg_off[k], msg_sz[k] )
                     : !memcmp( q, pub + 32UL*k, 32 ) && !memcmp( q + 32, sig + 64UL*k, 64 ) &&
                       !memcmp( q + 96, blob + msg_off[k], msg_sz[k] );
          mism += !ok; checked++;
        }
        seq++;
        if( seq - fseq >= 64UL ) { fseq = seq; out_fseq.store( seq, std::memory_order_release ); }
        continue;
      }
      if( __atomic_load_n( &tile_rc, __ATOMIC_ACQUIRE ) == 1 &&          /* tile finished and nothing left */
          __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != seq ) break;
      if( fseq != seq ) { fseq = seq; out_fseq.store( seq, std::memory_order_release ); }
    }
    if( check && !lap ) {     /* frags that should have been published and were not */
      ulong want = 0;
      for( ulong s=0; s<frag_cnt; s++ ) want += !expect_err[s % pool_n];
      if( want > checked ) mism += want - checked;
    }
  } );
  ulong const * ofs = (ulong const *)&out_fseq;
  pin_to( 0 );
  int rc = fd_verify_amd_tile_run( tile, in_mc.data(), depth, dcache, 0UL, &in_fseq, out_mc.data(), out_depth, 0UL, ofs,
                                   frag_cnt, NULL, &diag, lat.data(), frag_cnt );
  ulong t1 = now_ns();
  __atomic_store_n( &tile_rc, 1, __ATOMIC_RELEASE );
  if( rc ) __atomic_store_n( &in_fseq, ~0UL >> 1, __ATOMIC_RELEASE );   /* unblock the producer */
  prod.join(); cons.join();
  if( pin ) (void)pthread_setaffinity_np( pthread_self(), sizeof saved, &saved );
  for( auto const & mv : moved ) (void)sched_setaffinity( mv.first, sizeof mv.second, &mv.second );
  ulong const pass_max = tile->pass_max_ns;
  ulong const stg[6] = { tile->n_pass, tile->n_hand, tile->n_stop_window, tile->n_stop_frames, tile->n_stop_bmax, tile->n_stop_pass };
  ulong const n_steal = tile->n_steal;
  double ph_ns[4];
  for( int k=0; k<4; k++ ) ph_ns[k] = (double)tile->ph_tick[k] * tsc_clock().ns_per_tick / (double)std::max( tile->ph_frags, 1UL );
  copier_stall_ns.store( 0UL, std::memory_order_relaxed );
  fd_verify_amd_tile_delete( tile );
  free( dcache );
  if( rc ) return rc;
  ulong n = std::min( (ulong)diag.out_cnt, frag_cnt );
  for( int k=0; k<49; k++ ) out[k] = 0.0;
  for( int k=0; k<4; k++ ) out[44 + k] = ph_ns[k];
  out[41] = (double)n_steal;
  out[42] = (double)diag.gpu_chunk_quad_cnt; out[43] = (double)diag.gpu_frag_quad_cnt; out[48] = (double)diag.quad_pair_cnt;
  if( t90 > t10 && t10 && s90 > s10 ) out[40] = (double)(s90 - s10) / ((double)(t90 - t10) * 1e-9);
  /* decomposition (before lat is sorted: the samples are per published frag) */
  /* paced runs: percentiles over the steady state (n_st samples); the
     all-frags p50 / p99 go to out[38], out[39] */
  std::vector<uint> lat_all;
  ulong n_st = n;
  if( !steady.empty() && rate > 0.0 ) {
    lat_all.assign( lat.begin(), lat.begin() + (long)n );
    n_st = 0;
    for( ulong i=0; i<n; i++ ) if( steady[i] ) { lat[n_st] = lat[i]; if( !parts.empty() ) memmove( &parts[4*n_st], &parts[4*i], 16 ); n_st++; }
    if( !n_st ) { n_st = n; lat.assign( lat_all.begin(), lat_all.end() ); lat.resize( frag_cnt ); }
  }
  if( !parts.empty() && n_st ) {
    std::vector<uint> v[7];
    for( auto & x : v ) x.reserve( n_st );
    for( ulong i=0; i<n_st; i++ ) {
      uint const * p = parts.data() + 4UL * i;
      uint const svc = p[2] & 0x7fffffffu;
      ulong sum = (ulong)p[0] + p[1] + svc + p[3];
      v[0].push_back( p[0] ); v[1].push_back( p[1] ); v[2].push_back( svc ); v[3].push_back( p[3] );
      v[4].push_back( (ulong)lat[i] > sum ? (uint)((ulong)lat[i] - sum) : 0u );
      v[(p[2] >> 31) ? 5 : 6].push_back( svc );
    }
    auto q = []( std::vector<uint> & x, double f ) -> double {
      if( x.empty() ) return 0.0;
      ulong k = std::min( x.size() - 1UL, (ulong)(f * (double)x.size()) );
      std::nth_element( x.begin(), x.begin() + (long)k, x.end() );
      return (double)x[k];
    };
    for( int k=0; k<5; k++ ) { out[17 + 2*k] = q( v[k], 0.50 ); out[18 + 2*k] = q( v[k], 0.99 ); }
    out[27] = q( v[5], 0.50 ); out[28] = q( v[6], 0.50 );
    out[30] = (double)n_st;
  }
  out[29] = (double)diag.mode_switch_cnt;
  for( int k=0; k<6; k++ ) out[32 + k] = (double)stg[k];
  std::sort( lat.begin(), lat.begin() + (long)n_st );
  auto pct = [&]( double q ) -> double { return n_st && !lap ? (double)lat[ std::min( n_st-1UL, (ulong)(q * (double)n_st) ) ] : 0.0; };
  if( !lat_all.empty() ) {
    std::sort( lat_all.begin(), lat_all.end() );
    out[38] = (double)lat_all[ std::min( n-1UL, (ulong)(0.50 * (double)n) ) ];
    out[39] = (double)lat_all[ std::min( n-1UL, (ulong)(0.99 * (double)n) ) ];
  }
  { ulong const ts = __atomic_load_n( &t_prod0, __ATOMIC_ACQUIRE );
    out[0] = (double)diag.in_cnt / ((double)(t1 - (ts ? ts : t0)) * 1e-9); }
  out[1] = pct( 0.50 ); out[2] = pct( 0.99 ); out[3] = pct( 0.999 );
  out[4] = diag.batch_cnt ? (double)diag.batch_sig_cnt / (double)diag.batch_cnt : 0.0;
  out[5] = (double)diag.out_cnt; out[6] = (double)diag.sv_filt_cnt; out[7] = (double)diag.ovrn_cnt;
  out[8] = (double)mism; out[9] = (double)checked;
  out[10] = (double)diag.gpu_chunk_lat_cnt; out[11] = (double)diag.gpu_chunk_thr_cnt;
  out[12] = (double)diag.gpu_frag_lat_cnt;  out[13] = (double)diag.gpu_frag_thr_cnt;
  out[14] = (double)late_max; out[15] = (double)pass_max; out[16] = (double)gap_max; out[31] = (double)credit_max;
  return FD_ED25519_AMD_OK;
}

#ifdef FD_AMD_DIAG
/* ------------------------------------------------------------------ */
/* Diagnostics build only (tools/tile_synth.py): k_tile_persist's chunk
   pipeline on frags already in device memory, without the host hand-off.
   frames: nframes frames of FD_VERIFY_AMD_FRAME_SZ bytes (pub | sig | msg),
   fsz their sizes; ring entry j takes frame j % nframes.  out_ms: the
   launch's time; verdict: per entry the verdict, or 99 if its result word
   is missing.  where (flags): 1 ring entries, 2 results, 4 frames in
   mapped coherent host memory, 8 frames in mapped non-coherent host
   memory, 16 one more wave polling mapped host control words meanwhile
   (the scout's load) */
extern "C" int
fd_amd_tile_synth( int device, uint32_t waves, uint32_t iters, int eight, uint32_t where,
                   uint8_t const * frames, uint32_t nframes, uint32_t const * fsz, double * out_ms, int8_t * verdict ) {
  if( !frames || !nframes || !fsz || !out_ms || !verdict || !waves || !iters || waves > 65536u || iters > 4096u ) return FD_ED25519_AMD_ERR_INVAL;
  for( uint32_t f=0; f<nframes; f++ ) if( fsz[f] < 96u || fsz[f] > 96u + FD_ED25519_AMD_MSG_MAX ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  ulong const k = eight == 1 ? 8UL : eight == 2 ? 16UL : 64UL, n = (ulong)waves * iters * k;   /* eight: 0 throughput, 1 latency, 2 quad */
  ulong R = 1UL; while( R < n ) R <<= 1;
  std::vector<fd_amd_tile_ent_t> ent( R );
  for( ulong j=0; j<R; j++ ) ent[j] = fd_amd_tile_ent_t{ (uint32_t)((j % nframes) * FRAME_CHUNKS), 0u, fsz[j % nframes], 0u };
  uint8_t * d_fr = NULL; fd_amd_tile_ent_t * d_ent = NULL; uint64_t * d_res = NULL;
  fd_amd_tile_dctl_t * d_ctl = NULL; uint8_t * d_scr = NULL;
  fd_amd_tile_hctl_t * h_ctl = NULL; void * h_ctl_dev = NULL;
  void * hm[3] = { NULL, NULL, NULL };   /* host allocations of ring, results, frames */
  hipStream_t st = NULL; hipEvent_t e0 = NULL, e1 = NULL;
  int rc = FD_ED25519_AMD_ERR_DEVICE;
  std::vector<uint64_t> res( 2UL * R );
  fd_amd_tile_args_t A;
  float ms = 0.f;
  auto halloc = [&]( int k, ulong sz, unsigned fl, void ** dev ) -> bool {
    return hipHostMalloc( &hm[k], sz, hipHostMallocMapped | fl ) == hipSuccess && hipHostGetDevicePointer( dev, hm[k], 0 ) == hipSuccess;
  };
  unsigned const frfl = (where & 4u) ? hipHostMallocCoherent : hipHostMallocNonCoherent;
  if( ( (where & 12u) ? !halloc( 2, (ulong)nframes * FD_VERIFY_AMD_FRAME_SZ, frfl, (void **)&d_fr )
                      : hipMalloc( (void **)&d_fr, (ulong)nframes * FD_VERIFY_AMD_FRAME_SZ ) != hipSuccess ) ||
      ( (where & 1u) ? !halloc( 0, R * sizeof(fd_amd_tile_ent_t), hipHostMallocCoherent, (void **)&d_ent )
                     : hipMalloc( (void **)&d_ent, R * sizeof(fd_amd_tile_ent_t) ) != hipSuccess ) ||
      ( (where & 2u) ? !halloc( 1, 2UL * R * sizeof(uint64_t), hipHostMallocCoherent, (void **)&d_res )
                     : hipMalloc( (void **)&d_res, 2UL * R * sizeof(uint64_t) ) != hipSuccess ) ||
      ( (where & 16u) && ( hipHostMalloc( (void **)&h_ctl, sizeof(fd_amd_tile_hctl_t), hipHostMallocMapped | hipHostMallocCoherent ) != hipSuccess ||
                           hipHostGetDevicePointer( &h_ctl_dev, h_ctl, 0 ) != hipSuccess ) ) ||
      hipMalloc( (void **)&d_ctl, sizeof(fd_amd_tile_dctl_t) ) != hipSuccess ||
      hipMalloc( (void **)&d_scr, (ulong)waves * fd_amd_tile_scratch_stride() ) != hipSuccess ||
      hipStreamCreateWithFlags( &st, hipStreamNonBlocking ) != hipSuccess ||
      hipEventCreate( &e0 ) != hipSuccess || hipEventCreate( &e1 ) != hipSuccess ||
      hipMemcpy( hm[2] ? hm[2] : (void *)d_fr, frames, (ulong)nframes * FD_VERIFY_AMD_FRAME_SZ, hipMemcpyDefault ) != hipSuccess ||
      hipMemcpy( hm[0] ? hm[0] : (void *)d_ent, ent.data(), R * sizeof(fd_amd_tile_ent_t), hipMemcpyDefault ) != hipSuccess ||
      hipMemset( hm[1] ? hm[1] : (void *)d_res, 0, 2UL * R * sizeof(uint64_t) ) != hipSuccess ||
      hipMemset( d_ctl, 0, sizeof(fd_amd_tile_dctl_t) ) != hipSuccess ) goto done;
  memset( &A, 0, sizeof A );
  if( h_ctl ) memset( h_ctl, 0, sizeof(fd_amd_tile_hctl_t) );
  A.ent = d_ent; A.res_tag = d_res; A.res_word = d_res + R; A.mask = R - 1UL; A.src = d_fr; A.out = NULL; A.dctl = d_ctl; A.scratch = d_scr;
  A.hctl = (fd_amd_tile_hctl_t *)h_ctl_dev; A.watchdog = 1000000000UL;
  A.prof = (where & 32u) ? 1u : 0u;     /* per-phase clocks of every chunk, summed (stderr) */
  if( hipEventRecord( e0, st ) != hipSuccess || fd_amd_launch_tile_synth( &A, waves + (h_ctl ? 1u : 0u), iters, eight, st ) ||
      hipEventRecord( e1, st ) != hipSuccess || hipStreamSynchronize( st ) != hipSuccess ||
      hipEventElapsedTime( &ms, e0, e1 ) != hipSuccess ||
      hipMemcpy( res.data(), hm[1] ? hm[1] : (void *)d_res, 2UL * R * sizeof(uint64_t), hipMemcpyDefault ) != hipSuccess ) goto done;
  *out_ms = (double)ms;
  if( A.prof ) {
    fd_amd_tile_dctl_t dc;
    if( hipMemcpy( &dc, d_ctl, sizeof dc, hipMemcpyDeviceToHost ) != hipSuccess ) goto done;
    /* s_memrealtime runs at 100 MHz: per chunk per wave, in us */
    double const c = (double)waves * iters * 100.;
    fprintf( stderr, "tile_synth prof (us per chunk): gather %.1f prep %.1f decomp %.1f dsm %.1f results %.1f\n",
             (double)dc.prof[0] / c, (double)dc.prof[6] / c, (double)dc.prof[1] / c, (double)dc.prof[2] / c, (double)dc.prof[3] / c );
  }
  for( ulong j=0; j<n; j++ ) verdict[j] = (res[R + j] >> 8) == j + 1UL ? (int8_t)(uint8_t)(res[R + j] & 0xffUL) : (int8_t)99;
  rc = FD_ED25519_AMD_OK;
done:
  if( st ) (void)hipStreamSynchronize( st );
  if( e0 ) (void)hipEventDestroy( e0 );
  if( e1 ) (void)hipEventDestroy( e1 );
  if( st ) (void)hipStreamDestroy( st );
  if( d_fr && !hm[2] ) (void)hipFree( d_fr );
  if( d_ent && !hm[0] ) (void)hipFree( d_ent );
  if( d_res && !hm[1] ) (void)hipFree( d_res );
  for( int k=0; k<3; k++ ) if( hm[k] ) (void)hipHostFree( hm[k] );
  if( h_ctl ) (void)hipHostFree( h_ctl );
  if( d_ctl ) (void)hipFree( d_ctl );
  if( d_scr ) (void)hipFree( d_scr );
  return rc;
}
#endif /* FD_AMD_DIAG */
