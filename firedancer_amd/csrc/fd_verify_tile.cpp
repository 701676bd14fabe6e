/* firedancer_amd/csrc/fd_verify_tile.cpp
 *
 * Tango-compatible streaming verify tile on the MI355X engine
 * (include/fd_tango_amd.h).
 *
 * The reference verify tile (src/app/frank/load/fd_frank_verify_synth_load.c:
 * 300-425) verifies one frag per fd_ed25519_verify call.  Here the run loop
 * is split into a host side that never blocks on the GPU and a GPU side that
 * verifies whole batches:
 *
 *   poll   -- read the next input frag metadata (seq-checked, overrun-aware)
 *   dedup  -- HA tag cache (tag = first 8 signature bytes), FD_TCACHE_INSERT
 *             semantics (src/tango/tcache/fd_tcache.h:372-403): a tag is a
 *             duplicate iff it is one of the last `depth` distinct tags
 *   stage  -- reserve a frame of the tile-owned output dcache; copy mode:
 *             copy the frag into it, re-check the mcache line, release the
 *             input frag; zero-copy: hand the GPU (chunk, size) only
 *   launch -- adaptive batching: launch when the batch is full, or when the
 *             GPU is idle (no batch in flight), or when the oldest staged
 *             frag waited batch_wait_ns; up to 4 batches in flight
 *   publish-- when the oldest batch completes, publish its passing frags in
 *             arrival order (fd_mcache_publish protocol) out of the output
 *             dcache, with the GPU's SHA-512-derived dedup tag as meta.sig;
 *             failures count SV_FILT; zero-copy releases the batch's input
 *             frags only now
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
#include <x86intrin.h>
#include <thread>
#include <sched.h>
#include <pthread.h>
#include <vector>
#include <atomic>
#include <mutex>
#include <algorithm>

#include "../../include/fd_ed25519_amd.h"
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

struct pending_t {            /* one staged / in-flight frag */
  ulong  seq;                 /* input sequence number */
  ulong  frame;               /* output frame reservation (monotonic) */
  ushort sz, ctl;
  uint   tsorig;
  uint   fidx;                /* frame % frame_cnt (kept incrementally: no division per frag) */
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

inline bool use_tsc( void ) {   /* FD_AMD_TILE_CLOCK=mono selects clock_gettime (A/B) */
  char const * v = getenv( "FD_AMD_TILE_CLOCK" );
  return !(v && !strcmp( v, "mono" ));
}

inline ulong now_ns( void ) {
  static bool        const tsc = use_tsc();   /* thread-safe one-time init */
  static tsc_clock_t const c;
  if( !tsc ) return mono_ns();
  return c.ns0 + (ulong)((double)(long)(__rdtsc() - c.tsc0) * c.ns_per_tick);
}

} /* namespace */

#define FRAME_CHUNKS ((uint)(FD_VERIFY_AMD_FRAME_SZ >> FD_CHUNK_LG_SZ))
#define FRAME_FREE   (~0UL)
#define TXN_SIG_MAX_AT_MTU (19UL)   /* most signatures fd_amd_txn_slots1 reserves for a 1232-B payload */

struct tile_slot_t {
  uint32_t * h_meta;             /* pinned, mapped: [ichunk n | ochunk n | fsz n | tbase n+1] of the batch */
  uint32_t * m_meta;             /* its device address (the kernels read it in place) */
  uint8_t  * d_mir;              /* device frames of the batch, FD_VERIFY_AMD_FRAME_SZ apart */
  std::vector<pending_t> pend;
  std::vector<uint32_t>  ich, fsz, tb;
  ulong seq_lo;                  /* first input seq of the batch (zero-copy release point) */
  ulong frame_hi;                /* frame reservation counter after the batch's last frame */
  ulong nsig;                    /* signature slots (TXN) */
};

struct fd_verify_amd_tile {
  fd_ed25519_amd_t * eng;
  ulong              batch_max;
  ulong              wait_ns;
  tcache_t           tc;
  int                nslot;
  int                framing;   /* FD_VERIFY_AMD_FRAMING_* */
  uint8_t *          reg_base;  /* host data region mapped into the GPU (zero copy) */
  ulong              reg_sz;
  uint8_t *          reg_dev;
  /* the tile-owned output dcache: frame_cnt frames, pinned and mapped */
  uint8_t *          out_base;
  uint8_t *          out_dev;
  ulong              frame_cnt;
  std::vector<ulong> frame_pub;  /* out seq of the frag a frame last carried (FRAME_FREE: none) */
  ulong              frame_next, frame_retired;
  ulong              frame_next_idx;   /* frame_next % frame_cnt */
  ulong              out_seq_end;   /* out seq after the last run's last publish (a run continuing it keeps frame_pub) */
  tile_slot_t        ts[FD_AMD_SLOT_MAX];
  /* persistent consumer (PUB_SIG_MSG framing, k_tile_persist) */
  hipStream_t          pst;
  hipEvent_t           pdone;
  fd_amd_tile_hctl_t * hctl;  void * hctl_dev;
  fd_amd_tile_ent_t *  ring;  void * ring_dev;
  fd_amd_tile_desc_t * desc;  void * desc_dev;   /* chunk descriptors (same size as the ring) */
  uint64_t *           res;   void * res_dev;   /* results: R tags, then R verdict words */
  fd_amd_tile_dctl_t * dctl;
  uint8_t *            scratch;
  ulong                R;          /* ring size (power of 2) */
  ulong                window;     /* frags in flight at most (handed to the GPU, not yet published) */
  uint32_t             waves;
  ulong                light_frags;   /* hand-offs while fewer frags are in flight are cut into latency chunks */
  ulong                chunk_wait_ns; /* throughput mode: longest a partial chunk waits for company */
  ulong                pass_max_ns;   /* longest pass of the last run's loop (stall diagnosis) */
  bool                 counted;       /* in the per-device live tile count */
  ulong                desc_seq;      /* descriptors published, monotonic over the tile's life */
  std::vector<pending_t> ppend;    /* per ring slot */
  ulong                ring_seq;   /* ring index of the next frag, monotonic over the tile's life */
  bool                 batched;    /* FD_AMD_TILE_BATCHED=1: the multi-stream batch path for every framing (A/B) */
};

static ulong
env_ulong( char const * name, ulong dflt ) {
  char const * v = getenv( name );
  return ( v && *v ) ? strtoul( v, NULL, 0 ) : dflt;
}

extern "C" int
fd_verify_amd_tile_register_dcache( fd_verify_amd_tile_t * t, void * base, ulong sz ) {
  if( !t || !base || !sz ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( t->eng->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  if( t->reg_base ) { (void)hipHostUnregister( t->reg_base ); t->reg_base = NULL; t->reg_dev = NULL; t->reg_sz = 0; }
  uintptr_t lo = (uintptr_t)base & ~(uintptr_t)4095, hi = ((uintptr_t)base + sz + 4095) & ~(uintptr_t)4095;
  if( hipHostRegister( (void *)lo, hi - lo, hipHostRegisterMapped ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  void * dev = NULL;
  if( hipHostGetDevicePointer( &dev, (void *)lo, 0 ) != hipSuccess ) {
    (void)hipHostUnregister( (void *)lo );
    return FD_ED25519_AMD_ERR_DEVICE;
  }
  t->reg_base = (uint8_t *)lo; t->reg_sz = hi - lo; t->reg_dev = (uint8_t *)dev;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_verify_amd_tile_set_framing( fd_verify_amd_tile_t * t, int framing ) {
  if( !t || (framing != FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG && framing != FD_VERIFY_AMD_FRAMING_TXN) )
    return FD_ED25519_AMD_ERR_INVAL;
  /* every transaction must fit an empty batch, else the tile could never stage it */
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

#define TILE_NSLOT (4)   /* batches in flight (FD_AMD_TILE_NSLOT overrides; 6 or 8 measured: higher
                            p50 at every batch_max, higher saturated rate only at 16384): one wave's verify takes ~0.7 ms, so small
                            batches need several in flight to keep the GPU busy */

/* Live tiles per device (process-wide): a run's persistent kernel takes
   the wave slots of 8 x CUs / (tiles on its device), so tiles created on
   one GPU before any of them runs share it instead of the first run
   holding every slot (FD_AMD_TILE_WAVES fixes the count instead). */
namespace {
std::mutex g_tile_mu;
int        g_tile_cnt[64];
}

static void
tile_count( int device, int d ) {
  if( device < 0 || device >= 64 ) return;
  std::lock_guard<std::mutex> g( g_tile_mu );
  g_tile_cnt[device] += d;
}

static uint32_t
tile_run_waves( fd_verify_amd_tile_t const * t ) {
  if( getenv( "FD_AMD_TILE_WAVES" ) ) return t->waves;
  int n = 1;
  if( t->eng->device >= 0 && t->eng->device < 64 ) {
    std::lock_guard<std::mutex> g( g_tile_mu );
    n = std::max( 1, g_tile_cnt[t->eng->device] );
  }
  return std::max( 2u, t->waves / (uint32_t)n );
}

extern "C" uint
fd_verify_amd_tickcount( void ) {
  return (uint)now_ns();
}

extern "C" void
fd_verify_amd_tile_delete( fd_verify_amd_tile_t * t ) {
  if( !t ) return;
  if( t->counted ) tile_count( t->eng->device, -1 );
  (void)hipSetDevice( t->eng->device );
  fd_ed25519_amd_delete( t->eng );   /* synchronises every slot stream first */
  if( t->reg_base ) (void)hipHostUnregister( t->reg_base );
  for( int k=0; k<FD_AMD_SLOT_MAX; k++ ) {
    if( t->ts[k].h_meta ) (void)hipHostFree( t->ts[k].h_meta );
    if( t->ts[k].d_mir  ) (void)hipFree( t->ts[k].d_mir );
  }
  if( t->out_base ) (void)hipHostFree( t->out_base );
  if( t->pst )     (void)hipStreamDestroy( t->pst );
  if( t->pdone )   (void)hipEventDestroy( t->pdone );
  if( t->hctl )    (void)hipHostFree( t->hctl );
  if( t->ring )    (void)hipHostFree( t->ring );
  if( t->desc )    (void)hipHostFree( t->desc );
  if( t->res )     (void)hipHostFree( t->res );
  if( t->dctl )    (void)hipFree( t->dctl );
  if( t->scratch ) (void)hipFree( t->scratch );
  delete t;
}


/* The persistent consumer's resources: control words, ring and results in
   mapped coherent host memory, the device control block, per-wave scratch.
   Window (frags in flight): 64 x batch_max, at least 2^13, at most 2^18
   (FD_AMD_TILE_WINDOW overrides): a larger batch_max buys throughput with
   latency at saturation, as more batches in flight did in the batch path.
   Waves: 8 per CU, every wave slot of a kernel at 2 waves per SIMD
   (FD_AMD_TILE_WAVES overrides, e.g. to share a GPU between tiles). */
static int
tile_persist_alloc( fd_verify_amd_tile_t * t ) {
  ulong W = t->batch_max >= (1UL << 12) ? (1UL << 18) : std::max( 64UL * t->batch_max, 1UL << 13 );
  W = env_ulong( "FD_AMD_TILE_WINDOW", W );
  if( W > t->frame_cnt ) W = t->frame_cnt;
  if( !W ) return FD_ED25519_AMD_ERR_INVAL;
  ulong R = 1UL; while( R < W ) R <<= 1;
  int cus = 0;
  if( hipDeviceGetAttribute( &cus, hipDeviceAttributeMultiprocessorCount, t->eng->device ) != hipSuccess || cus <= 0 ) cus = 256;
  ulong waves = env_ulong( "FD_AMD_TILE_WAVES", 8UL * (ulong)cus );
  if( waves < 2UL || waves > 65536UL ) return FD_ED25519_AMD_ERR_INVAL;
  t->window = W; t->R = R; t->waves = (uint32_t)waves;
  /* latency chunks (8 frags, 8 lanes per signature) while at most one such
     chunk per SIMD is in flight: 8 x 4 x CUs frags */
  t->light_frags = env_ulong( "FD_AMD_TILE_LIGHT_FRAGS", 32UL * (ulong)cus );
  t->chunk_wait_ns = env_ulong( "FD_AMD_TILE_CHUNK_WAIT_NS", 50000UL );
  unsigned const hf = hipHostMallocMapped | hipHostMallocCoherent;
  if( hipStreamCreateWithFlags( &t->pst, hipStreamNonBlocking ) != hipSuccess ||
      hipEventCreateWithFlags( &t->pdone, hipEventDisableTiming ) != hipSuccess ||
      hipHostMalloc( (void **)&t->hctl, sizeof(fd_amd_tile_hctl_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->hctl_dev, t->hctl, 0 ) != hipSuccess ||
      hipHostMalloc( (void **)&t->ring, R * sizeof(fd_amd_tile_ent_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->ring_dev, t->ring, 0 ) != hipSuccess ||
      hipHostMalloc( (void **)&t->desc, R * sizeof(fd_amd_tile_desc_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->desc_dev, t->desc, 0 ) != hipSuccess ||
      hipHostMalloc( (void **)&t->res, 2UL * R * sizeof(uint64_t), hf ) != hipSuccess ||
      hipHostGetDevicePointer( &t->res_dev, t->res, 0 ) != hipSuccess ||
      hipMalloc( (void **)&t->dctl, sizeof(fd_amd_tile_dctl_t) ) != hipSuccess ||
      hipMalloc( (void **)&t->scratch, waves * fd_amd_tile_scratch_stride() ) != hipSuccess )
    return FD_ED25519_AMD_ERR_DEVICE;
  memset( t->hctl, 0, sizeof(fd_amd_tile_hctl_t) );
  memset( t->ring, 0, R * sizeof(fd_amd_tile_ent_t) );
  memset( t->desc, 0, R * sizeof(fd_amd_tile_desc_t) );
  t->desc_seq = 0UL;
  memset( t->res,  0, 2UL * R * sizeof(uint64_t) );   /* word 0 never matches an index + 1 */
  t->ppend.resize( R );
  t->ring_seq = 0UL;
  return FD_ED25519_AMD_OK;
}

extern "C" fd_verify_amd_tile_t *
fd_verify_amd_tile_new( int device, ulong batch_max, ulong batch_wait_ns, ulong tcache_depth, ulong out_frame_cnt ) {
  if( !batch_max || batch_max > (1UL<<20) ) return NULL;
  int nslot = TILE_NSLOT;
  if( char const * v = getenv( "FD_AMD_TILE_NSLOT" ) ) nslot = atoi( v );
  if( nslot < 2 || nslot > FD_AMD_SLOT_MAX ) return NULL;
  if( !out_frame_cnt ) {   /* the frags in flight (window, or the batch path's slots) + the staging group + the consumer's lag */
    ulong W = batch_max >= (1UL << 12) ? (1UL << 18) : std::max( 64UL * batch_max, 1UL << 13 );
    W = env_ulong( "FD_AMD_TILE_WINDOW", W );
    out_frame_cnt = 4096UL + batch_max + std::max( W, (ulong)nslot * batch_max );
  }
  if( out_frame_cnt > (0xFFFFFFFFUL / FRAME_CHUNKS) ) return NULL;   /* chunk indices are 32-bit */
  /* the engine's own staging is unused by the tile (frags reach the GPU
     through the output frames), so it is sized for a single message */
  fd_ed25519_amd_t * eng = fd_amd_engine_new( device, batch_max, FD_ED25519_AMD_MSG_MAX, nslot );
  if( !eng ) return NULL;
  fd_verify_amd_tile_t * t = new fd_verify_amd_tile_t();
  t->eng = eng; t->batch_max = batch_max; t->wait_ns = batch_wait_ns; t->nslot = nslot;
  t->framing = FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG;
  t->tc.init( tcache_depth );
  bool ok = true;
  for( int k=0; k<nslot && ok; k++ ) {
    tile_slot_t & s = t->ts[k];
    ok = !fd_amd_slot_alloc_aux( &eng->slot[k], batch_max ) &&
         hipHostMalloc( (void **)&s.h_meta, 4UL*(4UL*batch_max + 1UL), hipHostMallocMapped ) == hipSuccess &&
         hipHostGetDevicePointer( (void **)&s.m_meta, s.h_meta, 0 ) == hipSuccess &&
         hipMalloc( (void **)&s.d_mir, batch_max * FD_VERIFY_AMD_FRAME_SZ + 64UL ) == hipSuccess;
    s.pend.resize( batch_max ); s.ich.resize( batch_max ); s.fsz.resize( batch_max ); s.tb.resize( batch_max + 1UL );
  }
  ok = ok && hipHostMalloc( (void **)&t->out_base, out_frame_cnt * FD_VERIFY_AMD_FRAME_SZ, hipHostMallocMapped ) == hipSuccess &&
       hipHostGetDevicePointer( (void **)&t->out_dev, t->out_base, 0 ) == hipSuccess;
  t->frame_cnt = out_frame_cnt;
  t->frame_pub.assign( out_frame_cnt, FRAME_FREE );
  t->out_seq_end = ~0UL;
  t->batched = env_ulong( "FD_AMD_TILE_BATCHED", 0UL ) != 0UL;
  ok = ok && ( t->batched || !tile_persist_alloc( t ) );
  if( !ok ) { fd_verify_amd_tile_delete( t ); return NULL; }
  t->counted = true; tile_count( device, 1 );
  return t;
}

/* Launch the staged batch of tile slot k (n frags; nsig signature slots
   for TXN framing).  src: the mapped region the GPU copies the frags from
   (input dcache in zero-copy mode, the output dcache in copy mode); out:
   the mapped output dcache when the GPU must fill the output frames. */
static int
tile_launch( fd_verify_amd_tile_t * t, int k, ulong n, bool txn, uint8_t const * src, uint8_t * out ) {
  slot_t *      s  = &t->eng->slot[k];
  tile_slot_t & ts = t->ts[k];
  uint32_t * hm = ts.h_meta;
  memcpy( hm, ts.ich.data(), 4UL*n );
  for( ulong i=0; i<n; i++ ) hm[n + i] = (uint32_t)((ts.pend[i].frame % t->frame_cnt) * FRAME_CHUNKS);
  memcpy( hm + 2UL*n, ts.fsz.data(), 4UL*n );
  uint32_t const * m_tbase = ts.m_meta + 3UL*n;
  if( txn ) memcpy( hm + 3UL*n, ts.tb.data(), 4UL*(n + 1UL) );
  if( fd_amd_launch_tile_gather( (uint32_t)n, ts.m_meta, src, out, ts.d_mir, (uint32_t)FD_VERIFY_AMD_FRAME_SZ, txn ? 1 : 0,
                                 s->d_pub, s->d_sig, txn ? s->d_toff : s->d_off, txn ? s->d_tsz : s->d_sz, s->stream ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  /* tile batches are small next to the GPU, so the 4-lane latency kernels
     are used even with 4 in flight.  Measured (profiles/r01_tile_policy_ab.txt):
     switching batches of >= 4096/8192 to the 1-lane kernel while others were
     in flight lowered the saturated rate at every batch_max and doubled
     latency; the in-flight work (4 x batch_max) is too small for the 1-lane
     kernel to fill the GPU.  The 8-lane k_dsm8 only when batch_max <= 2048:
     four of its batches then still fit one wave per SIMD (batch_max 256:
     p50 650 -> 589 us; above, its doubled wave count oversubscribes the
     SIMDs; profiles/r02_tile_dsm8_ab.txt).  Transaction batches carry up to
     12 signatures per frag and keep the size rule. */
  int mode = fd_amd_batch_dsm_mode( (uint32_t)(txn ? ts.nsig : n), txn ? 0xFFFFFFFFu : (uint32_t)t->batch_max );
  if( txn ) {
    ulong nsig = ts.nsig;
    if( fd_amd_launch_txn_parse( (uint32_t)n, ts.d_mir, s->d_toff, s->d_tsz, s->d_fp, NULL, 0, m_tbase,
                                 s->d_pub, s->d_sig, s->d_off, s->d_sz, s->d_skip, s->stream ) )
      return FD_ED25519_AMD_ERR_DEVICE;
    if( nsig && fd_amd_launch_verify( (uint32_t)nsig, s->d_pub, s->d_sig, s->d_off, s->d_sz, ts.d_mir, s->d_err,
                                      s->d_ws, s->stream, 0, NULL, s->d_skip, mode ) )
      return FD_ED25519_AMD_ERR_DEVICE;
    if( fd_amd_launch_txn_reduce( (uint32_t)n, s->d_fp, m_tbase, s->d_err, s->d_terr, s->stream ) )
      return FD_ED25519_AMD_ERR_DEVICE;
    if( fd_amd_slot_out( s, s->h_terr, s->d_terr, n ) ) return FD_ED25519_AMD_ERR_DEVICE;
    if( nsig ) {
      ws_layout_t L = fd_amd_ws_layout( nsig );
      if( fd_amd_slot_out( s, s->h_tag, (uint8_t *)s->d_ws + L.tag, 8UL*nsig ) ) return FD_ED25519_AMD_ERR_DEVICE;
    }
  } else {
    if( fd_amd_launch_verify( (uint32_t)n, s->d_pub, s->d_sig, s->d_off, s->d_sz, ts.d_mir, s->d_err, s->d_ws,
                              s->stream, 1, NULL, NULL, mode ) )
      return FD_ED25519_AMD_ERR_DEVICE;
    if( fd_amd_slot_out( s, s->h_err, s->d_err, n ) ) return FD_ED25519_AMD_ERR_DEVICE;
    ws_layout_t L = fd_amd_ws_layout( n );
    if( fd_amd_slot_out( s, s->h_tag, (uint8_t *)s->d_ws + L.tag, 8UL*n ) ) return FD_ED25519_AMD_ERR_DEVICE;
  }
  if( hipEventRecord( s->done, s->stream ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  s->out = s->t_out = s->s_out = NULL;
  s->n = n; s->t_n = n; s->busy = 1;
  s->chk_err = txn ? 0 : n; s->chk_terr = txn ? n : 0;
  return FD_ED25519_AMD_OK;
}

/* Error exit of the batch path: wait for every batch still in flight (a
   queued k_tile_gather reads its slot's mapped metadata in place, which the
   next run rewrites) and forget them. */
static int
tile_quiesce( fd_verify_amd_tile_t * t, int rc ) {
  for( int k=0; k<t->nslot; k++ ) {
    slot_t * s = &t->eng->slot[k];
    if( s->busy ) (void)hipEventSynchronize( s->done );
    s->out = s->t_out = s->s_out = NULL;
    s->busy = 0;
  }
  return rc;
}

static int
tile_run_persist( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth, void const * in_chunk0,
                  ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache, ulong out_depth, ulong out_seq0,
                  ulong const * out_fseq, ulong frag_cnt, int const * stop, fd_verify_amd_diag_t * diag, uint * lat,
                  ulong lat_max, uint8_t const * zc_dev, ulong zc_lim );

/* The multi-stream batch path: TXN framing (and every framing under
   FD_AMD_TILE_BATCHED=1). */
static int
tile_run_batched( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth, void const * in_chunk0,
                  ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache, ulong out_depth, ulong out_seq0,
                  ulong const * out_fseq, ulong frag_cnt, int const * stop, fd_verify_amd_diag_t * diag, uint * lat,
                  ulong lat_max, uint8_t const * zc_dev, ulong zc_lim );

extern "C" int
fd_verify_amd_tile_run( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth,
                        void const * in_chunk0, ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache,
                        ulong out_depth, ulong out_seq0, ulong const * out_fseq, ulong frag_cnt, int const * stop,
                        fd_verify_amd_diag_t * diag, uint * lat, ulong lat_max ) {
  if( !t || !in_mcache || !in_depth || (in_depth & (in_depth-1UL)) || !in_chunk0 || !out_mcache || !out_depth ||
      (out_depth & (out_depth-1UL)) || !diag || (!frag_cnt && !stop) ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( t->eng->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  bool txn = t->framing == FD_VERIFY_AMD_FRAMING_TXN;
  if( txn && t->batch_max < TXN_SIG_MAX_AT_MTU ) return FD_ED25519_AMD_ERR_INVAL;

  /* Output session.  A run whose out_seq0 continues the previous run's
     output keeps the frames' publication record, so a frame a lagging
     consumer may still read is not reused before out_fseq passes it; any
     other out_seq0 starts a new session (a new consumer), with every frame
     free. */
  if( out_seq0 != t->out_seq_end ) std::fill( t->frame_pub.begin(), t->frame_pub.end(), FRAME_FREE );
  t->frame_next = t->frame_retired = t->frame_next_idx = 0UL;

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
  if( !txn && !t->batched )
    return tile_run_persist( t, in_mcache, in_depth, in_chunk0, in_seq0, in_fseq, out_mcache, out_depth, out_seq0, out_fseq,
                             frag_cnt, stop, diag, lat, lat_max, zc_dev, zc_lim );
  return tile_run_batched( t, in_mcache, in_depth, in_chunk0, in_seq0, in_fseq, out_mcache, out_depth, out_seq0, out_fseq,
                           frag_cnt, stop, diag, lat, lat_max, zc_dev, zc_lim );
}

static int
tile_run_batched( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth, void const * in_chunk0,
                  ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache, ulong out_depth, ulong out_seq0,
                  ulong const * out_fseq, ulong frag_cnt, int const * stop, fd_verify_amd_diag_t * diag, uint * lat,
                  ulong lat_max, uint8_t const * zc_dev, ulong zc_lim ) {
  fd_ed25519_amd_t * e = t->eng;
  bool txn = t->framing == FD_VERIFY_AMD_FRAMING_TXN;
  ulong const F = t->frame_cnt;
  ulong in_seq = in_seq0, out_seq = out_seq0, lat_n = 0;
  int   K = t->nslot;
  int   stage = 0;                 /* slot being filled; slots are used round robin, so the */
  int   oldest = 0, nfly = 0;      /* in-flight ones are oldest, oldest+1, ... (mod K)      */
  ulong staged = 0, slots = 0, stage_t0 = 0;
  int   rc;
  /* Flow-control state shared with other threads is exchanged in strides,
     not per frag (the reference's tiles publish fseq and refresh credits
     in housekeeping, fd_fctl): diag->in_cnt and in_fseq are published per
     staging pass; out_fseq is re-read only when a cached value runs out. */
  ulong in_cnt = diag->in_cnt, out_cr = 0, cons = out_seq0, fseq_pub = ~0UL;
  /* debug (FD_AMD_TILE_DEBUG): host TSC ticks in retire+publish, staging,
     launch, and spinning with every slot in flight */
  bool const hdbg = env_ulong( "FD_AMD_TILE_DEBUG", 0UL ) != 0UL;
  ulong hpt[4] = { 0, 0, 0, 0 }, hspin = 0, ht = hdbg ? __rdtsc() : 0UL, ht0 = ht, hns0 = hdbg ? now_ns() : 0UL, hin0 = in_cnt;
# define HSTAMP( k_ ) do { if( hdbg ) { ulong t_ = __rdtsc(); hpt[k_] += t_ - ht; ht = t_; } } while(0)

  auto publish = [&]( int k ) -> int {
    slot_t *      s  = &e->slot[k];
    tile_slot_t & ts = t->ts[k];
    if( (rc = fd_amd_slot_drain( s )) ) return rc;
    ulong cnt = s->n;
    for( ulong i=0; i<cnt; i++ ) {
      pending_t const & m = ts.pend[i];
      /* zero copy: the GPU read the frag some time before now; if its mcache
         line has been lapped since, the producer may have rewritten it */
      if( zc_dev && __atomic_load_n( &in_mcache[ m.seq & (in_depth-1UL) ].seq, __ATOMIC_ACQUIRE ) != m.seq ) {
        diag->ovrn_cnt++;
        continue;
      }
      int bad = txn ? s->h_terr[i] : s->h_err[i];
      if( bad ) { diag->sv_filt_cnt++; diag->sv_filt_sz += m.sz; continue; }
      /* dedup tag: the verify's SHA-512 tag of the (first) signature */
      ulong tag = txn ? s->h_tag[ ts.tb[i] ] : s->h_tag[i];
      if( out_fseq && (long)(out_seq - out_cr) >= 0 ) {   /* credit check against the slowest consumer */
        out_cr = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE ) + out_depth;
        if( (long)(out_seq - out_cr) >= 0 ) {
          diag->backp_cnt++;
          do out_cr = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE ) + out_depth; while( (long)(out_seq - out_cr) >= 0 );
        }
      }
      ulong f = m.fidx;
      t->frame_pub[f] = out_seq;
      uint tspub = fd_verify_amd_tickcount();
      fd_mcache_publish( out_mcache, out_depth, out_seq, tag, f * FRAME_CHUNKS, m.sz, m.ctl, m.tsorig, tspub );
      if( lat && lat_n < lat_max ) lat[lat_n++] = tspub - m.tsorig;
      out_seq++; diag->out_cnt++; diag->out_sz += m.sz;
    }
    t->frame_retired = ts.frame_hi;
    return FD_ED25519_AMD_OK;
  };

  for( ;; ) {
    /* 1. retire the oldest batch if it is done (publication stays in
          arrival order: batches retire in launch order) */
    while( nfly ) {
      int r = fd_amd_slot_ready( &e->slot[oldest] );
      if( r < 0 ) return tile_quiesce( t, r );
      if( !r ) break;
      if( (rc = publish( oldest )) ) return tile_quiesce( t, rc );
      oldest = (oldest + 1) % K; nfly--;
    }
    HSTAMP( 0 );
    /* producer credit: copy mode is done with a frag once it is copied;
       zero copy only once the batch holding it has retired */
    if( in_fseq ) {
      ulong rel = !zc_dev ? in_seq : nfly ? t->ts[oldest].seq_lo : staged ? t->ts[stage].seq_lo : in_seq;
      if( rel != fseq_pub ) { __atomic_store_n( in_fseq, rel, __ATOMIC_RELEASE ); fseq_pub = rel; }
    }
    bool done_in = frag_cnt ? (in_seq - in_seq0 >= frag_cnt) : (__atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0);
    if( done_in && !staged && !nfly ) break;
    if( nfly == K ) { hspin++; HSTAMP( 3 ); continue; }   /* every slot in flight: the staging slot is busy */

    /* 2. stage input frags into the free slot */
    tile_slot_t & ts = t->ts[stage];
    bool idle_in = false, full = false;
    while( !done_in && staged < t->batch_max ) {
      if( frag_cnt && in_seq - in_seq0 >= frag_cnt ) break;
      fd_frag_meta_t const * m = in_mcache + (in_seq & (in_depth-1UL));
      ulong seq_found = __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE );
      long  d = (long)(seq_found - in_seq);
      if( d < 0 ) { idle_in = true; break; }                             /* not yet published */
      if( d > 0 ) { diag->ovrn_cnt += (ulong)d; in_seq = seq_found; continue; }   /* overrun: resync */
      ulong chunk = m->chunk, sz = m->sz, ctl = m->ctl, tsorig = m->tsorig;
      __atomic_thread_fence( __ATOMIC_ACQUIRE );
      if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != in_seq ) { diag->ovrn_cnt++; in_seq++; continue; }
      if( (txn ? (!sz || sz > FD_ED25519_AMD_MSG_MAX) : (sz < 96UL || sz - 96UL > FD_ED25519_AMD_MSG_MAX)) ||
          (zc_dev && (chunk << FD_CHUNK_LG_SZ) + ((sz + 63UL) & ~63UL) > zc_lim) ) {
        diag->bad_frag_cnt++; in_seq++; in_cnt++; continue;
      }
      /* reserve the next output frame: not staged or in flight, and no
         longer read by a consumer that honours flow control */
      ulong fr = t->frame_next, f = t->frame_next_idx;
      if( fr - t->frame_retired >= F ) { full = true; break; }
      if( out_fseq && t->frame_pub[f] != FRAME_FREE && (long)(t->frame_pub[f] - cons) >= 0 ) {
        cons = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE );
        if( (long)(t->frame_pub[f] - cons) >= 0 ) { diag->backp_cnt++; full = true; break; }
      }
      uchar const * p = (uchar const *)fd_chunk_to_laddr_const( in_chunk0, chunk );
      if( !zc_dev ) {
        /* copy mode: the frame is the tile's copy; a frag lapped while it
           was copied is dropped (speculative read, then seq re-check) */
        uint8_t * dst = t->out_base + f * FD_VERIFY_AMD_FRAME_SZ;
        memcpy( dst, p, sz );
        __atomic_thread_fence( __ATOMIC_ACQUIRE );
        if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != in_seq ) { diag->ovrn_cnt++; in_seq++; continue; }
        p = dst;
      }
      ulong k2 = 0;
      if( txn ) {
        /* wire transaction (fd_txn.h layout): dedup on its first signature */
        k2 = fd_amd_txn_slots1( p, sz );
        if( slots + k2 > t->batch_max ) { full = true; break; }        /* no room for its signatures: next batch */
      }
      in_seq++; in_cnt++;
      ulong ha_tag = 0;
      if( !txn )   memcpy( &ha_tag, p + 32, 8 );                        /* first 8 signature bytes */
      else if( k2 ) memcpy( &ha_tag, p + 1, 8 );
      if( (!txn || k2) && t->tc.insert( ha_tag ) ) { diag->ha_filt_cnt++; diag->ha_filt_sz += sz; continue; }
      t->frame_pub[f] = FRAME_FREE;
      t->frame_next++;
      if( ++t->frame_next_idx == F ) t->frame_next_idx = 0UL;
      ts.ich[staged] = zc_dev ? (uint32_t)chunk : (uint32_t)(f * FRAME_CHUNKS);
      ts.fsz[staged] = (uint32_t)sz;
      ts.tb[staged]  = (uint32_t)slots;
      slots += k2;
      ts.pend[staged] = pending_t{ in_seq - 1UL, fr, (ushort)sz, (ushort)ctl, (uint)tsorig, (uint)f };
      if( !staged ) { stage_t0 = now_ns(); ts.seq_lo = in_seq - 1UL; }
      staged++;
    }
    __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
    if( in_fseq && !zc_dev && in_seq != fseq_pub ) { __atomic_store_n( in_fseq, in_seq, __ATOMIC_RELEASE ); fseq_pub = in_seq; }
    done_in = frag_cnt ? (in_seq - in_seq0 >= frag_cnt) : (__atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0);
    HSTAMP( 1 );

    /* 3. adaptive launch (a free slot exists here): full batch, input
          momentarily drained (greedy: under light load batches stay small
          and latency low; under load every slot is busy and batches grow
          toward batch_max), end of input, no frame or signature room left,
          or the oldest staged frag waited batch_wait_ns.  A nonzero
          batch_wait_ns turns the greedy rule off while another batch is in
          flight. */
    bool greedy = idle_in && (!t->wait_ns || !nfly);
    if( staged && ( staged == t->batch_max || full || greedy || done_in ||
                    (t->wait_ns && now_ns() - stage_t0 >= t->wait_ns) ) ) {
      ts.tb[staged] = (uint32_t)slots;
      ts.nsig = slots;
      ts.frame_hi = t->frame_next;
      uint8_t const * src = zc_dev ? zc_dev : t->out_dev;
      if( (rc = tile_launch( t, stage, staged, txn, src, zc_dev ? t->out_dev : NULL )) ) return tile_quiesce( t, rc );
      diag->batch_sig_cnt += txn ? slots : staged;
      diag->batch_cnt++;
      nfly++;
      stage = (stage + 1) % K; staged = 0; slots = 0;
    }
    HSTAMP( 2 );
  }
# undef HSTAMP
  if( hdbg ) {
    double const tot = (double)(__rdtsc() - ht0);
    fprintf( stderr, "tile debug (batch path, host): publish %.1f%% stage %.1f%% launch %.1f%% all-slots-busy %.1f%% (%lu spins), "
             "%.1f ns/frag\n", 100.0*(double)hpt[0]/tot, 100.0*(double)hpt[1]/tot, 100.0*(double)hpt[2]/tot,
             100.0*(double)hpt[3]/tot, hspin, (double)(now_ns() - hns0) / (double)(in_cnt - hin0 + 1UL) );
  }
  __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
  if( in_fseq ) __atomic_store_n( in_fseq, in_seq, __ATOMIC_RELEASE );
  t->out_seq_end = out_seq;
  return FD_ED25519_AMD_OK;
}

/* The persistent path (PUB_SIG_MSG framing).  One k_tile_persist launch
   per run; the host thread polls, dedups and stages frags into the ring,
   hands them over by advancing the ring head, and publishes verdicts in
   ring order as the GPU's result words arrive.  Nothing here waits on a
   HIP call: the GPU side is driven entirely through mapped memory.

     stage   -- as the batch path (poll, dedup, reserve an output frame;
                copy mode: copy the frag there), then write the frag's
                ring entry
     hand    -- advance the ring head (the GPU's claimable range): when
                batch_max frags are staged, the input is momentarily
                drained (greedy; with batch_wait_ns only while nothing is
                in flight), the input ended, the window or the frames ran
                out, or the oldest staged frag waited batch_wait_ns
     publish -- the next frag in ring order whose result word carries its
                index: lapped (zero copy) -> overrun, failed -> SV_FILT,
                else fd_mcache_publish out of its output frame

   The window (t->window frags handed over and not yet published) bounds
   the GPU's work in flight; with the output frames it is the tile's
   backpressure on the producer. */
/* The persistent path's hand-off rule (tile_run_persist step 3): of the
   staged frags [handed, staged), how far to hand over now, and in which
   chunk mode (*lat_mode: 8-frag latency chunks, else 64-frag throughput
   chunks).  Latency mode while fewer than light_frags frags are in flight
   (handed - pubd): everything, as soon as the input is momentarily drained
   (with wait_ns only while nothing is in flight).  Throughput mode: whole
   64-frag chunks only, a remainder once its oldest frag waited
   chunk_wait_ns.  Either mode: everything at batch_max staged, when the
   window or the frames ran out (full), at the end of the input, or once the
   oldest waited wait_ns (nonzero).  Pure; exported for the CPU tests. */
extern "C" ulong
fd_verify_amd_tile_cut( ulong staged, ulong handed, ulong pubd, ulong light_frags, ulong batch_max, ulong waited_ns,
                        ulong wait_ns, ulong chunk_wait_ns, int idle_in, int full, int done_in, int * lat_mode ) {
  bool const lat = handed - pubd < light_frags;
  if( lat_mode ) *lat_mode = lat ? 1 : 0;
  if( staged == handed ) return handed;
  bool const flush = staged - handed >= batch_max || full || done_in || (wait_ns && waited_ns >= wait_ns) ||
                     (!lat && waited_ns >= chunk_wait_ns);
  if( flush || (lat && idle_in && (!wait_ns || handed == pubd)) ) return staged;
  return lat ? handed : handed + ((staged - handed) & ~63UL);
}

static int
tile_run_persist( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth, void const * in_chunk0,
                  ulong in_seq0, ulong * in_fseq, fd_frag_meta_t * out_mcache, ulong out_depth, ulong out_seq0,
                  ulong const * out_fseq, ulong frag_cnt, int const * stop, fd_verify_amd_diag_t * diag, uint * lat,
                  ulong lat_max, uint8_t const * zc_dev, ulong zc_lim ) {
  ulong const F = t->frame_cnt, mask = t->R - 1UL, W = t->window, base = t->ring_seq;
  fd_amd_tile_hctl_t * H = t->hctl;

  /* seed the control words, then launch: the kernel's ticket counter and
     the mirrors start at this run's first descriptor */
  ulong const dbase = t->desc_seq;
  __atomic_store_n( &H->head, dbase, __ATOMIC_RELAXED );
  __atomic_store_n( &H->stop, 0u, __ATOMIC_RELAXED );
  __atomic_store_n( &H->kerr, 0u, __ATOMIC_RELAXED );
  ulong beat = __atomic_load_n( &H->beat, __ATOMIC_RELAXED );
  {
    fd_amd_tile_dctl_t d0;
    memset( &d0, 0, sizeof d0 );
    d0.ticket = dbase;
    for( int x=0; x<FD_AMD_TILE_MIRRORS; x++ ) d0.mw[x].w = dbase;
    if( hipMemcpyAsync( t->dctl, &d0, sizeof d0, hipMemcpyHostToDevice, t->pst ) != hipSuccess ||
        hipStreamSynchronize( t->pst ) != hipSuccess )
      return FD_ED25519_AMD_ERR_DEVICE;
  }
  fd_amd_tile_args_t A;
  memset( &A, 0, sizeof A );
  A.hctl = (fd_amd_tile_hctl_t *)t->hctl_dev;
  A.ent  = (fd_amd_tile_ent_t const *)t->ring_dev;
  A.desc = (fd_amd_tile_desc_t const *)t->desc_dev;
  A.res_tag  = (uint64_t *)t->res_dev;
  A.res_word = (uint64_t *)t->res_dev + t->R;
  A.mask = mask;
  A.src  = zc_dev ? zc_dev : t->out_dev;
  A.out  = zc_dev ? t->out_dev : NULL;
  A.dctl = t->dctl;
  A.scratch = t->scratch;
  A.watchdog = 500000000UL;   /* 5 s of s_memrealtime (100 MHz) without a heartbeat */
  A.prof = (uint32_t)env_ulong( "FD_AMD_TILE_DEBUG", 0UL );
  uint32_t const waves = tile_run_waves( t );
  if( fd_amd_launch_tile_persist( &A, waves, t->pst ) || hipEventRecord( t->pdone, t->pst ) != hipSuccess ) {
    (void)hipStreamSynchronize( t->pst );
    return FD_ED25519_AMD_ERR_DEVICE;
  }

  ulong in_seq = in_seq0, out_seq = out_seq0, lat_n = 0;
  ulong staged = base, handed = base, pubd = base, hand_t0 = 0UL;
  ulong in_cnt = diag->in_cnt, out_cr = 0, cons = out_seq0, fseq_pub = ~0UL;
  ulong idle = 0UL;
  int   rc = FD_ED25519_AMD_OK;
  uchar const * in_chunk0b = (uchar const *)in_chunk0;

  ulong iter = 0UL, pass_t = now_ns(), pass_max = 0UL;
  /* debug (FD_AMD_TILE_DEBUG): host TSC ticks in publish, staging, hand-off and empty passes */
  bool const hdbg = A.prof != 0u;
  ulong hpt[3] = { 0, 0, 0 }, ht = hdbg ? __rdtsc() : 0UL, ht0 = ht, hns0 = hdbg ? now_ns() : 0UL, hin0 = in_cnt, hpass = 0;
# define HSTAMP( k_ ) do { if( hdbg ) { ulong t_ = __rdtsc(); hpt[k_] += t_ - ht; ht = t_; } } while(0)
  for( ;; ) {
    /* the kernel's watchdog needs a heartbeat now and then, not every
       pass: each store after a GPU read of the line is a cache-line
       ownership round trip */
    if( !(++iter & 63UL) ) __atomic_store_n( &H->beat, ++beat, __ATOMIC_RELAXED );
    bool progress = false;
    { ulong const tn = now_ns(); pass_max = std::max( pass_max, tn - pass_t ); pass_t = tn; }

    /* 1. publish in ring order: count the results that are in, then (zero
          copy) check once that the oldest of them was not lapped -- lapping
          goes in sequence order, so if its mcache line is intact now, after
          the GPU read every frag of the pass, so are the newer ones' -- then
          publish them with one timestamp */
    ulong ready = 0UL;
    while( pubd + ready != handed && ready < 4096UL ) {
      ulong w = __atomic_load_n( t->res + t->R + ((pubd + ready) & mask), __ATOMIC_ACQUIRE );
      if( (w >> 8) != pubd + ready + 1UL ) break;
      ready++;
    }
    if( ready ) {
      progress = true;
      bool lap_ok = true;
      if( zc_dev ) {
        ulong const s0 = t->ppend[pubd & mask].seq;
        lap_ok = __atomic_load_n( &in_mcache[ s0 & (in_depth-1UL) ].seq, __ATOMIC_ACQUIRE ) == s0;
      }
      uint const tspub = fd_verify_amd_tickcount();
      for( ulong end = pubd + ready; pubd != end; ) {
        ulong const j = pubd & mask;
        ulong const w = t->res[ t->R + j ];
        pending_t const & m = t->ppend[j];
        pubd++;
        t->frame_retired = m.frame + 1UL;
        /* zero copy: the GPU read the frag some time before now; if its
           mcache line has been lapped since, the producer may have
           rewritten it */
        if( !lap_ok && __atomic_load_n( &in_mcache[ m.seq & (in_depth-1UL) ].seq, __ATOMIC_ACQUIRE ) != m.seq ) {
          diag->ovrn_cnt++;
          continue;
        }
        if( (schar)(uchar)(w & 0xffUL) ) { diag->sv_filt_cnt++; diag->sv_filt_sz += m.sz; continue; }
        ulong tag = t->res[ j ];   /* the verify's SHA-512 tag (dedup tile) */
        if( out_fseq && (long)(out_seq - out_cr) >= 0 ) {   /* credit check against the slowest consumer */
          out_cr = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE ) + out_depth;
          if( (long)(out_seq - out_cr) >= 0 ) {
            diag->backp_cnt++;
            do {
              __atomic_store_n( &H->beat, ++beat, __ATOMIC_RELAXED );
              out_cr = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE ) + out_depth;
            } while( (long)(out_seq - out_cr) >= 0 );
          }
        }
        ulong f = m.fidx;
        t->frame_pub[f] = out_seq;
        fd_mcache_publish( out_mcache, out_depth, out_seq, tag, f * FRAME_CHUNKS, m.sz, m.ctl, m.tsorig, tspub );
        if( lat && lat_n < lat_max ) lat[lat_n++] = tspub - m.tsorig;
        out_seq++; diag->out_cnt++; diag->out_sz += m.sz;
      }
    }
    HSTAMP( 0 );
    /* producer credit: copy mode is done with a frag once it is copied,
       zero copy once it is published (or dropped) */
    if( in_fseq ) {
      ulong rel = ( !zc_dev || pubd == staged ) ? in_seq : t->ppend[pubd & mask].seq;
      if( rel != fseq_pub ) { __atomic_store_n( in_fseq, rel, __ATOMIC_RELEASE ); fseq_pub = rel; }
    }
    bool done_in = frag_cnt ? (in_seq - in_seq0 >= frag_cnt) : (__atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0);
    if( done_in && pubd == staged ) break;

    /* 2. stage */
    bool idle_in = false, full = false;
    while( !done_in && staged - handed < t->batch_max ) {
      if( frag_cnt && in_seq - in_seq0 >= frag_cnt ) break;
      if( staged - pubd >= W ) { full = true; break; }
      fd_frag_meta_t const * m = in_mcache + (in_seq & (in_depth-1UL));
      __builtin_prefetch( in_mcache + ((in_seq + 16UL) & (in_depth-1UL)) );
      ulong seq_found = __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE );
      long  d = (long)(seq_found - in_seq);
      if( d < 0 ) { idle_in = true; break; }                             /* not yet published */
      if( d > 0 ) { diag->ovrn_cnt += (ulong)d; in_seq = seq_found; continue; }   /* overrun: resync */
      ulong chunk = m->chunk, sz = m->sz, ctl = m->ctl, tsorig = m->tsorig;
      __atomic_thread_fence( __ATOMIC_ACQUIRE );
      if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != in_seq ) { diag->ovrn_cnt++; in_seq++; continue; }
      if( sz < 96UL || sz - 96UL > FD_ED25519_AMD_MSG_MAX ||
          (zc_dev && (chunk << FD_CHUNK_LG_SZ) + ((sz + 63UL) & ~63UL) > zc_lim) ) {
        diag->bad_frag_cnt++; in_seq++; in_cnt++; continue;
      }
      /* reserve the next output frame: not in flight, and no longer read
         by a consumer that honours flow control */
      ulong fr = t->frame_next, f = t->frame_next_idx;
      if( fr - t->frame_retired >= F ) { full = true; break; }
      if( out_fseq && t->frame_pub[f] != FRAME_FREE && (long)(t->frame_pub[f] - cons) >= 0 ) {
        cons = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE );
        if( (long)(t->frame_pub[f] - cons) >= 0 ) { diag->backp_cnt++; full = true; break; }
      }
      uchar const * p = (uchar const *)fd_chunk_to_laddr_const( in_chunk0b, chunk );
      if( !zc_dev ) {
        /* copy mode: the frame is the tile's copy; a frag lapped while it
           was copied is dropped (speculative read, then seq re-check) */
        uint8_t * dst = t->out_base + f * FD_VERIFY_AMD_FRAME_SZ;
        memcpy( dst, p, sz );
        __atomic_thread_fence( __ATOMIC_ACQUIRE );
        if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != in_seq ) { diag->ovrn_cnt++; in_seq++; continue; }
        p = dst;
      }
      in_seq++; in_cnt++;
      if( t->tc.depth ) {   /* HA dedup on the first 8 signature bytes (reads the frag: a cache miss in zero copy) */
        ulong ha_tag; memcpy( &ha_tag, p + 32, 8 );
        if( t->tc.insert( ha_tag ) ) { diag->ha_filt_cnt++; diag->ha_filt_sz += sz; continue; }
      }
      t->frame_pub[f] = FRAME_FREE;
      t->frame_next++;
      if( ++t->frame_next_idx == F ) t->frame_next_idx = 0UL;
      fd_amd_tile_ent_t * en = t->ring + (staged & mask);
      en->src_chunk = zc_dev ? (uint32_t)chunk : (uint32_t)(f * FRAME_CHUNKS);
      en->out_chunk = (uint32_t)(f * FRAME_CHUNKS);
      en->sz        = (uint32_t)sz;
      t->ppend[staged & mask] = pending_t{ in_seq - 1UL, fr, (ushort)sz, (ushort)ctl, (uint)tsorig, (uint)f };
      if( staged == handed ) hand_t0 = now_ns();
      staged++; progress = true;
    }
    __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
    if( in_fseq && !zc_dev && in_seq != fseq_pub ) { __atomic_store_n( in_fseq, in_seq, __ATOMIC_RELEASE ); fseq_pub = in_seq; }
    done_in = frag_cnt ? (in_seq - in_seq0 >= frag_cnt) : (__atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0);
    HSTAMP( 1 );

    /* 3. hand over: cut staged frags into chunks and publish their
          descriptors (x86 stores are ordered: entries and descriptors are
          visible before the head).  A chunk takes one wave whatever its
          size, so the cut follows the load:
            latency mode (fewer than light_frags in flight): everything
              staged, in chunks of up to 8 frags (8 lanes per signature),
              when the input is momentarily drained (greedy; with
              batch_wait_ns only while nothing is in flight) or the oldest
              waited batch_wait_ns;
            throughput mode: whole 64-frag chunks only (1 lane per
              signature), a remainder once its oldest frag waited
              chunk_wait_ns -- small hand-offs under load would otherwise
              become small chunks, each holding a wave for a full chunk's
              time.
          Either mode hands over everything at batch_max staged frags, when
          the window or the frames ran out, and at the end of the input. */
    if( staged != handed ) {
      int lat_mode;
      ulong const upto = fd_verify_amd_tile_cut( staged, handed, pubd, t->light_frags, t->batch_max, now_ns() - hand_t0,
                                                 t->wait_ns, t->chunk_wait_ns, idle_in, full, done_in, &lat_mode );
      if( upto != handed ) {
        ulong K = lat_mode ? 8UL : 64UL, ds = t->desc_seq;
        for( ulong c = handed; c < upto; c += K, ds++ ) {
          fd_amd_tile_desc_t * dd = t->desc + (ds & mask);
          dd->first = c;
          dd->count = (uint32_t)std::min( K, upto - c ) | (lat_mode ? FD_AMD_TILE_LAT : 0u);
        }
        t->desc_seq = ds;
        __atomic_store_n( &H->head, ds, __ATOMIC_RELEASE );
        diag->batch_cnt++; diag->batch_sig_cnt += upto - handed;
        handed = upto; progress = true;
        if( staged != handed ) hand_t0 = now_ns();
      }
    }

    HSTAMP( 2 );
    if( hdbg && !progress ) hpass++;
    /* 4. an idle tile checks now and then that the kernel is still there */
    if( progress ) idle = 0UL;
    else if( ++idle >= 4096UL ) {
      idle = 0UL;
      hipError_t q = hipEventQuery( t->pdone );
      if( q != hipErrorNotReady ) {
        fprintf( stderr, "fd_verify_amd_tile_run: the tile kernel exited early (%s, watchdog %u)\n",
                 hipGetErrorString( q ), __atomic_load_n( &H->kerr, __ATOMIC_ACQUIRE ) );
        rc = FD_ED25519_AMD_ERR_DEVICE;
        break;
      }
    }
  }

# undef HSTAMP
  if( hdbg ) {
    double const tot = (double)(__rdtsc() - ht0);
    fprintf( stderr, "tile debug (persistent, host): publish %.1f%% stage %.1f%% hand-off %.1f%%, %lu empty passes, %.1f ns/frag\n",
             100.0*(double)hpt[0]/tot, 100.0*(double)hpt[1]/tot, 100.0*(double)hpt[2]/tot, hpass,
             (double)(now_ns() - hns0) / (double)(in_cnt - hin0 + 1UL) );
  }
  /* stop: the waves exit once nothing is left to claim */
  __atomic_store_n( &H->stop, 1u, __ATOMIC_RELEASE );
  if( hipEventSynchronize( t->pdone ) != hipSuccess ) rc = FD_ED25519_AMD_ERR_DEVICE;
  ulong st[4] = { 0, 0, 0, 0 };
  if( hipMemcpy( st, t->dctl->stat, sizeof st, hipMemcpyDeviceToHost ) != hipSuccess ) rc = FD_ED25519_AMD_ERR_DEVICE;
  if( __atomic_load_n( &H->kerr, __ATOMIC_ACQUIRE ) ) rc = FD_ED25519_AMD_ERR_DEVICE;
  if( env_ulong( "FD_AMD_TILE_DEBUG", 0UL ) ) {   /* per-phase wave time (k_tile_persist, args.prof) */
    ulong pf[8];
    if( hipMemcpy( pf, t->dctl->prof, sizeof pf, hipMemcpyDeviceToHost ) == hipSuccess ) {
      double w = (double)(waves - 1U) * 1e5;   /* ticks are 10 ns: per-wave ms */
      fprintf( stderr, "tile debug: per-wave ms  gather %.2f front %.2f dsm %.2f results %.2f wait %.2f fence %.2f"
               "  (chunks %lu latency + %lu throughput)\n", pf[0]/w, pf[1]/w, pf[2]/w, pf[3]/w, pf[4]/w, pf[5]/w,
               st[0], st[1] );
    }
  }
  diag->gpu_chunk_lat_cnt += st[0]; diag->gpu_chunk_thr_cnt += st[1];
  diag->gpu_frag_lat_cnt  += st[2]; diag->gpu_frag_thr_cnt  += st[3];
  t->ring_seq = staged;
  t->pass_max_ns = pass_max;
  __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
  if( in_fseq ) __atomic_store_n( in_fseq, in_seq, __ATOMIC_RELEASE );
  t->out_seq_end = out_seq;
  return rc;
}

/* ------------------------------------------------------------------ */
/* Measurement aid (tools/tile_synth.py): k_tile_persist's chunk pipeline
   on frags already in device memory, without the host hand-off.  frames:
   nframes frames of FD_VERIFY_AMD_FRAME_SZ bytes (pub | sig | msg), fsz
   their sizes; ring entry j takes frame j % nframes.  out_ms: the launch's
   time; verdict: per entry the verdict, or 99 if its result word is
   missing. */
/* where (flags): 1 ring entries, 2 results, 4 frames in mapped coherent
   host memory, 8 frames in mapped non-coherent host memory, 16 one more
   wave polling mapped host control words meanwhile (the scout's load) */
extern "C" int
fd_amd_tile_synth( int device, uint32_t waves, uint32_t iters, int eight, uint32_t where,
                   uint8_t const * frames, uint32_t nframes, uint32_t const * fsz, double * out_ms, int8_t * verdict ) {
  if( !frames || !nframes || !fsz || !out_ms || !verdict || !waves || !iters || waves > 65536u || iters > 4096u ) return FD_ED25519_AMD_ERR_INVAL;
  for( uint32_t f=0; f<nframes; f++ ) if( fsz[f] < 96u || fsz[f] > 96u + FD_ED25519_AMD_MSG_MAX ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  ulong const k = eight ? 8UL : 64UL, n = (ulong)waves * iters * k;
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
  if( hipEventRecord( e0, st ) != hipSuccess || fd_amd_launch_tile_synth( &A, waves + (h_ctl ? 1u : 0u), iters, eight, st ) ||
      hipEventRecord( e1, st ) != hipSuccess || hipStreamSynchronize( st ) != hipSuccess ||
      hipEventElapsedTime( &ms, e0, e1 ) != hipSuccess ||
      hipMemcpy( res.data(), hm[1] ? hm[1] : (void *)d_res, 2UL * R * sizeof(uint64_t), hipMemcpyDefault ) != hipSuccess ) goto done;
  *out_ms = (double)ms;
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

/* ------------------------------------------------------------------ */
/* streaming benchmark and end-to-end check: producer -> tile -> consumer */

extern "C" int
fd_verify_amd_bench_stream( int device, ulong batch_max, ulong batch_wait_ns, double rate, int flags,
                            ulong dcache_frames, ulong pool_n, uchar const * pub, uchar const * sig,
                            uint const * msg_off, uint const * msg_sz, uchar const * blob, schar const * expect_err,
                            ulong const * expect_tag, ulong frag_cnt, double * out ) {
  if( !pool_n || !frag_cnt || !out || frag_cnt > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  for( ulong k=0; k<pool_n; k++ ) if( msg_sz[k] > FD_ED25519_AMD_MSG_MAX ) return FD_ED25519_AMD_ERR_INVAL;
  bool zero_copy = !!(flags & FD_VERIFY_AMD_BENCH_ZERO_COPY);
  bool writes    = !!(flags & FD_VERIFY_AMD_BENCH_WRITE);
  bool lap       = writes && (flags & FD_VERIFY_AMD_BENCH_LAP);
  bool check     = expect_err && expect_tag;
  ulong byte_mask = (flags & FD_VERIFY_AMD_BENCH_SAMPLE_BYTES) ? 15UL : 0UL;   /* compare bytes of every 16th frag */
  ulong depth = 1UL; while( depth < 8UL*batch_max + 1024UL ) depth <<= 1;   /* > batches in flight + staging */
  ulong out_depth = 1UL; while( out_depth < 2UL*batch_max + 1024UL ) out_depth <<= 1;
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
  auto put_frame = [&]( uchar * p, ulong k ) {
    memcpy( p, pub + 32UL*k, 32 ); memcpy( p + 32, sig + 64UL*k, 64 ); memcpy( p + 96, blob + msg_off[k], msg_sz[k] );
  };
  if( !writes ) for( ulong k=0; k<pool_n; k++ ) put_frame( dcache + k * frame, k );

  fd_verify_amd_tile_t * tile = fd_verify_amd_tile_new( device, batch_max, batch_wait_ns, 0UL, 0UL );
  if( !tile ) { free( dcache ); return FD_ED25519_AMD_ERR_DEVICE; }
  if( zero_copy && fd_verify_amd_tile_register_dcache( tile, dcache, region ) ) {
    fd_verify_amd_tile_delete( tile ); free( dcache ); return FD_ED25519_AMD_ERR_DEVICE;
  }
  uchar const * out_chunk0 = (uchar const *)fd_verify_amd_tile_out_chunk0( tile );

  /* the three spinning threads (producer, tile, consumer) each get a CPU of
     their own from the process's allowed set, so the scheduler does not
     stack them (the saturated rate otherwise varies run to run): the
     highest-numbered allowed CPUs, away from CPU 0, which takes most of the
     machine's interrupts (tile passes of 1-5 ms and p99 spikes were seen
     with the tile thread on CPU 0) */
  cpu_set_t allowed, saved; CPU_ZERO( &allowed ); CPU_ZERO( &saved );
  int cpus[3] = { -1, -1, -1 }, ncpu = 0;
  bool pin = !sched_getaffinity( 0, sizeof allowed, &allowed ) && CPU_COUNT( &allowed ) >= 4;
  if( pin ) {
    saved = allowed;
    for( int c=CPU_SETSIZE-1; c>0 && ncpu<3; c-- ) if( CPU_ISSET( c, &allowed ) ) cpus[ncpu++] = c;
    pin = ncpu == 3;
  }
  auto pin_to = [&]( int k ) {
    if( !pin ) return;
    cpu_set_t one; CPU_ZERO( &one ); CPU_SET( cpus[k], &one );
    (void)pthread_setaffinity_np( pthread_self(), sizeof one, &one );
  };

  ulong in_fseq = 0UL;                                   /* the tile's credit to the producer */
  std::atomic<ulong> out_fseq( 0UL );                    /* consumer progress (the tile's output credit) */
  std::vector<uint> lat( frag_cnt );
  fd_verify_amd_diag_t diag; memset( &diag, 0, sizeof diag );
  int tile_rc = 0;
  ulong mism = 0, checked = 0, late_max = 0, gap_max = 0;
  ulong t0 = now_ns();

  std::thread prod( [&]() {
    pin_to( 1 );
    ulong p0 = now_ns(), cr = 0;   /* cr: first seq not covered by the cached credit */
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
      if( !lap ) while( seq >= cr ) cr = __atomic_load_n( &in_fseq, __ATOMIC_ACQUIRE ) + lim;
      ulong sz = 96UL + msg_sz[k];
      ulong fr = writes ? fw : k;
      if( writes ) put_frame( dcache + fr * frame, k );
      /* tsorig = the scheduled send time when paced, so producer stalls
         count as latency; the input seq when lapping (the check needs it) */
      if( !due && !(seq & 31UL) ) tnow = fd_verify_amd_tickcount();
      uint tso = lap ? (uint)seq : due ? (uint)due : tnow;
      fd_mcache_publish( in_mc.data(), depth, seq, 0UL, fr * frame_c, sz, 3UL, tso, 0UL );
    }
  } );
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
          uchar const * q = out_chunk0 + (chunk << FD_CHUNK_LG_SZ);
          bool ok = s_in < frag_cnt && !expect_err[k] && tag == expect_tag[k] && sz == 96UL + msg_sz[k];
          if( ok && !(checked & byte_mask) )
            ok = !memcmp( q, pub + 32UL*k, 32 ) && !memcmp( q + 32, sig + 64UL*k, 64 ) &&
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
  ulong const pass_max = tile->pass_max_ns;
  fd_verify_amd_tile_delete( tile );
  free( dcache );
  if( rc ) return rc;
  ulong n = std::min( (ulong)diag.out_cnt, frag_cnt );
  std::sort( lat.begin(), lat.begin() + (long)n );
  auto pct = [&]( double q ) -> double { return n && !lap ? (double)lat[ std::min( n-1UL, (ulong)(q * (double)n) ) ] : 0.0; };
  out[0] = (double)diag.in_cnt / ((double)(t1 - t0) * 1e-9);
  out[1] = pct( 0.50 ); out[2] = pct( 0.99 ); out[3] = pct( 0.999 );
  out[4] = diag.batch_cnt ? (double)diag.batch_sig_cnt / (double)diag.batch_cnt : 0.0;
  out[5] = (double)diag.out_cnt; out[6] = (double)diag.sv_filt_cnt; out[7] = (double)diag.ovrn_cnt;
  out[8] = (double)mism; out[9] = (double)checked;
  out[10] = (double)diag.gpu_chunk_lat_cnt; out[11] = (double)diag.gpu_chunk_thr_cnt;
  out[12] = (double)diag.gpu_frag_lat_cnt;  out[13] = (double)diag.gpu_frag_thr_cnt;
  out[14] = (double)late_max; out[15] = (double)pass_max; out[16] = (double)gap_max;
  return FD_ED25519_AMD_OK;
}
