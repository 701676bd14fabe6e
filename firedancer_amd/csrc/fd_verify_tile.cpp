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
 *   stage  -- copy pub/sig/msg into the pinned staging of the free engine slot
 *   launch -- adaptive batching: launch when the batch is full, or when the
 *             GPU is idle (no batch in flight), or when the oldest staged
 *             frag waited batch_wait_ns; two slots, so one batch stages
 *             while the other verifies
 *   publish-- when the oldest batch completes, publish its passing frags in
 *             arrival order (fd_mcache_publish protocol) with the GPU's
 *             SHA-512-derived dedup tag as meta.sig; failures count SV_FILT
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
  uint   chunk;
  ushort sz, ctl;
  uint   tsorig;
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
  std::vector<pending_t> meta[FD_AMD_SLOT_MAX];
};

extern "C" int
fd_verify_amd_tile_register_dcache( fd_verify_amd_tile_t * t, void * base, ulong sz ) {
  if( !t || !base || !sz ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( t->eng->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
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
  t->framing = framing;
  return FD_ED25519_AMD_OK;
}

#define TILE_NSLOT (4)   /* batches in flight (FD_AMD_TILE_NSLOT overrides; 6 or 8 measured: higher
                            p50 at every batch_max, higher saturated rate only at 16384): one wave's verify takes ~0.7 ms, so small
                            batches need several in flight to keep the GPU busy */

extern "C" uint
fd_verify_amd_tickcount( void ) {
  return (uint)now_ns();
}

extern "C" fd_verify_amd_tile_t *
fd_verify_amd_tile_new( int device, ulong batch_max, ulong batch_wait_ns, ulong tcache_depth ) {
  if( !batch_max ) return NULL;
  int nslot = TILE_NSLOT;
  if( char const * v = getenv( "FD_AMD_TILE_NSLOT" ) ) nslot = atoi( v );
  if( nslot < 2 || nslot > FD_AMD_SLOT_MAX ) return NULL;
  fd_ed25519_amd_t * eng = fd_amd_engine_new( device, batch_max, batch_max * FD_ED25519_AMD_MSG_MAX, nslot );
  if( !eng ) return NULL;
  for( int k=0; k<nslot; k++ )
    if( fd_amd_slot_alloc_aux( &eng->slot[k], batch_max ) ) { fd_ed25519_amd_delete( eng ); return NULL; }
  fd_verify_amd_tile_t * t = new fd_verify_amd_tile_t();
  t->eng = eng; t->batch_max = batch_max; t->wait_ns = batch_wait_ns; t->nslot = nslot;
  t->framing = FD_VERIFY_AMD_FRAMING_PUB_SIG_MSG;
  t->tc.init( tcache_depth );
  for( int k=0; k<nslot; k++ ) t->meta[k].resize( batch_max );
  return t;
}

extern "C" void
fd_verify_amd_tile_delete( fd_verify_amd_tile_t * t ) {
  if( !t ) return;
  if( t->reg_base ) { (void)hipSetDevice( t->eng->device ); (void)hipHostUnregister( t->reg_base ); }
  fd_ed25519_amd_delete( t->eng );
  delete t;
}

extern "C" int
fd_verify_amd_tile_run( fd_verify_amd_tile_t * t, fd_frag_meta_t const * in_mcache, ulong in_depth,
                        void const * in_chunk0, ulong in_seq0, fd_frag_meta_t * out_mcache, ulong out_depth,
                        ulong out_seq0, ulong const * out_fseq, ulong frag_cnt, int const * stop,
                        fd_verify_amd_diag_t * diag, uint * lat, ulong lat_max ) {
  if( !t || !in_mcache || !in_depth || (in_depth & (in_depth-1UL)) || !out_mcache || !out_depth ||
      (out_depth & (out_depth-1UL)) || !diag || (!frag_cnt && !stop) ) return FD_ED25519_AMD_ERR_INVAL;
  fd_ed25519_amd_t * e = t->eng;
  if( hipSetDevice( e->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;

  ulong in_seq = in_seq0, out_seq = out_seq0, lat_n = 0;
  int   K = t->nslot;
  int   stage = 0;                 /* slot being filled; slots are used round robin, so the */
  int   oldest = 0, nfly = 0;      /* in-flight ones are oldest, oldest+1, ... (mod K)      */
  ulong staged = 0, blob_at = 0, stage_t0 = 0, slots = 0;
  int   rc;
  /* Flow-control state shared with other threads is exchanged in strides,
     not per frag (the reference's tiles publish fseq and refresh credits
     in housekeeping, fd_fctl): diag->in_cnt is published every 256 frags
     and at the end of each staging pass; out_fseq is re-read only when the
     cached credit runs out. */
  ulong in_cnt = diag->in_cnt, out_cr = 0;

  bool txn = t->framing == FD_VERIFY_AMD_FRAMING_TXN;
  /* zero copy: the input data region is mapped into the GPU; frags are
     handed over as (chunk, size) and gathered on the device */
  uint8_t const * zc_dev = NULL;
  if( t->reg_base && (uint8_t const *)in_chunk0 >= t->reg_base &&
      (uint8_t const *)in_chunk0 < t->reg_base + t->reg_sz &&
      t->reg_sz - (ulong)((uint8_t const *)in_chunk0 - t->reg_base) <= (1UL << 32) )
    zc_dev = t->reg_dev + ((uint8_t const *)in_chunk0 - t->reg_base);
  auto publish = [&]( int k ) -> int {
    slot_t * s = &e->slot[k];
    if( (rc = fd_amd_slot_drain( s )) ) return rc;
    ulong cnt = txn ? s->t_n : s->n;
    for( ulong i=0; i<cnt; i++ ) {
      pending_t const & m = t->meta[k][i];
      int bad = txn ? s->h_terr[i] : s->h_err[i];
      if( bad ) { diag->sv_filt_cnt++; diag->sv_filt_sz += m.sz; continue; }
      /* dedup tag: the verify's SHA-512 tag of the (first) signature */
      ulong tag = txn ? s->h_tag[ s->h_tbase[i] ] : s->h_tag[i];
      if( out_fseq && (long)(out_seq - out_cr) >= 0 ) {   /* credit check against the slowest consumer */
        out_cr = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE ) + out_depth;
        if( (long)(out_seq - out_cr) >= 0 ) {
          diag->backp_cnt++;
          do out_cr = __atomic_load_n( out_fseq, __ATOMIC_ACQUIRE ) + out_depth; while( (long)(out_seq - out_cr) >= 0 );
        }
      }
      uint tspub = fd_verify_amd_tickcount();
      fd_mcache_publish( out_mcache, out_depth, out_seq, tag, m.chunk, m.sz, m.ctl, m.tsorig, tspub );
      if( lat && lat_n < lat_max ) lat[lat_n++] = tspub - m.tsorig;
      out_seq++; diag->out_cnt++; diag->out_sz += m.sz;
    }
    return FD_ED25519_AMD_OK;
  };

  for( ;; ) {
    /* 1. retire the oldest batch if it is done (publication stays in
          arrival order: batches retire in launch order) */
    while( nfly ) {
      int r = fd_amd_slot_ready( &e->slot[oldest] );
      if( r < 0 ) return r;
      if( !r ) break;
      if( (rc = publish( oldest )) ) return rc;
      oldest = (oldest + 1) % K; nfly--;
    }
    bool done_in = frag_cnt ? (in_cnt >= frag_cnt) : (__atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0);
    if( done_in && !staged && !nfly ) break;
    if( nfly == K ) continue;      /* every slot in flight: the staging slot is busy */

    /* 2. stage input frags into the free slot */
    slot_t * s = &e->slot[stage];
    bool idle_in = false, full = false;
    while( !done_in && staged < t->batch_max ) {
      if( frag_cnt && in_cnt >= frag_cnt ) break;
      if( !(in_cnt & 255UL) ) __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
      fd_frag_meta_t const * m = in_mcache + (in_seq & (in_depth-1UL));
      ulong seq_found = __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE );
      long  d = (long)(seq_found - in_seq);
      if( d < 0 ) { idle_in = true; break; }                             /* not yet published */
      if( d > 0 ) { diag->ovrn_cnt += (ulong)d; in_seq = seq_found; continue; }   /* overrun: resync */
      ulong chunk = m->chunk, sz = m->sz, ctl = m->ctl, tsorig = m->tsorig;
      __atomic_thread_fence( __ATOMIC_ACQUIRE );
      if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != in_seq ) { diag->ovrn_cnt++; in_seq++; continue; }
      uchar const * p = (uchar const *)fd_chunk_to_laddr_const( in_chunk0, chunk );
      in_seq++;
      in_cnt++;
      if( !txn ) {
        if( sz < 96UL || sz - 96UL > FD_ED25519_AMD_MSG_MAX ) { diag->bad_frag_cnt++; continue; }
        ulong ha_tag; memcpy( &ha_tag, p + 32, 8 );                      /* first 8 signature bytes */
        if( t->tc.insert( ha_tag ) ) { diag->ha_filt_cnt++; diag->ha_filt_sz += sz; continue; }
        if( zc_dev ) {                                                   /* zero copy: metadata only */
          s->h_off[staged] = (uint32_t)chunk; s->h_sz[staged] = (uint32_t)sz;
        } else {
          ulong msz = sz - 96UL;                                         /* blob_cap = batch_max*MSG_MAX: fits */
          memcpy( s->h_pub + 32UL*staged, p,      32 );
          memcpy( s->h_sig + 64UL*staged, p + 32, 64 );
          memcpy( s->h_blob + blob_at,    p + 96, msz );
          s->h_off[staged] = (uint32_t)blob_at; s->h_sz[staged] = (uint32_t)msz;
          blob_at += msz;
        }
      } else {
        /* wire transaction (fd_txn.h layout): dedup on its first signature */
        if( sz > FD_ED25519_AMD_MSG_MAX ) { diag->bad_frag_cnt++; continue; }
        ulong k2 = fd_amd_txn_slots1( p, sz );
        if( slots + k2 > t->batch_max ) {                              /* no room for its signatures: next batch */
          in_seq--; in_cnt--;
          full = true;
          break;
        }
        if( k2 ) {
          ulong ha_tag; memcpy( &ha_tag, p + 1, 8 );
          if( t->tc.insert( ha_tag ) ) { diag->ha_filt_cnt++; diag->ha_filt_sz += sz; continue; }
        }
        if( zc_dev ) {                                                   /* zero copy: parsed in place */
          s->h_toff[staged] = (uint32_t)(chunk << FD_CHUNK_LG_SZ);
        } else {
          memcpy( s->h_blob + blob_at, p, sz );
          s->h_toff[staged] = (uint32_t)blob_at;
          blob_at += sz;
        }
        s->h_tsz[staged] = (uint32_t)sz; s->h_tbase[staged] = (uint32_t)slots;
        slots += k2;
      }
      t->meta[stage][staged] = pending_t{ (uint)chunk, (ushort)sz, (ushort)ctl, (uint)tsorig };
      if( !staged ) stage_t0 = now_ns();
      staged++;
    }
    __atomic_store_n( &diag->in_cnt, in_cnt, __ATOMIC_RELEASE );
    done_in = frag_cnt ? (in_cnt >= frag_cnt) : (__atomic_load_n( stop, __ATOMIC_ACQUIRE ) != 0);

    /* 3. adaptive launch (a free slot exists here): full batch, input
          momentarily drained (greedy: under light load batches stay small
          and latency low; under load every slot is busy and batches grow
          toward batch_max), end of input, or the oldest staged frag waited
          batch_wait_ns.  A nonzero batch_wait_ns turns the greedy rule off
          while another batch is in flight. */
    bool greedy = idle_in && (!t->wait_ns || !nfly);
    if( staged && ( staged == t->batch_max || full || greedy || done_in ||
                    (t->wait_ns && now_ns() - stage_t0 >= t->wait_ns) ) ) {
      /* kernel path by batch size: tile batches are small next to the GPU,
         so the 4-lane latency kernels are used even with 4 in flight.
         Measured (profiles/r01_tile_policy_ab.txt): switching batches
         of >= 4096/8192 to the 1-lane kernel while others were in flight
         lowered the saturated rate at every batch_max and doubled latency;
         the in-flight work (4 x batch_max) is too small for the 1-lane
         kernel to fill the GPU. */
      s->dsm_mode = 0;
      if( txn ) {
        s->h_tbase[staged] = (uint32_t)slots;
        if( (rc = fd_amd_slot_launch_txn( s, staged, slots, blob_at, NULL, NULL, 1, zc_dev )) ) return rc;
        diag->batch_sig_cnt += slots;
      } else if( zc_dev ) {
        if( (rc = fd_amd_slot_launch_zc( s, staged, zc_dev )) ) return rc;
        diag->batch_sig_cnt += staged;
      } else {
        if( (rc = fd_amd_slot_launch( s, staged, blob_at, NULL, 1 )) ) return rc;
        diag->batch_sig_cnt += staged;
      }
      diag->batch_cnt++;
      nfly++;
      stage = (stage + 1) % K; staged = 0; blob_at = 0; slots = 0;
    }
  }
  return FD_ED25519_AMD_OK;
}

/* ------------------------------------------------------------------ */
/* streaming benchmark: producer -> tile -> consumer                    */

extern "C" int
fd_verify_amd_bench_stream( int device, ulong batch_max, ulong batch_wait_ns, double rate, int zero_copy,
                            ulong pool_n, uchar const * pub, uchar const * sig, uint const * msg_off,
                            uint const * msg_sz, uchar const * blob, ulong frag_cnt, double * out ) {
  if( !pool_n || !frag_cnt || !out ) return FD_ED25519_AMD_ERR_INVAL;
  ulong depth = 1UL; while( depth < 8UL*batch_max + 1024UL ) depth <<= 1;   /* > batches in flight + staging */
  ulong mtu = 96UL + FD_ED25519_AMD_MSG_MAX;
  ulong chunk_mtu = ((mtu + 2UL*FD_CHUNK_SZ - 1UL) >> (1 + FD_CHUNK_LG_SZ)) << 1;
  /* The data region holds every pool frame once (what a NIC would have
     DMA'd): the producer publishes metadata only, so the bench measures the
     tile, not a producer-side memcpy. */
  ulong data_chunks = chunk_mtu * pool_n;
  std::vector<fd_frag_meta_t> in_mc( depth ), out_mc( depth );
  for( ulong i=0; i<depth; i++ ) { in_mc[i].seq = i - depth; out_mc[i].seq = i - depth; }   /* "never published" */
  uchar * dcache = (uchar *)aligned_alloc( 4096, ((data_chunks * FD_CHUNK_SZ + 4095UL) & ~4095UL) );
  if( !dcache ) return FD_ED25519_AMD_ERR_INVAL;
  for( ulong k=0; k<pool_n; k++ ) {
    uchar * p = dcache + k * chunk_mtu * FD_CHUNK_SZ;
    memcpy( p, pub + 32UL*k, 32 ); memcpy( p + 32, sig + 64UL*k, 64 ); memcpy( p + 96, blob + msg_off[k], msg_sz[k] );
  }

  fd_verify_amd_tile_t * tile = fd_verify_amd_tile_new( device, batch_max, batch_wait_ns, 0UL );
  if( !tile ) { free( dcache ); return FD_ED25519_AMD_ERR_DEVICE; }
  if( zero_copy && fd_verify_amd_tile_register_dcache( tile, dcache, data_chunks * FD_CHUNK_SZ ) ) {
    fd_verify_amd_tile_delete( tile ); free( dcache ); return FD_ED25519_AMD_ERR_DEVICE;
  }

  /* the three spinning threads (producer, tile, consumer) each get a CPU of
     their own from the process's allowed set, so the scheduler does not
     stack them (the saturated rate otherwise varies run to run) */
  cpu_set_t allowed, saved; CPU_ZERO( &allowed ); CPU_ZERO( &saved );
  int cpus[3] = { -1, -1, -1 }, ncpu = 0;
  bool pin = !sched_getaffinity( 0, sizeof allowed, &allowed ) && CPU_COUNT( &allowed ) >= 4;
  if( pin ) {
    saved = allowed;
    for( int c=0; c<CPU_SETSIZE && ncpu<3; c++ ) if( CPU_ISSET( c, &allowed ) ) cpus[ncpu++] = c;
    pin = ncpu == 3;
  }
  auto pin_to = [&]( int k ) {
    if( !pin ) return;
    cpu_set_t one; CPU_ZERO( &one ); CPU_SET( cpus[k], &one );
    (void)pthread_setaffinity_np( pthread_self(), sizeof one, &one );
  };

  std::atomic<ulong> in_fseq( 0UL ), out_fseq( 0UL );   /* consumer progress (credits) */
  std::vector<uint> lat( frag_cnt );
  fd_verify_amd_diag_t diag; memset( &diag, 0, sizeof diag );
  int tile_rc = 0;
  ulong t0 = now_ns();

  std::thread prod( [&]() {
    pin_to( 1 );
    ulong p0 = now_ns(), cr = 0;   /* cr: first seq not covered by the cached credit */
    for( ulong seq=0; seq<frag_cnt; seq++ ) {
      ulong due = rate > 0.0 ? p0 + (ulong)((double)seq * 1e9 / rate) : 0UL;   /* paced: open loop */
      if( due ) while( now_ns() < due ) { /* spin */ }
      /* credit: do not lap the tile's consumption of the input mcache
         (refreshed only when the cached credit runs out) */
      while( seq >= cr ) cr = __atomic_load_n( &diag.in_cnt, __ATOMIC_ACQUIRE ) + depth - 16UL;
      ulong k = seq % pool_n, sz = 96UL + msg_sz[k];
      /* tsorig = the scheduled send time when paced, so producer stalls count as latency */
      uint tso = due ? (uint)due : fd_verify_amd_tickcount();
      fd_mcache_publish( in_mc.data(), depth, seq, 0UL, k * chunk_mtu, sz, 3UL, tso, 0UL );
    }
  } );
  std::thread cons( [&]() {
    pin_to( 2 );
    ulong seq = 0, fseq = 0;   /* fseq: last value published to out_fseq (every 64 frags, or when idle) */
    for( ;; ) {
      if( __atomic_load_n( &tile_rc, __ATOMIC_ACQUIRE ) == 1 ) {   /* tile finished: drain what is there */
        fd_frag_meta_t const * m = &out_mc[ seq & (depth-1UL) ];
        if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) != seq ) break;
      }
      fd_frag_meta_t const * m = &out_mc[ seq & (depth-1UL) ];
      if( __atomic_load_n( &m->seq, __ATOMIC_ACQUIRE ) == seq ) {
        seq++;
        if( seq - fseq >= 64UL ) { fseq = seq; out_fseq.store( seq, std::memory_order_release ); }
      } else if( fseq != seq ) { fseq = seq; out_fseq.store( seq, std::memory_order_release ); }
    }
  } );
  ulong const * ofs = (ulong const *)&out_fseq;
  pin_to( 0 );
  int rc = fd_verify_amd_tile_run( tile, in_mc.data(), depth, dcache, 0UL, out_mc.data(), depth, 0UL, ofs,
                                   frag_cnt, NULL, &diag, lat.data(), frag_cnt );
  ulong t1 = now_ns();
  __atomic_store_n( &tile_rc, 1, __ATOMIC_RELEASE );
  prod.join(); cons.join();
  if( pin ) (void)pthread_setaffinity_np( pthread_self(), sizeof saved, &saved );
  fd_verify_amd_tile_delete( tile );
  free( dcache );
  if( rc ) return rc;
  ulong n = std::min( (ulong)diag.out_cnt, frag_cnt );
  std::sort( lat.begin(), lat.begin() + (long)n );
  auto pct = [&]( double q ) -> double { return n ? (double)lat[ std::min( n-1UL, (ulong)(q * (double)n) ) ] : 0.0; };
  out[0] = (double)diag.in_cnt / ((double)(t1 - t0) * 1e-9);
  out[1] = pct( 0.50 ); out[2] = pct( 0.99 ); out[3] = pct( 0.999 );
  out[4] = diag.batch_cnt ? (double)diag.batch_sig_cnt / (double)diag.batch_cnt : 0.0;
  out[5] = (double)diag.out_cnt; out[6] = (double)diag.sv_filt_cnt;
  (void)in_fseq;
  return FD_ED25519_AMD_OK;
}
