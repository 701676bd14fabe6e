/* firedancer_amd/csrc/fd_ed25519_engine.cpp
 *
 * Host side of the C-ABI boundary (include/fd_ed25519_amd.h): the batch
 * engine (device buffers, pinned double-buffered staging, per-engine HIP
 * streams), the device-resident entry point, and the reference's drop-in
 * fd_ed25519_verify / fd_ed25519_strerror.
 *
 * Reference interfaces replaced: src/ballet/ed25519/fd_ed25519.h:96-109
 * (verify, strerror); the tile-side call site is
 * src/app/frank/load/fd_frank_verify_synth_load.c:380 (one verify per
 * fragment); the batch API is new (SURVEY.md s8 b).
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <thread>

#include "../../include/fd_ed25519_amd.h"
#include "../../include/fd_txn_amd.h"
#include "fd_ed25519_kernels.h"

#define HIPCHK( x ) do { hipError_t _e = (x); if( _e != hipSuccess ) {                          \
    fprintf( stderr, "fd_ed25519_amd: %s failed: %s (%s:%d)\n", #x, hipGetErrorString( _e ),     \
             __FILE__, __LINE__ );                                                              \
    return FD_ED25519_AMD_ERR_DEVICE; } } while(0)

#include "fd_ed25519_engine.h"

/* Results go device -> host through a small kernel that writes the mapped,
   coherent pinned buffer, not through a DMA copy: the copy engine serves
   the streams' commands in order, so a D2H queued behind one batch's
   kernels would hold up the next batch's H2D on another stream. */
static hipError_t
slot_out( slot_t * s, void * h_dst, void const * d_src, ulong n ) {
  void * d_dst = h_dst == (void *)s->h_err  ? s->m_err  :
                 h_dst == (void *)s->h_terr ? s->m_terr :
                 h_dst == (void *)s->h_tag  ? s->m_tag  : NULL;
  if( !d_dst ) return hipErrorInvalidValue;
  return fd_amd_launch_copy_out( d_dst, d_src, n, s->stream ) ? hipErrorLaunchFailure : hipSuccess;
}

int
fd_amd_slot_out( slot_t * s, void * h_dst, void const * d_src, ulong n ) {
  return slot_out( s, h_dst, d_src, n ) == hipSuccess ? 0 : -1;
}

static void
slot_free( slot_t * s ) {
  if( s->d_pub  ) (void)hipFree( s->d_pub );
  if( s->d_sig  ) (void)hipFree( s->d_sig );
  if( s->d_blob ) (void)hipFree( s->d_blob );
  if( s->d_off  ) (void)hipFree( s->d_off );
  if( s->d_sz   ) (void)hipFree( s->d_sz );
  if( s->d_err  ) (void)hipFree( s->d_err );
  if( s->d_ws   ) (void)hipFree( s->d_ws );
  if( s->h_pub  ) (void)hipHostFree( s->h_pub );
  if( s->h_sig  ) (void)hipHostFree( s->h_sig );
  if( s->h_blob ) (void)hipHostFree( s->h_blob );
  if( s->h_off  ) (void)hipHostFree( s->h_off );
  if( s->h_sz   ) (void)hipHostFree( s->h_sz );
  if( s->h_err  ) (void)hipHostFree( s->h_err );
  if( s->d_pack ) (void)hipFree( s->d_pack );
  if( s->h_pack ) (void)hipHostFree( s->h_pack );
  if( s->d_toff ) (void)hipFree( s->d_toff );
  if( s->d_tsz  ) (void)hipFree( s->d_tsz );
  if( s->d_fp   ) (void)hipFree( s->d_fp );
  if( s->d_tbase) (void)hipFree( s->d_tbase );
  if( s->d_terr ) (void)hipFree( s->d_terr );
  if( s->d_skip ) (void)hipFree( s->d_skip );
  if( s->h_toff ) (void)hipHostFree( s->h_toff );
  if( s->h_tsz  ) (void)hipHostFree( s->h_tsz );
  if( s->h_tbase) (void)hipHostFree( s->h_tbase );
  if( s->h_terr ) (void)hipHostFree( s->h_terr );
  if( s->h_tag  ) (void)hipHostFree( s->h_tag );
  if( s->stream ) (void)hipStreamDestroy( s->stream );
  if( s->done   ) (void)hipEventDestroy( s->done );
  memset( s, 0, sizeof(*s) );
}

static int
slot_alloc( slot_t * s, ulong cap, ulong blob_cap ) {
  memset( s, 0, sizeof(*s) );
  ws_layout_t L = fd_amd_ws_layout( cap );
  HIPCHK( hipMalloc( (void **)&s->d_pub,  32UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_sig,  64UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_blob, blob_cap + 64UL ) );
  HIPCHK( hipMalloc( (void **)&s->d_off,  4UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_sz,   4UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_err,  cap ) );
  HIPCHK( hipMalloc( &s->d_ws, L.total ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_pub,  32UL*cap, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_sig,  64UL*cap, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_blob, blob_cap + 64UL, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_off,  4UL*cap, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_sz,   4UL*cap, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_err,  cap, hipHostMallocMapped | hipHostMallocCoherent ) );
  HIPCHK( hipHostGetDevicePointer( &s->m_err, s->h_err, 0 ) );
  HIPCHK( hipMalloc( (void **)&s->d_pack, 104UL*cap + blob_cap + 64UL ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_pack, 104UL*cap + blob_cap + 64UL, hipHostMallocMapped | hipHostMallocCoherent ) );
  HIPCHK( hipHostGetDevicePointer( (void **)&s->m_pack, s->h_pack, 0 ) );
  HIPCHK( hipStreamCreateWithFlags( &s->stream, hipStreamNonBlocking ) );
  HIPCHK( hipEventCreateWithFlags( &s->done, hipEventDisableTiming ) );
  /* first use of a stream (its hardware queue) and of a staging pair costs
     ~8 ms inside the first hipMemcpyAsync: pay it here, not in a batch */
  memset( s->h_pack, 0, 104UL*cap + blob_cap + 64UL );
  HIPCHK( hipMemcpyAsync( s->d_pack, s->h_pack, 104UL*cap + blob_cap + 64UL, hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipStreamSynchronize( s->stream ) );
  return FD_ED25519_AMD_OK;
}

extern "C" fd_ed25519_amd_t *
fd_ed25519_amd_new( int device, ulong batch_max, ulong blob_max ) {
  int nslot = 2;
  char const * ev = getenv( "FD_ED25519_AMD_NSLOT" );
  if( ev && atoi( ev ) >= 2 && atoi( ev ) <= FD_AMD_SLOT_MAX ) nslot = atoi( ev );
  return fd_amd_engine_new( device, batch_max, blob_max, nslot );
}

fd_ed25519_amd_t *
fd_amd_engine_new( int device, ulong batch_max, ulong blob_max, int nslot ) {
  if( nslot < 2 || nslot > FD_AMD_SLOT_MAX ) return NULL;
  if( !batch_max ) batch_max = 1;
  if( batch_max > (1UL<<26) ) return NULL;
  if( blob_max < FD_ED25519_AMD_MSG_MAX ) blob_max = FD_ED25519_AMD_MSG_MAX;
  if( blob_max > (1UL<<32) - 4096UL ) return NULL;
  int cnt = 0;
  if( hipGetDeviceCount( &cnt ) != hipSuccess || device < 0 || device >= cnt ) {
    fprintf( stderr, "fd_ed25519_amd: no HIP device %d (count %d)\n", device, cnt );
    return NULL;
  }
  if( hipSetDevice( device ) != hipSuccess ) return NULL;
  fd_ed25519_amd_t * e = (fd_ed25519_amd_t *)calloc( 1, sizeof(fd_ed25519_amd_t) );
  if( !e ) return NULL;
  e->device = device; e->cap = batch_max; e->blob_cap = blob_max; e->nslot = nslot;
  /* the pinned staging on the GPU's NUMA node (the thread's own policy is
     restored afterwards; fd_numa.cpp) */
  int pmode = 0; unsigned long pmask[16];
  int pnode = fd_amd_numa_prefer_begin( device, &pmode, pmask );
  int bad = 0;
  for( int k=0; k<nslot && !bad; k++ ) bad = slot_alloc( &e->slot[k], batch_max, blob_max );
  if( pnode >= 0 ) fd_amd_numa_prefer_end( pmode, pmask );
  if( bad ) { fd_ed25519_amd_delete( e ); return NULL; }
  return e;
}

extern "C" void
fd_ed25519_amd_delete( fd_ed25519_amd_t * e ) {
  if( !e ) return;
  (void)hipSetDevice( e->device );
  for( int k=0; k<FD_AMD_SLOT_MAX; k++ ) { if( e->slot[k].stream ) (void)hipStreamSynchronize( e->slot[k].stream ); slot_free( &e->slot[k] ); }
  free( e );
}

int
fd_amd_slot_alloc_aux( slot_t * s, ulong cap ) {
  if( s->d_toff ) return FD_ED25519_AMD_OK;
  HIPCHK( hipMalloc( (void **)&s->d_toff,  4UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_tsz,   4UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_fp,    4UL*cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_tbase, 4UL*(cap+1UL) ) );
  HIPCHK( hipMalloc( (void **)&s->d_terr,  cap ) );
  HIPCHK( hipMalloc( (void **)&s->d_skip,  cap ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_toff,  4UL*cap, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_tsz,   4UL*cap, hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_tbase, 4UL*(cap+1UL), hipHostMallocDefault ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_terr,  cap, hipHostMallocMapped | hipHostMallocCoherent ) );
  HIPCHK( hipHostGetDevicePointer( &s->m_terr, s->h_terr, 0 ) );
  HIPCHK( hipHostMalloc( (void **)&s->h_tag,   8UL*cap, hipHostMallocMapped | hipHostMallocCoherent ) );
  HIPCHK( hipHostGetDevicePointer( &s->m_tag, s->h_tag, 0 ) );
  return FD_ED25519_AMD_OK;
}

/* Wait for a slot's chunk and deliver its verdicts. */
int
fd_amd_slot_drain( slot_t * s ) {
  if( !s->busy ) return FD_ED25519_AMD_OK;
  HIPCHK( hipEventSynchronize( s->done ) );
  /* k_dsmp's hang guard marks every verdict of its launch (k_fin) */
  bool fault = ( s->chk_err  && s->h_err[0] == (int8_t)FD_AMD_VERDICT_DEVICE ) ||
               ( s->chk_terr && memchr( s->h_terr, (uint8_t)FD_AMD_VERDICT_DEVICE, s->chk_terr ) );
  if( fault ) fprintf( stderr, "fd_ed25519_amd: the pooled double-scalar multiply hit its step guard\n" );
  else {
    if( s->out   ) memcpy( s->out,   s->h_err,  s->n );
    if( s->t_out ) memcpy( s->t_out, s->h_terr, s->t_n );
    if( s->s_out ) memcpy( s->s_out, s->h_err,  s->s_n );
  }
  s->out = s->t_out = s->s_out = NULL;
  s->busy = 0;
  return fault ? FD_ED25519_AMD_ERR_DEVICE : FD_ED25519_AMD_OK;
}

/* Error exit of a batch call: wait for every chunk still in flight and
   forget where its verdicts were to go, so no later call writes into the
   caller's (by then possibly freed) output arrays. */
static int
engine_quiesce( fd_ed25519_amd_t * e, int rc ) {
  for( int k=0; k<FD_AMD_SLOT_MAX; k++ ) {
    slot_t * s = &e->slot[k];
    if( s->busy ) (void)hipEventSynchronize( s->done );
    s->out = s->t_out = s->s_out = NULL;
    s->busy = 0;
  }
  return rc;
}

int
fd_amd_slot_launch_packed( slot_t * s, ulong n, ulong blob_sz, schar * out ) {
  /* latency path: k_front reads the staging in place over PCIe (one pass,
     ~300 B per signature), which saves the H2D and its launch gap; larger
     batches copy first (their kernels re-read the inputs) */
  uint8_t * d = s->m_pack;
  if( !fd_amd_uses_latency_path( (uint32_t)n, 0 ) ) {
    d = s->d_pack;
    HIPCHK( hipMemcpyAsync( d, s->h_pack, 104UL*n + blob_sz, hipMemcpyHostToDevice, s->stream ) );
  }
  bool const lat = fd_amd_uses_latency_path( (uint32_t)n, 0 ) != 0;
  if( fd_amd_launch_verify( (uint32_t)n, d, d + 32UL*n, (uint32_t *)(d + 96UL*n), (uint32_t *)(d + 100UL*n),
                            d + 104UL*n, s->d_err, s->d_ws, s->stream, 1, NULL, NULL, 0,
                            lat ? (int8_t *)s->m_err : NULL ) )   /* latency path: verdicts written in place */
    return FD_ED25519_AMD_ERR_DEVICE;
  if( !lat ) HIPCHK( slot_out( s, s->h_err, s->d_err, n ) );
  HIPCHK( hipEventRecord( s->done, s->stream ) );
  s->out = out; s->n = n; s->busy = 1; s->want_tag = 0;
  s->chk_err = n; s->chk_terr = 0;
  return FD_ED25519_AMD_OK;
}

int
fd_amd_slot_ready( slot_t * s ) {
  if( !s->busy ) return 1;
  hipError_t e = hipEventQuery( s->done );
  if( e == hipSuccess ) return 1;
  if( e == hipErrorNotReady ) return 0;
  fprintf( stderr, "fd_ed25519_amd: hipEventQuery failed: %s\n", hipGetErrorString( e ) );
  return FD_ED25519_AMD_ERR_DEVICE;
}

/* Launch a staged transaction chunk: c transactions (payload bytes in
   h_blob, rebased offsets in h_toff/h_tsz, signature-slot bases in
   h_tbase[0..c]), nslot = h_tbase[c] signature slots. */
int
fd_amd_slot_launch_txn( slot_t * s, ulong c, ulong nslot, ulong blob_sz, schar * t_out, schar * s_out, int want_tag,
                        uint8_t const * d_payload ) {
  HIPCHK( hipMemcpyAsync( s->d_toff,  s->h_toff,  4UL*c,        hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_tsz,   s->h_tsz,   4UL*c,        hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_tbase, s->h_tbase, 4UL*(c+1UL),  hipMemcpyHostToDevice, s->stream ) );
  uint8_t const * pl = d_payload;
  if( !pl ) {
    pl = s->d_blob;
    if( blob_sz ) HIPCHK( hipMemcpyAsync( s->d_blob, s->h_blob, blob_sz, hipMemcpyHostToDevice, s->stream ) );
  }
  if( fd_amd_launch_txn_parse( (uint32_t)c, pl, s->d_toff, s->d_tsz, s->d_fp, NULL, 0, s->d_tbase,
                               s->d_pub, s->d_sig, s->d_off, s->d_sz, s->d_skip, s->stream ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  if( nslot && fd_amd_launch_verify( (uint32_t)nslot, s->d_pub, s->d_sig, s->d_off, s->d_sz, pl, s->d_err,
                                     s->d_ws, s->stream, 0, NULL, s->d_skip, s->dsm_mode ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  if( fd_amd_launch_txn_reduce( (uint32_t)c, s->d_fp, s->d_tbase, s->d_err, s->d_terr, s->stream ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  HIPCHK( slot_out( s, s->h_terr, s->d_terr, c ) );
  if( s_out && nslot ) HIPCHK( slot_out( s, s->h_err, s->d_err, nslot ) );
  if( want_tag && nslot ) {
    ws_layout_t L = fd_amd_ws_layout( nslot );
    HIPCHK( slot_out( s, s->h_tag, (uint8_t *)s->d_ws + L.tag, 8UL*nslot ) );
  }
  HIPCHK( hipEventRecord( s->done, s->stream ) );
  s->t_out = t_out; s->t_n = c;
  s->s_out = nslot ? s_out : NULL; s->s_n = nslot;
  s->chk_err = (s_out && nslot) ? nslot : 0; s->chk_terr = c;
  s->busy = 1;
  return FD_ED25519_AMD_OK;
}

/* Generic chunked, double-buffered driver.  get(i, &msg, &sz, &sig, &pub)
   returns signature i's inputs. */
template<typename GET>
static int
run_chunked( fd_ed25519_amd_t * e, ulong n, schar * err, GET get ) {
  if( hipSetDevice( e->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  for( ulong j=0; j<n; j++ ) {          /* every message must fit one chunk: checked before anything launches */
    uint8_t const * msg; ulong sz; uint8_t const * sig; uint8_t const * pub;
    get( j, &msg, &sz, &sig, &pub );
    if( sz > e->blob_cap || (sz && !msg) ) return FD_ED25519_AMD_ERR_INVAL;
  }
  ulong i = 0; int k = 0; int rc = FD_ED25519_AMD_OK;
  while( i < n ) {
    slot_t * s = &e->slot[k];
    if( (rc = fd_amd_slot_drain( s )) ) return engine_quiesce( e, rc );
    /* size the chunk first, then stage it packed: [pub|sig|off|sz|blob] */
    ulong c = 0, bsz = 0;
    while( i + c < n && c < e->cap ) {
      uint8_t const * msg; ulong sz; uint8_t const * sig; uint8_t const * pub;
      get( i + c, &msg, &sz, &sig, &pub );
      if( bsz + sz > e->blob_cap ) break;
      bsz += sz; c++;
    }
    uint8_t * hp = s->h_pack;
    uint8_t * h_pub = hp, * h_sig = hp + 32UL*c, * h_blob = hp + 104UL*c;
    uint32_t * h_off = (uint32_t *)(hp + 96UL*c), * h_sz = (uint32_t *)(hp + 100UL*c);
    bsz = 0;
    for( ulong j=0; j<c; j++ ) {
      uint8_t const * msg; ulong sz; uint8_t const * sig; uint8_t const * pub;
      get( i + j, &msg, &sz, &sig, &pub );
      memcpy( h_pub + 32UL*j, pub, 32 );
      memcpy( h_sig + 64UL*j, sig, 64 );
      if( sz ) memcpy( h_blob + bsz, msg, sz );
      h_off[j] = (uint32_t)bsz; h_sz[j] = (uint32_t)sz;
      bsz += sz;
    }
    if( (rc = fd_amd_slot_launch_packed( s, c, bsz, err + i )) ) return engine_quiesce( e, rc );
    i += c; k ^= 1;
  }
  for( int j=0; j<2; j++ ) if( (rc = fd_amd_slot_drain( &e->slot[j] )) ) return engine_quiesce( e, rc );
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_verify_batch( fd_ed25519_amd_t * e, ulong n, void const * const * msg, ulong const * sz,
                             void const * const * sig, void const * const * pub, schar * err ) {
  if( !e || (n && (!msg || !sz || !sig || !pub || !err)) ) return FD_ED25519_AMD_ERR_INVAL;
  return run_chunked( e, n, err, [&]( ulong i, uint8_t const ** m, ulong * s, uint8_t const ** g, uint8_t const ** p ) {
    *m = (uint8_t const *)msg[i]; *s = sz[i]; *g = (uint8_t const *)sig[i]; *p = (uint8_t const *)pub[i];
  } );
}

/* memcpy split over up to 4 host threads for large copies (the staging
   copy is the host-side limit of the SoA path: ~300 B per signature). */
static void
copy_par( void * dst, void const * src, ulong sz ) {
  ulong const min_part = 4UL << 20;
  int nt = (int)( sz / min_part ); if( nt > 4 ) nt = 4;
  if( nt < 2 ) { if( sz ) memcpy( dst, src, sz ); return; }
  std::thread th[3];
  ulong part = ( sz / (ulong)nt + 63UL ) & ~63UL;
  for( int t=1; t<nt; t++ ) {
    ulong lo = part*(ulong)t, hi = lo + part < sz ? lo + part : sz;
    if( lo < hi ) th[t-1] = std::thread( [=]{ memcpy( (uint8_t *)dst + lo, (uint8_t const *)src + lo, hi - lo ); } );
  }
  memcpy( dst, src, part < sz ? part : sz );
  for( int t=1; t<nt; t++ ) if( th[t-1].joinable() ) th[t-1].join();
}

/* SoA staging with block copies: pub and sig are contiguous per chunk, and
   when the chunk's messages sit in a window of the blob not much larger
   than their total size, the window is copied as one block and the offsets
   rebased (no per-message copy).  Other layouts gather message by message. */
static int
run_soa( fd_ed25519_amd_t * e, ulong n, uchar const * pub, uchar const * sig, uint const * msg_off,
         uint const * msg_sz, uchar const * blob, schar * err ) {
  if( hipSetDevice( e->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  ulong i = 0; int k = 0; int rc = FD_ED25519_AMD_OK;
  while( i < n ) {
    slot_t * s = &e->slot[k];
    if( (rc = fd_amd_slot_drain( s )) ) return engine_quiesce( e, rc );
    ulong c = 0, bsz = 0, lo = ~0UL, hi = 0UL;
    while( i + c < n && c < e->cap ) {
      ulong sz = msg_sz[i+c];                /* <= blob_cap: checked by the caller */
      if( bsz + sz > e->blob_cap ) break;
      if( sz ) { ulong o = msg_off[i+c]; lo = o < lo ? o : lo; hi = o + sz > hi ? o + sz : hi; }
      bsz += sz; c++;
    }
    uint8_t * hp = s->h_pack;
    uint8_t * h_blob = hp + 104UL*c;
    uint32_t * h_off = (uint32_t *)(hp + 96UL*c), * h_sz = (uint32_t *)(hp + 100UL*c);
    copy_par( hp, pub + 32UL*i, 32UL*c );
    copy_par( hp + 32UL*c, sig + 64UL*i, 64UL*c );
    memcpy( h_sz, msg_sz + i, 4UL*c );
    ulong win = hi > lo ? hi - lo : 0UL;
    if( win <= e->blob_cap && win <= bsz + bsz/4UL + 4096UL ) {
      copy_par( h_blob, blob + (hi > lo ? lo : 0UL), win );
      for( ulong j=0; j<c; j++ ) h_off[j] = msg_sz[i+j] ? (uint32_t)(msg_off[i+j] - lo) : 0U;
      bsz = win;
    } else {
      bsz = 0;
      for( ulong j=0; j<c; j++ ) {
        ulong sz = msg_sz[i+j];
        if( sz ) memcpy( h_blob + bsz, blob + msg_off[i+j], sz );
        h_off[j] = (uint32_t)bsz; bsz += sz;
      }
    }
    if( (rc = fd_amd_slot_launch_packed( s, c, bsz, err + i )) ) return engine_quiesce( e, rc );
    i += c; k = (k + 1) % e->nslot;
  }
  for( int j=0; j<e->nslot; j++ ) if( (rc = fd_amd_slot_drain( &e->slot[j] )) ) return engine_quiesce( e, rc );
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_verify_soa( fd_ed25519_amd_t * e, ulong n, uchar const * pub, uchar const * sig,
                           uint const * msg_off, uint const * msg_sz, uchar const * blob, ulong blob_sz,
                           schar * err ) {
  if( !e || (n && (!pub || !sig || !msg_off || !msg_sz || !err)) ) return FD_ED25519_AMD_ERR_INVAL;
  /* every message in bounds and small enough for one chunk: checked before
     anything launches, so an error never leaves a chunk in flight */
  for( ulong i=0; i<n; i++ )
    if( msg_sz[i] && ((ulong)msg_off[i] + msg_sz[i] > blob_sz || !blob || msg_sz[i] > e->blob_cap) )
      return FD_ED25519_AMD_ERR_INVAL;
  return run_soa( e, n, pub, sig, msg_off, msg_sz, blob, err );
}

/* ------------------------------------------------------------------ */
/* zero-copy host batches (caller memory registered once)               */

/* Registrations made through fd_ed25519_amd_host_register, with their
   device addresses: the latency path validates and translates a plane with
   a table lookup instead of four HIP pointer queries per plane (~25 runtime
   calls per batch of five planes, most of the host-side overhead of a
   0.5 ms call).  Memory registered by other means takes the query path. */
namespace {
struct reg_t { uintptr_t lo, hi; uintptr_t dev; };
std::mutex          g_reg_mu;
std::vector<reg_t>  g_reg;
}

extern "C" int
fd_ed25519_amd_host_register( void * base, ulong sz ) {
  if( !base || !sz ) return FD_ED25519_AMD_ERR_INVAL;
  /* portable: usable by every device's engine; mapped: small batches are
     read in place by the GPU (no copy at all) */
  if( hipHostRegister( base, sz, hipHostRegisterPortable | hipHostRegisterMapped ) != hipSuccess )
    return FD_ED25519_AMD_ERR_DEVICE;
  void * dev = NULL;
  if( hipHostGetDevicePointer( &dev, base, 0 ) == hipSuccess ) {
    std::lock_guard<std::mutex> g( g_reg_mu );
    g_reg.push_back( reg_t{ (uintptr_t)base, (uintptr_t)base + sz, (uintptr_t)dev } );
  } else (void)hipGetLastError();
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_host_unregister( void * base ) {
  if( !base ) return FD_ED25519_AMD_ERR_INVAL;
  {
    std::lock_guard<std::mutex> g( g_reg_mu );
    for( size_t k=0; k<g_reg.size(); k++ )
      if( g_reg[k].lo == (uintptr_t)base ) { g_reg[k] = g_reg.back(); g_reg.pop_back(); break; }
  }
  return hipHostUnregister( base ) == hipSuccess ? FD_ED25519_AMD_OK : FD_ED25519_AMD_ERR_DEVICE;
}

/* [p, p+sz) lies in ONE registration: its first and its last byte are
   registered host memory and map to device addresses sz-1 apart (two
   adjacent registrations map to unrelated device ranges).  The latency
   path reads the planes in place, so a plane registered only in part must
   be refused here, not faulted on by the GPU.  *dev: p's device address. */
static bool
host_registered( void const * p, ulong sz, void ** dev ) {
  {
    std::lock_guard<std::mutex> g( g_reg_mu );
    uintptr_t const a = (uintptr_t)p, b = a + (sz ? sz : 1UL);
    for( reg_t const & r : g_reg )
      if( a >= r.lo && b <= r.hi && b > a ) { *dev = (void *)(r.dev + (a - r.lo)); return true; }
  }
  hipPointerAttribute_t a;
  if( hipPointerGetAttributes( &a, p ) != hipSuccess ) { (void)hipGetLastError(); return false; }
  if( a.type != hipMemoryTypeHost ) return false;
  void * dp = NULL, * dq = NULL;
  if( hipHostGetDevicePointer( &dp, (void *)p, 0 ) != hipSuccess ) { (void)hipGetLastError(); return false; }
  *dev = dp;
  if( sz <= 1UL ) return true;
  void const * q = (uchar const *)p + (sz - 1UL);
  if( hipPointerGetAttributes( &a, q ) != hipSuccess ) { (void)hipGetLastError(); return false; }
  if( a.type != hipMemoryTypeHost ) return false;
  if( hipHostGetDevicePointer( &dq, (void *)q, 0 ) != hipSuccess ) { (void)hipGetLastError(); return false; }
  return (ulong)((uchar const *)dq - (uchar const *)dp) == sz - 1UL;
}

/* One chunk straight from registered caller memory: the pub/sig/off/sz
   slices and the message window [lo, lo+win) by DMA into the slot's
   device planes, offsets rebased on the device. */
static int
slot_launch_dma( slot_t * s, ulong c, uchar const * pub, uchar const * sig, uint const * off, uint const * sz,
                 uchar const * win_src, ulong win, uint lo, schar * out ) {
  HIPCHK( hipMemcpyAsync( s->d_pub, pub, 32UL*c, hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_sig, sig, 64UL*c, hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_off, off, 4UL*c,  hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_sz,  sz,  4UL*c,  hipMemcpyHostToDevice, s->stream ) );
  if( win ) HIPCHK( hipMemcpyAsync( s->d_blob, win_src, win, hipMemcpyHostToDevice, s->stream ) );
  if( fd_amd_launch_rebase_off( (uint32_t)c, s->d_off, s->d_sz, lo, s->stream ) ) return FD_ED25519_AMD_ERR_DEVICE;
  if( fd_amd_launch_verify( (uint32_t)c, s->d_pub, s->d_sig, s->d_off, s->d_sz, s->d_blob, s->d_err, s->d_ws, s->stream,
                            1, NULL ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  HIPCHK( slot_out( s, s->h_err, s->d_err, c ) );
  HIPCHK( hipEventRecord( s->done, s->stream ) );
  s->out = out; s->n = c; s->busy = 1; s->want_tag = 0;
  s->chk_err = c; s->chk_terr = 0;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_verify_soa_registered( fd_ed25519_amd_t * e, ulong n, uchar const * pub, uchar const * sig,
                                      uint const * msg_off, uint const * msg_sz, uchar const * blob, ulong blob_sz,
                                      schar * err ) {
  if( !e || (n && (!pub || !sig || !msg_off || !msg_sz || !err)) ) return FD_ED25519_AMD_ERR_INVAL;
  for( ulong i=0; i<n; i++ )
    if( msg_sz[i] && ((ulong)msg_off[i] + msg_sz[i] > blob_sz || !blob || msg_sz[i] > e->blob_cap) )
      return FD_ED25519_AMD_ERR_INVAL;
  if( !n ) return FD_ED25519_AMD_OK;
  void * d[5] = { NULL, NULL, NULL, NULL, NULL };   /* the planes' device addresses */
  if( !host_registered( pub, 32UL*n, &d[0] ) || !host_registered( sig, 64UL*n, &d[1] ) ||
      !host_registered( msg_off, 4UL*n, &d[2] ) || !host_registered( msg_sz, 4UL*n, &d[3] ) ||
      (blob && blob_sz && !host_registered( blob, blob_sz, &d[4] )) )
    return FD_ED25519_AMD_ERR_INVAL;
  if( !(blob && blob_sz) ) d[4] = d[0];   /* no message bytes: any valid address */
  if( hipSetDevice( e->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  int rc = FD_ED25519_AMD_OK;
  if( n <= e->cap && fd_amd_uses_latency_path( (uint32_t)n, 0 ) ) {
    /* a latency-path batch is read once, by k_front: it reads the caller's
       registered planes in place over PCIe, with no copy on either side */
    slot_t * s = &e->slot[0];
    if( (rc = fd_amd_slot_drain( s )) ) return engine_quiesce( e, rc );
    /* the DSM kernel writes the verdicts into the mapped h_err itself */
    if( fd_amd_launch_verify( (uint32_t)n, (uint8_t const *)d[0], (uint8_t const *)d[1], (uint32_t const *)d[2],
                              (uint32_t const *)d[3], (uint8_t const *)d[4], s->d_err, s->d_ws, s->stream, 1, NULL,
                              NULL, 0, (int8_t *)s->m_err ) )
      return engine_quiesce( e, FD_ED25519_AMD_ERR_DEVICE );
    if( hipEventRecord( s->done, s->stream ) != hipSuccess ) return engine_quiesce( e, FD_ED25519_AMD_ERR_DEVICE );
    s->out = err; s->n = n; s->busy = 1; s->want_tag = 0;
    s->chk_err = n; s->chk_terr = 0;
    if( (rc = fd_amd_slot_drain( s )) ) return engine_quiesce( e, rc );
    return FD_ED25519_AMD_OK;
  }
  ulong i = 0; int k = 0;
  while( i < n ) {
    slot_t * s = &e->slot[k];
    if( (rc = fd_amd_slot_drain( s )) ) return engine_quiesce( e, rc );
    ulong c = 0, bsz = 0, lo = ~0UL, hi = 0UL;
    while( i + c < n && c < e->cap ) {
      ulong sz = msg_sz[i+c];
      if( bsz + sz > e->blob_cap ) break;
      if( sz ) {
        ulong o = msg_off[i+c];
        ulong nlo = o < lo ? o : lo, nhi = o + sz > hi ? o + sz : hi;
        if( nhi - nlo > e->blob_cap ) break;     /* the window must fit the device blob */
        lo = nlo; hi = nhi;
      }
      bsz += sz; c++;
    }
    ulong win = hi > lo ? hi - lo : 0UL;
    if( win <= bsz + bsz/4UL + 4096UL ) {
      rc = slot_launch_dma( s, c, pub + 32UL*i, sig + 64UL*i, msg_off + i, msg_sz + i, blob + (win ? lo : 0UL), win,
                            (uint)(win ? lo : 0UL), err + i );
    } else {
      /* scattered messages: gather them through the pinned staging */
      uint8_t * hp = s->h_pack;
      uint8_t * h_blob = hp + 104UL*c;
      uint32_t * h_off = (uint32_t *)(hp + 96UL*c), * h_sz = (uint32_t *)(hp + 100UL*c);
      memcpy( hp, pub + 32UL*i, 32UL*c );
      memcpy( hp + 32UL*c, sig + 64UL*i, 64UL*c );
      memcpy( h_sz, msg_sz + i, 4UL*c );
      ulong b = 0;
      for( ulong j=0; j<c; j++ ) {
        ulong sz = msg_sz[i+j];
        if( sz ) memcpy( h_blob + b, blob + msg_off[i+j], sz );
        h_off[j] = (uint32_t)b; b += sz;
      }
      rc = fd_amd_slot_launch_packed( s, c, b, err + i );
    }
    if( rc ) return engine_quiesce( e, rc );
    i += c; k = (k + 1) % e->nslot;
  }
  for( int j=0; j<e->nslot; j++ ) if( (rc = fd_amd_slot_drain( &e->slot[j] )) ) return engine_quiesce( e, rc );
  return FD_ED25519_AMD_OK;
}

/* Signature slots the engine reserves for a payload: its first byte when
   that is a plausible signature count (fd_txn_parse.c:79-82 accept it),
   else 0.  Exact for every payload that parses. */
ulong
fd_amd_txn_slots1( uchar const * p, ulong sz ) {
  if( !sz ) return 0UL;
  ulong k = p[0];
  return ( k >= 1UL && k <= FD_TXN_SIG_MAX && 64UL*k <= sz - 1UL ) ? k : 0UL;
}

extern "C" int
fd_ed25519_amd_verify_txns( fd_ed25519_amd_t * e, ulong txn_cnt, uchar const * payload, uint const * txn_off,
                            uint const * txn_sz, ulong payload_sz, schar * txn_err, uint * sig_base, schar * sig_err ) {
  if( !e || (txn_cnt && (!payload || !txn_off || !txn_sz || !txn_err)) ) return FD_ED25519_AMD_ERR_INVAL;
  if( sig_err && !sig_base ) return FD_ED25519_AMD_ERR_INVAL;
  /* every transaction in bounds and stageable in one chunk (its bytes in
     blob_max, its signatures in batch_max): checked before anything
     launches, so the chunk loop always makes progress */
  for( ulong t=0; t<txn_cnt; t++ ) {
    if( txn_sz[t] > FD_TXN_AMD_MTU || (ulong)txn_off[t] + txn_sz[t] > payload_sz || txn_sz[t] > e->blob_cap )
      return FD_ED25519_AMD_ERR_INVAL;
    if( fd_amd_txn_slots1( payload + txn_off[t], txn_sz[t] ) > e->cap ) return FD_ED25519_AMD_ERR_INVAL;
  }
  if( hipSetDevice( e->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  int rc;
  for( int k=0; k<2; k++ ) if( (rc = fd_amd_slot_alloc_aux( &e->slot[k], e->cap )) ) return rc;
  /* global signature numbering (the caller-visible sig_base) */
  uint acc = 0U;
  if( sig_base ) {
    for( ulong t=0; t<txn_cnt; t++ ) { sig_base[t] = acc; acc += (uint)fd_amd_txn_slots1( payload + txn_off[t], txn_sz[t] ); }
    sig_base[txn_cnt] = acc;
  }
  ulong t = 0, gsig = 0; int k = 0;
  while( t < txn_cnt ) {
    slot_t * s = &e->slot[k];
    if( (rc = fd_amd_slot_drain( s )) ) return engine_quiesce( e, rc );
    ulong c = 0, bsz = 0, ns = 0;
    while( t + c < txn_cnt && c < e->cap ) {
      uchar const * p = payload + txn_off[t+c];
      ulong sz = txn_sz[t+c], k2 = fd_amd_txn_slots1( p, sz );
      if( bsz + sz > e->blob_cap || ns + k2 > e->cap ) break;
      if( sz ) memcpy( s->h_blob + bsz, p, sz );
      s->h_toff[c] = (uint32_t)bsz; s->h_tsz[c] = (uint32_t)sz; s->h_tbase[c] = (uint32_t)ns;
      bsz += sz; ns += k2; c++;
    }
    s->h_tbase[c] = (uint32_t)ns;
    if( (rc = fd_amd_slot_launch_txn( s, c, ns, bsz, txn_err + t, sig_err ? sig_err + gsig : NULL, 0, NULL )) )
      return engine_quiesce( e, rc );
    t += c; gsig += ns; k ^= 1;
  }
  for( int j=0; j<2; j++ ) if( (rc = fd_amd_slot_drain( &e->slot[j] )) ) return engine_quiesce( e, rc );
  return FD_ED25519_AMD_OK;
}

/* Device-resident transaction batch: workspace = verify workspace for
   slot_cnt signatures + the signature layout planes + footprints. */
namespace {
struct txn_ws_t { size_t vws, pub, sig, off, sz, skip, err, fp, total; };
inline size_t al256( size_t x ) { return (x + 255UL) & ~(size_t)255UL; }
txn_ws_t txn_ws_layout( ulong txn_cnt, ulong slot_cnt ) {
  txn_ws_t L; size_t o = 0; ulong S = slot_cnt ? slot_cnt : 1UL;
  L.vws  = o; o = al256( o + fd_amd_ws_layout( S ).total );
  L.pub  = o; o = al256( o + 32UL*S );
  L.sig  = o; o = al256( o + 64UL*S );
  L.off  = o; o = al256( o + 4UL*S );
  L.sz   = o; o = al256( o + 4UL*S );
  L.skip = o; o = al256( o + S );
  L.err  = o; o = al256( o + S );
  L.fp   = o; o = al256( o + 4UL*(txn_cnt ? txn_cnt : 1UL) );
  L.total = o;
  return L;
}
}

extern "C" ulong
fd_ed25519_amd_txn_workspace_footprint( ulong txn_cnt, ulong slot_cnt ) {
  return txn_ws_layout( txn_cnt, slot_cnt ).total;
}

extern "C" ulong
fd_ed25519_amd_txn_slots( ulong txn_cnt, uchar const * payload, uint const * txn_off, uint const * txn_sz,
                          uint * tbase ) {
  ulong acc = 0;
  for( ulong t=0; t<txn_cnt; t++ ) { tbase[t] = (uint)acc; acc += fd_amd_txn_slots1( payload + txn_off[t], txn_sz[t] ); }
  tbase[txn_cnt] = (uint)acc;
  return acc;
}

extern "C" int
fd_ed25519_amd_verify_txns_dev( ulong txn_cnt, ulong slot_cnt, uchar const * d_payload, uint const * d_txn_off,
                                uint const * d_txn_sz, uint const * d_tbase, schar * d_txn_err, schar * d_sig_err,
                                void * d_ws, void * stream ) {
  if( txn_cnt > 0xFFFFFFFFUL || slot_cnt > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  if( !txn_cnt ) return FD_ED25519_AMD_OK;
  if( !d_payload || !d_txn_off || !d_txn_sz || !d_tbase || !d_txn_err || !d_ws ) return FD_ED25519_AMD_ERR_INVAL;
  txn_ws_t L = txn_ws_layout( txn_cnt, slot_cnt );
  uint8_t * w = (uint8_t *)d_ws;
  hipStream_t st = (hipStream_t)stream;
  int8_t * err = d_sig_err ? (int8_t *)d_sig_err : (int8_t *)(w + L.err);
  if( fd_amd_launch_txn_parse( (uint32_t)txn_cnt, d_payload, d_txn_off, d_txn_sz, (uint32_t *)(w + L.fp), NULL, 0,
                               d_tbase, w + L.pub, w + L.sig, (uint32_t *)(w + L.off), (uint32_t *)(w + L.sz),
                               (int8_t *)(w + L.skip), st ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  if( slot_cnt && fd_amd_launch_verify( (uint32_t)slot_cnt, w + L.pub, w + L.sig, (uint32_t *)(w + L.off),
                                        (uint32_t *)(w + L.sz), d_payload, err, w + L.vws, st, 1, NULL,
                                        (int8_t *)(w + L.skip) ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  if( fd_amd_launch_txn_reduce( (uint32_t)txn_cnt, (uint32_t *)(w + L.fp), d_tbase, err, (int8_t *)d_txn_err, st ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_txn_amd_parse_dev( ulong txn_cnt, uchar const * d_payload, uint const * d_txn_off, uint const * d_txn_sz,
                      uint * d_footprint, uchar * d_out, ulong out_stride, void * stream ) {
  if( txn_cnt > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  if( !txn_cnt ) return FD_ED25519_AMD_OK;
  if( !d_payload || !d_txn_off || !d_txn_sz || !d_footprint ) return FD_ED25519_AMD_ERR_INVAL;
  if( d_out && (out_stride < FD_TXN_MAX_SZ || (out_stride & 1UL)) ) return FD_ED25519_AMD_ERR_INVAL;
  if( fd_amd_launch_txn_parse( (uint32_t)txn_cnt, d_payload, d_txn_off, d_txn_sz, d_footprint, d_out, out_stride,
                               NULL, NULL, NULL, NULL, NULL, NULL, (hipStream_t)stream ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_sign_dev( ulong n, uchar const * d_prv, uint const * d_msg_off, uint const * d_msg_sz,
                         uchar const * d_blob, uchar * d_pub, uchar * d_sig, void * stream ) {
  if( n > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  if( !n ) return FD_ED25519_AMD_OK;
  if( !d_prv || !d_msg_off || !d_msg_sz || !d_blob || !d_pub || !d_sig ) return FD_ED25519_AMD_ERR_INVAL;
  if( fd_amd_launch_sign( (uint32_t)n, d_prv, d_msg_off, d_msg_sz, d_blob, d_pub, d_sig, (hipStream_t)stream ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  return FD_ED25519_AMD_OK;
}

extern "C" ulong
fd_ed25519_amd_workspace_footprint( ulong n ) {
  return fd_amd_ws_layout( n ).total;
}

extern "C" int
fd_ed25519_amd_verify_dev( ulong n, uchar const * d_pub, uchar const * d_sig, uint const * d_msg_off,
                           uint const * d_msg_sz, uchar const * d_blob, schar * d_err, void * d_ws, void * stream ) {
  if( n > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  if( !n ) return FD_ED25519_AMD_OK;
  if( !d_pub || !d_sig || !d_msg_off || !d_msg_sz || !d_blob || !d_err || !d_ws ) return FD_ED25519_AMD_ERR_INVAL;
  if( fd_amd_launch_verify( (uint32_t)n, d_pub, d_sig, d_msg_off, d_msg_sz, d_blob, (int8_t *)d_err, d_ws,
                            (hipStream_t)stream, 1, NULL ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_verify_dev_ev( ulong n, uchar const * d_pub, uchar const * d_sig, uint const * d_msg_off,
                              uint const * d_msg_sz, uchar const * d_blob, schar * d_err, void * d_ws, void * stream,
                              void * const * ev ) {
  if( n > 0xFFFFFFFFUL ) return FD_ED25519_AMD_ERR_INVAL;
  if( !n ) return FD_ED25519_AMD_OK;
  if( !d_pub || !d_sig || !d_msg_off || !d_msg_sz || !d_blob || !d_err || !d_ws ) return FD_ED25519_AMD_ERR_INVAL;
  if( fd_amd_launch_verify( (uint32_t)n, d_pub, d_sig, d_msg_off, d_msg_sz, d_blob, (int8_t *)d_err, d_ws,
                            (hipStream_t)stream, 1, (hipEvent_t const *)ev ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_work_stats_dev( ulong n, void const * d_ws, uint * d_stats, void * stream ) {
  if( !n ) return FD_ED25519_AMD_OK;
  ws_layout_t L = fd_amd_ws_layout( n );
  uint8_t const * st = (uint8_t const *)d_ws + L.st;
  for( int k=0; k<3; k++ )
    HIPCHK( hipMemcpyAsync( d_stats + (ulong)k*n, st + 4UL*(ulong)k*L.N, 4UL*n, hipMemcpyDeviceToDevice, (hipStream_t)stream ) );
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_debug_digits_dev( ulong n, void const * d_ws, ushort * d_dig, int * d_top, void * stream ) {
  if( !n ) return FD_ED25519_AMD_OK;
  ws_layout_t L = fd_amd_ws_layout( n );
  uint8_t const * ws = (uint8_t const *)d_ws;
  if( fd_amd_launch_digits_dense( (uint32_t)n, d_ws, d_dig, (hipStream_t)stream ) ) return FD_ED25519_AMD_ERR_DEVICE;
  HIPCHK( hipMemcpyAsync( d_top, ws + L.top, 4UL*n,   hipMemcpyDeviceToDevice, (hipStream_t)stream ) );
  return FD_ED25519_AMD_OK;
}

/* ------------------------------------------------------------------ */
/* drop-in reference API                                                */

/* One engine per calling thread (the reference is reentrant with one
   fd_sha512_t per thread, fd_frank_verify.c:121-123), freed by a
   pthread-key destructor when the thread exits.  The reference boots N
   verify tiles as threads of one process (fd_frank_main.c:118-143), so the
   engine's device is a per-thread choice: the thread's own
   (fd_ed25519_amd_dropin_set_device), else FD_ED25519_AMD_DEVICE, else
   round robin over the GPUs local to the NUMA node of the CPU the thread
   first verifies on (fd_ed25519_amd_dropin_pick). */
namespace {
struct dropin_t { fd_ed25519_amd_t * eng; ulong blob; int want; int dev; };
pthread_key_t  dropin_key;
pthread_once_t dropin_once = PTHREAD_ONCE_INIT;
void dropin_free( void * p ) {
  dropin_t * d = (dropin_t *)p;
  if( d->eng ) fd_ed25519_amd_delete( d->eng );
  free( d );
}
void dropin_key_init( void ) { (void)pthread_key_create( &dropin_key, dropin_free ); }
dropin_t * dropin_self( void ) {
  (void)pthread_once( &dropin_once, dropin_key_init );
  dropin_t * d = (dropin_t *)pthread_getspecific( dropin_key );
  if( !d ) {
    d = (dropin_t *)calloc( 1, sizeof(dropin_t) );
    if( !d || pthread_setspecific( dropin_key, d ) ) { free( d ); return NULL; }
    d->want = FD_ED25519_AMD_DROPIN_AUTO; d->dev = -1;
  }
  return d;
}
/* threads given a default device so far, per NUMA node of their CPU (the
   last counter takes unknown and out-of-range nodes) */
std::atomic<ulong> dropin_ordinal[65];

/* The default device of a thread that set none. */
int dropin_default_device( void ) {
  char const * dv = getenv( "FD_ED25519_AMD_DEVICE" );
  if( dv && *dv ) return atoi( dv );
  int cnt = 0;
  if( hipGetDeviceCount( &cnt ) != hipSuccess || cnt <= 0 ) { (void)hipGetLastError(); return 0; }
  int node_of[FD_ED25519_AMD_DROPIN_DEV_MAX];
  cnt = std::min( cnt, (int)FD_ED25519_AMD_DROPIN_DEV_MAX );
  for( int k=0; k<cnt; k++ ) node_of[k] = fd_ed25519_amd_device_numa_node( k );
  unsigned cpu = 0, node = 0;
  int const cpu_node = syscall( SYS_getcpu, &cpu, &node, NULL ) ? -1 : (int)node;
  ulong const o = dropin_ordinal[ cpu_node >= 0 && cpu_node < 64 ? cpu_node : 64 ].fetch_add( 1UL );
  return fd_ed25519_amd_dropin_pick( node_of, cnt, cpu_node, o );
}
}

extern "C" int
fd_ed25519_amd_dropin_pick( int const * dev_node, int dev_cnt, int cpu_node, ulong ordinal ) {
  if( dev_cnt <= 0 || !dev_node ) return 0;
  int local = 0;
  if( cpu_node >= 0 ) for( int k=0; k<dev_cnt; k++ ) local += dev_node[k] == cpu_node;
  if( !local ) return (int)(ordinal % (ulong)dev_cnt);
  ulong j = ordinal % (ulong)local;
  for( int k=0; k<dev_cnt; k++ ) if( dev_node[k] == cpu_node && !j-- ) return k;
  return 0;   /* not reached */
}

extern "C" int
fd_ed25519_amd_dropin_set_device( int device ) {
  if( device < FD_ED25519_AMD_DROPIN_AUTO ) return FD_ED25519_AMD_ERR_INVAL;
  if( device >= 0 ) {
    int cnt = 0;
    if( hipGetDeviceCount( &cnt ) != hipSuccess ) { (void)hipGetLastError(); return FD_ED25519_AMD_ERR_DEVICE; }
    if( device >= cnt ) return FD_ED25519_AMD_ERR_INVAL;
  }
  dropin_t * d = dropin_self();
  if( !d ) return FD_ED25519_AMD_ERR_INVAL;
  d->want = device;
  return FD_ED25519_AMD_OK;
}

extern "C" int
fd_ed25519_amd_dropin_device( void ) {
  dropin_t * d = dropin_self();
  return d && d->eng ? d->dev : -1;
}

extern "C" int
fd_ed25519_verify( void const * msg, ulong sz, void const * sig, void const * public_key, fd_sha512_t * sha ) {
  (void)sha;   /* scratch of the reference; hashing happens on the GPU */
  dropin_t * d = dropin_self();
  if( !d ) {
    fprintf( stderr, "fd_ed25519_verify: out of memory\n" );
    abort();
  }
  if( sz > 0xFFFFFFFFUL - 4096UL ) {
    fprintf( stderr, "fd_ed25519_verify: message of %lu bytes exceeds the engine's 32-bit offsets\n", sz );
    abort();
  }
  /* the thread's device: its own choice, else the default picked once */
  int const dev = d->want >= 0 ? d->want : d->dev >= 0 ? d->dev : dropin_default_device();
  /* the engine grows when a message exceeds its staging (the reference
     accepts any size) and moves when the thread's device changed */
  if( !d->eng || sz > d->blob || dev != d->dev ) {
    ulong want = std::max( d->eng ? d->blob : 0UL, 64UL*FD_ED25519_AMD_MSG_MAX );
    while( want < sz ) want <<= 1;
    if( d->eng ) { fd_ed25519_amd_delete( d->eng ); d->eng = NULL; }
    d->eng = fd_ed25519_amd_new( dev, 64UL, want );
    if( !d->eng ) {
      fprintf( stderr, "fd_ed25519_verify: no usable MI355X/HIP device %d; this library has no CPU path\n", dev );
      abort();
    }
    d->blob = want; d->dev = dev;
  }
  static uint8_t const zero = 0;
  uint32_t off = 0, s32 = (uint32_t)sz;
  schar err = 0;
  int rc = fd_ed25519_amd_verify_soa( d->eng, 1UL, (uchar const *)public_key, (uchar const *)sig, &off, &s32,
                                      sz ? (uchar const *)msg : &zero, sz, &err );
  if( rc ) { fprintf( stderr, "fd_ed25519_verify: device error %d\n", rc ); abort(); }
  return (int)err;
}

extern "C" char const *
fd_ed25519_strerror( int err ) {
  switch( err ) {
  case FD_ED25519_SUCCESS:    return "success";
  case FD_ED25519_ERR_SIG:    return "bad signature";
  case FD_ED25519_ERR_PUBKEY: return "bad public key";
  case FD_ED25519_ERR_MSG:    return "bad message";
  default: break;
  }
  return "unknown";
}

extern "C" char const *
fd_ed25519_amd_version( void ) {
  return "fd_ed25519_amd 0.3 (gfx950; k_prep/k_decomp/k_dsm + k_front/k_dsm8/k_dsm4, txn front end, verify tile, multi-device, GPU signer)";
}

#ifdef FD_AMD_DIAG
#include <time.h>
#include <x86intrin.h>
#include <algorithm>
/* Diagnostics build only.  Latency-path A/B (profiles/r04_latency_ab.txt):
   one n-signature batch resident in HBM, verified `iters` times per way of
   launching and waiting, each call timed on the host clock:
     mode 0  k_front + k_dsm8 launched on a stream, hipEventSynchronize
     mode 1  the same launches, host spins on the verdicts k_dsm8 writes
             into mapped memory
     mode 2  the two launches captured once into a hipGraph, hipGraphLaunch
             + hipEventSynchronize
     mode 3  hipGraphLaunch + spin on the mapped verdicts
   out[4*m + 0..3] = p50 / p99 / min us of mode m and its GPU time (events
   around the launches, p50).  Every call's verdicts must equal the first
   call's (checked; ERR_DEVICE otherwise). */
extern "C" int
fd_amd_latency_ab( int device, uint32_t n, uint8_t const * pub, uint8_t const * sig, uint32_t const * off,
                   uint32_t const * sz, uint8_t const * blob, uint64_t blob_sz, uint32_t iters, double * out ) {
  if( !n || !iters || !out || !fd_amd_uses_latency_path( n, 0 ) ) return FD_ED25519_AMD_ERR_INVAL;
  if( hipSetDevice( device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  int rc = FD_ED25519_AMD_ERR_DEVICE;
  uint8_t * d_in = NULL, * d_ws = NULL; int8_t * d_err = NULL, * h_out = NULL, * d_out = NULL;
  hipStream_t st = NULL; hipEvent_t e0 = NULL, e1 = NULL, ed = NULL;
  hipGraph_t g = NULL; hipGraphExec_t ge = NULL;
  ulong const in_sz = 104UL*n + blob_sz;
  std::vector<int8_t> first( n );
  std::vector<double> t( iters ), gt( iters );
  ws_layout_t const L = fd_amd_ws_layout( n );
  uint8_t * p_pub, * p_sig, * p_blob; uint32_t * p_off, * p_sz;
  auto now = []() { struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts ); return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3; };
  if( hipMalloc( (void **)&d_in, in_sz ) != hipSuccess || hipMalloc( (void **)&d_ws, L.total ) != hipSuccess ||
      hipMalloc( (void **)&d_err, n ) != hipSuccess ||
      hipHostMalloc( (void **)&h_out, n, hipHostMallocMapped | hipHostMallocCoherent ) != hipSuccess ||
      hipHostGetDevicePointer( (void **)&d_out, h_out, 0 ) != hipSuccess ||
      hipStreamCreateWithFlags( &st, hipStreamNonBlocking ) != hipSuccess ||
      hipEventCreate( &e0 ) != hipSuccess || hipEventCreate( &e1 ) != hipSuccess || hipEventCreate( &ed ) != hipSuccess )
    goto done;
  p_pub = d_in; p_sig = d_in + 32UL*n; p_off = (uint32_t *)(d_in + 96UL*n); p_sz = (uint32_t *)(d_in + 100UL*n); p_blob = d_in + 104UL*n;
  if( hipMemcpy( p_pub, pub, 32UL*n, hipMemcpyHostToDevice ) != hipSuccess ||
      hipMemcpy( p_sig, sig, 64UL*n, hipMemcpyHostToDevice ) != hipSuccess ||
      hipMemcpy( p_off, off, 4UL*n, hipMemcpyHostToDevice ) != hipSuccess ||
      hipMemcpy( p_sz, sz, 4UL*n, hipMemcpyHostToDevice ) != hipSuccess ||
      ( blob_sz && hipMemcpy( p_blob, blob, blob_sz, hipMemcpyHostToDevice ) != hipSuccess ) ) goto done;
  /* the graph: the same two launches, captured */
  if( hipStreamBeginCapture( st, hipStreamCaptureModeThreadLocal ) != hipSuccess ) goto done;
  if( fd_amd_launch_verify( n, p_pub, p_sig, p_off, p_sz, p_blob, d_err, d_ws, st, 0, NULL, NULL, 0, d_out ) ) {
    (void)hipStreamEndCapture( st, &g ); goto done;
  }
  if( hipStreamEndCapture( st, &g ) != hipSuccess || hipGraphInstantiate( &ge, g, NULL, NULL, 0 ) != hipSuccess ) goto done;
  for( int m=0; m<4; m++ ) {
    bool const graph = m >= 2, spin = m & 1;
    for( uint32_t it=0; it<iters + 8u; it++ ) {   /* 8 untimed warm-up calls */
      memset( h_out, 0x7f, n );
      double const a = now();
      if( hipEventRecord( e0, st ) != hipSuccess ) goto done;
      if( graph ) { if( hipGraphLaunch( ge, st ) != hipSuccess ) goto done; }
      else if( fd_amd_launch_verify( n, p_pub, p_sig, p_off, p_sz, p_blob, d_err, d_ws, st, 0, NULL, NULL, 0, d_out ) ) goto done;
      if( hipEventRecord( e1, st ) != hipSuccess ) goto done;
      if( spin ) {
        /* every verdict lands in mapped memory; wait for the last unwritten one */
        for( uint32_t j=0; j<n; ) { if( ((int8_t volatile *)h_out)[j] != (int8_t)0x7f ) j++; else _mm_pause(); }
      } else if( hipEventSynchronize( e1 ) != hipSuccess ) goto done;
      double const b = now();
      if( hipEventSynchronize( e1 ) != hipSuccess ) goto done;
      float ms = 0.f;
      if( hipEventElapsedTime( &ms, e0, e1 ) != hipSuccess ) goto done;
      if( m == 0 && it == 0 ) memcpy( first.data(), h_out, n );
      else if( memcmp( first.data(), h_out, n ) ) { fprintf( stderr, "fd_amd_latency_ab: verdicts differ (mode %d call %u)\n", m, it ); goto done; }
      if( it >= 8u ) { t[it - 8u] = b - a; gt[it - 8u] = 1e3 * (double)ms; }
    }
    std::sort( t.begin(), t.end() ); std::sort( gt.begin(), gt.end() );
    out[4*m + 0] = t[iters / 2]; out[4*m + 1] = t[std::min( (ulong)iters - 1UL, (ulong)(0.99 * iters) )];
    out[4*m + 2] = t[0]; out[4*m + 3] = gt[iters / 2];
  }
  rc = FD_ED25519_AMD_OK;
done:
  if( st ) (void)hipStreamSynchronize( st );
  if( ge ) (void)hipGraphExecDestroy( ge );
  if( g ) (void)hipGraphDestroy( g );
  if( e0 ) (void)hipEventDestroy( e0 );
  if( e1 ) (void)hipEventDestroy( e1 );
  if( ed ) (void)hipEventDestroy( ed );
  if( st ) (void)hipStreamDestroy( st );
  if( h_out ) (void)hipHostFree( h_out );
  if( d_in ) (void)hipFree( d_in );
  if( d_ws ) (void)hipFree( d_ws );
  if( d_err ) (void)hipFree( d_err );
  return rc;
}
#endif /* FD_AMD_DIAG */
