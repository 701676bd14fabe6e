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
#include <mutex>

#include "../../include/fd_ed25519_amd.h"
#include "fd_ed25519_kernels.h"

#define HIPCHK( x ) do { hipError_t _e = (x); if( _e != hipSuccess ) {                          \
    fprintf( stderr, "fd_ed25519_amd: %s failed: %s (%s:%d)\n", #x, hipGetErrorString( _e ),     \
             __FILE__, __LINE__ );                                                              \
    return FD_ED25519_AMD_ERR_DEVICE; } } while(0)

namespace {

struct slot_t {
  /* device */
  uint8_t  * d_pub;  uint8_t * d_sig; uint8_t * d_blob;
  uint32_t * d_off;  uint32_t * d_sz; int8_t * d_err; void * d_ws;
  /* pinned host staging */
  uint8_t  * h_pub;  uint8_t * h_sig; uint8_t * h_blob;
  uint32_t * h_off;  uint32_t * h_sz; int8_t * h_err;
  hipStream_t stream;
  hipEvent_t  done;
  /* the chunk in flight: where its verdicts go */
  schar *    out;
  ulong      n;
  int        busy;
};

} /* namespace */

struct fd_ed25519_amd {
  int    device;
  ulong  cap;        /* signatures per chunk */
  ulong  blob_cap;   /* message bytes per chunk */
  slot_t slot[2];
};

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
  HIPCHK( hipHostMalloc( (void **)&s->h_err,  cap, hipHostMallocDefault ) );
  HIPCHK( hipStreamCreateWithFlags( &s->stream, hipStreamNonBlocking ) );
  HIPCHK( hipEventCreateWithFlags( &s->done, hipEventDisableTiming ) );
  return FD_ED25519_AMD_OK;
}

extern "C" fd_ed25519_amd_t *
fd_ed25519_amd_new( int device, ulong batch_max, ulong blob_max ) {
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
  e->device = device; e->cap = batch_max; e->blob_cap = blob_max;
  for( int k=0; k<2; k++ ) {
    if( slot_alloc( &e->slot[k], batch_max, blob_max ) ) { fd_ed25519_amd_delete( e ); return NULL; }
  }
  return e;
}

extern "C" void
fd_ed25519_amd_delete( fd_ed25519_amd_t * e ) {
  if( !e ) return;
  (void)hipSetDevice( e->device );
  for( int k=0; k<2; k++ ) { if( e->slot[k].stream ) (void)hipStreamSynchronize( e->slot[k].stream ); slot_free( &e->slot[k] ); }
  free( e );
}

/* Wait for a slot's chunk and deliver its verdicts. */
static int
slot_drain( slot_t * s ) {
  if( !s->busy ) return FD_ED25519_AMD_OK;
  HIPCHK( hipEventSynchronize( s->done ) );
  memcpy( s->out, s->h_err, s->n );
  s->busy = 0;
  return FD_ED25519_AMD_OK;
}

/* Launch the staged chunk of slot s (inputs already in pinned memory). */
static int
slot_launch( slot_t * s, ulong n, ulong blob_sz, schar * out ) {
  HIPCHK( hipMemcpyAsync( s->d_pub,  s->h_pub,  32UL*n, hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_sig,  s->h_sig,  64UL*n, hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_off,  s->h_off,  4UL*n,  hipMemcpyHostToDevice, s->stream ) );
  HIPCHK( hipMemcpyAsync( s->d_sz,   s->h_sz,   4UL*n,  hipMemcpyHostToDevice, s->stream ) );
  if( blob_sz ) HIPCHK( hipMemcpyAsync( s->d_blob, s->h_blob, blob_sz, hipMemcpyHostToDevice, s->stream ) );
  if( fd_amd_launch_verify( (uint32_t)n, s->d_pub, s->d_sig, s->d_off, s->d_sz, s->d_blob, s->d_err, s->d_ws, s->stream, 1, NULL ) )
    return FD_ED25519_AMD_ERR_DEVICE;
  HIPCHK( hipMemcpyAsync( s->h_err, s->d_err, n, hipMemcpyDeviceToHost, s->stream ) );
  HIPCHK( hipEventRecord( s->done, s->stream ) );
  s->out = out; s->n = n; s->busy = 1;
  return FD_ED25519_AMD_OK;
}

/* Generic chunked, double-buffered driver.  get(i, &msg, &sz, &sig, &pub)
   returns signature i's inputs. */
template<typename GET>
static int
run_chunked( fd_ed25519_amd_t * e, ulong n, schar * err, GET get ) {
  if( hipSetDevice( e->device ) != hipSuccess ) return FD_ED25519_AMD_ERR_DEVICE;
  ulong i = 0; int k = 0; int rc = FD_ED25519_AMD_OK;
  while( i < n ) {
    slot_t * s = &e->slot[k];
    if( (rc = slot_drain( s )) ) return rc;
    ulong c = 0, bsz = 0;
    while( i + c < n && c < e->cap ) {
      uint8_t const * msg; ulong sz; uint8_t const * sig; uint8_t const * pub;
      get( i + c, &msg, &sz, &sig, &pub );
      if( sz > e->blob_cap ) return FD_ED25519_AMD_ERR_INVAL;   /* cannot be staged in one chunk */
      if( bsz + sz > e->blob_cap ) break;
      memcpy( s->h_pub + 32UL*c, pub, 32 );
      memcpy( s->h_sig + 64UL*c, sig, 64 );
      if( sz ) memcpy( s->h_blob + bsz, msg, sz );
      s->h_off[c] = (uint32_t)bsz; s->h_sz[c] = (uint32_t)sz;
      bsz += sz; c++;
    }
    if( (rc = slot_launch( s, c, bsz, err + i )) ) return rc;
    i += c; k ^= 1;
  }
  for( int j=0; j<2; j++ ) if( (rc = slot_drain( &e->slot[j] )) ) return rc;
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

extern "C" int
fd_ed25519_amd_verify_soa( fd_ed25519_amd_t * e, ulong n, uchar const * pub, uchar const * sig,
                           uint const * msg_off, uint const * msg_sz, uchar const * blob, ulong blob_sz,
                           schar * err ) {
  if( !e || (n && (!pub || !sig || !msg_off || !msg_sz || !err)) ) return FD_ED25519_AMD_ERR_INVAL;
  for( ulong i=0; i<n; i++ )
    if( msg_sz[i] && ((ulong)msg_off[i] + msg_sz[i] > blob_sz || !blob) ) return FD_ED25519_AMD_ERR_INVAL;
  return run_chunked( e, n, err, [&]( ulong i, uint8_t const ** m, ulong * s, uint8_t const ** g, uint8_t const ** p ) {
    *m = blob + msg_off[i]; *s = msg_sz[i]; *g = sig + 64UL*i; *p = pub + 32UL*i;
  } );
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
  HIPCHK( hipMemcpyAsync( d_dig, ws + L.dig, 512UL*n, hipMemcpyDeviceToDevice, (hipStream_t)stream ) );
  HIPCHK( hipMemcpyAsync( d_top, ws + L.top, 4UL*n,   hipMemcpyDeviceToDevice, (hipStream_t)stream ) );
  return FD_ED25519_AMD_OK;
}

/* ------------------------------------------------------------------ */
/* drop-in reference API                                                */

extern "C" int
fd_ed25519_verify( void const * msg, ulong sz, void const * sig, void const * public_key, fd_sha512_t * sha ) {
  (void)sha;   /* scratch of the reference; hashing happens on the GPU */
  static thread_local fd_ed25519_amd_t * eng = NULL;
  if( !eng ) {
    char const * d = getenv( "FD_ED25519_AMD_DEVICE" );
    eng = fd_ed25519_amd_new( d ? atoi( d ) : 0, 64UL, 64UL*FD_ED25519_AMD_MSG_MAX );
    if( !eng ) {
      fprintf( stderr, "fd_ed25519_verify: no usable MI355X/HIP device; this library has no CPU path\n" );
      abort();
    }
  }
  static uint8_t const zero = 0;
  uint32_t off = 0, s32 = (uint32_t)sz;
  if( sz > 64UL*FD_ED25519_AMD_MSG_MAX ) {
    fprintf( stderr, "fd_ed25519_verify: message of %lu bytes exceeds the engine limit\n", sz );
    abort();
  }
  schar err = 0;
  int rc = fd_ed25519_amd_verify_soa( eng, 1UL, (uchar const *)public_key, (uchar const *)sig, &off, &s32,
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
  return "fd_ed25519_amd 0.1 (gfx950; k_prep/k_decomp/k_dsm, one signature per lane)";
}
