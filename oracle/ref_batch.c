/* oracle/ref_batch.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Multi-threaded driver around the COMPILED REFERENCE's fd_ed25519_verify
 * (oracle/_ref/libfdref.so = src/ballet/ed25519/fd_ed25519_user.c:345 built
 * from the reference's own sources), one fd_sha512_t per thread exactly as
 * the verify tile holds one (src/app/frank/fd_frank_verify.c:121-123).  Used
 * as bench.py's cpu_baseline ("kind": "reference") and as a second checker.
 */
#include <stdint.h>
#include <stdlib.h>
#include <pthread.h>

void * fd_sha512_new ( void * shmem );
void * fd_sha512_join( void * shsha );
int    fd_ed25519_verify( void const * msg, unsigned long sz, void const * sig, void const * pub, void * sha );

typedef struct {
  uint64_t lo, hi;
  uint8_t const * pub; uint8_t const * sig; uint32_t const * off; uint32_t const * sz; uint8_t const * blob;
  int8_t * err;
} rjob_t;

static void *
rjob( void * arg ) {
  rjob_t * j = (rjob_t *)arg;
  void * mem = aligned_alloc( 128, 256 );
  void * sha = fd_sha512_join( fd_sha512_new( mem ) );
  for( uint64_t i=j->lo; i<j->hi; i++ )
    j->err[i] = (int8_t)fd_ed25519_verify( j->blob + j->off[i], j->sz[i], j->sig + 64*i, j->pub + 32*i, sha );
  free( mem );
  return NULL;
}

int
ref_ed25519_verify_batch( uint64_t n, uint8_t const * pub, uint8_t const * sig, uint32_t const * off,
                          uint32_t const * sz, uint8_t const * blob, int8_t * err, int nthread ) {
  if( nthread < 1 ) nthread = 1;
  if( nthread > 512 ) nthread = 512;
  pthread_t th[512]; rjob_t jb[512];
  for( int t=0; t<nthread; t++ ) {
    jb[t] = (rjob_t){ n*(uint64_t)t/(uint64_t)nthread, n*(uint64_t)(t+1)/(uint64_t)nthread, pub, sig, off, sz, blob, err };
    pthread_create( &th[t], NULL, rjob, &jb[t] );
  }
  for( int t=0; t<nthread; t++ ) pthread_join( th[t], NULL );
  return 0;
}
