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

/* Multi-signer transactions through the compiled reference: fd_txn_parse
   (src/ballet/txn/fd_txn_parse.c) then fd_ed25519_verify of every
   signature against its account address over payload[message_off, sz)
   (fd_txn.h:159-217), first failing code in signature order; -4 when the
   payload does not parse (the rule of fd_ed25519_amd_verify_txns). */
unsigned long fd_txn_parse( uint8_t const * payload, unsigned long payload_sz, void * out_buf, void * counters_opt );

typedef struct {               /* leading fields of fd_txn_t (fd_txn.h:146-272) */
  uint8_t  transaction_version, signature_cnt;
  uint16_t signature_off, message_off;
  uint8_t  readonly_signed_cnt, readonly_unsigned_cnt;
  uint16_t acct_addr_cnt, acct_addr_off;
} ref_txn_head_t;

typedef struct {
  uint64_t lo, hi;
  uint8_t const * payload; uint32_t const * off; uint32_t const * sz;
  int8_t * err;
} tjob_t;

static void *
tjob( void * arg ) {
  tjob_t * j = (tjob_t *)arg;
  void * mem = aligned_alloc( 128, 256 );
  void * sha = fd_sha512_join( fd_sha512_new( mem ) );
  void * buf = aligned_alloc( 64, 4096 );   /* >= FD_TXN_MAX_SZ */
  for( uint64_t t=j->lo; t<j->hi; t++ ) {
    uint8_t const * p = j->payload + j->off[t];
    unsigned long sz = j->sz[t];
    if( !fd_txn_parse( p, sz, buf, NULL ) ) { j->err[t] = -4; continue; }
    ref_txn_head_t const * h = (ref_txn_head_t const *)buf;
    int8_t r = 0;
    for( unsigned i=0; i<h->signature_cnt && !r; i++ )
      r = (int8_t)fd_ed25519_verify( p + h->message_off, sz - h->message_off, p + h->signature_off + 64UL*i,
                                     p + h->acct_addr_off + 32UL*i, sha );
    j->err[t] = r;
  }
  free( buf ); free( mem );
  return NULL;
}

int
ref_txn_verify_batch( uint64_t n, uint8_t const * payload, uint32_t const * off, uint32_t const * sz, int8_t * err,
                      int nthread ) {
  if( nthread < 1 ) nthread = 1;
  if( nthread > 512 ) nthread = 512;
  pthread_t th[512]; tjob_t jb[512];
  for( int t=0; t<nthread; t++ ) {
    jb[t] = (tjob_t){ n*(uint64_t)t/(uint64_t)nthread, n*(uint64_t)(t+1)/(uint64_t)nthread, payload, off, sz, err };
    pthread_create( &th[t], NULL, tjob, &jb[t] );
  }
  for( int t=0; t<nthread; t++ ) pthread_join( th[t], NULL );
  return 0;
}
