/* tests/c/dropin_client.c -- a plain C caller of the drop-in boundary.
 *
 * What a Firedancer maintainer gets after relinking:
 * this file includes only the headers under include/, is compiled by gcc (no HIP headers,
 * no C++), and links libfd_ed25519_amd.so.  It exercises the reference's
 * API exactly as the reference's own callers do (src/ballet/ed25519/
 * fd_ed25519.h:40-109; the verify call of load/fd_frank_verify_synth_load.c:
 * 380), then the batch API.
 *
 *   dropin_client cpu   host-side entry points only (runs without a GPU):
 *                       RFC 8032 s7.1 test 1 keygen + sign bytes, strerror,
 *                       and fd_ed25519_amd_new refusing to start without a
 *                       device
 *   dropin_client gpu   everything: fd_ed25519_verify on valid / corrupted
 *                       inputs, then a 2000-signature batch through
 *                       fd_ed25519_amd_verify_soa and _verify_batch, each
 *                       verdict equal to the per-signature drop-in call
 *
 * Prints "dropin_client <mode>: OK" and exits 0, or names the failed check.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fd_ed25519_amd.h"
#include "fd_tango_amd.h"
#include "fd_txn_amd.h"

#define CHECK( c ) do { if( !(c) ) { fprintf( stderr, "dropin_client: FAIL %s (%s:%d)\n", #c, __FILE__, __LINE__ ); exit( 1 ); } } while(0)

static void
hex( uchar * out, char const * h, ulong n ) {
  for( ulong i=0; i<n; i++ ) { unsigned x; CHECK( sscanf( h + 2*i, "%2x", &x ) == 1 ); out[i] = (uchar)x; }
}

/* splitmix64: deterministic test inputs */
static ulong sm_state = 0x1234567ULL;
static ulong
sm64( void ) {
  ulong z = (sm_state += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

int
main( int argc, char ** argv ) {
  char const * mode = argc > 1 ? argv[1] : "cpu";
  /* the reference hands a 128-aligned fd_sha512_t scratch; this library
     never touches it, but a caller that owns one passes it as before */
  static __attribute__((aligned(128))) uchar sha_mem[ FD_SHA512_FOOTPRINT ];
  fd_sha512_t * sha = (fd_sha512_t *)sha_mem;

  /* RFC 8032 s7.1 TEST 1 (empty message) */
  uchar prv[32], pub_exp[32], sig_exp[64], pub[32], sig[64];
  hex( prv,     "9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60", 32 );
  hex( pub_exp, "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", 32 );
  hex( sig_exp, "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b", 64 );
  CHECK( fd_ed25519_public_from_private( pub, prv, sha ) == pub );
  CHECK( !memcmp( pub, pub_exp, 32 ) );
  CHECK( fd_ed25519_sign( sig, NULL, 0UL, pub, prv, sha ) == sig );
  CHECK( !memcmp( sig, sig_exp, 64 ) );
  CHECK( !strcmp( fd_ed25519_strerror( FD_ED25519_SUCCESS ), "success" ) );
  CHECK( fd_ed25519_strerror( FD_ED25519_ERR_MSG ) != NULL );
  CHECK( FD_ED25519_SIG_SZ == 64UL && sizeof( fd_ed25519_sig_t ) == 64UL );
  CHECK( sizeof( fd_frag_meta_t ) == 32UL );
  CHECK( fd_ed25519_amd_version() != NULL );

  if( !strcmp( mode, "cpu" ) ) {
    /* no device here: the batch engine must refuse to start (no CPU fallback) */
    CHECK( fd_ed25519_amd_new( 0, 64UL, 64UL*FD_ED25519_AMD_MSG_MAX ) == NULL );
    printf( "dropin_client cpu: OK\n" );
    return 0;
  }

  /* --- drop-in verify, as the verify tile calls it --- */
  CHECK( fd_ed25519_verify( NULL, 0UL, sig, pub, sha ) == FD_ED25519_SUCCESS );
  uchar bad[64]; memcpy( bad, sig, 64 ); bad[40] ^= 0x01;       /* s changed, still < L */
  CHECK( fd_ed25519_verify( NULL, 0UL, bad, pub, sha ) == FD_ED25519_ERR_MSG );
  memcpy( bad, sig, 64 ); bad[5] ^= 0x10;                        /* this R no longer decompresses */
  CHECK( fd_ed25519_verify( NULL, 0UL, bad, pub, sha ) == FD_ED25519_ERR_PUBKEY );
  memcpy( bad, sig, 64 ); bad[63] |= 0xF0;                      /* s >= 2^252: the s check */
  CHECK( fd_ed25519_verify( NULL, 0UL, bad, pub, sha ) == FD_ED25519_ERR_SIG );
  uchar msg1[1] = { 0x72 };
  CHECK( fd_ed25519_verify( msg1, 1UL, sig, pub, sha ) == FD_ED25519_ERR_MSG );

  /* --- batch API: n signed messages, ~10 % corrupted --- */
  ulong const n = 2000UL;
  uchar * P = malloc( 32UL*n ), * S = malloc( 64UL*n ), * blob = malloc( 1232UL*n + 1UL );
  uint  * off = malloc( 4UL*n ), * sz = malloc( 4UL*n );
  schar * err = malloc( n ), * err2 = malloc( n );
  void const ** mp = malloc( sizeof(void *)*n ), ** sp = malloc( sizeof(void *)*n ), ** pp = malloc( sizeof(void *)*n );
  ulong * szl = malloc( 8UL*n );
  CHECK( P && S && blob && off && sz && err && err2 && mp && sp && pp && szl );
  ulong o = 0;
  for( ulong i=0; i<n; i++ ) {
    uchar k[32];
    for( int j=0; j<32; j++ ) k[j] = (uchar)sm64();
    sz[i] = (uint)(sm64() % 1233UL); off[i] = (uint)o;
    for( uint j=0; j<sz[i]; j++ ) blob[o+j] = (uchar)sm64();
    fd_ed25519_public_from_private( P + 32UL*i, k, sha );
    fd_ed25519_sign( S + 64UL*i, blob + o, sz[i], P + 32UL*i, k, sha );
    ulong r = sm64();
    if( !(r % 10UL) ) {
      if( (r >> 8) & 1 ) S[64UL*i + ((r >> 16) % 64UL)] ^= (uchar)(1U << ((r >> 24) & 7U));
      else               P[32UL*i + ((r >> 16) % 32UL)] ^= (uchar)(1U << ((r >> 24) & 7U));
    }
    mp[i] = blob + o; sp[i] = S + 64UL*i; pp[i] = P + 32UL*i; szl[i] = sz[i];
    o += sz[i];
  }
  fd_ed25519_amd_t * eng = fd_ed25519_amd_new( 0, 512UL, 512UL*FD_ED25519_AMD_MSG_MAX );   /* chunked: 4 chunks */
  CHECK( eng != NULL );
  CHECK( fd_ed25519_amd_verify_soa( eng, n, P, S, off, sz, blob, o, err ) == FD_ED25519_AMD_OK );
  CHECK( fd_ed25519_amd_verify_batch( eng, n, mp, szl, sp, pp, err2 ) == FD_ED25519_AMD_OK );
  ulong ok = 0, rej = 0;
  for( ulong i=0; i<n; i++ ) {
    int e1 = fd_ed25519_verify( mp[i], szl[i], sp[i], pp[i], sha );
    if( e1 != err[i] || e1 != err2[i] ) {
      fprintf( stderr, "dropin_client: FAIL signature %lu: drop-in %d, soa %d, batch %d\n", i, e1, err[i], err2[i] );
      return 1;
    }
    if( e1 ) rej++; else ok++;
  }
  CHECK( rej > 100UL && ok > 1600UL );
  /* argument errors are reported, not crashed on */
  CHECK( fd_ed25519_amd_verify_soa( eng, 1UL, NULL, S, off, sz, blob, o, err ) == FD_ED25519_AMD_ERR_INVAL );
  fd_ed25519_amd_delete( eng );
  printf( "dropin_client gpu: OK (%lu accepted, %lu rejected, verdicts equal across the three entry points)\n", ok, rej );
  return 0;
}
