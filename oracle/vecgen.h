/* oracle/vecgen.h -- TEST INFRASTRUCTURE ONLY (build container).
 *
 * Seeded synthesis of ed25519 verify inputs for the parity harnesses
 * (check_vs_ref.c, gen_golden.c).  Valid signatures are produced by the
 * COMPILED REFERENCE (oracle/_ref/libfdref.so: fd_ed25519_public_from_private
 * and fd_ed25519_sign, src/ballet/ed25519/fd_ed25519_user.c:279-343); the
 * expected verdict of every vector is the reference's fd_ed25519_verify
 * (user.c:345-431) run on the exact same bytes.
 */
#ifndef ORACLE_VECGEN_H
#define ORACLE_VECGEN_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

typedef unsigned long ulong_t;

/* reference symbols (oracle/_ref/libfdref.so) */
void * fd_sha512_new ( void * shmem );
void * fd_sha512_join( void * shsha );
void * fd_ed25519_public_from_private( void * pub, void const * prv, void * sha );
void * fd_ed25519_sign( void * sig, void const * msg, ulong_t sz, void const * pub, void const * prv, void * sha );
int    fd_ed25519_verify( void const * msg, ulong_t sz, void const * sig, void const * pub, void * sha );

/* oracle symbols (oracle/liboracle.so) */
int    oracle_ed25519_verify( void const * msg, size_t sz, void const * sig, void const * pub );
void   oracle_sc_reduce( uint8_t out[32], uint8_t const in[64] );

/* splitmix64 */
static inline uint64_t sm64( uint64_t * s ) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15UL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9UL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebUL;
  return z ^ (z >> 31);
}
static inline void sm_bytes( uint64_t * s, uint8_t * p, size_t n ) {
  for( size_t i=0; i<n; i+=8 ) { uint64_t v = sm64( s ); for( size_t j=0; j<8 && i+j<n; j++ ) p[i+j] = (uint8_t)(v>>(8*j)); }
}

static void * vg_sha( void ) {
  static __thread void * sha = NULL;
  if( !sha ) { void * mem = aligned_alloc( 128, 256 ); sha = fd_sha512_join( fd_sha512_new( mem ) ); }
  return sha;
}

/* one vector */
typedef struct {
  uint8_t  pub[32];
  uint8_t  sig[64];
  uint32_t sz;
  uint8_t  cls;
  uint8_t  msg[1232];
} vec_t;

/* classes (mirrored in tests/golden/README.md and tests/_golden.py) */
enum {
  CLS_VALID = 0,       /* freshly signed by the reference signer */
  CLS_FLIP_SIG,        /* one random bit of sig flipped */
  CLS_FLIP_MSG,        /* one random bit of msg flipped */
  CLS_FLIP_PUB,        /* one random bit of pub flipped */
  CLS_S_WINDOW,        /* s[31]==0x10 and s[16..30]!=0: reference returns 0 (user.c:379) */
  CLS_S_RANGE,         /* s >= L / s[31]>0x10 / s == L exactly / s == L-1 */
  CLS_MALLEATE,        /* s' = s + L of a valid signature */
  CLS_OFFCURVE_A,      /* pub y with no square root */
  CLS_OFFCURVE_R,      /* R y with no square root */
  CLS_SMALL_ORDER,     /* A and/or R from the 8 torsion points, s = 0 */
  CLS_NONCANON,        /* y >= p, "-0", bit-255 encodings for A/R */
  CLS_FALSE_REJECT,    /* valid signatures the AVX limb compare rejects */
  CLS_RANDOM,          /* uniformly random pub/sig bytes */
  CLS_RFC8032,         /* RFC 8032 s7.1 secrets/messages signed by the reference */
  CLS_MAINNET,         /* src/ballet/txn/fixtures/transaction{1,2,3}.bin */
  CLS_ZERO_MSG,        /* sz == 0 */
  CLS_MAX_MSG,         /* sz == 1232 (MTU) */
  CLS_CNT
};

static void vg_sign( vec_t * v, uint8_t const prv[32] ) {
  fd_ed25519_public_from_private( v->pub, prv, vg_sha() );
  fd_ed25519_sign( v->sig, v->msg, v->sz, v->pub, prv, vg_sha() );
}

static void vg_valid( vec_t * v, uint64_t * rs, uint32_t szlo, uint32_t szhi ) {
  uint8_t prv[32]; sm_bytes( rs, prv, 32 );
  v->sz = szlo + (uint32_t)(sm64( rs ) % (uint64_t)(szhi - szlo + 1));
  sm_bytes( rs, v->msg, v->sz );
  vg_sign( v, prv );
  v->cls = CLS_VALID;
}

/* "mixed" stream: valid, 10 % with one flipped bit in sig, msg or pub */
static void vg_mixed( vec_t * v, uint64_t * rs, uint32_t szlo, uint32_t szhi ) {
  vg_valid( v, rs, szlo, szhi );
  uint64_t r = sm64( rs );
  if( r % 10 ) return;
  int which = (int)((r >> 8) % 3);
  if( which==1 && v->sz==0 ) which = 0;
  uint64_t bit = r >> 16;
  if( which==0 ) { v->sig[ (bit>>3) % 64 ] ^= (uint8_t)(1 << (bit&7)); v->cls = CLS_FLIP_SIG; }
  if( which==1 ) { v->msg[ (bit>>3) % v->sz ] ^= (uint8_t)(1 << (bit&7)); v->cls = CLS_FLIP_MSG; }
  if( which==2 ) { v->pub[ (bit>>3) % 32 ] ^= (uint8_t)(1 << (bit&7)); v->cls = CLS_FLIP_PUB; }
}

static int vg_hex( uint8_t * out, char const * hex ) {
  size_t n = strlen( hex ) / 2;
  for( size_t i=0; i<n; i++ ) { unsigned x; sscanf( hex + 2*i, "%2x", &x ); out[i] = (uint8_t)x; }
  return (int)n;
}

/* torsion points (computed as [L]P for random P) */
static char const * const VG_TORSION[8] = {
  "0100000000000000000000000000000000000000000000000000000000000000",
  "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
  "0000000000000000000000000000000000000000000000000000000000000000",
  "0000000000000000000000000000000000000000000000000000000000000080",
  "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
  "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
  "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
  "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
};

/* non-canonical encodings accepted by decompression */
static char const * const VG_NONCANON[6] = {
  "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f", /* y = p    */
  "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f", /* y = p+1  */
  "0100000000000000000000000000000000000000000000000000000000000080", /* -0 identity */
  "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff", /* y = p, bit 255 */
  "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff", /* y = p+1, bit 255 */
  "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff", /* (0,-1) with bit 255 */
};

static uint8_t const VG_L[32] = {
  0xed,0xd3,0xf5,0x5c,0x1a,0x63,0x12,0x58,0xd6,0x9c,0xf7,0xa2,0xde,0xf9,0xde,0x14,
  0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0x10 };

/* a += b (256-bit little endian) */
static void vg_add256( uint8_t * a, uint8_t const * b ) {
  unsigned c = 0;
  for( int i=0; i<32; i++ ) { unsigned s = (unsigned)a[i] + b[i] + c; a[i] = (uint8_t)s; c = s >> 8; }
}

/* y with no square root: find small y such that (y^2-1)/(dy^2+1) is a
   non-residue -- we simply use the reference/oracle to test candidate
   encodings y=2,3,... and keep those that return -2 on decompression. */

#endif
