/* firedancer_amd/csrc/fd_ed25519_host.cpp
 *
 * Host-side (CPU) pieces of the reference API that are NOT on the verify
 * hot path: fd_ed25519_public_from_private and fd_ed25519_sign
 * (reference: src/ballet/ed25519/fd_ed25519_user.c:279-343), plus a
 * multi-threaded batch signer used to synthesise workloads.
 *
 * Ed25519 signing is deterministic (RFC 8032 s5.1.6), so any correct
 * implementation produces the reference's bytes; this one uses radix-2^51
 * limbs with 128-bit products (value-level arithmetic, canonical outputs)
 * and a 64 x 16 fixed-window table of multiples of B.  Parity with the
 * reference signer is pinned by the golden fixtures (RFC 8032 s7.1 vectors
 * and the seeded-stream digests in tests/golden/).
 */
#include <stdint.h>
#include <string.h>
#include <mutex>
#include <thread>
#include <vector>

#include "fd_ed25519_consts.h"

namespace {

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t  u8;
typedef unsigned __int128 u128;

/* ------------------------------ SHA-512 ------------------------------ */

u64 const K512[80] = FD_AMD_SHA512_K;
u64 const H512[8]  = FD_AMD_SHA512_H0;

inline u64 rotr( u64 x, int n ) { return (x >> n) | (x << (64 - n)); }

struct sha512 {
  u64 st[8]; u8 buf[128]; u64 tot; u32 nbuf;
  sha512() { memcpy( st, H512, sizeof(st) ); tot = 0; nbuf = 0; }
  void block( u8 const * p ) {
    u64 w[80];
    for( int i=0; i<16; i++ ) { u64 v = 0; for( int j=0; j<8; j++ ) v = (v << 8) | p[8*i+j]; w[i] = v; }
    for( int i=16; i<80; i++ ) {
      u64 s0 = rotr( w[i-15], 1 ) ^ rotr( w[i-15], 8 ) ^ (w[i-15] >> 7);
      u64 s1 = rotr( w[i-2], 19 ) ^ rotr( w[i-2], 61 ) ^ (w[i-2] >> 6);
      w[i] = w[i-16] + s0 + w[i-7] + s1;
    }
    u64 a=st[0], b=st[1], c=st[2], d=st[3], e=st[4], f=st[5], g=st[6], h=st[7];
    for( int i=0; i<80; i++ ) {
      u64 t1 = h + (rotr( e, 14 ) ^ rotr( e, 18 ) ^ rotr( e, 41 )) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
      u64 t2 = (rotr( a, 28 ) ^ rotr( a, 34 ) ^ rotr( a, 39 )) + ((a & b) ^ (a & c) ^ (b & c));
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0]+=a; st[1]+=b; st[2]+=c; st[3]+=d; st[4]+=e; st[5]+=f; st[6]+=g; st[7]+=h;
  }
  void append( void const * data, size_t n ) {
    u8 const * p = (u8 const *)data; tot += n;
    while( n ) {
      size_t take = 128u - nbuf; if( take > n ) take = n;
      memcpy( buf + nbuf, p, take ); nbuf += (u32)take; p += take; n -= take;
      if( nbuf == 128u ) { block( buf ); nbuf = 0; }
    }
  }
  void fini( u8 out[64] ) {
    u64 bits = tot << 3;
    buf[nbuf++] = 0x80;
    if( nbuf > 112u ) { memset( buf + nbuf, 0, 128u - nbuf ); block( buf ); nbuf = 0; }
    memset( buf + nbuf, 0, 128u - nbuf );
    buf[119] = (u8)(tot >> 61);
    for( int i=0; i<8; i++ ) buf[127-i] = (u8)(bits >> (8*i));
    block( buf );
    for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (u8)(st[i] >> (56 - 8*j));
  }
};

/* --------------------------- scalars mod L --------------------------- */

u64 const L64[4] = { 0x5812631a5cf5d3edUL, 0x14def9dea2f79cd6UL, 0UL, 0x1000000000000000UL };

/* x (nbytes little-endian) mod L -> 32 bytes; byte-serial Horner */
void sc_mod( u8 out[32], u8 const * in, int nbytes ) {
  u64 r[5] = {0,0,0,0,0};
  for( int k=nbytes-1; k>=0; k-- ) {
    r[4] = (r[4] << 8) | (r[3] >> 56); r[3] = (r[3] << 8) | (r[2] >> 56);
    r[2] = (r[2] << 8) | (r[1] >> 56); r[1] = (r[1] << 8) | (r[0] >> 56);
    r[0] = (r[0] << 8) | in[k];
    u64 q = (r[3] >> 60) | (r[4] << 4);
    u128 c = 0; u64 ql[5];
    for( int i=0; i<4; i++ ) { u128 p = (u128)q * L64[i] + c; ql[i] = (u64)p; c = p >> 64; }
    ql[4] = (u64)c;
    u64 br = 0;
    for( int i=0; i<5; i++ ) { u128 d = (u128)r[i] - ql[i] - br; r[i] = (u64)d; br = (u64)(d >> 64) & 1u; }
    if( br ) { u128 s = 0; for( int i=0; i<4; i++ ) { s = (u128)r[i] + L64[i] + (u64)(s >> 64); r[i] = (u64)s; } r[4] += (u64)(s >> 64); }
  }
  for( ;; ) {   /* r < 2L: final conditional subtract */
    bool ge = r[4] != 0;
    if( !ge ) { ge = true; for( int i=3; i>=0; i-- ) { if( r[i] != L64[i] ) { ge = r[i] > L64[i]; break; } } }
    if( !ge ) break;
    u64 br = 0;
    for( int i=0; i<4; i++ ) { u128 d = (u128)r[i] - L64[i] - br; r[i] = (u64)d; br = (u64)(d >> 64) & 1u; }
    r[4] -= br;
  }
  for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (u8)(r[i] >> (8*j));
}

/* (a*b + c) mod L, all 32-byte little endian */
void sc_muladd( u8 out[32], u8 const a[32], u8 const b[32], u8 const c[32] ) {
  u64 A[4], B[4], C[4];
  memcpy( A, a, 32 ); memcpy( B, b, 32 ); memcpy( C, c, 32 );
  u64 p[9] = {0};
  for( int i=0; i<4; i++ ) {
    u128 carry = 0;
    for( int j=0; j<4; j++ ) { u128 t = (u128)A[i] * B[j] + p[i+j] + carry; p[i+j] = (u64)t; carry = t >> 64; }
    p[i+4] += (u64)carry;
  }
  u128 carry = 0;
  for( int i=0; i<9; i++ ) { u128 t = (u128)p[i] + (i < 4 ? C[i] : 0) + carry; p[i] = (u64)t; carry = t >> 64; }
  u8 wide[72]; memcpy( wide, p, 72 );
  sc_mod( out, wide, 72 );
}

/* --------------------------- field 2^255-19 -------------------------- */

struct f51 { u64 v[5]; };
u64 const M51 = (1UL << 51) - 1;

inline f51 fadd( f51 const & a, f51 const & b ) { f51 r; for( int i=0; i<5; i++ ) r.v[i] = a.v[i] + b.v[i]; return r; }
inline f51 fsub( f51 const & a, f51 const & b ) {   /* a + 4p - b */
  f51 r;
  r.v[0] = a.v[0] + 0x1FFFFFFFFFFFB4UL - b.v[0];
  for( int i=1; i<5; i++ ) r.v[i] = a.v[i] + 0x1FFFFFFFFFFFFCUL - b.v[i];
  return r;
}
inline f51 fcarry( u128 t0, u128 t1, u128 t2, u128 t3, u128 t4 ) {
  t1 += t0 >> 51; t0 &= M51;
  t2 += t1 >> 51; t1 &= M51;
  t3 += t2 >> 51; t2 &= M51;
  t4 += t3 >> 51; t3 &= M51;
  t0 += (t4 >> 51) * 19; t4 &= M51;
  t1 += t0 >> 51; t0 &= M51;
  f51 r; r.v[0] = (u64)t0; r.v[1] = (u64)t1; r.v[2] = (u64)t2; r.v[3] = (u64)t3; r.v[4] = (u64)t4;
  return r;
}
inline f51 fmul( f51 const & f, f51 const & g ) {
  u64 g1 = 19*g.v[1], g2 = 19*g.v[2], g3 = 19*g.v[3], g4 = 19*g.v[4];
  u128 t0 = (u128)f.v[0]*g.v[0] + (u128)f.v[1]*g4 + (u128)f.v[2]*g3 + (u128)f.v[3]*g2 + (u128)f.v[4]*g1;
  u128 t1 = (u128)f.v[0]*g.v[1] + (u128)f.v[1]*g.v[0] + (u128)f.v[2]*g4 + (u128)f.v[3]*g3 + (u128)f.v[4]*g2;
  u128 t2 = (u128)f.v[0]*g.v[2] + (u128)f.v[1]*g.v[1] + (u128)f.v[2]*g.v[0] + (u128)f.v[3]*g4 + (u128)f.v[4]*g3;
  u128 t3 = (u128)f.v[0]*g.v[3] + (u128)f.v[1]*g.v[2] + (u128)f.v[2]*g.v[1] + (u128)f.v[3]*g.v[0] + (u128)f.v[4]*g4;
  u128 t4 = (u128)f.v[0]*g.v[4] + (u128)f.v[1]*g.v[3] + (u128)f.v[2]*g.v[2] + (u128)f.v[3]*g.v[1] + (u128)f.v[4]*g.v[0];
  return fcarry( t0, t1, t2, t3, t4 );
}
inline f51 fsq( f51 const & f ) { return fmul( f, f ); }
inline f51 fconst( u64 x ) { f51 r = {{ x, 0, 0, 0, 0 }}; return r; }

f51 ffrombytes( u8 const s[32] ) {
  u64 w[4]; memcpy( w, s, 32 );
  f51 r;
  r.v[0] =  w[0]                        & M51;
  r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r.v[4] =  (w[3] >> 12)                 & M51;
  return r;
}

void ftobytes( u8 s[32], f51 const & a ) {
  f51 h = fcarry( a.v[0], a.v[1], a.v[2], a.v[3], a.v[4] );
  h = fcarry( h.v[0], h.v[1], h.v[2], h.v[3], h.v[4] );
  u64 q = (h.v[0] + 19) >> 51; q = (h.v[1] + q) >> 51; q = (h.v[2] + q) >> 51; q = (h.v[3] + q) >> 51; q = (h.v[4] + q) >> 51;
  h.v[0] += 19 * q;
  h.v[1] += h.v[0] >> 51; h.v[0] &= M51;
  h.v[2] += h.v[1] >> 51; h.v[1] &= M51;
  h.v[3] += h.v[2] >> 51; h.v[2] &= M51;
  h.v[4] += h.v[3] >> 51; h.v[3] &= M51;
  h.v[4] &= M51;
  u64 w[4];
  w[0] = h.v[0] | (h.v[1] << 51);
  w[1] = (h.v[1] >> 13) | (h.v[2] << 38);
  w[2] = (h.v[2] >> 26) | (h.v[3] << 25);
  w[3] = (h.v[3] >> 39) | (h.v[4] << 12);
  memcpy( s, w, 32 );
}

f51 finvert( f51 const & z ) {   /* z^(p-2) */
  f51 z2 = fsq( z );
  f51 t = fsq( fsq( z2 ) );
  f51 z9 = fmul( t, z );
  f51 z11 = fmul( z9, z2 );
  f51 z2_5 = fmul( fsq( z11 ), z9 );                         /* 2^5 - 1 */
  t = z2_5; for( int i=0; i<5; i++ ) t = fsq( t );
  f51 z2_10 = fmul( t, z2_5 );
  t = z2_10; for( int i=0; i<10; i++ ) t = fsq( t );
  f51 z2_20 = fmul( t, z2_10 );
  t = z2_20; for( int i=0; i<20; i++ ) t = fsq( t );
  f51 z2_40 = fmul( t, z2_20 );
  t = z2_40; for( int i=0; i<10; i++ ) t = fsq( t );
  f51 z2_50 = fmul( t, z2_10 );
  t = z2_50; for( int i=0; i<50; i++ ) t = fsq( t );
  f51 z2_100 = fmul( t, z2_50 );
  t = z2_100; for( int i=0; i<100; i++ ) t = fsq( t );
  f51 z2_200 = fmul( t, z2_100 );
  t = z2_200; for( int i=0; i<50; i++ ) t = fsq( t );
  f51 z2_250 = fmul( t, z2_50 );
  t = z2_250; for( int i=0; i<5; i++ ) t = fsq( t );
  return fmul( t, z11 );                                      /* 2^255 - 21 */
}

/* ------------------------------ points ------------------------------- */

struct gep { f51 X, Y, Z, T; };            /* extended */
struct gec { f51 YpX, YmX, Z, T2d; };      /* cached   */

f51 D2_51;

gep gadd( gep const & p, gec const & q ) {
  f51 a = fmul( fsub( p.Y, p.X ), q.YmX );
  f51 b = fmul( fadd( p.Y, p.X ), q.YpX );
  f51 c = fmul( p.T, q.T2d );
  f51 zz = fmul( p.Z, q.Z ); f51 d = fadd( zz, zz );
  f51 e = fsub( b, a ), f = fsub( d, c ), g = fadd( d, c ), h = fadd( b, a );
  gep r; r.X = fmul( e, f ); r.Y = fmul( g, h ); r.T = fmul( e, h ); r.Z = fmul( f, g );
  return r;
}

gep gdbl( gep const & p ) {
  f51 a = fsq( p.X ), b = fsq( p.Y ), zz = fsq( p.Z ), c = fadd( zz, zz );
  f51 h = fadd( a, b );
  f51 e = fsub( h, fsq( fadd( p.X, p.Y ) ) );
  f51 g = fsub( a, b );
  f51 f = fadd( c, g );
  gep r; r.X = fmul( e, f ); r.Y = fmul( g, h ); r.T = fmul( e, h ); r.Z = fmul( f, g );
  return r;
}

gec gcache( gep const & p ) {
  gec c; c.YpX = fadd( p.Y, p.X ); c.YmX = fsub( p.Y, p.X ); c.Z = p.Z; c.T2d = fmul( p.T, D2_51 );
  return c;
}

gep gidentity() { gep r; r.X = fconst( 0 ); r.Y = fconst( 1 ); r.Z = fconst( 1 ); r.T = fconst( 0 ); return r; }

/* table[i][j] = j * 16^i * B (cached), j = 0..15 */
gec TBL[64][16];
std::once_flag tbl_once;

f51 limbs_to_f51( int32_t const * l ) {
  /* value of a 10-limb 26/25 representation, reduced via bytes of an exact integer */
  /* compute sum l_k 2^{ceil(25.5 k)} as signed big integer mod p */
  static int const sh[10] = { 0, 26, 51, 77, 102, 128, 153, 179, 204, 230 };
  /* accumulate in 5 x 64-bit two's complement + reduce by adding 8p */
  __int128 acc[5] = {0,0,0,0,0};
  for( int k=0; k<10; k++ ) {
    int limb = sh[k] / 51, off = sh[k] % 51;
    __int128 v = (__int128)l[k] << off;
    acc[limb] += v;
  }
  /* normalise to non-negative by adding 16p (limb form) */
  acc[0] += (__int128)16 * ((1L << 51) - 19);
  for( int i=1; i<5; i++ ) acc[i] += (__int128)16 * ((1L << 51) - 1);
  for( int i=0; i<4; i++ ) { __int128 c = acc[i] >> 51; acc[i] -= c << 51; acc[i+1] += c; }
  __int128 c = acc[4] >> 51; acc[4] -= c << 51; acc[0] += c * 19;
  c = acc[0] >> 51; acc[0] -= c << 51; acc[1] += c;
  f51 r; for( int i=0; i<5; i++ ) r.v[i] = (u64)acc[i];
  return r;
}

void tbl_init() {
  int32_t const d2l[10] = FD_AMD_FE_D2;
  D2_51 = limbs_to_f51( d2l );
  /* B from the generated Bi table: Bi[0] rows y+x, y-x */
  int32_t const bi[8][3][10] = FD_AMD_BI_PRECOMP;
  f51 ypx = limbs_to_f51( bi[0][0] ), ymx = limbs_to_f51( bi[0][1] );
  /* x = (ypx - ymx)/2, y = (ypx + ymx)/2 */
  f51 inv2;  { u8 b[32] = {0}; b[0] = 0xf7; for( int i=1; i<31; i++ ) b[i] = 0xff; b[31] = 0x3f; inv2 = ffrombytes( b ); } /* (p+1)/2 */
  gep B; B.X = fmul( fsub( ypx, ymx ), inv2 ); B.Y = fmul( fadd( ypx, ymx ), inv2 ); B.Z = fconst( 1 ); B.T = fmul( B.X, B.Y );
  gep base = B;
  for( int i=0; i<64; i++ ) {
    gep acc = gidentity();
    gec cb = gcache( base );
    for( int j=0; j<16; j++ ) { TBL[i][j] = gcache( acc ); acc = gadd( acc, cb ); }
    for( int k=0; k<4; k++ ) base = gdbl( base );
  }
}

gep scalarmult_base( u8 const a[32] ) {
  std::call_once( tbl_once, tbl_init );
  gep r = gidentity();
  for( int i=0; i<64; i++ ) {
    int e = (a[i >> 1] >> (4 * (i & 1))) & 15;
    if( e ) r = gadd( r, TBL[i][e] );
  }
  return r;
}

void gencode( u8 s[32], gep const & p ) {
  f51 zi = finvert( p.Z );
  f51 x = fmul( p.X, zi ), y = fmul( p.Y, zi );
  u8 xb[32]; ftobytes( xb, x ); ftobytes( s, y );
  s[31] ^= (u8)((xb[0] & 1) << 7);
}

void pub_from_prv( u8 pub[32], u8 const prv[32] ) {
  u8 h[64]; sha512 s; s.append( prv, 32 ); s.fini( h );
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  gencode( pub, scalarmult_base( h ) );
}

void sign1( u8 sig[64], u8 const * msg, size_t sz, u8 const pub[32], u8 const prv[32] ) {
  u8 h[64]; { sha512 s; s.append( prv, 32 ); s.fini( h ); }
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  u8 r64[64]; { sha512 s; s.append( h + 32, 32 ); if( sz ) s.append( msg, sz ); s.fini( r64 ); }
  u8 r[32]; sc_mod( r, r64, 64 );
  gencode( sig, scalarmult_base( r ) );
  u8 k64[64]; { sha512 s; s.append( sig, 32 ); s.append( pub, 32 ); if( sz ) s.append( msg, sz ); s.fini( k64 ); }
  u8 k[32]; sc_mod( k, k64, 64 );
  sc_muladd( sig + 32, k, h, r );
}

} /* namespace */

extern "C" {

void *
fd_ed25519_public_from_private( void * public_key, void const * private_key, void * sha ) {
  (void)sha;
  pub_from_prv( (u8 *)public_key, (u8 const *)private_key );
  return public_key;
}

void *
fd_ed25519_sign( void * sig, void const * msg, unsigned long sz, void const * public_key,
                 void const * private_key, void * sha ) {
  (void)sha;
  sign1( (u8 *)sig, (u8 const *)msg, sz, (u8 const *)public_key, (u8 const *)private_key );
  return sig;
}

/* Batch keygen + sign over the engine's SoA layout, nthread host threads:
   prv[n][32] -> pub[n][32], sig[n][64] over blob[msg_off[i] .. +msg_sz[i]). */
int
fd_ed25519_amd_sign_batch( unsigned long n, uint8_t const * prv, uint8_t const * blob, uint32_t const * msg_off,
                           uint32_t const * msg_sz, uint8_t * pub, uint8_t * sig, int nthread ) {
  std::call_once( tbl_once, tbl_init );
  if( nthread < 1 ) nthread = 1;
  if( nthread > 256 ) nthread = 256;
  std::vector<std::thread> th;
  for( int t=0; t<nthread; t++ ) {
    th.emplace_back( [=]() {
      unsigned long lo = n * (unsigned long)t / (unsigned long)nthread, hi = n * (unsigned long)(t+1) / (unsigned long)nthread;
      for( unsigned long i=lo; i<hi; i++ ) {
        pub_from_prv( pub + 32*i, prv + 32*i );
        sign1( sig + 64*i, blob + msg_off[i], msg_sz[i], pub + 32*i, prv + 32*i );
      }
    } );
  }
  for( auto & x : th ) x.join();
  return 0;
}

/* Workload synthesis for the transaction front end (config 4): txn_cnt
   well-formed wire transactions (fd_txn.h layout), legacy and v0 by turns,
   with nsig in [nsig_lo, nsig_hi] signers whose account addresses are the
   next public keys of pub[] (consumed in order) and a message of about
   [msg_lo, msg_hi] bytes, capped so a payload fits the 1232-byte MTU.
   Signature fields are left zero; per signature s the caller gets where
   its message starts/ends (sig_msg_off / sig_msg_sz, offsets in payload)
   and where its 64 bytes go (sig_at).  Returns the number of signatures
   (0 if payload_cap or pub_cnt is too small). */
unsigned long
fd_ed25519_amd_synth_txns( unsigned long seed, unsigned long txn_cnt, uint32_t nsig_lo, uint32_t nsig_hi,
                           uint32_t msg_lo, uint32_t msg_hi, uint8_t const * pub, unsigned long pub_cnt,
                           uint8_t * payload, unsigned long payload_cap, uint32_t * txn_off, uint32_t * txn_sz,
                           uint32_t * sig_msg_off, uint32_t * sig_msg_sz, uint32_t * sig_at ) {
  uint64_t s = seed * 0x9E3779B97F4A7C15UL + 0x1234567UL;
  auto rnd = [&]() -> uint64_t {
    uint64_t z = (s += 0x9e3779b97f4a7c15UL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9UL; z = (z ^ (z >> 27)) * 0x94d049bb133111ebUL; return z ^ (z >> 31);
  };
  auto cu16 = [&]( uint8_t * p, uint32_t v ) -> uint32_t {
    if( v < 0x80u ) { p[0] = (uint8_t)v; return 1u; }
    if( v < 0x4000u ) { p[0] = (uint8_t)(0x80u | (v & 0x7fu)); p[1] = (uint8_t)(v >> 7); return 2u; }
    p[0] = (uint8_t)(0x80u | (v & 0x7fu)); p[1] = (uint8_t)(0x80u | ((v >> 7) & 0x7fu)); p[2] = (uint8_t)(v >> 14); return 3u;
  };
  unsigned long at = 0, ns = 0;
  if( nsig_lo < 1 ) nsig_lo = 1;
  if( nsig_hi < nsig_lo ) nsig_hi = nsig_lo;
  for( unsigned long t=0; t<txn_cnt; t++ ) {
    uint32_t nsig = nsig_lo + (uint32_t)(rnd() % (nsig_hi - nsig_lo + 1u));
    if( ns + nsig > pub_cnt || at + 1232UL > payload_cap ) return 0UL;
    int v0 = (int)(t & 1u);
    uint32_t nx = nsig >= 10u ? 1u : 1u + (uint32_t)(rnd() % 3u), nacct = nsig + nx;
    uint32_t fixed = 1u + 64u*nsig + (v0 ? 1u : 0u) + 3u + 1u + 32u*nacct + 32u + 1u + 1u + 1u + 2u + 2u + (v0 ? 1u : 0u);
    uint32_t want = msg_lo + (uint32_t)(rnd() % (msg_hi - msg_lo + 1u));
    uint32_t total = fixed + (want > fixed - 1u - 64u*nsig ? want - (fixed - 1u - 64u*nsig) : 0u);
    if( total > 1232u ) total = 1232u;
    uint32_t dlen = total - fixed;
    if( fixed > 1232u ) return 0UL;
    uint8_t * p = payload + at;
    uint32_t o = 0;
    p[o++] = (uint8_t)nsig;
    for( uint32_t j=0; j<nsig; j++ ) { sig_at[ns + j] = (uint32_t)(at + o); memset( p + o, 0, 64 ); o += 64u; }
    uint32_t moff = o;
    if( v0 ) p[o++] = 0x80u;
    p[o++] = (uint8_t)nsig; p[o++] = (uint8_t)(rnd() % nsig); p[o++] = (uint8_t)(rnd() % (nx + 1u));
    o += cu16( p + o, nacct );
    for( uint32_t j=0; j<nsig; j++ ) { memcpy( p + o, pub + 32UL*(ns + j), 32 ); o += 32u; }
    for( uint32_t j=0; j<32u*nx + 32u; j++ ) p[o++] = (uint8_t)rnd();          /* other accounts + blockhash */
    p[o++] = 1u;                                                               /* one instruction */
    p[o++] = (uint8_t)(1u + rnd() % (nacct - 1u));
    p[o++] = 2u; p[o++] = 0u; p[o++] = (uint8_t)(nacct - 1u);
    o += cu16( p + o, dlen );
    for( uint32_t j=0; j<dlen; j++ ) p[o++] = (uint8_t)rnd();
    if( v0 ) p[o++] = 0u;                                                      /* no lookup tables */
    txn_off[t] = (uint32_t)at; txn_sz[t] = o;
    for( uint32_t j=0; j<nsig; j++ ) { sig_msg_off[ns + j] = (uint32_t)(at + moff); sig_msg_sz[ns + j] = o - moff; }
    at += o; ns += nsig;
  }
  return ns;
}

} /* extern "C" */
