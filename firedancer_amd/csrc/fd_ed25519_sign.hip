/* firedancer_amd/csrc/fd_ed25519_sign.hip
 *
 * GPU keygen + sign: synthesises large verify workloads
 * (2^24 signatures for config 4) on the device instead of host threads.
 * Ed25519 signing is deterministic (RFC 8032 s5.1.6), so the output bytes
 * equal the reference's fd_ed25519_public_from_private / fd_ed25519_sign
 * (src/ballet/ed25519/fd_ed25519_user.c:279-343) for any correct
 * algorithm; tests compare every byte with the host signer, which the
 * golden RFC 8032 vectors pin.  One signature per lane:
 *
 *   h = SHA-512(seed); a = clamp(h[0:32]); A = [a]B   -> public key
 *   r = SHA-512(h[32:64] || M) mod L; R = [r]B
 *   k = SHA-512(R || A || M) mod L;  S = (r + k a) mod L  -> R || S
 *
 * [x]B is the signed radix-16 fixed-base method over the 32 x 8 table
 * BASE[j][k] = (k+1) 256^j B (tools/gen_consts.py): 64 mixed additions and
 * 4 doublings; points are encoded with one inversion each.  Not constant
 * time: workload synthesis only, never for real keys.
 */
#include "fd_ed25519_dev.h"
#include "fd_ed25519_kernels.h"

typedef int8_t i8;

namespace {

__device__ static i32 const BASE[32][8][3][10] = FD_AMD_BASE_COMB;

/* SHA-512 over NPRE prefix words (big-endian-loaded u64s, in message byte
   order as little-endian words like k_prep's R||A) followed by M[0..sz) */
template<int NPRE>
__device__ void
sha512_pm( u64 st[8], u64 const pre[NPRE], u8 const * M, u32 sz ) {
  u64 const H0[8] = FD_AMD_SHA512_H0;
  _Pragma("unroll") for( int k=0; k<8; k++ ) st[k] = H0[k];
  u32 nblk = (8u*NPRE + sz + 17u + 127u) / 128u;
  u64 bitlen = (u64)(8u*NPRE + sz) << 3;
  for( u32 blk=0; blk<nblk; blk++ ) {
    u64 w[16];
    _Pragma("unroll") for( int k=0; k<16; k++ ) {
      u32 kk = blk*16u + (u32)k;
      u64 v;
      if( kk < (u32)NPRE ) v = pre[kk < (u32)NPRE ? kk : 0];
      else                 v = msg_word( M, sz, 8u*(kk - (u32)NPRE) );
      v = bswap64( v );
      if( blk == nblk-1u && k == 15 ) v |= bitlen;
      w[k] = v;
    }
    sha512_compress( st, w );
  }
}

/* digest -> 16 little-endian u32 words (the byte string as an integer) */
__device__ __forceinline__ void
digest_words( u32 hd[16], u64 const st[8] ) {
  _Pragma("unroll") for( int a=0; a<8; a++ ) {
    hd[2*a]   = __builtin_bswap32( (u32)(st[a] >> 32) );
    hd[2*a+1] = __builtin_bswap32( (u32)st[a] );
  }
}

/* z^(p-2) by the standard 2^255-21 addition chain (254 squarings) */
__device__ fe
fe_invert( fe const & z ) {
  fe t0 = fe_sq( z );                       /* 2 */
  fe t1 = fe_sq_iter( t0, 2 );              /* 8 */
  t1 = fe_mul( z, t1 );                     /* 9 */
  t0 = fe_mul( t0, t1 );                    /* 11 */
  fe t2 = fe_sq( t0 );                      /* 22 */
  t1 = fe_mul( t1, t2 );                    /* 2^5 - 1 */
  t2 = fe_sq_iter( t1, 5 );  t1 = fe_mul( t2, t1 );     /* 2^10 - 1 */
  t2 = fe_sq_iter( t1, 10 ); t2 = fe_mul( t2, t1 );     /* 2^20 - 1 */
  fe t3 = fe_sq_iter( t2, 20 ); t2 = fe_mul( t3, t2 );  /* 2^40 - 1 */
  t2 = fe_sq_iter( t2, 10 ); t1 = fe_mul( t2, t1 );     /* 2^50 - 1 */
  t2 = fe_sq_iter( t1, 50 ); t2 = fe_mul( t2, t1 );     /* 2^100 - 1 */
  t3 = fe_sq_iter( t2, 100 ); t2 = fe_mul( t3, t2 );    /* 2^200 - 1 */
  t2 = fe_sq_iter( t2, 50 ); t1 = fe_mul( t2, t1 );     /* 2^250 - 1 */
  t1 = fe_sq_iter( t1, 5 );                              /* 2^255 - 2^5 */
  return fe_mul( t1, t0 );                               /* 2^255 - 21 */
}

/* canonical little-endian encoding (limb offsets 0,26,51,...,230) */
__device__ void
fe_tobytes_w( u32 w[8], fe const & f ) {
  i32 h[10];
  fe_reduce( h, f );
  int const off[10] = { 0, 26, 51, 77, 102, 128, 153, 179, 204, 230 };
  _Pragma("unroll") for( int k=0; k<8; k++ ) w[k] = 0u;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    u32 v = (u32)h[k];
    int wi = off[k] >> 5, sh = off[k] & 31;
    w[wi] |= v << sh;
    if( sh && wi < 7 ) w[wi+1] |= v >> (32 - sh);
  }
}

struct gp3 { fe X, Y, Z, T; };

/* h += sign*BASE[j][|d|-1] (mixed addition with a Duif-form table entry) */
__device__ __forceinline__ void
madd_base( gp3 & h, int j, int d ) {
  if( !d ) return;
  int a = d < 0 ? -d : d;
  fe ypx, ymx, xy2d;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    ypx.v[k] = BASE[j][a-1][0][k]; ymx.v[k] = BASE[j][a-1][1][k]; xy2d.v[k] = BASE[j][a-1][2][k];
  }
  if( d < 0 ) { fe t = ypx; ypx = ymx; ymx = t; xy2d = fe_neg( xy2d ); }
  fe A = fe_mul( fe_add( h.Y, h.X ), ypx );
  fe Bv = fe_mul( fe_sub( h.Y, h.X ), ymx );
  fe C = fe_mul( xy2d, h.T );
  fe D = fe_add( h.Z, h.Z );
  fe X3 = fe_sub( A, Bv ), Y3 = fe_add( A, Bv ), Z3 = fe_add( D, C ), T3 = fe_sub( D, C );
  h.X = fe_mul( X3, T3 ); h.Y = fe_mul( Y3, Z3 ); h.Z = fe_mul( Z3, T3 ); h.T = fe_mul( X3, Y3 );
}

__device__ __forceinline__ void
dbl( gp3 & h ) {
  fe XX = fe_sq( h.X ), YY = fe_sq( h.Y ), B = fe_sqn<2>( h.Z ), A = fe_sq( fe_add( h.X, h.Y ) );
  fe Y3 = fe_add( YY, XX ), Z3 = fe_sub( YY, XX ), X3 = fe_sub( A, Y3 ), T3 = fe_sub( B, Z3 );
  h.X = fe_mul( X3, T3 ); h.Y = fe_mul( Y3, Z3 ); h.Z = fe_mul( Z3, T3 ); h.T = fe_mul( X3, Y3 );
}

/* [s]B for a 256-bit scalar s (8 LE words, s < 2^255), encoded */
__device__ void
scalarmult_base_enc( u32 enc[8], u32 const s[8] ) {
  /* signed radix-16 digits e[0..63] in [-8,8], packed 4 per word as int8 */
  u32 dig[16];
  int carry = 0;
  _Pragma("unroll") for( int i=0; i<64; i++ ) {
    int e = (int)((s[i >> 3] >> (4 * (i & 7))) & 15u) + carry;
    carry = (e + 8) >> 4;
    e -= carry << 4;
    if( i == 63 ) e += carry << 4;             /* s < 2^255: the top digit absorbs the final carry */
    if( (i & 3) == 0 ) dig[i >> 2] = 0u;
    dig[i >> 2] |= ((u32)(e & 0xff)) << (8 * (i & 3));
  }
  auto D = [&]( int i ) -> int { return (int)(i8)(dig[i >> 2] >> (8 * (i & 3))); };
  gp3 h; h.X = fe_zero(); h.Y = fe_one(); h.Z = fe_one(); h.T = fe_zero();
  for( int i=1; i<64; i+=2 ) madd_base( h, i >> 1, D( i ) );
  dbl( h ); dbl( h ); dbl( h ); dbl( h );
  for( int i=0; i<64; i+=2 ) madd_base( h, i >> 1, D( i ) );
  fe zi = fe_invert( h.Z );
  fe x = fe_mul( h.X, zi ), y = fe_mul( h.Y, zi );
  fe_tobytes_w( enc, y );
  i32 hx[10]; fe_reduce( hx, x );
  enc[7] |= ((u32)hx[0] & 1u) << 31;
}

/* (r + k a) mod L for canonical r, k, a < L (8 LE words each) */
__device__ void
sc_muladd( u32 out[8], u32 const k[8], u32 const a[8], u32 const r[8] ) {
  u32 prod[16];
  _Pragma("unroll") for( int i=0; i<16; i++ ) prod[i] = 0u;
  _Pragma("unroll") for( int i=0; i<8; i++ ) {
    u64 c = 0;
    _Pragma("unroll") for( int j=0; j<8; j++ ) {
      u64 t = (u64)k[i] * a[j] + prod[i+j] + c;
      prod[i+j] = (u32)t; c = t >> 32;
    }
    prod[i+8] = (u32)c;
  }
  u64 c = 0;
  _Pragma("unroll") for( int i=0; i<16; i++ ) {
    u64 t = (u64)prod[i] + (i < 8 ? r[i] : 0u) + c;
    prod[i] = (u32)t; c = t >> 32;
  }
  sc_reduce( out, prod );
}

} /* namespace */

__global__ void __launch_bounds__(64)
k_sign( u32 n, u8 const * __restrict__ prv, u32 const * __restrict__ moff, u32 const * __restrict__ msz,
        u8 const * __restrict__ blob, u8 * __restrict__ pub, u8 * __restrict__ sig ) {
  u32 i = blockIdx.x * 64u + threadIdx.x;
  if( i >= n ) return;
  u32 const * P = (u32 const *)(prv + 32UL*i);                      /* 32-aligned records */
  u64 seed[4];
  _Pragma("unroll") for( int k=0; k<4; k++ ) seed[k] = ((u64)P[2*k+1] << 32) | P[2*k];
  u64 st[8];
  sha512_pm<4>( st, seed, (u8 const *)0, 0u );
  u32 hw[16]; digest_words( hw, st );
  u32 a[8];
  _Pragma("unroll") for( int k=0; k<8; k++ ) a[k] = hw[k];
  a[0] &= ~7u; a[7] &= 0x7fffffffu; a[7] |= 0x40000000u;          /* clamp (RFC 8032 s5.1.5) */
  u32 A[8]; scalarmult_base_enc( A, a );
  u32 * PO = (u32 *)(pub + 32UL*i);
  _Pragma("unroll") for( int k=0; k<8; k++ ) PO[k] = A[k];

  u8 const * M = blob + moff[i];
  u32 sz = msz[i];
  u64 pre[4];
  _Pragma("unroll") for( int k=0; k<4; k++ ) pre[k] = ((u64)hw[8+2*k+1] << 32) | hw[8+2*k];
  sha512_pm<4>( st, pre, M, sz );
  u32 rw[16]; digest_words( rw, st );
  u32 r[8]; sc_reduce( r, rw );
  u32 R[8]; scalarmult_base_enc( R, r );

  u64 ra[8];
  _Pragma("unroll") for( int k=0; k<4; k++ ) { ra[k] = ((u64)R[2*k+1] << 32) | R[2*k]; ra[4+k] = ((u64)A[2*k+1] << 32) | A[2*k]; }
  sha512_pm<8>( st, ra, M, sz );
  u32 kw[16]; digest_words( kw, st );
  u32 kk[8]; sc_reduce( kk, kw );
  /* a itself may exceed L: reduce it first (ka mod L is unchanged) */
  u32 aw[16];
  _Pragma("unroll") for( int k=0; k<8; k++ ) { aw[k] = a[k]; aw[8+k] = 0u; }
  u32 ar[8]; sc_reduce( ar, aw );
  u32 S[8]; sc_muladd( S, kk, ar, r );
  u32 * SO = (u32 *)(sig + 64UL*i);
  _Pragma("unroll") for( int k=0; k<8; k++ ) { SO[k] = R[k]; SO[8+k] = S[k]; }
}

int
fd_amd_launch_sign( uint32_t n, uint8_t const * d_prv, uint32_t const * d_off, uint32_t const * d_sz,
                    uint8_t const * d_blob, uint8_t * d_pub, uint8_t * d_sig, hipStream_t stream ) {
  if( !n ) return 0;
  hipLaunchKernelGGL( k_sign, dim3((n + 63u)/64u), dim3(64), 0, stream, n, d_prv, d_off, d_sz, d_blob, d_pub, d_sig );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
