/* firedancer_amd/csrc/fd_ed25519_kernels.hip
 *
 * The ed25519 verify pipeline as three CDNA4 kernels, one signature per
 * lane (64 signatures per wave64):
 *
 *   k_prep   s-range check (fd_ed25519_user.c:362-393), SHA-512(R||A||M)
 *            (user.c:411-413), reduction mod L (user.c:414), signed
 *            sliding-window recoding of h and s (avx/fd_ed25519_ge.c:378-400)
 *            -> digit planes in HBM.
 *   k_decomp 2-point decompression (avx/fd_ed25519_ge.c:221-299), one lane
 *            per point (A and R of a signature on adjacent lanes), then the
 *            A := -A negation (user.c:406-407).
 *   k_dsm    [h](-A) + [s]B with the reference's AVX op flow
 *            (avx/fd_ed25519_ge.c:408-527) run as a per-lane op stream (no
 *            predicated adds; the Ai table in a per-lane HBM slab, the Bi
 *            table in LDS) and the limb compare (user.c:417-425).
 *
 * Verdict per signature: err[i] in {0,-1,-2,-3}; 1 marks "still pending"
 * between kernels.
 *
 * Workspace layout (N = n rounded up to 64; every plane is [element][N] so
 * that the 64 lanes of a wave touch 64 consecutive elements):
 *   dig  : u16    [N][256]     slide digit pairs (a_p = h digit, b_p = s digit) as
 *                              int8 (low, high), contiguous per lane
 *   top  : int32  [N]          highest nonzero digit position (-1 if none)
 *   A    : int32  [30][N]      -A.X, A.Y, -A.T   (A.Z == 1)
 *   R    : int32  [20][N]      R.X, R.Y
 *   Ai   : int32  [N][8][4][12] cached odd multiples of -A, rows [Z,Y-X,Y+X,2dT] of
 *                              10 limbs padded to 12: per-lane contiguous (one ADD gathers
 *                              192 contiguous bytes instead of 40 scattered dwords)
 *   st   : uint32 [3][N]       work statistics (iterations, nnz h, nnz s)
 *   ds   : uint8  [N][2]       decompression status of A / R (0 ok, 1 not on the
 *                              curve); k_dsm turns a failure into -2
 *   tag  : uint64 [N]          dedup tag: the first 8 bytes (little endian) of
 *                              SHA-512(R||A||M), 0 when the s check rejected
 *                              (app/frank/README.md:107-110: verify yields a
 *                              secure hash for dedup at no extra cost)
 */

#include "fd_ed25519_dev.h"
#include "fd_ed25519_kernels.h"
#include "fd_txn_dev.h"
#include <stdlib.h>

typedef int8_t i8;
typedef uint16_t u16;

/* ------------------------------------------------------------------ */
/* workspace                                                            */

__host__ __device__ constexpr size_t ws_al( size_t x ) { return (x + 255UL) & ~(size_t)255UL; }

/* constexpr so that a kernel with a fixed N (k_tile_persist, N = 64) folds
   every plane offset into an immediate */
__host__ __device__ constexpr ws_layout_t
ws_layout_const( size_t n ) {
  ws_layout_t L = {};
  size_t N = (n + 63UL) & ~(size_t)63UL; if( !N ) N = 64;
  size_t o = 0;
  L.N   = N;
  L.dig = o; o = ws_al( o + 2UL*128UL*N );   /* u16 [N][128] digit events: h [0,64), s [64,128) */
  L.evn = o; o = ws_al( o + 4UL*N );          /* u32 [N]: h event count | s count << 8 */
  L.top = o; o = ws_al( o + 4UL*N );
  L.A   = o; o = ws_al( o + 4UL*30UL*N );
  L.R   = o; o = ws_al( o + 4UL*20UL*N );
  L.Ai  = o; o = ws_al( o + 4UL*384UL*N );
  L.st  = o; o = ws_al( o + 4UL*3UL*N );
  L.tag = o; o = ws_al( o + 8UL*N );
  L.ds  = o; o = ws_al( o + 2UL*N );
  L.init = o; o = ws_al( o + 16UL*N );        /* uint4 [N]: k_dsmp op-stream start (k_ai) */
  L.ctr  = o; o = ws_al( o + 16UL );          /* u32 k_dsmp work counter (zeroed by k_ai) | u32 k_dsmp guard flag */
  L.total = o;
  return L;
}

ws_layout_t
fd_amd_ws_layout( size_t n ) {
  return ws_layout_const( n );
}

/* ------------------------------------------------------------------ */
/* k_prep                                                               */

/* fd_ed25519_ge_slide (avx/fd_ed25519_ge.c:378-400) on a 256-bit register
   shift window: bit 0 of w0 is always position `pos`, so every look-ahead
   index is static.  The reference's carry loop "for k>=i+b: if !r[k] set,
   break; else clear" is the big-integer increment B += 2^(i+b).  Scalars
   are < 2^253 so no carry leaves position 255.  emit(pos, digit). */
template<typename EMIT>
__device__ __forceinline__ void
slide_reg( u32 const a[8], EMIT emit ) {
  u64 w0 = ((u64)a[1] << 32) | a[0], w1 = ((u64)a[3] << 32) | a[2];
  u64 w2 = ((u64)a[5] << 32) | a[4], w3 = ((u64)a[7] << 32) | a[6];
  int pos = 0;
  while( (w0 | w1 | w2 | w3) != 0UL ) {
    /* skip to the next set bit */
    while( w0 == 0UL ) { w0 = w1; w1 = w2; w2 = w3; w3 = 0UL; pos += 64; }
    int tz = __builtin_ctzll( w0 );
    if( tz ) {
      w0 = (w0 >> tz) | (w1 << (64 - tz));
      w1 = (w1 >> tz) | (w2 << (64 - tz));
      w2 = (w2 >> tz) | (w3 << (64 - tz));
      w3 = (w3 >> tz);
      pos += tz;
    }
    int r = 1; w0 &= ~1UL;
    bool stop = false;
    _Pragma("unroll")
    for( int b=1; b<=6; b++ ) {
      bool bit = !stop && ((w0 >> b) & 1UL);
      if( bit ) {
        if( r + (1 << b) <= 15 ) { r += 1 << b; w0 &= ~(1UL << b); }
        else if( r - (1 << b) >= -15 ) {
          r -= 1 << b;
          u64 n0 = w0 + (1UL << b);                 /* B += 2^b (carry chain) */
          u64 c  = n0 < w0;
          w0 = n0; w1 += c; c = c && w1 == 0UL; w2 += c; c = c && w2 == 0UL; w3 += c;
        } else stop = true;
      }
    }
    emit( pos, r );
    /* step past pos */
    w0 = (w0 >> 1) | (w1 << 63); w1 = (w1 >> 1) | (w2 << 63); w2 = (w2 >> 1) | (w3 << 63); w3 >>= 1;
    pos += 1;
  }
}

__device__ __forceinline__ void
prep_body( u32 i, u32 n, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
           u32 const * __restrict__ msg_off, u32 const * __restrict__ msg_sz,
           u8 const * __restrict__ blob, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L,
           i8 const * __restrict__ skip ) {
  if( i >= n ) return;
  if( skip && skip[i] ) {   /* slot of a transaction that failed to parse (fd_txn_kernels.hip) */
    ((int *)(ws + L.top))[i] = -1;
    ((u32 *)(ws + L.evn))[i] = 0u;
    ((u64 *)(ws + L.tag))[i] = 0UL;
    err[i] = (i8)skip[i];
    return;
  }

  /* R || A as 16 LE dwords (sig / pub records are 64- / 32-byte aligned) */
  uint4 const * S4 = (uint4 const *)(sig + 64UL*i);
  uint4 const * P4 = (uint4 const *)(pub + 32UL*i);
  uint4 r0 = S4[0], r1 = S4[1], s0 = S4[2], s1 = S4[3], a0 = P4[0], a1 = P4[1];
  u32 sw[8] = { s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w };

  /* s-range check with the reference's early "return 0" window (user.c:373-379) */
  int code = 1;   /* pending */
  {
    u32 s31 = sw[7] >> 24;
    if( s31 > 0x10u ) code = -1;
    else if( s31 == 0x10u ) {
      if( (sw[4] | sw[5] | sw[6] | (sw[7] & 0x00ffffffu)) != 0u ) code = 0;   /* s[16..30] != 0 */
      else {
        /* s[0..15] vs l_low, compared from the top byte: s < l_low passes */
        u32 const ll[4] = { 0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu };
        bool less = false, decided = false;
        _Pragma("unroll") for( int k=3; k>=0; k-- ) {
          if( !decided && sw[k] != ll[k] ) { less = sw[k] < ll[k]; decided = true; }
        }
        if( !less ) code = -1;
      }
    }
  }

  u64 * evw = (u64 *)(ws + L.dig) + (size_t)i*32u;   /* this signature's event row: 16 words h, 16 words s */
  u32 nh = 0u, ns = 0u;
  int top = -1;
  u64 tag = 0UL;
  u64 st[8] = FD_AMD_SHA512_H0;
  if( code >= 0 ) {   /* pending, or accepted by the s window (the tag is still the hash) */
    u32 sz = msg_sz[i];
    u8 const * M = blob + msg_off[i];
    u32 nblk = (64u + sz + 17u + 127u) / 128u;
    u64 const ra[8] = { ((u64)r0.y << 32) | r0.x, ((u64)r0.w << 32) | r0.z, ((u64)r1.y << 32) | r1.x, ((u64)r1.w << 32) | r1.z,
                        ((u64)a0.y << 32) | a0.x, ((u64)a0.w << 32) | a0.z, ((u64)a1.y << 32) | a1.x, ((u64)a1.w << 32) | a1.z };
    u64 bitlen = (u64)(64u + sz) << 3;
    for( u32 blk=0; blk<nblk; blk++ ) {
      u64 w[16];
      _Pragma("unroll") for( int k=0; k<16; k++ ) {
        u32 kk = blk*16u + (u32)k;                 /* stream word index */
        u64 v;
        if( kk < 8u ) v = ra[k & 7];               /* only block 0 */
        else          v = msg_word( M, sz, 8u*(kk - 8u) );
        v = bswap64( v );
        if( blk == nblk-1u && k == 15 ) v |= bitlen;
        w[k] = v;
      }
      sha512_compress( st, w );
    }
    tag = bswap64( st[0] );
  }
  if( code == 1 ) {
    u32 hd[16];
    _Pragma("unroll") for( int a=0; a<8; a++ ) {
      hd[2*a]   = __builtin_bswap32( (u32)(st[a] >> 32) );
      hd[2*a+1] = __builtin_bswap32( (u32)st[a] );
    }
    u32 h[8];
    sc_reduce( h, hd );

    /* digits as sparse EVENTS, u16 = position | digit << 8, ascending, four
       per 64-bit word (the consumer walks them from the top).  Consecutive
       nonzero digits of the slide are >= 5 positions apart (bits i+1..i+4
       are always absorbed), so a 253-bit scalar has at most 52 events: the
       16-word halves never overflow.  Only the words holding events are
       written -- no dense 256-entry row, no zero fill. */
    u64 buf = 0UL;
    slide_reg( h, [&]( int pos, int r ) {
      buf |= (u64)((u32)pos | ((u32)(u8)(i8)r << 8)) << (16u*(nh & 3u));
      if( !(++nh & 3u) ) { evw[(nh >> 2) - 1u] = buf; buf = 0UL; }
      top = max( top, pos );
    } );
    if( nh & 3u ) evw[nh >> 2] = buf;
    buf = 0UL;
    slide_reg( sw, [&]( int pos, int r ) {
      buf |= (u64)((u32)pos | ((u32)(u8)(i8)r << 8)) << (16u*(ns & 3u));
      if( !(++ns & 3u) ) { evw[16u + (ns >> 2) - 1u] = buf; buf = 0UL; }
      top = max( top, pos );
    } );
    if( ns & 3u ) evw[16u + (ns >> 2)] = buf;
  }
  ((u32 *)(ws + L.evn))[i] = nh | (ns << 8);
  ((int *)(ws + L.top))[i] = top;
  ((u64 *)(ws + L.tag))[i] = tag;
  err[i] = (i8)code;
}

__global__ void __launch_bounds__(64)
k_prep( u32 n, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
        u32 const * __restrict__ msg_off, u32 const * __restrict__ msg_sz,
        u8 const * __restrict__ blob, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L,
        i8 const * __restrict__ skip ) {
  prep_body( blockIdx.x * 64u + threadIdx.x, n, pub, sig, msg_off, msg_sz, blob, err, ws, L, skip );
}

/* ------------------------------------------------------------------ */
/* k_decomp: lane 2i -> A = pub[i], lane 2i+1 -> R = sig[i][0:32]       */

#define FD_DECOMP_WAVES 2   /* k_decomp / k_front occupancy target (222 VGPRs) */
/* one point per lane: t = 2i (A = pub[i]) or 2i+1 (R = sig[i][0:32]).
   Independent of k_prep (reads no verdict) when `gate` is 0, so the two
   can run concurrently (k_front); with gate, signatures k_prep already
   decided are skipped. */
__device__ __forceinline__ void
decomp_body( u32 t, u32 n, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
             i8 const * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, bool gate ) {
  u32 i = t >> 1; u32 which = t & 1u;
  if( i >= n ) return;
  if( gate && err[i] != 1 ) return;
  u8 * ds = ws + L.ds;
  /* the point as 8 LE dwords in two 16-B loads (sig / pub records are 64- /
     32-byte aligned, as k_prep reads them; on the latency path these are
     reads over PCIe from host memory, so fewer, wider loads) */
  uint4 const * src = (uint4 const *)(which ? (sig + 64UL*i) : (pub + 32UL*i));
  uint4 const s0 = src[0], s1 = src[1];
  u32 const w[8] = { s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w };

  fe const D = {FD_AMD_FE_D};
  fe const SQRTM1 = {FD_AMD_FE_SQRTM1};

  fe Y = fe_frombytes( w );
  fe u = fe_sq( Y );
  fe v = fe_mul( u, D );
  u.v[0] -= 1;                      /* u = y^2-1 */
  v.v[0] += 1;                      /* v = dy^2+1 */
  fe v3 = fe_sq( v ); v3 = fe_mul( v3, v );          /* v^3 */
  fe x = fe_sq( v3 ); x = fe_mul( x, v ); x = fe_mul( x, u );   /* uv^7 */
  x = fe_pow22523( x );
  x = fe_mul( x, v3 ); x = fe_mul( x, u );          /* uv^3 (uv^7)^((p-5)/8) */
  fe vxx = fe_sq( x ); vxx = fe_mul( vxx, v );
  fe chk = fe_sub( vxx, u );
  if( fe_isnonzero( chk ) ) {
    chk = fe_add( vxx, u );
    if( fe_isnonzero( chk ) ) { ds[2u*i + which] = 1u; return; }
    x = fe_mul( x, SQRTM1 );
  }
  if( fe_isnegative( x ) != (int)(w[7] >> 31) ) x = fe_neg( x );
  fe T = fe_mul( x, Y );

  size_t N = L.N;
  if( !which ) {
    i32 * A = (i32 *)(ws + L.A);
    fe nx = fe_neg( x ), nt = fe_neg( T );     /* A := -A (user.c:406-407) */
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      A[(size_t)(k   )*N + i] = nx.v[k];
      A[(size_t)(10+k)*N + i] = Y.v[k];
      A[(size_t)(20+k)*N + i] = nt.v[k];
    }
  } else {
    i32 * R = (i32 *)(ws + L.R);
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      R[(size_t)(k   )*N + i] = x.v[k];
      R[(size_t)(10+k)*N + i] = Y.v[k];
    }
  }
  ds[2u*i + which] = 0u;
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FD_DECOMP_WAVES)))
k_decomp( u32 n, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
          i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L ) {
  decomp_body( blockIdx.x * 64u + threadIdx.x, n, pub, sig, err, ws, L, true );
}

/* k_front: k_prep and k_decomp as ONE launch, blocks [0, nbp) hashing and
   blocks [nbp, 3 nbp) decompressing, concurrently (latency path: a small
   batch does not fill the GPU, so the two stages overlap instead of
   queueing). */
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FD_DECOMP_WAVES)))
k_front( u32 n, u32 nbp, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
         u32 const * __restrict__ msg_off, u32 const * __restrict__ msg_sz,
         u8 const * __restrict__ blob, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L,
         i8 const * __restrict__ skip ) {
  if( blockIdx.x < nbp ) prep_body( blockIdx.x * 64u + threadIdx.x, n, pub, sig, msg_off, msg_sz, blob, err, ws, L, skip );
  else                   decomp_body( (blockIdx.x - nbp) * 64u + threadIdx.x, n, pub, sig, err, ws, L, false );
}

/* ------------------------------------------------------------------ */
/* k_dsm                                                                */

struct p1p1 { fe X, Y, Z, T; };
struct p3   { fe X, Y, Z, T; };

/* p2/p3 doubling, AVX flow (avx/fd_ed25519_ge.c:493-498):
   [(X+Y)^2, Y^2, X^2, 2Z^2] -> [a-b-c, b+c, b-c, d-b+c] */
__device__ __forceinline__ p1p1
ge_dbl( fe const & X, fe const & Y, fe const & Z ) {
  fe a = fe_sqn<1>( fe_add( X, Y ) );
  fe b = fe_sqn<1>( Y );
  fe c = fe_sqn<1>( X );
  fe d = fe_sqn<2>( Z );
  p1p1 t;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    t.X.v[k] = a.v[k] - b.v[k] - c.v[k];
    t.Y.v[k] = b.v[k] + c.v[k];
    t.Z.v[k] = b.v[k] - c.v[k];
    t.T.v[k] = d.v[k] - b.v[k] + c.v[k];
  }
  return t;
}

/* p1p1 -> p3, AVX lanes Z=Z*T, Y=Y*Z, X=X*T, T=X*Y (:502-504) */
__device__ __forceinline__ p3
ge_p1p1_to_p3( p1p1 const & t ) {
  p3 u;
  /* operand order chosen so the products share pre-multiples: g in {T, Y}
     (x19) and f in {Z, X} (x2); mul is commutative at the integer level */
  u.Z = fe_mul( t.Z, t.T );
  u.Y = fe_mul( t.Z, t.Y );
  u.X = fe_mul( t.X, t.T );
  u.T = fe_mul( t.X, t.Y );
  return u;
}

/* the same products as interleaved, carry-folded pairs (fe_mul_fold2w) */
__device__ __forceinline__ p3
ge_p1p1_to_p3_fold( p1p1 const & t ) {
  p3 u;
  fe_mul_fold2w( u.Z, t.Z, t.T, u.Y, t.Z, t.Y );
  fe_mul_fold2w( u.X, t.X, t.T, u.T, t.X, t.Y );
  return u;
}

/* the add/sub (and madd/msub when qZ==1) body (:505-518).  qZ_one: the
   table Z lane is 1 (base-point table) so Z*1 is the carry chain. */
template<bool QZ_ONE>
__device__ __forceinline__ p1p1
ge_add( p3 const & u, fe const & qZ, fe const & qYmX, fe const & qYpX, fe const & qT2d, bool neg ) {
  fe ymx = fe_sub( u.Y, u.X ), ypx = fe_add( u.Y, u.X );
  fe ZZ = QZ_ONE ? fe_mul_one( u.Z ) : fe_mul( u.Z, qZ );
  fe MM = fe_mul( ymx, neg ? qYpX : qYmX );
  fe PP = fe_mul( ypx, neg ? qYmX : qYpX );
  fe TT = fe_mul( u.T, qT2d );
  p1p1 t;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    i32 z2 = ZZ.v[k] + ZZ.v[k];
    t.X.v[k] = PP.v[k] - MM.v[k];
    t.Y.v[k] = PP.v[k] + MM.v[k];
    i32 zp = z2 + TT.v[k], zm = z2 - TT.v[k];
    t.Z.v[k] = neg ? zm : zp;
    t.T.v[k] = neg ? zp : zm;
  }
  return t;
}

/* p3 -> cached with the AVX "x[1,1,1,2d]" multiply (:440-446, :475-479) */
__device__ __forceinline__ void
ge_to_cached( fe & cZ, fe & cYmX, fe & cYpX, fe & cT2d, p3 const & u ) {
  fe const D2 = {FD_AMD_FE_D2};
  fe Z1 = fe_mul_one( u.Z ), Y1 = fe_mul_one( u.Y ), X1 = fe_mul_one( u.X );
  cT2d = fe_mul( u.T, D2 );
  cZ = Z1; cYmX = fe_sub( Y1, X1 ); cYpX = fe_add( Y1, X1 );
}

/* Base-point table in LDS, rows [Z(=1), Y-X, Y+X, 2dT] x 10 limbs per entry
   (table/fd_ed25519_ge_bi_precomp_avx.c:30-112 lane order). */
__constant__ static i32 const BI_TABLE[8][3][10] = FD_AMD_BI_PRECOMP;   /* rows y+x, y-x, 2dxy */

/* The base-point table in the Ai slab's row layout (rows [Z = 1 | Y-X |
   Y+X | 2dT] x 12 limbs, 10 used): an ADD-A row comes from the signature's
   Ai slab, an ADD-B row from here, with the same three 16-B loads through
   one generic pointer.  Filled by the wave before the DSM bodies run. */
__device__ __forceinline__ void
bi12_fill( i32 (* __restrict__ bi12)[48] ) {
  for( int k=threadIdx.x & 63; k<8*48; k+=64 ) {
    int e = k / 48, c = (k % 48) / 12, l = k % 12;
    i32 v = 0;
    if( l < 10 ) {
      if( c == 0 ) v = (l == 0);
      else if( c == 1 ) v = BI_TABLE[e][1][l];
      else if( c == 2 ) v = BI_TABLE[e][0][l];
      else v = BI_TABLE[e][2][l];
    }
    bi12[e][k % 48] = v;
  }
}

/* Branch-free per-lane select: v_cndmask_b32 on a wave lane mask (ballot).
   Plain ?: on the op-stream selects lets LLVM re-form divergent branches
   around the field muls (both sides then run with copies in between). */
__device__ __forceinline__ i32 vsel( u64 m, i32 t, i32 f ) {
  i32 r;
  asm( "v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m) );
  return r;
}

enum { PH_DBL = 0, PH_ADDA = 1, PH_ADDB = 2, PH_FIN = 3, PH_DONE = 4 };

/* One scalar's slide-digit events (k_prep), walked from the top.  The
   kernel first copies the signature's event row into LDS, so a pop is one
   ds_read_u16 (an LDS wait, not a memory wait, when it lands in a
   divergent branch). */
struct evq {
  u16 const * e;     /* the list in LDS */
  int j, pos, dig;   /* current event index (descending), its position (-1: none left) and digit */
  __device__ __forceinline__ void load() {
    u32 x = (j >= 0) ? (u32)e[j] : 0xffffu;
    pos = (j >= 0) ? (int)(x & 0xffu) : -1;
    dig = (int)(i8)(x >> 8);
  }
  __device__ __forceinline__ void init( u16 const * e_, int n ) { e = e_; j = n - 1; load(); }
  __device__ __forceinline__ void pop() { j--; load(); }
};

/* k_dsm: [h](-A) + [s]B as a per-lane STEP STREAM.
 *
 * The reference loop (avx/fd_ed25519_ge.c:488-523) is, per bit position p
 * from the top:  DBL ; [ADD Ai[|a_p|/2] if a_p] ; [MADD Bi[|b_p|/2] if b_p] ;
 * with p1p1->p3 before every add and p1p1->p2 before every doubling.
 * p1p1->p2 computes exactly the first three products of p1p1->p3
 * (X*T, Y*Z, Z*T), so every op of the stream has the same shape:
 *
 *     u  = p1p1->p3(t)                        4 field muls
 *     m0..m3 = op-specific 4 field muls        DBL: (X+Y)^2, Y^2, X^2, Z*2Z
 *                                              ADD: Z*qZ, (Y-X)*qM, (Y+X)*qP, T*qT
 *     t  = op-specific linear mix
 *
 * so each lane walks ITS OWN op sequence and every step does 8 useful field
 * muls on every lane (no predicated adds).  Bit-exactness: sq(f) == mul(f,f),
 * sq2(f) == mul(f,f+f) and mul(f,1) == carry(f) at the integer level
 * (SURVEY.md s7 "Measured equivalences"), so a uniform mul is the
 * reference's sq / sq2 / madd Z*1 bit for bit.  A lane whose last op is done
 * takes one more step (PH_FIN): its p1p1->p2 result is R', compared with
 * the limb memcmp of fd_ed25519_user.c:417-425, then it idles (PH_DONE).
 */
/* Streaming tile (k_tile_persist): the wave's issue priority follows the
   age of its chunk, claimed at s_memrealtime tc (100 MHz): 0 below 0.4 ms,
   then one level per 0.4 ms.  Two waves share a SIMD, and at equal priority
   the arbiter prefers the older WAVE -- in a persistent kernel always the
   same one, so one wave of each pair ran its chunks ~1.1 ms and the other
   ~5 ms, and the tile publishes in order behind the slow ones.  By chunk age
   the older CHUNK goes first.  Scalar only (SGPRs, s_setprio). */
__device__ __forceinline__ void
tile_age_prio( u64 tc, u32 & lvl ) {
  u64 const el = __builtin_amdgcn_s_memrealtime() - tc;
  u32 const want = el < 40000UL ? 0u : el < 80000UL ? 1u : el < 120000UL ? 2u : 3u;
  if( want == lvl ) return;
  lvl = want;
  if( want == 1u )      __builtin_amdgcn_s_setprio( 1 );
  else if( want == 2u ) __builtin_amdgcn_s_setprio( 2 );
  else if( want == 3u ) __builtin_amdgcn_s_setprio( 3 );
  else                  __builtin_amdgcn_s_setprio( 0 );
}

__device__ __forceinline__ void
dsm_lane_body( u32 i, u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats,
               i32 (* __restrict__ bi)[48], u64 (* __restrict__ evl)[33], u64 tc = 0UL ) {
  /* bi: the base-point table in the Ai slab's row layout (bi12_fill), so
     ADD-A and ADD-B operands load alike */
  bool act = (i < n) && (err[i] == 1);
  if( act && (ws[L.ds + 2u*i] | ws[L.ds + 2u*i + 1u]) ) { err[i] = (i8)-2; act = false; }   /* A or R undecodable */
  size_t N = L.N;
  u32 ii = (i < n) ? i : 0u;
  i32 * Ail = (i32 *)(ws + L.Ai) + (size_t)ii*384u;   /* this lane's 8 x 4 x 12 table */

  /* -A (p3, Z = 1) and its odd multiples Ai (:423-481) -> HBM */
  {
    p3 A;
    i32 const * Aw = (i32 const *)(ws + L.A);
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      A.X.v[k] = act ? Aw[(size_t)(k   )*N + ii] : 0;
      A.Y.v[k] = act ? Aw[(size_t)(10+k)*N + ii] : (k==0);
      A.T.v[k] = act ? Aw[(size_t)(20+k)*N + ii] : 0;
      A.Z.v[k] = (k==0);
    }
    fe cZ, cYmX, cYpX, cT2d;
    ge_to_cached( cZ, cYmX, cYpX, cT2d, A );
#   define AI_ROW( e, r, f ) do {                                                   \
      int4 * d_ = (int4 *)(Ail + (e)*48 + (r)*12);                                  \
      d_[0] = make_int4( f.v[0], f.v[1], f.v[2], f.v[3] );                          \
      d_[1] = make_int4( f.v[4], f.v[5], f.v[6], f.v[7] );                          \
      d_[2] = make_int4( f.v[8], f.v[9], 0, 0 );                                    \
    } while(0)
#   define AI_STORE( e ) do { AI_ROW( e, 0, cZ ); AI_ROW( e, 1, cYmX ); AI_ROW( e, 2, cYpX ); AI_ROW( e, 3, cT2d ); } while(0)
    if( act ) AI_STORE( 0 );
    p1p1 t = ge_dbl( A.X, A.Y, A.Z );
    p3 A2 = ge_p1p1_to_p3( t );
    for( int e=0; e<7; e++ ) {
      p1p1 s2 = ge_add<false>( A2, cZ, cYmX, cYpX, cT2d, false );
      p3 u = ge_p1p1_to_p3( s2 );
      ge_to_cached( cZ, cYmX, cYpX, cT2d, u );
      if( act ) AI_STORE( e+1 );
    }
#   undef AI_STORE
#   undef AI_ROW
  }

  /* lane state */
  u64 const * dg = (u64 const *)(ws + L.dig) + (size_t)ii*32u;
  int p   = act ? ((int const *)(ws + L.top))[ii] : -1;
  int ph  = act ? (p >= 0 ? PH_DBL : PH_FIN) : PH_DONE;
  evq eva, evb;                                      /* digit events of h and s */
  {
    u64 * row = evl[threadIdx.x];                    /* this wave's event rows (33: bank spread) */
    u32 ne = act ? ((u32 const *)(ws + L.evn))[ii] : 0u;
    u32 wa = ((ne & 0xffu) + 3u) >> 2, wb = (((ne >> 8) & 0xffu) + 3u) >> 2;
    for( u32 k=0; k<wa; k++ ) row[k]       = dg[k];
    for( u32 k=0; k<wb; k++ ) row[16u + k] = dg[16u + k];
    eva.init( (u16 const *)row,        (int)(ne & 0xffu) );
    evb.init( (u16 const *)(row + 16), (int)((ne >> 8) & 0xffu) );
  }
  i32 const * Rw = (i32 const *)(ws + L.R);
  u32 nha = 0, nhb = 0;
  u32 nit = (u32)(p + 1);
  bool qneg = false;

  /* the next op's table operand q = [qZ | qM | qP | qT] (40 limbs) */
  fe q[4];
  _Pragma("unroll") for( int r=0; r<4; r++ ) q[r] = fe_zero();
# define QV( R_, K_ ) q[R_].v[K_]
# define Q_SET( R_, K_, V_ ) ( q[R_].v[K_] = (V_) )
  p1p1 t;   /* identity as a completed point: p1p1->p3 gives (0,1,1,0) */
  t.X = fe_zero(); t.Y = fe_one(); t.Z = fe_one(); t.T = fe_one();
  u32 lvl = 0u;

  for( ;; ) {
    if( tc ) tile_age_prio( tc, lvl );
    /* p1p1 -> p3 (its X,Y,Z are the reference's p1p1 -> p2) */
    p3 u = ge_p1p1_to_p3_fold( t );

    bool fin = (ph == PH_FIN);
    /* R' = u's (X, Y, Z) parks in the lane's own Ai rows (no ADD op reads
       them any more); the compare runs once for the whole wave after the
       loop instead of once per distinct finishing step */
    if( __any( fin ) ) {
      if( fin ) {
        int4 * d_ = (int4 *)Ail;
        d_[0] = make_int4( u.X.v[0], u.X.v[1], u.X.v[2], u.X.v[3] );
        d_[1] = make_int4( u.X.v[4], u.X.v[5], u.X.v[6], u.X.v[7] );
        d_[2] = make_int4( u.X.v[8], u.X.v[9], u.Y.v[0], u.Y.v[1] );
        d_[3] = make_int4( u.Y.v[2], u.Y.v[3], u.Y.v[4], u.Y.v[5] );
        d_[4] = make_int4( u.Y.v[6], u.Y.v[7], u.Y.v[8], u.Y.v[9] );
        d_[5] = make_int4( u.Z.v[0], u.Z.v[1], u.Z.v[2], u.Z.v[3] );
        d_[6] = make_int4( u.Z.v[4], u.Z.v[5], u.Z.v[6], u.Z.v[7] );
        d_[7] = make_int4( u.Z.v[8], u.Z.v[9], 0, 0 );
        ph = PH_DONE;
      }
    }
    if( __all( ph == PH_DONE ) ) break;

    /* op body: 4 field muls with per-lane operands, paired so that DBL and
       ADD share what they can: m0 = (X+Y)*[(X+Y) | qP], m1 = [Y | Y-X]*[Y | qM],
       m2 = [X | Z]*[X | qZ], m3 = [Z | T]*[2Z | qT] */
    bool isD = (ph == PH_DBL);
    u64 mD = __builtin_amdgcn_ballot_w64( isD ), mN = __builtin_amdgcn_ballot_w64( qneg );
    fe m0, m1, m2, m3;
    {
      fe a0, b0, a1, b1, a2, b2, a3, b3;
      _Pragma("unroll") for( int k=0; k<10; k++ ) {
        i32 xy = u.X.v[k] + u.Y.v[k];
        a0.v[k] = xy;                                     b0.v[k] = vsel( mD, xy, QV( 2, k ) );
        a1.v[k] = vsel( mD, u.Y.v[k], u.Y.v[k] - u.X.v[k] ); b1.v[k] = vsel( mD, u.Y.v[k], QV( 1, k ) );
        /* DBL Z*2Z pairs with ADD Z*qZ (shared a = Z), DBL X^2 with ADD T*qT */
        a2.v[k] = u.Z.v[k];                              b2.v[k] = vsel( mD, u.Z.v[k] + u.Z.v[k], QV( 0, k ) );
        a3.v[k] = vsel( mD, u.X.v[k], u.T.v[k] );        b3.v[k] = vsel( mD, u.X.v[k], QV( 3, k ) );
      }
      /* m0, m1, m3 come back with their limbs' rounding offsets b (2^25
         even, 2^24 odd) still added: the mix below folds them into its
         own adds; m2 is exact */
      fe_mul_fold2w<true, true>( m0, a0, b0, m1, a1, b1 );
      fe_mul_fold2w<false, true>( m2, a2, b2, m3, a3, b3 );
    }
    /* lanes that are done (PH_DONE) keep computing on don't-care values:
       nothing they compute is stored.
       DBL mix [a-b-c, b+c, b-c, d-b+c] with a=m0 b=m1 c=m3 d=m2 (m2 = Z*2Z, m3 = X^2);
       ADD mix [P-M, P+M, 2Z+sT, 2Z-sT] with P=m0 M=m1 Z=m2 T=m3, s = neg ? -1 : 1.
       With sA3 = s'*m3 (s' = -1 on DBL lanes, one v_xad_u32), 11 ops per limb:
         X = (m0 - m1) + (sA3 & D)            Y = m1 + (D ? m3 : m0)
         Z = (D ? m1 : 2 m2) + sA3            T = (m2 << (D ? 0 : 2)) - Z
       plus per-lane offset corrections cX (DBL: +b), cZ (ADD: -s b) and the
       uniform -2b of Y, each folded into a v_add3_u32.  Limbs equal the
       reference's wrapping int32 adds (every identity holds mod 2^32). */
    {
      u64 mS = mD | mN;
      i32 Dv = vsel( mD, -1, 0 ), Sv = vsel( mS, -1, 0 ), Sn = vsel( mS, 1, 0 );
      i32 cXe = Dv & (1<<25), cXo = Dv & (1<<24);
      i32 cZe = vsel( mD, 0, vsel( mN, (1<<25), -(1<<25) ) ), cZo = vsel( mD, 0, vsel( mN, (1<<24), -(1<<24) ) );
      i32 const nb2e = (i32)fd_opaque( -(2L<<25) ), nb2o = (i32)fd_opaque( -(2L<<24) );   /* SGPR */
      i32 const sT = vsel( mD, 0, 2 );                     /* T = (m2 << sT) - Z: DBL m2 - Z, ADD 4 m2 - Z */
      _Pragma("unroll") for( int k=0; k<10; k++ ) {
        i32 cX = (k & 1) ? cXo : cXe, cZ = (k & 1) ? cZo : cZe;
        i32 A0 = m0.v[k], A1 = m1.v[k], A2 = m2.v[k], A3 = m3.v[k];
        i32 sA3 = fd_xad( A3, Sv, Sn );
        i32 z2 = A2 + A2;
        i32 Z = fd_add3( vsel( mD, A1, z2 ), sA3, cZ );
        t.X.v[k] = fd_add3( A0 - A1, sA3 & Dv, cX );
        t.Y.v[k] = fd_add3s( A1, vsel( mD, A3, A0 ), (k & 1) ? nb2o : nb2e );
        t.Z.v[k] = Z;
        t.T.v[k] = (i32)((u32)A2 << (u32)sT) - Z;
      }
    }

    /* advance the lane's op stream: the event just executed is consumed; the next op follows from the
       event heads (an event at position p means a digit at p) */
    bool const wasA = ph == PH_ADDA, wasB = ph == PH_ADDB, wasD = ph == PH_DBL;
    eva.j -= (int)wasA; evb.j -= (int)wasB;
    eva.load(); evb.load();
    bool const toA = wasD && eva.pos == p;
    bool const toB = !toA && (wasD || wasA) && evb.pos == p;
    bool const adv = (wasD || wasA || wasB) && !toA && !toB;
    p -= (int)adv;
    ph = toA ? PH_ADDA : toB ? PH_ADDB : adv ? ((p < 0) ? PH_FIN : PH_DBL) : ph;
    nha += (u32)toA; nhb += (u32)toB;

    /* stage the next op's operand into q (consumed after the next
       p1p1->p3, so the load latency hides under 4 field muls); every lane
       loads, only an ADD reads it; ADD-A from the Ai slab, ADD-B from the
       LDS table, through one generic pointer (no branch) */
    {
      int const d = toA ? eva.dig : evb.dig;
      int const e = ((d < 0 ? -d : d) >> 1) & 7;
      qneg = d < 0;
      int4 const * src = toA ? (int4 const *)(Ail + e*48) : (int4 const *)&bi[e][0];
      int rowM = qneg ? 2 : 1, rowP = qneg ? 1 : 2;
#     define Q_ROW( r, c ) do {                                                      \
        int4 x0 = src[3*(c)], x1 = src[3*(c)+1], x2 = src[3*(c)+2];                \
        Q_SET( r, 0, x0.x ); Q_SET( r, 1, x0.y ); Q_SET( r, 2, x0.z ); Q_SET( r, 3, x0.w ); \
        Q_SET( r, 4, x1.x ); Q_SET( r, 5, x1.y ); Q_SET( r, 6, x1.z ); Q_SET( r, 7, x1.w ); \
        Q_SET( r, 8, x2.x ); Q_SET( r, 9, x2.y );                                  \
      } while(0)
      Q_ROW( 0, 0 ); Q_ROW( 1, rowM ); Q_ROW( 2, rowP ); Q_ROW( 3, 3 );
#     undef Q_ROW
    }
  }
# undef QV
# undef Q_SET

  /* the limb compare of fd_ed25519_user.c:417-425, once per wave */
  if( act ) {
    int4 const * s_ = (int4 const *)Ail;
    int4 w0 = s_[0], w1 = s_[1], w2 = s_[2], w3 = s_[3], w4 = s_[4], w5 = s_[5], w6 = s_[6], w7 = s_[7];
    fe X = {{ w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y }};
    fe Y = {{ w2.z, w2.w, w3.x, w3.y, w3.z, w3.w, w4.x, w4.y, w4.z, w4.w }};
    fe Z = {{ w5.x, w5.y, w5.z, w5.w, w6.x, w6.y, w6.z, w6.w, w7.x, w7.y }};
    fe RX, RY;
    _Pragma("unroll") for( int k=0; k<10; k++ ) { RX.v[k] = Rw[(size_t)k*N + ii]; RY.v[k] = Rw[(size_t)(10+k)*N + ii]; }
    fe xZ, yZ;
    fe_mul_fold2w( xZ, Z, RX, yZ, Z, RY );
    bool eq = true;
    _Pragma("unroll") for( int k=0; k<8; k++ ) eq = eq && (xZ.v[k] == X.v[k]) && (yZ.v[k] == Y.v[k]);
    err[i] = (i8)(eq ? 0 : -3);
  }
  if( want_stats && i < n ) {
    u32 * st = (u32 *)(ws + L.st);
    st[i] = act ? nit : 0u; st[N + i] = act ? nha : 0u; st[2*N + i] = act ? nhb : 0u;
  }
}

__global__ void __launch_bounds__(64)
k_dsm( u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats ) {
  __shared__ __attribute__((aligned(16))) i32 bi[8][48];
  __shared__ u64 evl[64][33];
  bi12_fill( bi );
  __syncthreads();
  dsm_lane_body( blockIdx.x * 64u + threadIdx.x, n, err, ws, L, want_stats, bi, evl );
}

/* ------------------------------------------------------------------ */
/* k_dsm4: the same op stream with FOUR lanes per signature (16 signatures
 * per wave), for latency: a small batch leaves most SIMDs idle and the
 * verify time is one lane's sequential op stream.  Every step of the op
 * stream is 4 independent field muls (p1p1->p3) followed by 4 independent
 * muls (the op body); lane q of a quad does the q-th mul of each group and
 * the quad exchanges results with DPP quad_perm broadcasts (the AVX build's
 * 4-lane split of fd_ed25519_ge.c:408-527, mapped to a lane quad instead of
 * a ymm register).  The linear mixes are recomputed by all four lanes, so
 * every lane holds the full point between the two mul groups.  Same field
 * ops in the same order as k_dsm: identical limbs.
 *
 *   p1p1->p3 : q0 Z*T -> u.Z   q1 Z*Y -> u.Y   q2 X*T -> u.X   q3 X*Y -> u.T
 *   DBL body : q0 (X+Y)^2      q1 Y^2          q2 X^2          q3 Z*2Z
 *   ADD body : q0 (Y+X)*qP     q1 (Y-X)*qM     q2 Z*qZ         q3 T*qT
 *   FIN      : q0 Z*RX         q1 Z*RY  (then the limb compare, quad AND)
 * Each lane loads only the table row its mul needs (qP/qM/qZ/qT).
 */
template<int K>
__device__ __forceinline__ i32 qb( i32 v ) {   /* broadcast lane K of each quad: DPP quad_perm(K,K,K,K) */
  return __builtin_amdgcn_mov_dpp( v, K * 0x55, 0xf, 0xf, false );
}
__device__ __forceinline__ void qgather( fe const & mine, fe & f0, fe & f1, fe & f2, fe & f3 ) {
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    f0.v[k] = qb<0>( mine.v[k] ); f1.v[k] = qb<1>( mine.v[k] );
    f2.v[k] = qb<2>( mine.v[k] ); f3.v[k] = qb<3>( mine.v[k] );
  }
}
/* per-lane choice among four values by quad position (lane masks m1,m2:
   bit 0 / bit 1 of q) */
__device__ __forceinline__ i32 q4( u64 m1, u64 m2, i32 a0, i32 a1, i32 a2, i32 a3 ) {
  return vsel( m2, vsel( m1, a3, a2 ), vsel( m1, a1, a0 ) );
}

/* p1p1 -> p3 on a quad: every lane ends with the full u */
__device__ __forceinline__ void
quad_p3( p3 & u, p1p1 const & t, u64 m1, u64 m2 ) {
  fe a, b;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    a.v[k] = vsel( m2, t.X.v[k], t.Z.v[k] );                               /* Z Z X X */
    b.v[k] = vsel( m1, t.Y.v[k], t.T.v[k] );                               /* T Y T Y */
  }
  fe pm = fe_mul( a, b );
  qgather( pm, u.Z, u.Y, u.X, u.T );
}

/* DPP quad_perm with a per-destination source lane: lane q reads lane s_q */
template<int S0, int S1, int S2, int S3>
__device__ __forceinline__ i32 qp( i32 v ) {
  return __builtin_amdgcn_mov_dpp( v, S0 | (S1 << 2) | (S2 << 4) | (S3 << 6), 0xf, 0xf, false );
}

/* Own-coordinate form of the step: after the body mul,
   lane q computes only the ONE p1p1 coordinate C = (Z, T, X, Y)[q] that it
   owns, as x*A + y*B + z*D over three DPP-read products with per-lane
   coefficients in {-1,0,1,2} (three v_mad_i64_i32, low 32 bits = the
   reference's wrapping limb adds), instead of every lane mixing all four
   coordinates.  The next p1p1->p3 then reads its operands a = (Z,Z,X,X)[q],
   b = (T,Y,T,Y)[q] with two quad_perm DPP reads per limb.
     DBL  Z = m1-m2   T = m3-m1+m2   X = m0-m1-m2   Y = m1+m2
     ADD  Z = 2m2+-m3 T = 2m2-+m3    X = m0-m1      Y = m0+m1
   A/B/D sources: q0,q1 <- m1,m2,m3; q2,q3 <- m0,m1,m2. */
__device__ __forceinline__ fe
quad_p3_ownc( fe const & C ) {
  fe a, b;
  _Pragma("unroll") for( int k=0; k<10; k++ ) { a.v[k] = qp<0,0,2,2>( C.v[k] ); b.v[k] = qp<1,3,1,3>( C.v[k] ); }
  return fe_mul_fold1( a, b );
}

__device__ __forceinline__ i32
lin3( i32 x, i32 A, i32 y, i32 B, i32 z, i32 D ) {
  i64 acc = fd_pin( (i64)x * (i64)A );
  acc = fd_pin( (i64)y * (i64)B + acc );
  acc = fd_pin( (i64)z * (i64)D + acc );
  return (i32)acc;
}

__device__ __forceinline__ i32
lin2( i32 x, i32 A, i32 y, i32 B ) {
  i64 acc = fd_pin( (i64)x * (i64)A );
  acc = fd_pin( (i64)y * (i64)B + acc );
  return (i32)acc;
}

__device__ __forceinline__ void
quad_body_ownc( fe & C, fe const & pm, fe const & qrow, bool isD, bool neg, u64 mD, int qd ) {
  /* operand a = c1*P1 + c2*P2 with P1 = quad_perm(2,2,2,0) -> X X X Z and
     P2 = quad_perm(1,1,0,3) -> Y Y Z T:  DBL a = [X+Y, Y, X, Z],
     ADD a = [X+Y, Y-X, Z, T];  b = DBL ? a << (q==3) : qrow */
  i32 c1 = (qd == 0) ? 1 : (qd == 1) ? (isD ? 0 : -1) : (isD ? 1 : 0);
  i32 c2 = (qd <= 1 || !isD) ? 1 : 0;
  i32 sh = (qd == 3) ? 1 : 0;
  asm( "" : "+v"(c1), "+v"(c2) );
  fe a, b;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    i32 av = lin2( c1, qp<2,2,2,0>( pm.v[k] ), c2, qp<1,1,0,3>( pm.v[k] ) );
    a.v[k] = av;
    b.v[k] = vsel( mD, (i32)((u32)av << sh), qrow.v[k] );
  }
  fe m = fe_mul_fold1( a, b );
  i32 s0 = neg ? -1 : 1;
  i32 x = isD ? (qd == 1 ? -1 : (qd == 3 ? 0 : 1)) : (qd >= 2 ? 1 : 0);
  i32 y = isD ? ((qd & 1) ? 1 : -1)               : (qd <= 1 ? 2 : (qd == 2 ? -1 : 1));
  i32 z = isD ? (qd == 0 ? 0 : (qd == 2 ? -1 : 1)) : (qd == 0 ? s0 : (qd == 1 ? -s0 : 0));
  asm( "" : "+v"(x), "+v"(y), "+v"(z) );   /* opaque: keep full v_mad_i64_i32 (no small-range rewrites) */
  _Pragma("unroll") for( int k=0; k<10; k++ )
    C.v[k] = lin3( x, qp<1,1,0,0>( m.v[k] ), y, qp<2,2,1,1>( m.v[k] ), z, qp<3,3,2,2>( m.v[k] ) );
}

/* op body + mix on a quad.  qrow: this lane's table row (ADD); isD/neg per
   lane (uniform within the quad). */
__device__ __forceinline__ void
quad_body( p1p1 & t, p3 const & u, fe const & qrow, u64 mD, u64 mN, u64 m1, u64 m2 ) {
  fe a, b;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    i32 X = u.X.v[k], Y = u.Y.v[k], Z = u.Z.v[k], T = u.T.v[k];
    i32 xy = X + Y;
    i32 aD = q4( m1, m2, xy, Y, X, Z );
    i32 bD = q4( m1, m2, xy, Y, X, Z + Z );
    i32 aA = q4( m1, m2, xy, Y - X, Z, T );
    a.v[k] = vsel( mD, aD, aA );
    b.v[k] = vsel( mD, bD, qrow.v[k] );
  }
  fe m = fe_mul( a, b );
  fe M0, M1, M2, M3;
  qgather( m, M0, M1, M2, M3 );
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    i32 A0 = M0.v[k], A1 = M1.v[k], A2 = M2.v[k], A3 = M3.v[k];
    i32 z2 = A2 + A2;
    i32 dX = A0 - A1 - A2, dY = A1 + A2, dZ = A1 - A2, dT = A3 - A1 + A2;
    i32 aX = A0 - A1,      aY = A0 + A1;
    i32 zp = z2 + A3, zm = z2 - A3;
    i32 aZ = vsel( mN, zm, zp ), aT = vsel( mN, zp, zm );
    t.X.v[k] = vsel( mD, dX, aX );
    t.Y.v[k] = vsel( mD, dY, aY );
    t.Z.v[k] = vsel( mD, dZ, aZ );
    t.T.v[k] = vsel( mD, dT, aT );
  }
}

/* p3 -> this lane's cached row (q0 Z*1, q1 Y1-X1, q2 Y1+X1, q3 T*2d) */
__device__ __forceinline__ fe
quad_cached_row( p3 const & u, u64 m1, u64 m2 ) {
  fe const D2 = {FD_AMD_FE_D2};
  fe Z1 = fe_mul_one( u.Z ), Y1 = fe_mul_one( u.Y ), X1 = fe_mul_one( u.X );
  fe T2 = fe_mul( u.T, D2 );
  fe r;
  _Pragma("unroll") for( int k=0; k<10; k++ ) r.v[k] = q4( m1, m2, Z1.v[k], Y1.v[k] - X1.v[k], Y1.v[k] + X1.v[k], T2.v[k] );
  return r;
}

/* -A and its odd multiples as cached rows on a quad (k_dsm4, k_dsm8):
   lane q computes row q ([Z, Y-X, Y+X, 2dT]) of every entry and,
   when wr, writes it to the signature's Ai slab Ail; the same ops as
   ge_to_cached / ge_dbl / ge_add (k_ai), so the same limbs. */
__device__ __forceinline__ void
ai_table_quad( bool act, bool wr, int qd, u64 m1, u64 m2, i32 const * __restrict__ Aw, size_t N, u32 ii,
               i32 * __restrict__ Ail ) {
  p3 A;
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    A.X.v[k] = act ? Aw[(size_t)(k   )*N + ii] : 0;
    A.Y.v[k] = act ? Aw[(size_t)(10+k)*N + ii] : (k==0);
    A.T.v[k] = act ? Aw[(size_t)(20+k)*N + ii] : 0;
    A.Z.v[k] = (k==0);
  }
  fe row = quad_cached_row( A, m1, m2 );
# define AI_ROW4( e ) do {                                                          \
    int4 * d_ = (int4 *)(Ail + (e)*48 + qd*12);                                     \
    d_[0] = make_int4( row.v[0], row.v[1], row.v[2], row.v[3] );                   \
    d_[1] = make_int4( row.v[4], row.v[5], row.v[6], row.v[7] );                   \
    d_[2] = make_int4( row.v[8], row.v[9], 0, 0 );                                 \
  } while(0)
  if( wr ) AI_ROW4( 0 );
  u64 const all = ~0UL, none = 0UL;
  p1p1 t; fe z0 = fe_zero();
  quad_body( t, A, z0, all, none, m1, m2 );            /* DBL(A) */
  p3 A2; quad_p3( A2, t, m1, m2 );
  for( int e=0; e<7; e++ ) {
    fe R0, R1, R2, R3;
    qgather( row, R0, R1, R2, R3 );                    /* rows Z, Y-X, Y+X, 2dT of entry e */
    fe br;
    _Pragma("unroll") for( int k=0; k<10; k++ ) br.v[k] = q4( m1, m2, R2.v[k], R1.v[k], R0.v[k], R3.v[k] );
    quad_body( t, A2, br, none, none, m1, m2 );        /* A2 + Ai[e] */
    p3 u; quad_p3( u, t, m1, m2 );
    row = quad_cached_row( u, m1, m2 );
    if( wr ) AI_ROW4( e+1 );
  }
# undef AI_ROW4
}

/* k_dsm4's body for lane gt of the launch (signature gt >> 2); bi12 filled
   (bi12_fill), evl: 16 event rows of 33 words for the wave's 16 signatures.
   Also the streaming tile's quad chunks (k_tile_persist). */
__device__ __forceinline__ void
dsm4_body( u32 gt, u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats,
           i32 (* __restrict__ bi12)[48], u64 (* __restrict__ evl)[33], u64 tc = 0UL ) {
  u32 i = gt >> 2;
  int qd = (int)(threadIdx.x & 3u);
  bool act = (i < n) && (err[i] == 1);
  if( act && (ws[L.ds + 2u*i] | ws[L.ds + 2u*i + 1u]) ) {            /* A or R undecodable */
    act = false;
    if( qd == 0 ) err[i] = (i8)-2;
  }
  size_t N = L.N;
  u32 ii = (i < n) ? i : 0u;
  i32 * Ail = (i32 *)(ws + L.Ai) + (size_t)ii*384u;
  u64 const m1 = __builtin_amdgcn_ballot_w64( qd & 1 ), m2 = __builtin_amdgcn_ballot_w64( qd & 2 );

  /* -A and its odd multiples (cached rows; lane q writes row q) */
  ai_table_quad( act, act, qd, m1, m2, (i32 const *)(ws + L.A), N, ii, Ail );

  u64 const * dg = (u64 const *)(ws + L.dig) + (size_t)ii*32u;
  int p   = act ? ((int const *)(ws + L.top))[ii] : -1;
  int ph  = act ? (p >= 0 ? PH_DBL : PH_FIN) : PH_DONE;
  evq eva, evb;                                      /* digit events of h and s */
  {
    u64 * row = evl[(threadIdx.x & 63u) >> 2];       /* one row per signature of the wave */
    u32 ne = act ? ((u32 const *)(ws + L.evn))[ii] : 0u;
    u32 wa = ((ne & 0xffu) + 3u) >> 2, wb = (((ne >> 8) & 0xffu) + 3u) >> 2;
    for( u32 k=(u32)qd; k<wa; k+=4u ) row[k]       = dg[k];        /* the quad copies the row together */
    for( u32 k=(u32)qd; k<wb; k+=4u ) row[16u + k] = dg[16u + k];
    __syncthreads();
    eva.init( (u16 const *)row,        (int)(ne & 0xffu) );
    evb.init( (u16 const *)(row + 16), (int)((ne >> 8) & 0xffu) );
  }
  i32 const * Rw = (i32 const *)(ws + L.R);
  u32 nha = 0, nhb = 0;
  u32 nit = (u32)(p + 1);
  bool qneg = false;
  fe qrow = fe_zero();
  fe C = (qd == 2) ? fe_zero() : fe_one();   /* identity: own coordinate (Z, T, X, Y)[q] = (1, 1, 0, 1) */
  u32 lvl = 0u;

  for( ;; ) {
    if( tc ) tile_age_prio( tc, lvl );
    fe pm = quad_p3_ownc( C );              /* q0 u.Z, q1 u.Y, q2 u.X, q3 u.T */

    bool fin = (ph == PH_FIN);
    /* each lane parks its own p1p1->p3 product in its row of entry 0 of the
       signature's Ai table (no ADD op reads it any more); the compare runs
       once after the loop */
    if( __any( fin ) ) {
      if( fin ) {
        int4 * d_ = (int4 *)(Ail + qd*12);
        d_[0] = make_int4( pm.v[0], pm.v[1], pm.v[2], pm.v[3] );
        d_[1] = make_int4( pm.v[4], pm.v[5], pm.v[6], pm.v[7] );
        d_[2] = make_int4( pm.v[8], pm.v[9], 0, 0 );
        ph = PH_DONE;
      }
    }
    if( __all( ph == PH_DONE ) ) break;

    bool isD = (ph == PH_DBL);
    u64 mD = __builtin_amdgcn_ballot_w64( isD );
    quad_body_ownc( C, pm, qrow, isD, qneg, mD, qd );

    /* the event just executed is consumed; the next op follows from the
       event heads (an event at position p means a digit at p) */
    /* branch-free, as in k_dsm8 */
    bool const wasA = ph == PH_ADDA, wasB = ph == PH_ADDB, wasD = ph == PH_DBL;
    eva.j -= (int)wasA; evb.j -= (int)wasB;
    eva.load(); evb.load();
    bool const toA = wasD && eva.pos == p;
    bool const toB = !toA && (wasD || wasA) && evb.pos == p;
    bool const adv = (wasD || wasA || wasB) && !toA && !toB;
    p -= (int)adv;
    ph = toA ? PH_ADDA : toB ? PH_ADDB : adv ? ((p < 0) ? PH_FIN : PH_DBL) : ph;
    nha += (u32)toA; nhb += (u32)toB;

    /* this lane's row of the next op's operand: q0 qP, q1 qM, q2 qZ, q3 qT;
       rows of an entry are [Z, Y-X, Y+X, 2dT], a negative digit swaps Y-X/Y+X */
    {
      int const d = toA ? eva.dig : evb.dig;
      int const e = ((d < 0 ? -d : d) >> 1) & 7;
      qneg = d < 0;
      int const row = (qd == 0) ? (qneg ? 1 : 2) : (qd == 1) ? (qneg ? 2 : 1) : (qd == 2) ? 0 : 3;
      int4 const * src = toA ? (int4 const *)(Ail + e*48 + row*12) : (int4 const *)&bi12[e][row*12];
      int4 x0 = src[0], x1 = src[1], x2 = src[2];
      qrow.v[0] = x0.x; qrow.v[1] = x0.y; qrow.v[2] = x0.z; qrow.v[3] = x0.w;
      qrow.v[4] = x1.x; qrow.v[5] = x1.y; qrow.v[6] = x1.z; qrow.v[7] = x1.w;
      qrow.v[8] = x2.x; qrow.v[9] = x2.y;
    }
  }

  /* the limb compare (fd_ed25519_user.c:417-425), once per wave, all lanes
     converged: q0 Z*RX vs X, q1 Z*RY vs Y, quad AND */
  {
    fe pm;
    int4 const * s_ = (int4 const *)(Ail + qd*12);
    int4 x0 = s_[0], x1 = s_[1], x2 = s_[2];
    pm.v[0] = x0.x; pm.v[1] = x0.y; pm.v[2] = x0.z; pm.v[3] = x0.w;
    pm.v[4] = x1.x; pm.v[5] = x1.y; pm.v[6] = x1.z; pm.v[7] = x1.w;
    pm.v[8] = x2.x; pm.v[9] = x2.y;
    _Pragma("unroll") for( int k=0; k<10; k++ ) qrow.v[k] = Rw[(size_t)((qd & 1)*10 + k)*N + ii];
    fe Z, ref;
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      Z.v[k] = qb<0>( pm.v[k] );
      ref.v[k] = qp<2,1,2,1>( pm.v[k] );    /* q0 <- X (lane 2), q1 <- Y (own) */
    }
    fe xz = fe_mul_fold1( Z, qrow );
    bool eq = true;
    _Pragma("unroll") for( int k=0; k<8; k++ ) eq = eq && (xz.v[k] == ref.v[k]);
    int e01 = (int)eq;
    int both = qb<0>( e01 ) & qb<1>( e01 );
    if( act && qd == 0 ) err[i] = (i8)(both ? 0 : -3);
  }

  if( want_stats && i < n && qd == 0 ) {
    u32 * st = (u32 *)(ws + L.st);
    st[i] = act ? nit : 0u; st[N + i] = act ? nha : 0u; st[2*N + i] = act ? nhb : 0u;
  }
}

__global__ void __launch_bounds__(64)
k_dsm4( u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats, i8 * __restrict__ out ) {
  __shared__ __attribute__((aligned(16))) i32 bi12[8][48];   /* the base-point table in the Ai slab's row layout */
  __shared__ u64 evl[16][33];
  bi12_fill( bi12 );
  __syncthreads();
  u32 const gt = blockIdx.x * 64u + threadIdx.x;
  dsm4_body( gt, n, err, ws, L, want_stats, bi12, evl );
  /* every verdict, straight to mapped host memory, by the lane that wrote it */
  if( out && (gt >> 2) < n && !(threadIdx.x & 3u) ) out[gt >> 2] = err[gt >> 2];
}

/* ------------------------------------------------------------------ */
/* k_dsm8: k_dsm4's op stream on EIGHT lanes per signature (8 signatures per
 * wave): two lane quads hold the same state, and every field mul of the
 * step is split between lane l (h = 0, even columns) and lane l ^ 4 (h = 1,
 * odd columns), 50 products each, so one step issues half the
 * multiply-accumulates per lane.  The instruction stream stays uniform:
 * lane h = 1 sees G shifted down one limb (G[j] = g_{j+1}, its wrap entry
 * G19[9] = g_0) and F undoubled, so slot (c, i) of both halves is
 * f_i * g_{2c+h-i} with that column's reference factors (x2 when i and j are
 * odd, x19 when i + j >= 10, on the wrapped int32 pre-multiples).  The five
 * 64-bit column sums are swapped between the two lanes with DPP
 * row_shl/row_shr 4 under bank masks, and the pair finishes the reference
 * carry chain on pre-biased sums, each lane running one of its two
 * interleaved runs (fe_mul_half5): the same limbs as fe_mul. */
struct half_t { u64 mH; i32 shF; i64 bias; i64 m4, k5; u32 shz, mo0; i32 bo0; };
__device__ __forceinline__ half_t half_ctx( int hh ) {
  half_t H;
  H.mH = __builtin_amdgcn_ballot_w64( hh != 0 );
  H.shF = hh ? 0 : 1;
  H.bias = hh ? (1L<<24) : (1L<<25);
  H.m4  = hh ? -1L : (1L<<26) - 1;           /* split carry (fe_mul_half5): see there */
  H.k5  = hh ? -1L : 0L;
  H.shz = hh ? 25u : 0u;
  H.mo0 = hh ? (1u<<25) - 1u : (1u<<26) - 1u;
  H.bo0 = hh ? (1<<24) : (1<<25);
  asm( "" : "+v"(H.shF), "+v"(H.m4), "+v"(H.k5), "+v"(H.shz), "+v"(H.mo0), "+v"(H.bo0) );
  return H;
}

/* the partner lane's value (lane l ^ 4 of the 8-lane group) where `mine`
   is the h = 0 / h = 1 slot: E keeps h = 0's own value and takes the partner's
   on h = 1 lanes, O the other way round */
__device__ __forceinline__ u32 half_from_lo( u32 v ) {   /* h = 1 lanes read lane - 4 (banks 1, 3) */
  return (u32)__builtin_amdgcn_update_dpp( (int)v, (int)v, 0x114, 0xf, 0xa, false );
}
__device__ __forceinline__ u32 half_from_hi( u32 v ) {   /* h = 0 lanes read lane + 4 (banks 0, 2) */
  return (u32)__builtin_amdgcn_update_dpp( (int)v, (int)v, 0x104, 0xf, 0x5, false );
}

/* The split field mul: after the column sums, the two lanes of a pair run
   the two halves of the reference carry chain side by side (rather than
   both running all of it), and each returns five limbs (fe5); fe_join5 makes the full
   element when an operation needs it.  The chain of fe_carry_b is two
   interleaved runs, 0->1->2->3->(4) and 4->5->6->7->8->9->(0); in slots
   s0..s5 lane h = 0 holds h0..h4 (s5 = 0) and lane h = 1 holds h4..h9, so
   one instruction stream advances both runs (the widths 26,25,26,25,26
   agree; only the mask of step 4 differs: t4 = (h4 & M26) + h3>>25 on
   h = 0, h8 += h7>>25 on h = 1).  The two cross terms, c4b into limb 5 and
   h9>>25 into limb 0, are swapped with DPP after the run.  Limbs out:
   h = 0 -> (r0, r1, r2, r3, r4), h = 1 -> (r9, r5, r6, r7, r8).  The same
   limbs as fe_carry_b, so the same as the reference's fe_mul. */
struct fe5 { i32 v[5]; };

__device__ __forceinline__ i64 dpp64_from_lo( i64 old, i64 src ) {   /* h = 1 lanes take lane - 4's src */
  u32 lo = (u32)__builtin_amdgcn_update_dpp( (int)(u32)old, (int)(u32)src, 0x114, 0xf, 0xa, false );
  u32 hi = (u32)__builtin_amdgcn_update_dpp( (int)(u32)((u64)old >> 32), (int)(u32)((u64)src >> 32), 0x114, 0xf, 0xa, false );
  return (i64)(((u64)hi << 32) | lo);
}
__device__ __forceinline__ i64 dpp64_from_hi( i64 old, i64 src ) {   /* h = 0 lanes take lane + 4's src */
  u32 lo = (u32)__builtin_amdgcn_update_dpp( (int)(u32)old, (int)(u32)src, 0x104, 0xf, 0x5, false );
  u32 hi = (u32)__builtin_amdgcn_update_dpp( (int)(u32)((u64)old >> 32), (int)(u32)((u64)src >> 32), 0x104, 0xf, 0x5, false );
  return (i64)(((u64)hi << 32) | lo);
}

__device__ __forceinline__ fe5
fe_mul_half5( fe const & F, fe const & G, half_t const & H ) {
  i32 gs[9], g19[10], f2[10];
  _Pragma("unroll") for( int j=0; j<9; j++ ) gs[j] = vsel( H.mH, G.v[j+1], G.v[j] );
  _Pragma("unroll") for( int j=1; j<9; j++ ) g19[j] = wmul( gs[j], 19 );
  g19[9] = vsel( H.mH, G.v[0], wmul( G.v[9], 19 ) );
  _Pragma("unroll") for( int i=1; i<10; i+=2 ) f2[i] = (i32)((u32)F.v[i] << (u32)H.shF);
  i64 a[5];
  _Pragma("unroll") for( int c=0; c<5; c++ ) a[c] = H.bias;
  _Pragma("unroll") for( int i=0; i<10; i++ ) {
    _Pragma("unroll") for( int c=0; c<5; c++ ) {
      int j = 2*c - i;
      i32 g = (j >= 0) ? gs[j] : g19[j + 10];
      i32 f = (i & 1) ? f2[i] : F.v[i];
      a[c] = mac( f, g, a[c] );
    }
  }
  /* a[c] is column 2c (h = 0) or 2c+1 (h = 1), pre-biased */
  i64 s1 = dpp64_from_hi( a[2], a[0] );    /* h1 | h5 */
  i64 s0 = dpp64_from_lo( a[0], a[2] );    /* h0 | h4 */
  i64 s2 = dpp64_from_lo( a[1], a[3] );    /* h2 | h6 */
  i64 s3 = dpp64_from_hi( a[3], a[1] );    /* h3 | h7 */
  i64 s4 = dpp64_from_lo( a[2], a[4] );    /* h4 | h8 */
  i64 s5 = a[4] & H.k5;                    /* 0  | h9 */
  s1 += s0 >> 26;
  s2 += s1 >> 25;
  s3 += s2 >> 26;
  s4 = (s4 & H.m4) + (s3 >> 25);           /* t4 | h8 */
  s5 += s4 >> 26;                          /* c4b | h9 */
  i64 const y = s5 >> H.shz;               /* c4b | h9 >> 25 */
  u32 const ylo = (u32)y, yhi = (u32)((u64)y >> 32);
  u32 zl = (u32)__builtin_amdgcn_update_dpp( (int)ylo, (int)ylo, 0x104, 0xf, 0x5, false );
  zl = (u32)__builtin_amdgcn_update_dpp( (int)zl, (int)ylo, 0x114, 0xf, 0xa, false );
  u32 const zh = (u32)__builtin_amdgcn_update_dpp( (int)yhi, (int)yhi, 0x104, 0xf, 0x5, false );
  i64 const z = (i64)(((u64)zh << 32) | zl);   /* h = 0: h9 >> 25; h = 1: c4b (low word) */
  i64 const t0 = (s0 & ((1L<<26) - 1)) + z * 19;
  i32 const cin = vsel( H.mH, (i32)zl, (i32)(t0 >> 26) );
  u32 const w0 = (u32)vsel( H.mH, (i32)(u32)s5, (i32)(u32)t0 );
  fe5 o;
  o.v[0] = (i32)(w0 & H.mo0) - H.bo0;
  o.v[1] = (i32)((u32)s1 & ((1u<<25) - 1u)) - (1<<24) + cin;
  o.v[2] = (i32)((u32)s2 & ((1u<<26) - 1u)) - (1<<25);
  o.v[3] = (i32)((u32)s3 & ((1u<<25) - 1u)) - (1<<24);
  o.v[4] = (i32)((u32)s4 & ((1u<<26) - 1u)) - (1<<25);
  return o;
}

__device__ __forceinline__ fe fe_join5( fe5 const & o ) {
  fe r;
  r.v[0] = (i32)half_from_lo( (u32)o.v[0] );
  r.v[9] = (i32)half_from_hi( (u32)o.v[0] );
  _Pragma("unroll") for( int k=1; k<5; k++ ) {
    r.v[k]   = (i32)half_from_lo( (u32)o.v[k] );
    r.v[k+4] = (i32)half_from_hi( (u32)o.v[k] );
  }
  return r;
}

__device__ __forceinline__ fe5
quad8_p3_ownc5( fe const & C, half_t const & H ) {
  fe a, b;
  _Pragma("unroll") for( int k=0; k<10; k++ ) { a.v[k] = qp<0,0,2,2>( C.v[k] ); b.v[k] = qp<1,3,1,3>( C.v[k] ); }
  return fe_mul_half5( a, b, H );
}

/* quad8_body_ownc on split limbs: every per-limb step (the operand
   combination, the mix) runs on the lane's five limbs, and the pair joins
   the operand before the mul and the mixed coordinate after it */
__device__ __forceinline__ void
quad8_body_ownc5( fe & C, fe5 const & pm, fe const & qrow, bool isD, bool neg, u64 mD, int qd, half_t const & H ) {
  i32 c1 = (qd == 0) ? 1 : (qd == 1) ? (isD ? 0 : -1) : (isD ? 1 : 0);
  i32 c2 = (qd <= 1 || !isD) ? 1 : 0;
  i32 sh = (qd == 3) ? 1 : 0;
  asm( "" : "+v"(c1), "+v"(c2) );
  fe5 a5;
  _Pragma("unroll") for( int k=0; k<5; k++ )
    a5.v[k] = lin2( c1, qp<2,2,2,0>( pm.v[k] ), c2, qp<1,1,0,3>( pm.v[k] ) );
  fe const a = fe_join5( a5 );
  fe b;
  _Pragma("unroll") for( int k=0; k<10; k++ ) b.v[k] = vsel( mD, (i32)((u32)a.v[k] << sh), qrow.v[k] );
  fe5 const m = fe_mul_half5( a, b, H );
  i32 s0 = neg ? -1 : 1;
  i32 x = isD ? (qd == 1 ? -1 : (qd == 3 ? 0 : 1)) : (qd >= 2 ? 1 : 0);
  i32 y = isD ? ((qd & 1) ? 1 : -1)               : (qd <= 1 ? 2 : (qd == 2 ? -1 : 1));
  i32 z = isD ? (qd == 0 ? 0 : (qd == 2 ? -1 : 1)) : (qd == 0 ? s0 : (qd == 1 ? -s0 : 0));
  asm( "" : "+v"(x), "+v"(y), "+v"(z) );
  fe5 c5;
  _Pragma("unroll") for( int k=0; k<5; k++ )
    c5.v[k] = lin3( x, qp<1,1,0,0>( m.v[k] ), y, qp<2,2,1,1>( m.v[k] ), z, qp<3,3,2,2>( m.v[k] ) );
  C = fe_join5( c5 );
}

/* k_dsm8's body for lane gt of the launch (signature gt >> 3); bi12 filled
   (bi12_fill), evl: 8 event rows of 33 words for the wave's 8 signatures.
   Also the streaming tile's latency chunks (k_tile_persist). */
__device__ __forceinline__ void
dsm8_body( u32 gt, u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats,
           i32 (* __restrict__ bi12)[48], u64 (* __restrict__ evl)[33], u64 tc = 0UL ) {
  u32 i = gt >> 3;
  int qd = (int)(threadIdx.x & 3u);
  int hh = (int)((threadIdx.x >> 2) & 1u);            /* which half of every field mul this lane computes */
  bool act = (i < n) && (err[i] == 1);
  if( act && (ws[L.ds + 2u*i] | ws[L.ds + 2u*i + 1u]) ) {            /* A or R undecodable */
    act = false;
    if( qd == 0 && !hh ) err[i] = (i8)-2;
  }
  size_t N = L.N;
  u32 ii = (i < n) ? i : 0u;
  i32 * Ail = (i32 *)(ws + L.Ai) + (size_t)ii*384u;
  u64 const m1 = __builtin_amdgcn_ballot_w64( qd & 1 ), m2 = __builtin_amdgcn_ballot_w64( qd & 2 );
  half_t const H = half_ctx( hh );

  /* -A and its odd multiples (cached rows; lane q writes row q, the h = 0 half) */
  ai_table_quad( act, act && !hh, qd, m1, m2, (i32 const *)(ws + L.A), N, ii, Ail );

  u64 const * dg = (u64 const *)(ws + L.dig) + (size_t)ii*32u;
  int p   = act ? ((int const *)(ws + L.top))[ii] : -1;
  int ph  = act ? (p >= 0 ? PH_DBL : PH_FIN) : PH_DONE;
  evq eva, evb;                                      /* digit events of h and s */
  {
    u64 * row = evl[(threadIdx.x & 63u) >> 3];       /* one row per signature of the wave */
    u32 ne = act ? ((u32 const *)(ws + L.evn))[ii] : 0u;
    u32 wa = ((ne & 0xffu) + 3u) >> 2, wb = (((ne >> 8) & 0xffu) + 3u) >> 2;
    for( u32 k=threadIdx.x & 7u; k<wa; k+=8u ) row[k]       = dg[k];   /* the 8 lanes copy the row together */
    for( u32 k=threadIdx.x & 7u; k<wb; k+=8u ) row[16u + k] = dg[16u + k];
    __syncthreads();
    eva.init( (u16 const *)row,        (int)(ne & 0xffu) );
    evb.init( (u16 const *)(row + 16), (int)((ne >> 8) & 0xffu) );
  }
  i32 const * Rw = (i32 const *)(ws + L.R);
  u32 nha = 0, nhb = 0;
  u32 nit = (u32)(p + 1);
  bool qneg = false;
  fe qrow = fe_zero();
  fe C = (qd == 2) ? fe_zero() : fe_one();   /* identity: own coordinate (Z, T, X, Y)[q] = (1, 1, 0, 1) */
  u32 lvl = 0u;

  for( ;; ) {
    if( tc ) tile_age_prio( tc, lvl );
    fe5 pm5 = quad8_p3_ownc5( C, H );          /* q0 u.Z, q1 u.Y, q2 u.X, q3 u.T (split limbs) */

    bool fin = (ph == PH_FIN);
    /* each lane parks its own p1p1->p3 product in its row of entry 0 of the
       signature's Ai table (no ADD op reads it any more); the compare runs
       once after the loop */
    if( __any( fin ) ) {
      fe const pm = fe_join5( pm5 );           /* all 8 lanes of a signature finish together */
      if( fin ) {
        int4 * d_ = (int4 *)(Ail + qd*12);
        d_[0] = make_int4( pm.v[0], pm.v[1], pm.v[2], pm.v[3] );
        d_[1] = make_int4( pm.v[4], pm.v[5], pm.v[6], pm.v[7] );
        d_[2] = make_int4( pm.v[8], pm.v[9], 0, 0 );
        ph = PH_DONE;
      }
    }
    if( __all( ph == PH_DONE ) ) break;

    bool isD = (ph == PH_DBL);
    u64 mD = __builtin_amdgcn_ballot_w64( isD );
    quad8_body_ownc5( C, pm5, qrow, isD, qneg, mD, qd, H );

    /* the event just executed is consumed; the next op follows from the
       event heads (an event at position p means a digit at p).  Branch-free:
       on one wave per SIMD every exec-mask branch is an issue slot. */
    bool const wasA = ph == PH_ADDA, wasB = ph == PH_ADDB, wasD = ph == PH_DBL;
    eva.j -= (int)wasA; evb.j -= (int)wasB;
    eva.load(); evb.load();
    bool const toA = wasD && eva.pos == p;
    bool const toB = !toA && (wasD || wasA) && evb.pos == p;
    bool const adv = (wasD || wasA || wasB) && !toA && !toB;
    p -= (int)adv;
    ph = toA ? PH_ADDA : toB ? PH_ADDB : adv ? ((p < 0) ? PH_FIN : PH_DBL) : ph;
    nha += (u32)toA; nhb += (u32)toB;

    /* this lane's row of the next op's operand: q0 qP, q1 qM, q2 qZ, q3 qT;
       rows of an entry are [Z, Y-X, Y+X, 2dT], a negative digit swaps Y-X/Y+X
       (loaded by every lane; only an ADD reads it) */
    {
      int const d = toA ? eva.dig : evb.dig;
      int const e = ((d < 0 ? -d : d) >> 1) & 7;
      qneg = d < 0;
      int const row = (qd == 0) ? (qneg ? 1 : 2) : (qd == 1) ? (qneg ? 2 : 1) : (qd == 2) ? 0 : 3;
      int4 const * src = toA ? (int4 const *)(Ail + e*48 + row*12) : (int4 const *)&bi12[e][row*12];
      int4 x0 = src[0], x1 = src[1], x2 = src[2];
      qrow.v[0] = x0.x; qrow.v[1] = x0.y; qrow.v[2] = x0.z; qrow.v[3] = x0.w;
      qrow.v[4] = x1.x; qrow.v[5] = x1.y; qrow.v[6] = x1.z; qrow.v[7] = x1.w;
      qrow.v[8] = x2.x; qrow.v[9] = x2.y;
    }
  }

  /* the limb compare (fd_ed25519_user.c:417-425), once per wave, all lanes
     converged: q0 Z*RX vs X, q1 Z*RY vs Y, quad AND */
  {
    fe pm;
    int4 const * s_ = (int4 const *)(Ail + qd*12);
    int4 x0 = s_[0], x1 = s_[1], x2 = s_[2];
    pm.v[0] = x0.x; pm.v[1] = x0.y; pm.v[2] = x0.z; pm.v[3] = x0.w;
    pm.v[4] = x1.x; pm.v[5] = x1.y; pm.v[6] = x1.z; pm.v[7] = x1.w;
    pm.v[8] = x2.x; pm.v[9] = x2.y;
    _Pragma("unroll") for( int k=0; k<10; k++ ) qrow.v[k] = Rw[(size_t)((qd & 1)*10 + k)*N + ii];
    fe Z, ref;
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      Z.v[k] = qb<0>( pm.v[k] );
      ref.v[k] = qp<2,1,2,1>( pm.v[k] );    /* q0 <- X (lane 2), q1 <- Y (own) */
    }
    fe xz = fe_mul_fold1( Z, qrow );
    bool eq = true;
    _Pragma("unroll") for( int k=0; k<8; k++ ) eq = eq && (xz.v[k] == ref.v[k]);
    int e01 = (int)eq;
    int both = qb<0>( e01 ) & qb<1>( e01 );
    if( act && qd == 0 && !hh ) err[i] = (i8)(both ? 0 : -3);
  }

  if( want_stats && i < n && qd == 0 && !hh ) {
    u32 * st = (u32 *)(ws + L.st);
    st[i] = act ? nit : 0u; st[N + i] = act ? nha : 0u; st[2*N + i] = act ? nhb : 0u;
  }
}

__global__ void __launch_bounds__(64)
k_dsm8( u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats, i8 * __restrict__ out ) {
  __shared__ __attribute__((aligned(16))) i32 bi12[8][48];
  __shared__ u64 evl[8][33];
  bi12_fill( bi12 );
  __syncthreads();
  u32 const gt = blockIdx.x * 64u + threadIdx.x;
  dsm8_body( gt, n, err, ws, L, want_stats, bi12, evl );
  /* every verdict, straight to mapped host memory, by the lane that wrote it */
  if( out && (gt >> 3) < n && !(threadIdx.x & 7u) ) out[gt >> 3] = err[gt >> 3];
}

/* ------------------------------------------------------------------ */
/* Pooled DSM for large batches: k_ai -> k_dsmp -> k_fin.
 *
 * k_dsm runs every op of a signature's stream (DBL / ADD-A / ADD-B, see
 * above) as the same 8-mul step, so a lane that doubles while its
 * neighbours add still computes general products: each step pays for
 * p1p1->p3 (4 muls) + 4 general muls + per-lane operand selects.  In the
 * reference's own flow (avx/fd_ed25519_ge.c:488-523) a doubling costs
 * p1p1->p2 (3 muls) + 4 squares (55 products each, not 100), and DBLs are
 * about three quarters of the stream.  k_dsmp keeps a POOL of FD_POOL_P
 * signatures per wave in LDS (their p1p1 state and op-stream cursor) and,
 * every step, runs 64 of them that want the SAME op class: a DBL step
 * (p2 + 4 squares) or an ADD step (p3 + 4 muls; ADD-A and ADD-B differ only
 * in where the table operand comes from).  With P >= 128 a full class
 * always exists (nA < 64 => nD > 64); at P = 112 nearly always.  Same field
 * ops as the reference, in the same order per signature: identical limbs.
 *
 *   k_ai    one lane per signature: k_dsm's activity check (-2 on an
 *           undecodable point) and Ai table of odd multiples of -A, plus
 *           the op-stream start init[i] = { -, heads, p|ja<<16|jb<<24, op }
 *           (heads: the top remaining h / s digit events, 0xffff = none).
 *   k_dsmp  one wave per workgroup, gridDim.x waves; waves claim
 *           signatures for their free pool slots from a shared counter.  A
 *           finished signature parks its final p1p1 in its own Ai slab.
 *   k_fin   one lane per signature: p1p1 -> p2 and the limb compare of
 *           fd_ed25519_user.c:417-425; work statistics.
 */
#ifndef FD_POOL_P
#define FD_POOL_P 112
#endif
enum { OP_D = 0, OP_AA = 1, OP_AB = 2, OP_EMPTY = 3, OP_NONE = 4 };

/* the base-point table in the Ai slab's row layout: entry e = rows
   [Z = 1 | Y-X | Y+X | 2dT] x 12 limbs (10 used), so ADD-A and ADD-B load
   their operand with the same code from different bases */
__device__ i32 g_bi12[8][48];
#ifdef FD_AMD_DIAG
__device__ u32 g_pool_dbg[4];   /* steps, live lanes, ADD steps, refill-only steps (summed over waves) */
__device__ u64 g_pool_dbg_t[8192][4];   /* per wave: wall_clock64 at start, at exhaustion of the counter, at exit; steps after exhaustion | lanes << 32 */
#endif

#ifndef FD_AI_WAVES
#define FD_AI_WAVES 2
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FD_AI_WAVES)))
k_ai( u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L ) {
  if( blockIdx.x == 0 ) {
    for( int k=threadIdx.x; k<8*48; k+=64 ) {
      int e = k / 48, c = (k % 48) / 12, l = k % 12;
      i32 v = 0;
      if( l < 10 ) {
        if( c == 0 ) v = (l == 0);
        else if( c == 1 ) v = BI_TABLE[e][1][l];
        else if( c == 2 ) v = BI_TABLE[e][0][l];
        else v = BI_TABLE[e][2][l];
      }
      g_bi12[e][k % 48] = v;
    }
  }
  u32 i = blockIdx.x * 64u + threadIdx.x;
  if( i == 0u ) { ((u32 *)(ws + L.ctr))[0] = 0u; ((u32 *)(ws + L.ctr))[1] = 0u; }   /* work counter, guard flag */
  bool act = (i < n) && (err[i] == 1);
  if( act && (ws[L.ds + 2u*i] | ws[L.ds + 2u*i + 1u]) ) { err[i] = (i8)-2; act = false; }
  size_t N = L.N;
  u32 ii = (i < n) ? i : 0u;
  /* the wave's 64 tables are written one entry at a time through LDS: lane
     l stages its 192-B entry, then the wave stores the 64 entries as 12
     contiguous 1-KB rows (whole 64-B lines; a lane writing its own table
     touches 64 lines per store and took ~0.36 of k_ai's 0.78 ms).  Lanes past
     n or inactive write don't-care tables into their own slabs (< N, never
     read). */
  __shared__ int4 s_ai[64 * 13];                   /* 13: a lane's entry starts 52 dwords after the last one's */
  int4 * const s_me = s_ai + threadIdx.x * 13u;
  int4 * const Ab = (int4 *)((i32 *)(ws + L.Ai) + (size_t)blockIdx.x * 64u * 384u);
  {
    p3 A;
    i32 const * Aw = (i32 const *)(ws + L.A);
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      A.X.v[k] = act ? Aw[(size_t)(k   )*N + ii] : 0;
      A.Y.v[k] = act ? Aw[(size_t)(10+k)*N + ii] : (k==0);
      A.T.v[k] = act ? Aw[(size_t)(20+k)*N + ii] : 0;
      A.Z.v[k] = (k==0);
    }
    fe cZ, cYmX, cYpX, cT2d;
    ge_to_cached( cZ, cYmX, cYpX, cT2d, A );
#   define AI_ROW( r, f ) do {                                                      \
      s_me[3*(r)  ] = make_int4( f.v[0], f.v[1], f.v[2], f.v[3] );                  \
      s_me[3*(r)+1] = make_int4( f.v[4], f.v[5], f.v[6], f.v[7] );                  \
      s_me[3*(r)+2] = make_int4( f.v[8], f.v[9], 0, 0 );                            \
    } while(0)
#   define AI_STORE( e ) do {                                                       \
      AI_ROW( 0, cZ ); AI_ROW( 1, cYmX ); AI_ROW( 2, cYpX ); AI_ROW( 3, cT2d );     \
      __syncthreads();                                                              \
      _Pragma("unroll") for( u32 q=0; q<12u; q++ ) {                                \
        u32 const x = q*64u + threadIdx.x, sg = x / 12u, c = x - 12u*sg;            \
        Ab[(size_t)sg*96u + (e)*12u + c] = s_ai[sg*13u + c];                        \
      }                                                                             \
      __syncthreads();                                                              \
    } while(0)
    AI_STORE( 0u );
    p1p1 t = ge_dbl( A.X, A.Y, A.Z );
    p3 A2 = ge_p1p1_to_p3( t );
    for( u32 e=0; e<7u; e++ ) {
      p1p1 s2 = ge_add<false>( A2, cZ, cYmX, cYpX, cT2d, false );
      p3 u = ge_p1p1_to_p3( s2 );
      ge_to_cached( cZ, cYmX, cYpX, cT2d, u );
      AI_STORE( e+1u );
    }
#   undef AI_STORE
#   undef AI_ROW
  }
  if( i < n ) {
    uint4 in = make_uint4( 0u, 0xffffffffu, 0u, (u32)OP_EMPTY );
    int p = act ? ((int const *)(ws + L.top))[i] : -1;
    if( p >= 0 ) {
      u32 ne = ((u32 const *)(ws + L.evn))[i];
      u32 na = ne & 0xffu, nb = (ne >> 8) & 0xffu;
      u16 const * ev = (u16 const *)(ws + L.dig) + (size_t)i*128u;
      u32 hA = na ? (u32)ev[na - 1u] : 0xffffu, hB = nb ? (u32)ev[64u + nb - 1u] : 0xffffu;
      in = make_uint4( 0u, hA | (hB << 16), ((u32)p & 0xffffu) | (na << 16) | (nb << 24), (u32)OP_D );
    }
    ((uint4 *)(ws + L.init))[i] = in;
  }
}

__device__ __forceinline__ void
pool_load_t( p1p1 & t, int4 const * s ) {
  _Pragma("unroll") for( int r=0; r<10; r++ ) {
    int4 x = s[r];
    i32 v[4] = { x.x, x.y, x.z, x.w };
    _Pragma("unroll") for( int c=0; c<4; c++ ) {
      int k = 4*r + c;                     /* limb k of [X | Y | Z | T] */
      if( k < 10 ) t.X.v[k] = v[c]; else if( k < 20 ) t.Y.v[k-10] = v[c];
      else if( k < 30 ) t.Z.v[k-20] = v[c]; else t.T.v[k-30] = v[c];
    }
  }
}

__device__ __forceinline__ void
pool_store_t( int4 * s, p1p1 const & t ) {
  _Pragma("unroll") for( int r=0; r<10; r++ ) {
    i32 v[4];
    _Pragma("unroll") for( int c=0; c<4; c++ ) {
      int k = 4*r + c;
      v[c] = (k < 10) ? t.X.v[k] : (k < 20) ? t.Y.v[k-10] : (k < 30) ? t.Z.v[k-20] : t.T.v[k-30];
    }
    s[r] = make_int4( v[0], v[1], v[2], v[3] );
  }
}

template<typename PTR>
__device__ __forceinline__ void
pool_load_ts( p1p1 & t, PTR s, u32 stride ) {
  _Pragma("unroll") for( int r=0; r<10; r++ ) {
    int4 x = s[(u32)r * stride];
    i32 v[4] = { x.x, x.y, x.z, x.w };
    _Pragma("unroll") for( int c=0; c<4; c++ ) {
      int k = 4*r + c;
      if( k < 10 ) t.X.v[k] = v[c]; else if( k < 20 ) t.Y.v[k-10] = v[c];
      else if( k < 30 ) t.Z.v[k-20] = v[c]; else t.T.v[k-30] = v[c];
    }
  }
}

template<typename PTR>
__device__ __forceinline__ void
pool_store_ts( PTR s, u32 stride, p1p1 const & t ) {
  _Pragma("unroll") for( int r=0; r<10; r++ ) {
    i32 v[4];
    _Pragma("unroll") for( int c=0; c<4; c++ ) {
      int k = 4*r + c;
      v[c] = (k < 10) ? t.X.v[k] : (k < 20) ? t.Y.v[k-10] : (k < 30) ? t.Z.v[k-20] : t.T.v[k-30];
    }
    s[(u32)r * stride] = make_int4( v[0], v[1], v[2], v[3] );
  }
}

/* a pure DBL step is chosen while its lane count is at least this percentage
   of a mixed step's.  100: only a full DBL step (64 lanes) beats a mixed one.
   The steps' cost ratio (~0.72) was the round-2 setting (78); a model of the
   pool's op streams and an interleaved A/B both favour 100: ADD slots wait
   less, so fewer signatures sit in the pool with nothing but an ADD to do
   (DSM stage -1 to -2 %, profiles/r03_pool_tune_ab.txt) */
#ifndef FD_POOL_DBL_PCT
#define FD_POOL_DBL_PCT 100u
#endif
/* k_dsmp's drain: issue priority by the signatures left in the pool */
#ifndef FD_POOL_DRAIN_PRIO
#define FD_POOL_DRAIN_PRIO 1
#endif
/* free slots that trigger a refill (one counter atomic + init loads) */
#ifndef FD_POOL_REFILL
#define FD_POOL_REFILL 8u
#endif


__device__ __forceinline__ u32 lane_rank( u64 m ) {   /* set bits of m below this lane */
  return __builtin_amdgcn_mbcnt_hi( (u32)(m >> 32), __builtin_amdgcn_mbcnt_lo( (u32)m, 0u ) );
}

/* The pool's op classes live in four wave-uniform 64-bit masks (slot s is
   bit s & 63 of word s >> 6): mD = DBL next, mA = ADD-A / ADD-B next,
   neither = free.  A step takes the first (up to) 64 slots of one class in
   slot order; lane l learns the l-th of them from a rank list in LDS, loads
   its slot's state from LDS, runs the op and writes the state back; the slots'
   new classes return to the masks through each slot's owner lane (s & 63),
   which pulls the processing lane's verdict with ds_bpermute. */
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_dsmp( u32 n, u8 * __restrict__ ws, ws_layout_t L, u64 iter_cap ) {
  constexpr u32 P = FD_POOL_P;
  static_assert( P >= 64 && P <= 128, "pool: each lane owns slots l and l + 64" );
  __shared__ int4  s_t[10][P];   /* p1p1 state [X | Y | Z | T], 16-B column r of slot s at [r][s]:
                                    a lane's b128 starts at bank 4 (s mod 16), not 8 (s mod 8) */
  __shared__ uint4 s_m[P];       /* { sig, heads, p | ja<<16 | jb<<24, op } */
  __shared__ u32   s_list[64];   /* slot of each rank in the step's selection */
  u32 const l = threadIdx.x, w = blockIdx.x;
  uint4 const * init = (uint4 const *)(ws + L.init);
  u16 const * dig = (u16 const *)(ws + L.dig);
  i32 * Ai = (i32 *)(ws + L.Ai);
  u64 const valid1 = (P >= 128u) ? ~0UL : ((1UL << (P - 64u)) - 1UL);   /* slots 64.. that exist */

  u64 mD0 = 0, mD1 = 0, mA0 = 0, mA1 = 0;
#ifdef FD_AMD_DIAG
  u64 dbg_t0 = wall_clock64(), dbg_te = 0; bool dbg_after = false; u64 dbg_sa = 0, dbg_la = 0;
#endif
  u32 * ctr = (u32 *)(ws + L.ctr);   /* next unclaimed signature, shared by all waves */
  bool more = true;                  /* wave-uniform: the counter has not passed n */
  /* hang guard: every step advances at least one op of at most 448 per
     signature, and a wave can claim at most all n signatures.  A wave that
     reaches it raises the launch's guard flag: k_fin then marks every
     verdict FD_AMD_VERDICT_DEVICE and the host call fails with
     FD_ED25519_AMD_ERR_DEVICE (iter_cap: a debug cap, ~0 normally). */
  u64 iter_max = ((u64)n + 2u*P) * 448u;
  if( iter_cap < iter_max ) iter_max = iter_cap;
  bool guard = true;
#ifdef FD_AMD_DIAG
  u32 dbg_steps = 0, dbg_lanes = 0, dbg_add = 0, dbg_idle = 0;
#endif
  for( u64 iter = 0; iter < iter_max; iter++ ) {
    u32 nD = (u32)(__builtin_popcountll( mD0 ) + __builtin_popcountll( mD1 ));
    u32 nA = (u32)(__builtin_popcountll( mA0 ) + __builtin_popcountll( mA1 ));
    u64 f0 = ~(mD0 | mA0), f1 = ~(mD1 | mA1) & valid1;   /* free slots */
    u32 nfree = (u32)(__builtin_popcountll( f0 ) + __builtin_popcountll( f1 ));
    /* refill in batches (one global round trip per 16 finished signatures),
       or whenever no class fills a wave */
    if( more && nfree && (nfree >= FD_POOL_REFILL || (nD < 64u && nA < 64u)) ) {
#ifdef FD_AMD_DIAG
      dbg_idle++;
#endif
      /* claim nfree signatures (one vector atomic; faster waves claim more,
         so the waves of a launch finish together) */
      u32 base = 0u;
      if( l == 0u ) base = atomicAdd( ctr, nfree );
      base = (u32)__builtin_amdgcn_readfirstlane( (int)base );
      if( base + nfree >= n || base + nfree < base ) {
        more = false;
#ifdef FD_AMD_DIAG
        dbg_te = wall_clock64(); dbg_after = true;
#endif
      }
      u32 pf0 = (u32)__builtin_popcountll( f0 );
      u64 s0 = (u64)base + lane_rank( f0 ), s1 = (u64)base + pf0 + lane_rank( f1 );
      bool r0 = ((f0 >> l) & 1u) && s0 < n, r1 = ((f1 >> l) & 1u) && s1 < n;
      uint4 in0 = init[r0 ? s0 : 0u], in1 = init[r1 ? s1 : 0u];
      r0 = r0 && in0.w == OP_D; r1 = r1 && in1.w == OP_D;   /* inactive signatures leave the slot free */
      p1p1 id;   /* new signatures enter with the identity (p1p1 whose p2 is (0,1,1)) */
      id.X = fe_zero(); id.Y = fe_one(); id.Z = fe_one(); id.T = fe_one();
      if( r0 ) { s_m[l] = make_uint4( (u32)s0, in0.y, in0.z, (u32)OP_D ); pool_store_ts( &s_t[0][l], P, id ); }
      if( r1 ) { s_m[l + 64u] = make_uint4( (u32)s1, in1.y, in1.z, (u32)OP_D ); pool_store_ts( &s_t[0][l + 64u], P, id ); }
      mD0 |= __builtin_amdgcn_ballot_w64( r0 );
      mD1 |= __builtin_amdgcn_ballot_w64( r1 );
      nD = (u32)(__builtin_popcountll( mD0 ) + __builtin_popcountll( mD1 ));
    }
    if( !(nD + nA) ) {
      if( !more ) { guard = false; break; }   /* pool empty, nothing left to take */
      continue;
    }
#if FD_POOL_DRAIN_PRIO
    /* drain: the wave with more signatures left issues first on its SIMD
       (at equal priority the arbiter prefers the older wave, whatever its
       pool holds), so the two waves of a SIMD empty their pools together */
    if( !more ) {
      u32 const left = nD + nA;
      if( left > 84u )      __builtin_amdgcn_s_setprio( 3 );
      else if( left > 56u ) __builtin_amdgcn_s_setprio( 2 );
      else if( left > 28u ) __builtin_amdgcn_s_setprio( 1 );
      else                  __builtin_amdgcn_s_setprio( 0 );
    }
#endif

    u32 kD = nD < 64u ? nD : 64u, kM = (nD + nA) < 64u ? (nD + nA) : 64u;
    bool mixed;
    u32 nsel, rk0, rk1;
    u64 S0, S1;
    if( !more ) {
      /* drain (nothing left to claim): the pool's last signatures set the
         launch's end.  The class is chosen as in the main phase; within it
         the (up to) 64 slots with the most ops left, p + ja + jb (remaining
         doublings and adds), go first -- in a mixed step every ADD slot
         ranks above every DBL slot.  A threshold search on those counts (10
         ballots) finds the 64th largest; ties go in slot order.  (Slot
         order alone left the youngest signatures waiting: 393 / 620 steps
         after the counter ran out, median / max, vs 382 / 479.) */
      mixed = 100u * kD < FD_POOL_DBL_PCT * kM;
      u64 const L0 = mixed ? (mA0 | mD0) : mD0, L1 = mixed ? (mA1 | mD1) : mD1;
      u32 const K = mixed ? kM : kD;
      u32 const z0 = s_m[l].z, z1 = s_m[l + 64u < P ? l + 64u : l].z;
      u32 const r0 = (z0 & 0xffffu) + ((z0 >> 16) & 0xffu) + (z0 >> 24) + (u32)vsel( mixed ? mA0 : 0UL, 512, 0 );
      u32 const r1 = (z1 & 0xffffu) + ((z1 >> 16) & 0xffu) + (z1 >> 24) + (u32)vsel( mixed ? mA1 : 0UL, 512, 0 );
      u32 T = 0u;
      _Pragma("unroll") for( int b=9; b>=0; b-- ) {   /* keys are below 1024 */
        u32 const Tb = T | (1u << b);
        u32 const c = (u32)(__builtin_popcountll( L0 & __builtin_amdgcn_ballot_w64( r0 >= Tb ) ) +
                            __builtin_popcountll( L1 & __builtin_amdgcn_ballot_w64( r1 >= Tb ) ));
        T = c >= K ? Tb : T;
      }
      u64 const G0 = L0 & __builtin_amdgcn_ballot_w64( r0 > T ), G1 = L1 & __builtin_amdgcn_ballot_w64( r1 > T );
      u64 const E0 = L0 & ~G0 & __builtin_amdgcn_ballot_w64( r0 >= T ), E1 = L1 & ~G1 & __builtin_amdgcn_ballot_w64( r1 >= T );
      u32 const need = K - (u32)(__builtin_popcountll( G0 ) + __builtin_popcountll( G1 ));
      u32 const e0 = (u32)__builtin_popcountll( E0 );
      S0 = G0 | (E0 & __builtin_amdgcn_ballot_w64( lane_rank( E0 ) < need ));
      S1 = G1 | (E1 & __builtin_amdgcn_ballot_w64( e0 + lane_rank( E1 ) < need ));
      rk0 = lane_rank( S0 ); rk1 = (u32)__builtin_popcountll( S0 ) + lane_rank( S1 );
      nsel = K;
    } else {
      /* the step: a pure DBL step (p2 + 4 squares) on up to 64 DBL slots,
         or a MIXED step (k_dsm's uniform 8-mul step) that takes every ADD
         slot first and fills the rest with DBL slots.  An ADD op costs the
         same in either, so ADDs always go through mixed steps; a DBL step
         runs only when it fills the wave (FD_POOL_DBL_PCT 100). */
      mixed = 100u * kD < FD_POOL_DBL_PCT * kM;
      nsel = mixed ? kM : kD;
      /* owner view: the rank of my slots in the selection order [ADD slots
         0..63, ADD slots 64.., DBL slots 0..63, DBL slots 64..] (ADDs only
         in a mixed step) is their processing lane.  Class bits are the
         wave-uniform masks used as lane masks (inverse ballot, v_cndmask):
         no per-lane shifts of the masks. */
      u64 const sA0 = mixed ? mA0 : 0UL, sA1 = mixed ? mA1 : 0UL;
      u32 const aoff = mixed ? nA : 0u;                         /* DBL ranks start after the ADDs */
      u32 const pa0 = (u32)__builtin_popcountll( sA0 ), pd0 = (u32)__builtin_popcountll( mD0 );
      rk0 = (u32)vsel( sA0, (i32)lane_rank( sA0 ), (i32)(aoff + lane_rank( mD0 )) );
      rk1 = (u32)vsel( sA1, (i32)(pa0 + lane_rank( sA1 )), (i32)(aoff + pd0 + lane_rank( mD1 )) );
      S0 = (sA0 | mD0) & __builtin_amdgcn_ballot_w64( rk0 < 64u );
      S1 = (sA1 | mD1) & __builtin_amdgcn_ballot_w64( rk1 < 64u );
    }
    bool in0 = __builtin_amdgcn_inverse_ballot_w64( S0 ), in1 = __builtin_amdgcn_inverse_ballot_w64( S1 );
    mA0 &= ~S0; mA1 &= ~S1; mD0 &= ~S0; mD1 &= ~S1;
#ifdef FD_AMD_DIAG
    dbg_steps++; dbg_lanes += nsel; dbg_add += mixed;
    if( dbg_after ) { dbg_sa++; dbg_la += nsel; }
#endif
    bool live = l < nsel;
    /* slot of rank l: each selected slot's owner writes it at its rank (the
       wave's LDS accesses complete in order: no barrier for a one-wave group) */
    if( in0 ) s_list[rk0] = l;
    if( in1 ) s_list[rk1] = l + 64u;
    __builtin_amdgcn_wave_barrier();
    u32 s = live ? s_list[l] : 0u;
    uint4 m = s_m[s];
    u32 op = live ? m.w : (u32)OP_D;    /* dead lanes: harmless reads, nothing stored */
    u32 si = live ? m.x : 0u;
    u32 hA = m.y & 0xffffu, hB = m.y >> 16;
    int p = (int)(short)(m.z & 0xffffu);
    u32 ja = (m.z >> 16) & 0xffu, jb = m.z >> 24;
    /* the consumed event's successor (popped after the op): its dword */
    u32 pidx = (op == OP_AA && ja >= 2u) ? ja - 2u : (op == OP_AB && jb >= 2u) ? 64u + jb - 2u : 0u;
    bool pop = (op == OP_AA && ja >= 2u) || (op == OP_AB && jb >= 2u);
    /* lanes that pop nothing read one shared, cache-resident word instead of
       their own event row (a load under a branch would wait at the join) */
    u32 const * nha = pop ? (u32 const *)(dig + (size_t)si*128u) + (pidx >> 1) : (u32 const *)&g_bi12[0][0];
    u32 nh = *nha;
    p1p1 t;
    pool_load_ts( t, &s_t[0][s], P );

    if( mixed ) {
      bool isadd = op == OP_AA || op == OP_AB;
      int dg = (op == OP_AA) ? (int)(i8)(hA >> 8) : (int)(i8)(hB >> 8);
      bool neg = isadd && dg < 0;
      int e = isadd ? ((dg < 0 ? -dg : dg) >> 1) & 7 : 0;
      i32 const * qb = (op == OP_AA) ? Ai + (size_t)si*384u + e*48 : &g_bi12[e][0];
      int const rowM = neg ? 2 : 1, rowP = neg ? 1 : 2;
      fe q[4];
#     define Q_ROW( R_, C_ ) do {                                                     \
        int4 const * src_ = (int4 const *)(qb + (C_)*12);                            \
        int4 x0 = src_[0], x1 = src_[1], x2 = src_[2];                               \
        q[R_].v[0] = x0.x; q[R_].v[1] = x0.y; q[R_].v[2] = x0.z; q[R_].v[3] = x0.w;  \
        q[R_].v[4] = x1.x; q[R_].v[5] = x1.y; q[R_].v[6] = x1.z; q[R_].v[7] = x1.w;  \
        q[R_].v[8] = x2.x; q[R_].v[9] = x2.y;                                        \
      } while(0)
      Q_ROW( 0, 0 ); Q_ROW( 1, rowM ); Q_ROW( 2, rowP ); Q_ROW( 3, 3 );
#     undef Q_ROW
      p3 u = ge_p1p1_to_p3_fold( t );
      /* the table operand is first touched here, after p1p1 -> p3 (its x19
         pre-multiples would otherwise be scheduled first and wait for it) */
      _Pragma("unroll") for( int r=0; r<4; r++ )
        asm volatile( "" : "+v"(q[r].v[0]), "+v"(q[r].v[1]), "+v"(q[r].v[2]), "+v"(q[r].v[3]), "+v"(q[r].v[4]),
                           "+v"(q[r].v[5]), "+v"(q[r].v[6]), "+v"(q[r].v[7]), "+v"(q[r].v[8]), "+v"(q[r].v[9])
                         : "v"(u.X.v[9]), "v"(u.T.v[9]) );
      /* k_dsm's op body and mix (see k_dsm) */
      u64 mD = __builtin_amdgcn_ballot_w64( !isadd ), mN = __builtin_amdgcn_ballot_w64( neg );
      fe m0, m1, m2, m3;
      {
        fe a0, b0, a1, b1, a2, b2, a3, b3;
        _Pragma("unroll") for( int k=0; k<10; k++ ) {
          i32 xy = u.X.v[k] + u.Y.v[k];
          a0.v[k] = xy;                                     b0.v[k] = vsel( mD, xy, q[2].v[k] );
          a1.v[k] = vsel( mD, u.Y.v[k], u.Y.v[k] - u.X.v[k] ); b1.v[k] = vsel( mD, u.Y.v[k], q[1].v[k] );
          a2.v[k] = u.Z.v[k];                              b2.v[k] = vsel( mD, u.Z.v[k] + u.Z.v[k], q[0].v[k] );
          a3.v[k] = vsel( mD, u.X.v[k], u.T.v[k] );        b3.v[k] = vsel( mD, u.X.v[k], q[3].v[k] );
        }
        fe_mul_fold2w<true, true>( m0, a0, b0, m1, a1, b1 );
        fe_mul_fold2w<false, true>( m2, a2, b2, m3, a3, b3 );
      }
      {
        u64 mS = mD | mN;
        i32 Dv = vsel( mD, -1, 0 ), Sv = vsel( mS, -1, 0 ), Sn = vsel( mS, 1, 0 );
        i32 cXe = Dv & (1<<25), cXo = Dv & (1<<24);
        i32 cZe = vsel( mD, 0, vsel( mN, (1<<25), -(1<<25) ) ), cZo = vsel( mD, 0, vsel( mN, (1<<24), -(1<<24) ) );
        i32 const nb2e = (i32)fd_opaque( -(2L<<25) ), nb2o = (i32)fd_opaque( -(2L<<24) );   /* SGPR */
        i32 const sT = vsel( mD, 0, 2 );
        _Pragma("unroll") for( int k=0; k<10; k++ ) {
          i32 cX = (k & 1) ? cXo : cXe, cZ = (k & 1) ? cZo : cZe;
          i32 A0 = m0.v[k], A1 = m1.v[k], A2 = m2.v[k], A3 = m3.v[k];
          i32 sA3 = fd_xad( A3, Sv, Sn );
          i32 z2 = A2 + A2;
          i32 Z = fd_add3( vsel( mD, A1, z2 ), sA3, cZ );
          t.X.v[k] = fd_add3( A0 - A1, sA3 & Dv, cX );
          t.Y.v[k] = fd_add3s( A1, vsel( mD, A3, A0 ), (k & 1) ? nb2o : nb2e );
          t.Z.v[k] = Z;
          t.T.v[k] = (i32)((u32)A2 << (u32)sT) - Z;
        }
      }
    } else {
      /* p1p1 -> p2 (the first three products of p1p1 -> p3), then the
         doubling (avx/fd_ed25519_ge.c:493-498) with squares */
      fe uZ, uY, uX;
      fe_mul_fold2w( uZ, t.Z, t.T, uY, t.Z, t.Y );
      uX = fe_mul_fold1( t.X, t.T );
      fe xy = fe_add( uX, uY );
      fe a, b, c, d;
      fe_sq_fold2w<false, false>( a, xy, b, uY );
      fe_sq_fold2w<false, true>( c, uX, d, uZ );
      _Pragma("unroll") for( int k=0; k<10; k++ ) {
        i32 z = b.v[k] - c.v[k];
        t.X.v[k] = a.v[k] - b.v[k] - c.v[k];
        t.Y.v[k] = b.v[k] + c.v[k];
        t.Z.v[k] = z;
        t.T.v[k] = d.v[k] - z;
      }
    }

    /* advance the op stream: pop the consumed event, then the next op
       (branch-free: every select is a lane mask) */
    bool const isAA = op == OP_AA, isAB = op == OP_AB, isDb = op == OP_D;
    {
      u32 ev = __builtin_amdgcn_ubfe( nh, (pidx & 1u) << 4, 16u );
      ja -= (u32)isAA; jb -= (u32)isAB;
      hA = isAA ? (ja ? ev : 0xffffu) : hA;
      hB = isAB ? (jb ? ev : 0xffffu) : hB;
    }
    bool const toAA = isDb && hA != 0xffffu && (hA & 0xffu) == (u32)p;
    bool const toAB = !toAA && (isDb || isAA) && hB != 0xffffu && (hB & 0xffu) == (u32)p;
    p -= (int)!(toAA || toAB);
    u32 nop = !live ? (u32)OP_EMPTY : toAA ? (u32)OP_AA : toAB ? (u32)OP_AB : (p < 0) ? (u32)OP_EMPTY : (u32)OP_D;
    if( live ) {
      if( nop == OP_EMPTY ) {
        pool_store_t( (int4 *)(Ai + (size_t)si*384u), t );   /* park the final p1p1 for k_fin */
      } else {
        pool_store_ts( &s_t[0][s], P, t );
        s_m[s] = make_uint4( si, hA | (hB << 16), ((u32)p & 0xffffu) | (ja << 16) | (jb << 24), nop );
      }
    }
    /* the slots' new classes, at their owner lanes */
    u32 v0 = (u32)__builtin_amdgcn_ds_bpermute( (int)(rk0 << 2), (int)nop );
    u32 v1 = (u32)__builtin_amdgcn_ds_bpermute( (int)((rk1 & 63u) << 2), (int)nop );
    u64 const d0 = __builtin_amdgcn_ballot_w64( v0 == OP_D ), d1 = __builtin_amdgcn_ballot_w64( v1 == OP_D );
    u64 const x0 = __builtin_amdgcn_ballot_w64( v0 < OP_EMPTY ), x1 = __builtin_amdgcn_ballot_w64( v1 < OP_EMPTY );
    mD0 |= S0 & d0; mA0 |= S0 & x0 & ~d0;                       /* OP_AA / OP_AB: below OP_EMPTY, not OP_D */
    mD1 |= S1 & d1; mA1 |= S1 & x1 & ~d1;
  }
  if( guard && l == 0u ) atomicOr( (u32 *)(ws + L.ctr) + 1, 1u );
#ifdef FD_AMD_DIAG
  if( l == 0u ) { atomicAdd( &g_pool_dbg[0], dbg_steps ); atomicAdd( &g_pool_dbg[1], dbg_lanes ); atomicAdd( &g_pool_dbg[2], dbg_add ); atomicAdd( &g_pool_dbg[3], dbg_idle ); }
  if( l == 0u && w < 8192u ) { g_pool_dbg_t[w][0] = dbg_t0; g_pool_dbg_t[w][1] = dbg_te; g_pool_dbg_t[w][2] = wall_clock64(); g_pool_dbg_t[w][3] = dbg_sa | (dbg_la << 32); }
#else
  (void)w;
#endif
}

#ifdef FD_AMD_DIAG
extern "C" int
fd_amd_pool_debug( unsigned * out, int reset ) {
  if( hipMemcpyFromSymbol( out, HIP_SYMBOL( g_pool_dbg ), sizeof(unsigned)*4 ) != hipSuccess ) return -1;
  if( reset ) { unsigned z[4] = { 0, 0, 0, 0 }; if( hipMemcpyToSymbol( HIP_SYMBOL( g_pool_dbg ), z, sizeof(z) ) != hipSuccess ) return -1; }
  return 0;
}
extern "C" int
fd_amd_pool_debug_times( unsigned long * out /* [8192][4] */ ) {
  return hipMemcpyFromSymbol( out, HIP_SYMBOL( g_pool_dbg_t ), sizeof(unsigned long)*8192*4 ) == hipSuccess ? 0 : -1;
}
#endif

__global__ void __launch_bounds__(64)
k_fin( u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats ) {
  u32 i = blockIdx.x * 64u + threadIdx.x;
  if( i >= n ) return;
  size_t N = L.N;
  if( ((u32 const *)(ws + L.ctr))[1] ) { err[i] = (i8)FD_AMD_VERDICT_DEVICE; return; }   /* k_dsmp's guard tripped */
  bool act = err[i] == 1;
  int top = ((int const *)(ws + L.top))[i];
  if( act ) {
    p1p1 t;
    if( top < 0 ) { t.X = fe_zero(); t.Y = fe_one(); t.Z = fe_one(); t.T = fe_one(); }
    else pool_load_t( t, (int4 const *)((i32 const *)(ws + L.Ai) + (size_t)i*384u) );
    fe uZ, uY, uX;
    fe_mul_fold2w( uZ, t.Z, t.T, uY, t.Z, t.Y );
    uX = fe_mul_fold1( t.X, t.T );
    i32 const * Rw = (i32 const *)(ws + L.R);
    fe RX, RY;
    _Pragma("unroll") for( int k=0; k<10; k++ ) { RX.v[k] = Rw[(size_t)k*N + i]; RY.v[k] = Rw[(size_t)(10+k)*N + i]; }
    fe xZ, yZ;
    fe_mul_fold2w( xZ, uZ, RX, yZ, uZ, RY );
    bool eq = true;
    _Pragma("unroll") for( int k=0; k<8; k++ ) eq = eq && (xZ.v[k] == uX.v[k]) && (yZ.v[k] == uY.v[k]);
    err[i] = (i8)(eq ? 0 : -3);
  }
  if( want_stats ) {
    u32 ne = ((u32 const *)(ws + L.evn))[i];
    u32 * st = (u32 *)(ws + L.st);
    st[i] = act ? (u32)(top + 1) : 0u; st[N + i] = act ? (ne & 0xffu) : 0u; st[2*N + i] = act ? ((ne >> 8) & 0xffu) : 0u;
  }
}

/* ------------------------------------------------------------------ */
/* k_tile_persist: the streaming tile's persistent consumer.
 *
 * The reference verify tile (src/app/frank/load/fd_frank_verify_synth_load.c:
 * 219-437) verifies one frag per call on one core; N tiles scale it.  Here
 * one launch per tile run holds every wave slot of the GPU (one single-wave
 * workgroup per slot) and verifies what the tile's host thread hands over
 * through mapped host memory: the frags' ring entries, and CHUNK
 * descriptors {first ring index, count, mode} that the host cuts from each
 * hand-off (mode: 8 lanes per signature while the GPU is lightly loaded,
 * for latency; 1 lane per signature under load, for throughput).
 *
 *   wave 0 (scout)   the only poller of host memory: it mirrors the host's
 *                    descriptor head, its stop request and a heartbeat into
 *                    one word per XCD (device memory, one line each);
 *   waves 1..        take a TICKET (one atomic add per chunk, never
 *                    retried), wait on their XCD's mirror word until
 *                    descriptor `ticket` exists, read it, and verify the
 *                    chunk alone: copy the frags in (and, zero-copy, out to
 *                    their output frames), k_prep's body, k_decomp's body,
 *                    then k_dsm8's body or k_dsm's body, then verdict + tag
 *                    to the mapped result ring, released after a
 *                    system-scope fence so the host sees them in full.
 *
 * Contention is what this layout avoids: a first version let every idle
 * wave load the shared head and CAS a claim counter; 2000 waves on one
 * line made every atomic take ~20 us and stalled the CUs' memory pipelines
 * (every phase, the DSM loop included, ran 8-10x slow).  Now each chunk
 * costs one atomic add, and a waiting wave polls its XCD's mirror with a
 * back-off proportional to how far its ticket is from the head.  Every
 * spin is bounded: the scout flags an error after `watchdog` ticks without
 * a host heartbeat, a waiting wave exits after `watchdog` ticks with an
 * unchanged mirror word, so the grid always drains.
 *
 * Same bodies as the batch kernels, same workspace layout (one N = 64
 * workspace per wave): identical limbs and verdicts. */

#define TILE_FRAME (1408u)   /* FD_VERIFY_AMD_FRAME_SZ */
#define TILE_MODE_THR   (0u)   /* 1 lane per signature, <= 64 slots (k_dsm's body) */
#define TILE_MODE_LAT8  (1u)   /* 8 lanes per signature, <= 8 slots (k_dsm8's body) */
#define TILE_MODE_QUAD4 (2u)   /* 4 lanes per signature, <= 16 slots (k_dsm4's body) */

__device__ __forceinline__ u64 ld_sys64( u64 const * p ) { return __hip_atomic_load( (u64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM ); }
__device__ __forceinline__ u32 ld_sys32( u32 const * p ) { return __hip_atomic_load( (u32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM ); }
__device__ __forceinline__ void st_sys64( u64 * p, u64 v ) { __hip_atomic_store( p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM ); }
__device__ __forceinline__ void st_sys32( u32 * p, u32 v ) { __hip_atomic_store( p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM ); }
__device__ __forceinline__ u64 ld_dev64( u64 const * p ) { return __hip_atomic_load( (u64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
__device__ __forceinline__ u32 ld_dev32( u32 const * p ) { return __hip_atomic_load( (u32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
__device__ __forceinline__ void st_dev32( u32 * p, u32 v ) { __hip_atomic_store( p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
__device__ __forceinline__ void st_dev64( u64 * p, u64 v ) { __hip_atomic_store( p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
__device__ __forceinline__ u64 rfl64( u64 v ) {
  return ((u64)(u32)__builtin_amdgcn_readfirstlane( (int)(u32)(v >> 32) ) << 32) | (u32)__builtin_amdgcn_readfirstlane( (int)(u32)v );
}

/* mirror word: descriptor head | scout heartbeat << 48 | err << 62 | stop << 63 */
#define TILE_MW_HEAD(w)  ((w) & ((1UL << 48) - 1UL))
#define TILE_MW_ERR      (1UL << 62)
#define TILE_MW_STOP     (1UL << 63)

/* per-wave scratch: an N = 64 workspace, then the chunk's frames and planes */
struct tile_scratch_t { size_t mir, pub, sig, off, sz, err, skp, tx, total; };
__host__ __device__ constexpr tile_scratch_t tile_scratch_layout( void ) {
  tile_scratch_t S = {}; size_t o = ws_al( ws_layout_const( 64 ).total );
  S.mir = o; o = ws_al( o + 64UL*TILE_FRAME );
  S.pub = o; o = ws_al( o + 64UL*32UL );
  S.sig = o; o = ws_al( o + 64UL*64UL );
  S.off = o; o = ws_al( o + 64UL*4UL );
  S.sz  = o; o = ws_al( o + 64UL*4UL );
  S.err = o; o = ws_al( o + 64UL );
  S.skp = o; o = ws_al( o + 64UL );          /* TXN: per slot, nonzero = its transaction failed to parse */
  S.tx  = o; o = ws_al( o + 64UL*4UL );      /* TXN: per entry, first slot | slots << 8 | parsed << 31 */
  S.total = o;
  return S;
}

size_t fd_amd_tile_scratch_stride( void ) { return tile_scratch_layout().total; }

/* The scout (wave 0, lane 0): host words -> the XCDs' mirror words, and
   back to the host every ~10 us its clock (the host maps the waves' time
   stamps onto its own clock with it; its first store tells the host the
   kernel started) and the count of finished chunks (the host's progress
   watchdog). */
#ifdef FD_AMD_SCOUT_NOINLINE   /* A/B only: the round-4 called scout (profiles/r05_scout_stop_cause.txt) */
__device__ __noinline__ void
#else
__device__ __forceinline__ void
#endif
tile_scout( fd_amd_tile_dctl_t * D, fd_amd_tile_hctl_t * H, u64 watchdog ) {
  __builtin_amdgcn_s_setprio( 3 );   /* beside the workers' aged chunks on its SIMD */
  u64 word = ld_dev64( &D->mw[0].w ), lastb = ~0UL, beat = 0UL;
  u64 tb = __builtin_amdgcn_s_memrealtime(), tpub = tb, tclk = tb;
  st_sys64( &H->gclock, tb );
  for( ;; ) {
    u64 h = ld_sys64( &H->head ), b = ld_sys64( &H->beat );
    u32 st = ld_sys32( &H->stop );
    u64 now = __builtin_amdgcn_s_memrealtime();
    if( now - tclk >= 1000UL ) {
      tclk = now;
      st_sys64( &H->gdone, ld_dev64( &D->done ) );
      st_sys64( &H->gclock, now );
    }
    if( b != lastb ) { lastb = b; tb = now; }
    bool dead = now - tb > watchdog;
    if( dead ) st_sys32( &H->kerr, 1u );
    /* the heartbeat field advances at most every 10 us (it only keeps the
       waiting waves' own watchdog quiet) */
    if( now - tpub > 1000UL && now - tb < 1000UL ) { beat++; tpub = now; }
    u64 w = (h & ((1UL << 48) - 1UL)) | ((beat & 0x3fffUL) << 48) | (dead ? TILE_MW_ERR : 0UL) | (st ? TILE_MW_STOP : 0UL);
    if( w != word ) {
      word = w;
      _Pragma("unroll") for( int x=0; x<FD_AMD_TILE_MIRRORS; x++ ) st_dev64( &D->mw[x].w, w );
    }
    if( st || dead ) break;
    __builtin_amdgcn_s_sleep( 2 );
  }
}

/* nw little-endian words from an unaligned address inside a frame: nw + 1
   aligned dword loads funnel-shifted by the misalignment (the frame has
   room for the extra word: frames are FD_VERIFY_AMD_FRAME_SZ >= MTU + 4). */
template<int NW>
__device__ __forceinline__ void
ld_words_unaligned( u8 const * p, u32 (&o)[NW] ) {
  u32 const * a = (u32 const *)((size_t)p & ~(size_t)3);
  u32 const sh = (u32)(size_t)p & 3u;
  u32 w[NW + 1];
  _Pragma("unroll") for( int k=0; k<=NW; k++ ) w[k] = a[k];
  _Pragma("unroll") for( int k=0; k<NW; k++ ) o[k] = __builtin_amdgcn_alignbyte( w[k+1], w[k], sh );   /* byte shift */
}

/* TXN framing: the chunk's k ring entries are wire transactions (frames
   0..k-1 of mir) carrying e_k signature slots each (the host's count,
   fd_amd_txn_slots1; the chunk's total <= 64).  Lane q < k parses
   transaction q (fd_txn_parse semantics, fd_txn_dev.h); lane s < n then
   lays slot s out for the verify bodies: signature i of its transaction
   with account address i over the shared message bytes in mir
   (fd_txn.h:159-217), or skip = FD_TXN_AMD_ERR_PARSE when the transaction
   failed to parse (or parsed to a signature count other than the host's:
   fail closed).  tx[q] keeps the entry's first slot, slot count and parse
   flag for the per-transaction reduce.  lds: >= 64 x 5 words of scratch
   LDS (the DSM bodies' event rows, unused until then).  Returns n, the
   chunk's signature slots (wave-uniform). */
__device__ __forceinline__ u32
tile_txn_layout( u32 l, u32 k, u32 e_sz, u32 e_k, u8 const * __restrict__ mir, u8 * __restrict__ pub,
                 u8 * __restrict__ sig, u32 * __restrict__ off, u32 * __restrict__ sz, i8 * __restrict__ skp,
                 u32 * __restrict__ tx, u32 * __restrict__ lds ) {
  u32 const kk = l < k ? e_k : 0u;
  u32 inc = kk;
  _Pragma("unroll") for( int d=1; d<64; d<<=1 ) {
    u32 const o = (u32)__shfl_up( (int)inc, (unsigned)d );
    if( l >= (u32)d ) inc += o;
  }
  u32 const base = inc - kk;
  u32 const n = min( (u32)__shfl( (int)inc, 63 ), 64u );
  u32 * own  = lds;            /* [64]: slot -> entry */
  u32 * info = lds + 64;       /* [64][5]: sig_off, acct_off, msg_off (~0: not parsed), frag size, first slot */
  if( l < k ) {
    u32 nsig = 0u, sig_off = 0u, acct_off = 0u, msg_off = 0u;
    u32 const fp = fd_txn_dev::txn_parse( mir + (size_t)l * TILE_FRAME, e_sz, (u8 *)0, &nsig, &sig_off, &acct_off, &msg_off );
    u32 const ok = fp != 0u && nsig == kk && base + kk <= 64u;   /* the host packs <= 64 slots per chunk */
    for( u32 i=0u; i<kk && base + i < 64u; i++ ) own[base + i] = l;
    u32 * in = info + 5u*l;
    in[0] = sig_off; in[1] = acct_off; in[2] = ok ? msg_off : 0xFFFFFFFFu; in[3] = e_sz; in[4] = base;
    tx[l] = base | (kk << 8) | (ok << 31);
  }
  __syncthreads();
  if( l < n ) {
    u32 const q = own[l];
    u32 const * in = info + 5u*q;
    u32 const i = l - in[4];
    u32 const msg_off = in[2];
    if( msg_off != 0xFFFFFFFFu ) {
      u8 const * f = mir + (size_t)q * TILE_FRAME;
      u32 a[8], g[16];
      ld_words_unaligned<8>( f + in[1] + 32u*i, a );
      ld_words_unaligned<16>( f + in[0] + 64u*i, g );
      uint4 * P = (uint4 *)(pub + 32u*l);
      uint4 * G = (uint4 *)(sig + 64u*l);
      P[0] = make_uint4( a[0], a[1], a[2], a[3] );   P[1] = make_uint4( a[4], a[5], a[6], a[7] );
      G[0] = make_uint4( g[0], g[1], g[2], g[3] );   G[1] = make_uint4( g[4], g[5], g[6], g[7] );
      G[2] = make_uint4( g[8], g[9], g[10], g[11] ); G[3] = make_uint4( g[12], g[13], g[14], g[15] );
      off[l] = q * TILE_FRAME + msg_off; sz[l] = in[3] - msg_off; skp[l] = 0;
    } else {
      off[l] = 0u; sz[l] = 0u; skp[l] = (i8)TXN_ERR_PARSE;
    }
  }
  return n;
}

/* Copy a chunk's k frags in: frame q (16-B word w of it) by lane 16 (q % 4)
   + (w % 16) of round q / 4; four rounds (16 frames) have every load
   issued before any store, so a 64-frag chunk waits four round trips to
   the frames' memory (host memory over PCIe in zero-copy mode), not
   sixteen (gather 92 -> 62 us per chunk at saturation, paced service p50
   1.30 -> 1.25 ms: profiles/r05_tile_pool_experiment.txt).  Frames are
   <= 1328 B = 83 words, chunk-aligned (every 16-B word whole): up to six
   words per lane per round.  Zero copy: every word also goes out to the
   frag's output frame; PUB_SIG_MSG: pub and sig to their planes. */
__device__ __forceinline__ void
tile_gather( fd_amd_tile_args_t const & A, u32 k, u32 l, u32 e_src, u32 e_out, u32 e_sz, u8 * __restrict__ mir,
             u8 * __restrict__ pub, u8 * __restrict__ sig, bool txn ) {
  u32 const g = l >> 4, j = l & 15u;
  for( u32 q0 = 0; q0 < k; q0 += 16u ) {
    uint4 v[4][6];
    u32 nv[4];
    _Pragma("unroll") for( int h=0; h<4; h++ ) {
      u32 const q = q0 + 4u*(u32)h + g;
      u32 const src = (u32)__shfl( (int)e_src, (int)(q & 63u) );
      u32 const fs  = (u32)__shfl( (int)e_sz,  (int)(q & 63u) );
      nv[h] = q < k ? (fs + 15u) >> 4 : 0u;
      uint4 const * s = (uint4 const *)(A.src + ((size_t)src << 6));
      _Pragma("unroll") for( int r=0; r<6; r++ ) {
        u32 w = j + 16u*(u32)r;
        v[h][r] = w < nv[h] ? s[w] : make_uint4( 0u, 0u, 0u, 0u );
      }
    }
    _Pragma("unroll") for( int h=0; h<4; h++ ) {
      u32 const q = q0 + 4u*(u32)h + g;
      u32 const oc = (u32)__shfl( (int)e_out, (int)(q & 63u) );
      uint4 * m = (uint4 *)(mir + (size_t)(q & 63u) * TILE_FRAME);
      uint4 * o = A.out ? (uint4 *)(A.out + ((size_t)oc << 6)) : (uint4 *)0;
      _Pragma("unroll") for( int r=0; r<6; r++ ) {
        u32 w = j + 16u*(u32)r;
        if( w < nv[h] ) { m[w] = v[h][r]; if( o ) o[w] = v[h][r]; }
      }
      if( q < k && !txn ) {
        if( j < 2u )      ((uint4 *)(pub + 32u*q))[j]      = v[h][0];
        else if( j < 6u ) ((uint4 *)(sig + 64u*q))[j - 2u] = v[h][0];
      }
    }
  }
}

#ifdef FD_AMD_TILE_QUAD_NOINLINE
__device__ __noinline__ void
tile_dsm4_call( u32 l, u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, i32 (* __restrict__ bi)[48],
                u64 (* __restrict__ evl)[33], u64 tc ) {
  dsm4_body( l, n, err, ws, L, 0, bi, evl, tc );
}
#endif

/* Verify ring entries [c0, c0 + k) (k <= 64) on this wave, claimed at
   s_memrealtime tc, in chunk mode `mode` (TILE_MODE_*: 1 lane per signature,
   8 lanes (k_dsm8's body) or 4 lanes (k_dsm4's body); the host keeps a
   chunk's slots within the mode's 64 / 8 / 16 lanes).  PUB_SIG_MSG: entry q is signature slot q.  TXN
   (A.txn): entry q is a wire transaction whose slots tile_txn_layout lays
   out, and its result is the transaction's verdict. */
__device__ __forceinline__ void
tile_chunk( fd_amd_tile_args_t const & A, u64 c0, u32 k, u32 mode, u8 * __restrict__ scr, ws_layout_t L,
            tile_scratch_t const & S, i32 (* __restrict__ bi)[48], u64 (* __restrict__ evl)[33], u64 * pt, u64 tc,
            u32 pp = 0u ) {
  /* pp = pair | pair_seq << 2 (quad pairs, FD_AMD_TILE_PAIR); pair: 0 none;
     1 sub 0 -- the front of all k entries, then the pair's flag =
     pair_seq + 1, then entries [0, 16); 2 sub 1 (the caller saw that flag)
     -- entries [16, k) on sub 0's front */
  u32 const pair = pp & 3u;
  /* pt (A.prof, set by the diagnostics build's host only): s_memrealtime
     ticks spent in gather [0], prep [6], decomp [1], DSM [2], results [3];
     wave-uniform */
  u64 ts = A.prof ? __builtin_amdgcn_s_memrealtime() : 0UL;
# define TILE_STAMP( k_ ) do { if( A.prof ) { u64 t_ = __builtin_amdgcn_s_memrealtime(); if( !threadIdx.x ) pt[k_] += t_ - ts; ts = t_; } } while(0)
  /* opaque per chunk: otherwise the compiler hoists every per-lane address
     of the bodies out of the persistent loop and spills them */
  {
    __attribute__((address_space(1))) u8 * g = (__attribute__((address_space(1))) u8 *)scr;
    asm volatile( "" : "+s"(g) );
    scr = (u8 *)g;     /* still known global: global, not flat, accesses */
  }
  u32 l = threadIdx.x;
  asm volatile( "" : "+v"(l) );
  u8 * ws = scr; u8 * mir = scr + S.mir; u8 * pub = scr + S.pub; u8 * sig = scr + S.sig;
  u32 * off = (u32 *)(scr + S.off); u32 * sz = (u32 *)(scr + S.sz); i8 * err = (i8 *)(scr + S.err);

  /* 1. the chunk's ring entries, lane q holds entry q (host memory: system-scope loads) */
  bool const txn = A.txn != 0u;
  /* a pair's sub 1 runs the front on no entries (its barriers only: a
     branch round the front costs the loop a VGPR spill) */
  u32 const kf = pair == 2u ? 0u : k;
  u32 e_src = 0u, e_out = 0u, e_sz = 96u, e_k = 0u;
  if( l < kf ) {
    u64 const * ep = (u64 const *)(A.ent + ((c0 + l) & A.mask));
    u64 w0 = ld_sys64( ep ), w1 = ld_sys64( ep + 1 );
    e_src = (u32)w0; e_out = (u32)(w0 >> 32); e_sz = (u32)w1; e_k = (u32)(w1 >> 32);
  }
  /* 2. copy the frags in (tile_gather) */
  tile_gather( A, kf, l, e_src, e_out, e_sz, mir, pub, sig, txn );
  if( l < kf && !txn ) { off[l] = l * TILE_FRAME + 96u; sz[l] = e_sz - 96u; }
  __syncthreads();
  /* TXN: parse and lay the chunk's signature slots out (n of them) */
  i8 * skp = (i8 *)(scr + S.skp);
  u32 * tx = (u32 *)(scr + S.tx);
  u32 const n = txn ? tile_txn_layout( l, k, e_sz, e_k, mir, pub, sig, off, sz, skp, tx, (u32 *)&evl[0][0] ) : kf;
  if( txn ) __syncthreads();
  TILE_STAMP( 0 );
  /* 3. the verify pipeline on the chunk (k_prep, k_decomp, k_dsm / k_dsm8 / k_dsm4 bodies) */
  prep_body( l, n, pub, sig, off, sz, mir, err, ws, L, txn ? (i8 const *)skp : (i8 const *)0 );
  __syncthreads();
  TILE_STAMP( 6 );
  decomp_body( l, n, pub, sig, err, ws, L, true );                 /* points 0..63: signatures 0..31 */
  if( n > 32u ) decomp_body( l + 64u, n, pub, sig, err, ws, L, true );
  __syncthreads();
  TILE_STAMP( 1 );
  if( pair == 1u ) {
    /* the pair's front is done: every lane's workspace writes out of this
       XCD's L2 (agent-scope release), then the flag sub 1 waits on */
    __builtin_amdgcn_fence( __ATOMIC_RELEASE, "agent" );
    __syncthreads();
    if( l == 0u ) st_dev32( A.pair_flag + ((pp >> 2) & A.pair_mask), (pp >> 2) + 1u );
  }
  /* this wave's signatures: all k, or a pair sub's 16 */
  u32 const g0 = pair == 2u ? 64u : 0u;                 /* k_dsm4's lane index: signature (g0 + l) >> 2 */
  u32 const nd = pair == 1u ? min( k, 16u ) : pair == 2u ? k : n;
#if defined(FD_AMD_TILE_QUAD_LAST)   /* A/B: code placement of the three bodies */
  if( mode == TILE_MODE_THR )        dsm_lane_body( l, n, err, ws, L, 0, bi, evl, tc );
  else if( mode == TILE_MODE_LAT8 )  dsm8_body( l, n, err, ws, L, 0, bi, evl, tc );
  else                               dsm4_body( l, n, err, ws, L, 0, bi, evl, tc );
#elif defined(FD_AMD_TILE_QUAD_NOINLINE)
  if( mode == TILE_MODE_LAT8 )       dsm8_body( l, n, err, ws, L, 0, bi, evl, tc );
  else if( mode == TILE_MODE_QUAD4 ) tile_dsm4_call( l, n, err, ws, L, bi, evl, tc );
  else                               dsm_lane_body( l, n, err, ws, L, 0, bi, evl, tc );
#else
  if( mode == TILE_MODE_LAT8 )       dsm8_body( l, n, err, ws, L, 0, bi, evl, tc );
#ifndef FD_AMD_TILE_NO_QUAD   /* A/B only: the tile kernel without the quad body (quad chunks run 1 lane each) */
  else if( mode == TILE_MODE_QUAD4 ) dsm4_body( g0 + l, nd, err, ws, L, 0, bi, evl, tc );
#endif
  else                               dsm_lane_body( l, n, err, ws, L, 0, bi, evl, tc );
#endif
  __builtin_amdgcn_s_setprio( 0 );
  __syncthreads();
  TILE_STAMP( 2 );
  /* 4. results: tags (and, zero-copy, the output frames above) first, one
        system-scope release, then the words the host polls.  TXN: an entry's
        verdict is its parse failure, else the first failing signature's
        code in signature order, else 0 (k_txn_reduce); its tag is its first
        signature's */
  u32 const e0 = pair == 2u ? 16u : 0u, e1 = pair == 1u ? min( k, 16u ) : k;   /* this wave's entries */
  u32 const q = e0 + l;
  u64 const idx = c0 + q, j = idx & A.mask;
  u64 tag = 0UL; i8 v = 0;
  if( q < e1 ) {
    if( !txn ) { tag = ((u64 const *)(ws + L.tag))[q]; v = err[q]; }
    else {
      u32 const w = tx[l], b = w & 0xffu, kk = (w >> 8) & 0xffu;
      if( !(w >> 31) ) v = (i8)TXN_ERR_PARSE;
      else for( u32 i=0u; i<kk; i++ ) { i8 const e = err[b + i]; if( e ) { v = e; break; } }
      if( kk ) tag = ((u64 const *)(ws + L.tag))[b];
    }
    st_sys64( A.res_tag + j, tag );
  }
  if( A.res_time && q < e1 ) st_sys64( A.res_time + j, (u64)(u32)tc | ((u64)(u32)__builtin_amdgcn_s_memrealtime() << 32) );
  __builtin_amdgcn_fence( __ATOMIC_RELEASE, "" );
  asm volatile( "s_waitcnt vmcnt(0)" ::: "memory" );
  u64 const wd = ((idx + 1UL) << 8) | (u64)(u8)v;
  if( q < e1 ) st_sys64( A.res_word + j, wd );
  TILE_STAMP( 3 );
# undef TILE_STAMP
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_tile_persist( fd_amd_tile_args_t A ) {
  constexpr ws_layout_t    L = ws_layout_const( 64 );   /* every plane offset an immediate */
  constexpr tile_scratch_t S = tile_scratch_layout();
  __shared__ __attribute__((aligned(16))) i32 bi[8][48];
  __shared__ u64 evl[64][33];
  fd_amd_tile_dctl_t * D = A.dctl;
  u32 const l = threadIdx.x;
  if( blockIdx.x == 0u ) {
    if( l == 0u ) tile_scout( D, A.hctl, A.watchdog );
    return;
  }
  bi12_fill( bi );
  __syncthreads();
#ifdef FD_AMD_TILE_SCRATCH_TOUCH
  /* experiment only (profiles/r06_scout_stop_fix.txt): every dword of the
     wave's private segment (FD_AMD_TILE_SCRATCH_TOUCH bytes, the kernel's
     private_segment_fixed_size) written once under full exec before the
     persistent loop, so the loop's spill slots are not first touched inside
     it */
  _Pragma("unroll") for( int o = 0; o < FD_AMD_TILE_SCRATCH_TOUCH; o += 4 )
    asm volatile( "scratch_store_dword off, %0, off offset:%1" :: "v"(0), "i"(o) : "memory" );
  asm volatile( "s_waitcnt vmcnt(0)" ::: "memory" );
#endif
  /* this wave's mirror word: its XCD's (HW_REG_XCC_ID) */
  u32 const xcc = __builtin_amdgcn_s_getreg( 20 | (0 << 6) | (3 << 11) ) % FD_AMD_TILE_MIRRORS;
  u64 const * mw = &D->mw[xcc].w;
  u8 * scr = A.scratch + (size_t)blockIdx.x * S.total;
  /* per-wave tallies in LDS, not registers (the DSM bodies want every VGPR):
     [0..7] diagnostics build (A.prof) gather, front, DSM, results, wait,
     fence, -, -; [8..13] dctl->stat: latency chunks, throughput chunks,
     their frags, quad chunks, their frags */
  __shared__ u64 s_tally[16];
  if( l < 16u ) s_tally[l] = 0UL;
  u64 * const pt = s_tally;
  /* A run-time flag (the host sets it only in the diagnostics build), not a
     compile-time constant: with the profiling branches folded away the
     compiler gives this kernel all 256 VGPRs, and at 256 its scout wave
     stopped ~0.7 ms into every run, called or inlined (profiles/
     r04_tile_scout_vgpr_ab.txt, r05_scout_stop_cause.txt); build.py refuses
     a build at 256. */
#ifdef FD_AMD_TILE_PROF_CONST   /* A/B only: folds the profiling branches, 256 VGPRs */
  bool const prof = false;
#else
  bool const prof = A.prof != 0u;
#endif
  for( ;; ) {
    u64 t = 0;
    if( l == 0u ) t = atomicAdd( (unsigned long long *)&D->ticket, 1ULL );
    t = rfl64( t );
    /* wait for descriptor t: poll the mirror, backing off with the
       distance to the head (the next in line polls every ~0.2 us) */
    u64 t0 = __builtin_amdgcn_s_memrealtime(), tw = t0, last = ~0UL;
    bool go = false;
    for( ;; ) {
      u64 const w = rfl64( l == 0u ? ld_dev64( mw ) : 0UL );
      if( TILE_MW_HEAD( w ) > t ) { go = true; break; }
      if( w & (TILE_MW_ERR | TILE_MW_STOP) ) break;
      u64 const now = __builtin_amdgcn_s_memrealtime();
      if( w != last ) { last = w; tw = now; }
      else if( now - tw > A.watchdog ) break;       /* no scout (or host) for that long: give up */
      u64 const d = t - TILE_MW_HEAD( w );
      u32 const nap = d < 2UL ? 1u : d < 64UL ? (u32)d : 64u;
      for( u32 z = 0; z < nap; z++ ) __builtin_amdgcn_s_sleep( 4 );
    }
    if( prof && !l ) pt[4] += __builtin_amdgcn_s_memrealtime() - t0;
    if( !go ) break;
    u64 const tc = __builtin_amdgcn_s_memrealtime();   /* claimed */
    /* descriptor t (host memory): { first ring index, count | FD_AMD_TILE_LAT | FD_AMD_TILE_QUAD } */
    u64 c = 0, cm = 0;
    if( l == 0u ) {
      u64 const * dp = (u64 const *)(A.desc + (t & A.mask));
      c = ld_sys64( dp ); cm = ld_sys64( dp + 1 );
    }
    c = rfl64( c ); cm = rfl64( cm );
    u32 const take = FD_AMD_TILE_COUNT( (u32)cm );
    u32 const md = ((u32)cm & FD_AMD_TILE_LAT) ? TILE_MODE_LAT8 : ((u32)cm & FD_AMD_TILE_QUAD) ? TILE_MODE_QUAD4 : TILE_MODE_THR;
    /* quad pair: its shared workspace and flag; sub 1 first waits for sub 0's front */
    u32 const pr = ((u32)cm & FD_AMD_TILE_PAIR) && A.pair_ws && !A.txn && md == TILE_MODE_QUAD4 ? 1u + (u32)((cm >> 32) & 1UL) : 0u;
    u32 const pseq = (u32)(cm >> 33) & 0x3fffffffu;
    u8 * cscr = pr ? A.pair_ws + (size_t)(pseq & A.pair_mask) * S.total : scr;
    u32 * pf = pr ? A.pair_flag + (pseq & A.pair_mask) : (u32 *)0;
    bool pok = true;
    if( pr == 2u ) {
      u64 const tp = __builtin_amdgcn_s_memrealtime();
      for( ;; ) {
        u32 const f = (u32)__builtin_amdgcn_readfirstlane( (int)(l == 0u ? ld_dev32( pf ) : 0u) );
        if( f == pseq + 1u ) break;
        u64 const w = rfl64( l == 0u ? ld_dev64( mw ) : 0UL );
        if( (w & TILE_MW_ERR) || __builtin_amdgcn_s_memrealtime() - tp > A.watchdog ) { pok = false; break; }
        __builtin_amdgcn_s_sleep( 2 );
      }
      __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "agent" );   /* sub 0's workspace writes (another XCD's L2) */
    }
    /* the frames were written by the host (copy mode) or the producer
       (zero-copy) into host memory: drop this CU's stale lines first */
    u64 const tf = prof ? __builtin_amdgcn_s_memrealtime() : 0UL;
    __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "" );
    asm volatile( "s_waitcnt vmcnt(0)" ::: "memory" );
    if( prof && !l ) pt[5] += __builtin_amdgcn_s_memrealtime() - tf;
    if( take && take <= 64u && pok && (!pr || (take > 16u && take <= 32u)) )
      tile_chunk( A, c, take, md, cscr, L, S, bi, evl, pt, tc, pr | pseq << 2 );
    if( !l ) {
      /* dctl->stat slots: chunks, frags -- latency 0, 2; throughput 1, 3; quad 4, 5 (a pair sub is a quad chunk) */
      u32 const tc_ = md == TILE_MODE_LAT8 ? 0u : md == TILE_MODE_THR ? 1u : 4u;
      u32 const tf_ = md == TILE_MODE_LAT8 ? 2u : md == TILE_MODE_THR ? 3u : 5u;
      s_tally[8u + tc_] += 1UL; s_tally[8u + tf_] += pr == 1u ? 16u : pr == 2u ? take - 16u : take;
      atomicAdd( (unsigned long long *)&D->done, 1ULL );   /* progress, mirrored to the host by the scout */
    }
  }
  if( l == 0u ) {
    _Pragma("unroll") for( int q=0; q<6; q++ ) atomicAdd( (unsigned long long *)&D->stat[q], (unsigned long long)s_tally[8 + q] );
    if( prof ) { _Pragma("unroll") for( int q=0; q<8; q++ ) atomicAdd( (unsigned long long *)&D->prof[q], (unsigned long long)pt[q] ); }
  }
}

#ifdef FD_AMD_DIAG
/* Diagnostics build only.  Measurement aid: k_tile_persist's chunk pipeline without the host
   hand-off (no tickets, no polling, nothing in mapped memory): wave w runs
   `iters` chunks of k ring entries, [(w iters + it) k, +k), with every
   argument in device memory (fd_amd_tile_synth, tools/tile_synth.py). */
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_tile_synth( fd_amd_tile_args_t A, u32 iters, u32 eight ) {
  constexpr ws_layout_t    L = ws_layout_const( 64 );
  constexpr tile_scratch_t S = tile_scratch_layout();
  __shared__ __attribute__((aligned(16))) i32 bi[8][48];
  __shared__ u64 evl[64][33];
  bi12_fill( bi );
  __syncthreads();
  __shared__ u64 pt[8];
  if( threadIdx.x < 8u ) pt[threadIdx.x] = 0UL;
  __syncthreads();
  u32 const md = eight == 1u ? TILE_MODE_LAT8 : eight == 2u ? TILE_MODE_QUAD4 : TILE_MODE_THR;   /* eight: 0 / 1 / 2 */
  u32 const k = md == TILE_MODE_LAT8 ? 8u : md == TILE_MODE_QUAD4 ? 16u : 64u;
  if( A.hctl && blockIdx.x == gridDim.x - 1u ) {
    /* A/B: a scout-like wave polling the host control words until the
       others are done (bounded by the watchdog) */
    if( threadIdx.x == 0u ) {
      u64 const t0 = __builtin_amdgcn_s_memrealtime();
      u64 acc = 0;
      while( __hip_atomic_load( (u64 *)&A.dctl->stat[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ) < (u64)(gridDim.x - 1u) &&
             __builtin_amdgcn_s_memrealtime() - t0 < A.watchdog ) {
        acc += ld_sys64( &A.hctl->head ) + ld_sys64( &A.hctl->beat ) + ld_sys32( &A.hctl->stop );
        __builtin_amdgcn_s_sleep( 2 );
      }
      A.dctl->stat[1] = acc;
    }
    return;
  }
  u8 * scr = A.scratch + (size_t)blockIdx.x * S.total;
  for( u32 it = 0; it < iters; it++ )
    tile_chunk( A, ((u64)blockIdx.x * iters + it) * k, k, md, scr, L, S, bi, evl, pt, 0UL );
  if( A.prof && threadIdx.x == 0u ) {
    _Pragma("unroll") for( int q=0; q<8; q++ ) atomicAdd( (unsigned long long *)&A.dctl->prof[q], (unsigned long long)pt[q] );
  }
  if( A.hctl && threadIdx.x == 0u ) atomicAdd( (unsigned long long *)&A.dctl->stat[0], 1ULL );
}

int
fd_amd_launch_tile_synth( fd_amd_tile_args_t const * a, uint32_t waves, uint32_t iters, int eight, hipStream_t stream ) {
  if( !waves || !iters ) return -1;
  hipLaunchKernelGGL( k_tile_synth, dim3(waves), dim3(64), 0, stream, *a, iters, (u32)eight );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif /* FD_AMD_DIAG */

int
fd_amd_launch_tile_persist( fd_amd_tile_args_t const * a, uint32_t waves, hipStream_t stream ) {
  if( waves < 2u ) return -1;
  (void)hipGetLastError();   /* the check below is the launch's own: every earlier call checked its return code */
  hipLaunchKernelGGL( k_tile_persist, dim3(waves), dim3(64), 0, stream, *a );
  hipError_t const e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;   /* the HIP error, for the caller's message */
}

/* ------------------------------------------------------------------ */
/* launch                                                               */

/* debug: dense u16 [n][256] digits from the event lists */
__global__ void __launch_bounds__(64)
k_digits_dense( u32 n, u8 const * __restrict__ ws, ws_layout_t L, u16 * __restrict__ out ) {
  u32 i = blockIdx.x * 64u + threadIdx.x;
  if( i >= n ) return;
  u16 * o = out + (size_t)i*256u;
  for( int k=0; k<256; k++ ) o[k] = 0;
  u32 ne = ((u32 const *)(ws + L.evn))[i];
  u16 const * ev = (u16 const *)(ws + L.dig) + (size_t)i*128u;
  for( u32 j=0; j<(ne & 0xffu); j++ )        { u16 e = ev[j];      o[e & 0xffu] = (u16)(o[e & 0xffu] | (e >> 8)); }
  for( u32 j=0; j<((ne >> 8) & 0xffu); j++ ) { u16 e = ev[64u + j]; o[e & 0xffu] = (u16)(o[e & 0xffu] | (e & 0xff00u)); }
}

int
fd_amd_launch_digits_dense( uint32_t n, void const * d_ws, uint16_t * d_dig, hipStream_t stream ) {
  if( !n ) return 0;
  hipLaunchKernelGGL( k_digits_dense, dim3((n + 63u)/64u), dim3(64), 0, stream, n, (u8 const *)d_ws, fd_amd_ws_layout( n ), d_dig );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Registered-memory batches: message offsets arrive as the caller wrote
   them (into its whole blob); the chunk's message window [lo, ...) was
   copied to the start of the device blob, so rebase them (empty messages
   point at 0, never outside the window). */
__global__ void __launch_bounds__(256)
k_rebase_off( u32 n, u32 * __restrict__ off, u32 const * __restrict__ sz, u32 lo ) {
  u32 i = blockIdx.x * 256u + threadIdx.x;
  if( i < n ) off[i] = sz[i] ? off[i] - lo : 0u;
}

int
fd_amd_launch_rebase_off( uint32_t n, uint32_t * d_off, uint32_t const * d_sz, uint32_t lo, hipStream_t stream ) {
  if( !n ) return 0;
  hipLaunchKernelGGL( k_rebase_off, dim3((n + 255u)/256u), dim3(256), 0, stream, n, d_off, d_sz, lo );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* device -> mapped host result copy: 16 B per lane where both ends are
   16-aligned (every result buffer is), bytes otherwise. */
__global__ void __launch_bounds__(256)
k_copy_out( u8 * __restrict__ dst, u8 const * __restrict__ src, size_t n ) {
  size_t i = (size_t)blockIdx.x * 256u + threadIdx.x, stride = (size_t)gridDim.x * 256u;
  size_t nv = (((size_t)dst | (size_t)src) & 15u) ? 0 : (n >> 4);
  for( size_t k = i; k < nv; k += stride ) ((uint4 *)dst)[k] = ((uint4 const *)src)[k];
  for( size_t k = (nv << 4) + i; k < n; k += stride ) dst[k] = src[k];
}

int
fd_amd_launch_copy_out( void * d_dst, void const * d_src, size_t n, hipStream_t stream ) {
  if( !n ) return 0;
  size_t nb = ( (n >> 4) + 256u ) / 256u;
  if( nb > 4096u ) nb = 4096u;
  hipLaunchKernelGGL( k_copy_out, dim3((unsigned)nb), dim3(256), 0, stream, (u8 *)d_dst, (u8 const *)d_src, n );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Kernel choice by batch size: up to g_dsm8_max signatures k_dsm8 (8 lanes
   per signature: the shortest op stream, but twice k_dsm4's waves), up to
   g_dsm4_max k_dsm4, larger batches k_dsm.  Measured (profiles/
   r02_k_dsm4_latency_experiments.txt): k_dsm8 is faster while its waves fit
   one per SIMD (n <= 8192 on 1024 SIMDs), slower beyond. */
static volatile u32 g_dsm4_max = 16384u;
static volatile u32 g_dsm8_max = 8192u;
static volatile u32 g_pool_min = 1u << 19;   /* k_dsmp from 2^19 signatures (pooled A/B) */
static volatile u64 g_pool_iter_cap = ~0UL;   /* debug: cap on k_dsmp's step loop (its hang guard) */

extern "C" void
fd_ed25519_amd_debug_set_pool_iter_cap( unsigned long cap ) {
  g_pool_iter_cap = cap ? cap : ~0UL;
}

extern "C" void
fd_ed25519_amd_set_pool_batch_min( unsigned long n ) {
  g_pool_min = n > 0xFFFFFFFFUL ? 0xFFFFFFFFu : (u32)n;
}

/* k_dsmp grid: one single-wave workgroup per resident wave slot (8 per CU:
   LDS-bound at FD_POOL_P slots, VGPR-bound at 2 waves per SIMD), fewer
   when the batch would leave pools nearly empty */
static u32
pool_waves( u32 n ) {
  static int cus = 0;
  if( !cus ) {
    int dev = 0, v = 0;
    if( hipGetDevice( &dev ) != hipSuccess || hipDeviceGetAttribute( &v, hipDeviceAttributeMultiprocessorCount, dev ) != hipSuccess || v <= 0 ) v = 256;
    cus = v;
  }
  u32 wmax = 8u * (u32)cus;
#ifdef FD_AMD_DIAG
  if( char const * e = getenv( "FD_POOL_WAVES" ) ) { u32 v = (u32)atoi( e ); if( v ) wmax = v; }
#endif
  u32 want = (n + 63u) / 64u;
  return want < wmax ? (want ? want : 1u) : wmax;
}

extern "C" void
fd_ed25519_amd_set_small_batch_max( unsigned long n ) {
  g_dsm4_max = n > 0xFFFFFFFFUL ? 0xFFFFFFFFu : (u32)n;
}

extern "C" void
fd_ed25519_amd_set_latency_batch_max( unsigned long n ) {
  g_dsm8_max = n > 0xFFFFFFFFUL ? 0xFFFFFFFFu : (u32)n;
}

/* the streaming tile keeps up to 4 batches in flight: k_dsm8 when four of
   its largest batches (cap) still fit one wave per SIMD (cap <= g_dsm8_max
   / 4), k_dsm4 up to g_dsm4_max, k_dsm beyond.  Deciding per batch size
   instead lets k_dsm8's partial batches oversubscribe the SIMDs beside full
   k_dsm4 ones (profiles/r02_tile_dsm8_ab.txt) */
int
fd_amd_batch_dsm_mode( uint32_t n, uint32_t cap ) {
  return cap <= g_dsm8_max / 4u ? 3 : n <= g_dsm4_max ? 2 : 1;
}

int
fd_amd_uses_latency_path( uint32_t n, int dsm_mode ) {
  return dsm_mode == 2 || dsm_mode == 3 || (dsm_mode == 0 && (n <= g_dsm4_max || n <= g_dsm8_max));
}

int
fd_amd_launch_verify( u32 n, u8 const * d_pub, u8 const * d_sig, u32 const * d_off, u32 const * d_sz,
                      u8 const * d_blob, i8 * d_err, void * d_ws, hipStream_t stream, int want_stats,
                      hipEvent_t const * ev, i8 const * d_skip, int dsm_mode, i8 * d_out ) {
  if( !n ) return 0;
  ws_layout_t L = fd_amd_ws_layout( n );
  u8 * ws = (u8 *)d_ws;
  u32 nb = (n + 63u) / 64u;
  bool small = fd_amd_uses_latency_path( n, dsm_mode );
  bool eight = dsm_mode == 3 || (dsm_mode == 0 && n <= g_dsm8_max);
  if( ev ) (void)hipEventRecord( ev[0], stream );
  if( small ) {   /* latency path: one front launch (hash || decompress), then k_dsm8 or k_dsm4 */
    hipLaunchKernelGGL( k_front, dim3(3u*nb), dim3(64), 0, stream, n, nb, d_pub, d_sig, d_off, d_sz, d_blob, d_err, ws, L, d_skip );
    if( ev ) { (void)hipEventRecord( ev[1], stream ); (void)hipEventRecord( ev[2], stream ); }
    if( eight ) hipLaunchKernelGGL( k_dsm8, dim3((n + 7u)/8u), dim3(64), 0, stream, n, d_err, ws, L, want_stats, d_out );
    else        hipLaunchKernelGGL( k_dsm4, dim3((n + 15u)/16u), dim3(64), 0, stream, n, d_err, ws, L, want_stats, d_out );
  } else {
    bool pooled = dsm_mode == 4 || (dsm_mode == 0 && n >= g_pool_min);
    hipLaunchKernelGGL( k_prep,   dim3(nb),    dim3(64), 0, stream, n, d_pub, d_sig, d_off, d_sz, d_blob, d_err, ws, L, d_skip );
    if( ev ) (void)hipEventRecord( ev[1], stream );
    hipLaunchKernelGGL( k_decomp, dim3(2u*nb), dim3(64), 0, stream, n, d_pub, d_sig, d_err, ws, L );
    if( ev ) (void)hipEventRecord( ev[2], stream );
    if( pooled ) {
      hipLaunchKernelGGL( k_ai,   dim3(nb),    dim3(64), 0, stream, n, d_err, ws, L );
      hipLaunchKernelGGL( k_dsmp, dim3(pool_waves( n )), dim3(64), 0, stream, n, ws, L, (u64)g_pool_iter_cap );
      hipLaunchKernelGGL( k_fin,  dim3(nb),    dim3(64), 0, stream, n, d_err, ws, L, want_stats );
    } else {
      hipLaunchKernelGGL( k_dsm,  dim3(nb),    dim3(64), 0, stream, n, d_err, ws, L, want_stats );
    }
  }
  if( ev ) (void)hipEventRecord( ev[3], stream );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
