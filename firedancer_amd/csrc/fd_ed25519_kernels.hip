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
 *            (avx/fd_ed25519_ge.c:408-527; the Ai table in a per-lane HBM
 *            slab, the Bi table in LDS) and the limb compare
 *            (user.c:417-425).
 *
 * Verdict per signature: err[i] in {0,-1,-2,-3}; 1 marks "still pending"
 * between kernels.
 *
 * Workspace layout (N = n rounded up to 64; every plane is [element][N] so
 * that the 64 lanes of a wave touch 64 consecutive elements):
 *   dig  : int8   [2][256][N]  slide digits of h (plane 0) and s (plane 1)
 *   top  : int32  [N]          highest nonzero digit position (-1 if none)
 *   A    : int32  [30][N]      -A.X, A.Y, -A.T   (A.Z == 1)
 *   R    : int32  [20][N]      R.X, R.Y
 *   Ai   : int32  [8][40][N]   cached odd multiples of -A, lanes [Z,Y-X,Y+X,2dT]
 *   st   : uint32 [3][N]       work statistics (iterations, nnz h, nnz s)
 */

#include "fd_ed25519_dev.h"
#include "fd_ed25519_kernels.h"

typedef int8_t i8;

/* ------------------------------------------------------------------ */
/* workspace                                                            */

static inline size_t ws_al( size_t x ) { return (x + 255UL) & ~(size_t)255UL; }

ws_layout_t
fd_amd_ws_layout( size_t n ) {
  ws_layout_t L;
  size_t N = (n + 63UL) & ~(size_t)63UL; if( !N ) N = 64;
  size_t o = 0;
  L.N   = N;
  L.dig = o; o = ws_al( o + 2UL*256UL*N );
  L.top = o; o = ws_al( o + 4UL*N );
  L.A   = o; o = ws_al( o + 4UL*30UL*N );
  L.R   = o; o = ws_al( o + 4UL*20UL*N );
  L.Ai  = o; o = ws_al( o + 4UL*320UL*N );
  L.st  = o; o = ws_al( o + 4UL*3UL*N );
  L.total = o;
  return L;
}

/* ------------------------------------------------------------------ */
/* k_prep                                                               */

/* byte p of the SHA input stream R || A || M || pad || len */
__device__ __forceinline__ u32
stream_byte( u32 p, u8 const * __restrict__ sig, u8 const * __restrict__ pub,
             u8 const * __restrict__ msg, u32 sz, u32 padded ) {
  if( p < 32u ) return sig[p];
  if( p < 64u ) return pub[p-32u];
  u32 m = p - 64u;
  if( m < sz ) return msg[m];
  if( m == sz ) return 0x80u;
  if( p >= padded - 8u ) {                 /* low 64 bits of the 128-bit bit-length */
    u64 bits = (u64)(64u + sz) << 3;
    u32 k = padded - 1u - p;               /* byte k of the big-endian length, from the end */
    return (u32)(bits >> (8u*k)) & 0xffu;
  }
  return 0u;
}

/* fd_ed25519_ge_slide (avx/fd_ed25519_ge.c:378-400) on an LDS column:
   r[i] lives at lds[i*64 + lane]. */
__device__ __forceinline__ void
slide_lds( i8 * lds, int lane, u32 const a[8] ) {
  for( int i=0; i<256; i++ ) lds[i*64 + lane] = (i8)((a[i>>5] >> (i&31)) & 1u);
  for( int i=0; i<256; i++ ) {
    int ri = lds[i*64 + lane];
    if( !ri ) continue;
    for( int b=1; b<=6 && i+b<256; b++ ) {
      int rb = lds[(i+b)*64 + lane];
      if( !rb ) continue;
      if( ri + (rb << b) <= 15 ) { ri += rb << b; lds[(i+b)*64 + lane] = 0; }
      else if( ri - (rb << b) >= -15 ) {
        ri -= rb << b;
        for( int k=i+b; k<256; k++ ) {
          if( !lds[k*64 + lane] ) { lds[k*64 + lane] = 1; break; }
          lds[k*64 + lane] = 0;
        }
      } else break;
    }
    lds[i*64 + lane] = (i8)ri;
  }
}

__global__ void __launch_bounds__(64)
k_prep( u32 n, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
        u32 const * __restrict__ msg_off, u32 const * __restrict__ msg_sz,
        u8 const * __restrict__ blob, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L ) {
  __shared__ i8 lds[256*64];
  int lane = (int)threadIdx.x;
  u32 i = blockIdx.x * 64u + (u32)lane;
  bool live = i < n;

  u8 const * S  = sig + 64UL*(size_t)(live ? i : 0u);
  u8 const * P  = pub + 32UL*(size_t)(live ? i : 0u);
  u8 const * s  = S + 32;
  int code = 1;   /* pending */

  /* s-range check with the reference's early "return 0" window (user.c:373-379) */
  if( live ) {
    u8 s31 = s[31];
    if( s31 > 0x10 ) code = -1;
    else if( s31 == 0x10 ) {
      u32 any = 0; for( int k=16; k<31; k++ ) any |= s[k];
      if( any ) code = 0;
      else {
        const u8 l_low[16] = { 0xED,0xD3,0xF5,0x5C,0x1A,0x63,0x12,0x58,0xD6,0x9C,0xF7,0xA2,0xDE,0xF9,0xDE,0x14 };
        int k;
        for( k=15; k>=0; k-- ) {
          if( s[k] < l_low[k] ) break;
          if( s[k] > l_low[k] ) { code = -1; break; }
        }
        if( k<0 ) code = -1;
      }
    }
  } else code = 0;

  u32 h[16]; u32 sw[8];
  _Pragma("unroll") for( int k=0; k<8; k++ ) sw[k] = 0;
  if( code == 1 ) {
    u32 sz = msg_sz[i];
    u8 const * M = blob + msg_off[i];
    u32 padded = ((64u + sz + 17u + 127u) / 128u) * 128u;
    u64 st[8] = FD_AMD_SHA512_H0;
    for( u32 blk=0; blk<padded; blk+=128u ) {
      u64 w[16];
      _Pragma("unroll") for( int k=0; k<16; k++ ) {
        u64 v = 0;
        _Pragma("unroll") for( int j=0; j<8; j++ ) v = (v << 8) | (u64)stream_byte( blk + 8u*(u32)k + (u32)j, S, P, M, sz, padded );
        w[k] = v;
      }
      sha512_compress( st, w );
    }
    /* digest bytes little-endian into 16 words: byte 8a+b of the digest is
       byte (7-b) of st[a] */
    u32 hd[16];
    _Pragma("unroll") for( int a=0; a<8; a++ ) {
      u64 x = st[a];
      u32 bswhi = __builtin_bswap32( (u32)(x >> 32) );
      u32 bswlo = __builtin_bswap32( (u32)x );
      hd[2*a] = bswhi; hd[2*a+1] = bswlo;
    }
    sc_reduce( h, hd );   /* h[0..7] */
    _Pragma("unroll") for( int k=0; k<8; k++ )
      sw[k] = (u32)s[4*k] | ((u32)s[4*k+1] << 8) | ((u32)s[4*k+2] << 16) | ((u32)s[4*k+3] << 24);
  } else {
    _Pragma("unroll") for( int k=0; k<16; k++ ) h[k] = 0;
  }

  size_t N = L.N;
  i8 * dig = (i8 *)(ws + L.dig);
  int top = -1;
  /* h digits (plane 0) then s digits (plane 1); non-pending lanes write zeros */
  for( int plane=0; plane<2; plane++ ) {
    slide_lds( lds, lane, plane ? sw : h );
    if( live ) {
      for( int p=0; p<256; p++ ) {
        i8 d = lds[p*64 + lane];
        dig[((size_t)plane*256u + (size_t)p)*N + i] = d;
        if( d ) top = max( top, p );
      }
    }
  }
  if( live ) {
    ((int *)(ws + L.top))[i] = top;
    err[i] = (i8)code;
  }
}

/* ------------------------------------------------------------------ */
/* k_decomp: lane 2i -> A = pub[i], lane 2i+1 -> R = sig[i][0:32]       */

__global__ void __launch_bounds__(64)
k_decomp( u32 n, u8 const * __restrict__ pub, u8 const * __restrict__ sig,
          i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L ) {
  u32 t = blockIdx.x * 64u + threadIdx.x;
  u32 i = t >> 1; u32 which = t & 1u;
  if( i >= n ) return;
  if( err[i] != 1 ) return;
  u8 const * src = which ? (sig + 64UL*i) : (pub + 32UL*i);
  u32 w[8];
  _Pragma("unroll") for( int k=0; k<8; k++ )
    w[k] = (u32)src[4*k] | ((u32)src[4*k+1] << 8) | ((u32)src[4*k+2] << 16) | ((u32)src[4*k+3] << 24);

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
    if( fe_isnonzero( chk ) ) { err[i] = (i8)-2; return; }
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
  u.Z = fe_mul( t.Z, t.T );
  u.Y = fe_mul( t.Y, t.Z );
  u.X = fe_mul( t.X, t.T );
  u.T = fe_mul( t.X, t.Y );
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

__device__ __forceinline__ int wave_max( int v ) {
  _Pragma("unroll") for( int o=32; o>0; o>>=1 ) v = max( v, __shfl_xor( v, o, 64 ) );
  return v;
}

__constant__ static i32 const BI_TABLE[8][3][10] = FD_AMD_BI_PRECOMP;   /* rows y+x, y-x, 2dxy */

__global__ void __launch_bounds__(64)
k_dsm( u32 n, i8 * __restrict__ err, u8 * __restrict__ ws, ws_layout_t L, int want_stats ) {
  __shared__ i32 bi[8][3][10];
  for( int k=threadIdx.x; k<8*3*10; k+=64 ) (&bi[0][0][0])[k] = (&BI_TABLE[0][0][0])[k];
  __syncthreads();

  u32 i = blockIdx.x * 64u + threadIdx.x;
  bool act = (i < n) && (err[i] == 1);
  size_t N = L.N;
  u32 ii = (i < n) ? i : 0u;

  i8 const * dig = (i8 const *)(ws + L.dig);
  i32 * Aiw = (i32 *)(ws + L.Ai);
  int top = act ? ((int const *)(ws + L.top))[ii] : -1;

  /* -A (p3, Z = 1) */
  p3 A;
  {
    i32 const * Aw = (i32 const *)(ws + L.A);
    _Pragma("unroll") for( int k=0; k<10; k++ ) {
      A.X.v[k] = act ? Aw[(size_t)(k   )*N + ii] : 0;
      A.Y.v[k] = act ? Aw[(size_t)(10+k)*N + ii] : (k==0);
      A.T.v[k] = act ? Aw[(size_t)(20+k)*N + ii] : 0;
      A.Z.v[k] = (k==0);
    }
  }

  /* Ai = {1,3,...,15}(-A) in cached form (:423-481) -> HBM slab */
  {
    fe cZ, cYmX, cYpX, cT2d;
    ge_to_cached( cZ, cYmX, cYpX, cT2d, A );
#   define AI_STORE( e ) do {                                                       \
      _Pragma("unroll") for( int k=0; k<10; k++ ) {                                 \
        Aiw[((size_t)(e)*40 + 0 + k)*N + ii] = cZ.v[k];                             \
        Aiw[((size_t)(e)*40 + 10 + k)*N + ii] = cYmX.v[k];                          \
        Aiw[((size_t)(e)*40 + 20 + k)*N + ii] = cYpX.v[k];                          \
        Aiw[((size_t)(e)*40 + 30 + k)*N + ii] = cT2d.v[k];                          \
      } } while(0)
    if( act ) AI_STORE( 0 );
    p1p1 t = ge_dbl( A.X, A.Y, A.Z );
    p3 A2 = ge_p1p1_to_p3( t );
    for( int e=0; e<7; e++ ) {
      p1p1 s = ge_add<false>( A2, cZ, cYmX, cYpX, cT2d, false );
      p3 u = ge_p1p1_to_p3( s );
      ge_to_cached( cZ, cYmX, cYpX, cT2d, u );
      if( act ) AI_STORE( e+1 );
    }
#   undef AI_STORE
  }

  fe X = fe_zero(), Y = fe_one(), Z = fe_one();
  int itop = wave_max( top );
  u32 nit = 0, nha = 0, nhb = 0;
  for( int p=itop; p>=0; p-- ) {
    p1p1 t = ge_dbl( X, Y, Z );
    int da = act ? (int)dig[(size_t)p*N + ii] : 0;
    int db = act ? (int)dig[((size_t)256 + (size_t)p)*N + ii] : 0;
    if( p <= top ) nit++;
    if( da ) {
      nha++;
      p3 u = ge_p1p1_to_p3( t );
      int e = (da < 0 ? -da : da) >> 1;
      fe qZ, qYmX, qYpX, qT2d;
      _Pragma("unroll") for( int k=0; k<10; k++ ) {
        qZ.v[k]   = Aiw[((size_t)e*40 + 0 + k)*N + ii];
        qYmX.v[k] = Aiw[((size_t)e*40 + 10 + k)*N + ii];
        qYpX.v[k] = Aiw[((size_t)e*40 + 20 + k)*N + ii];
        qT2d.v[k] = Aiw[((size_t)e*40 + 30 + k)*N + ii];
      }
      t = ge_add<false>( u, qZ, qYmX, qYpX, qT2d, da < 0 );
    }
    if( db ) {
      nhb++;
      p3 u = ge_p1p1_to_p3( t );
      int e = (db < 0 ? -db : db) >> 1;
      fe qYmX, qYpX, qT2d;
      _Pragma("unroll") for( int k=0; k<10; k++ ) {
        qYpX.v[k] = bi[e][0][k];
        qYmX.v[k] = bi[e][1][k];
        qT2d.v[k] = bi[e][2][k];
      }
      t = ge_add<true>( u, qYmX /*unused*/, qYmX, qYpX, qT2d, db < 0 );
    }
    X = fe_mul( t.X, t.T );
    Y = fe_mul( t.Y, t.Z );
    Z = fe_mul( t.Z, t.T );
  }

  if( want_stats && i < n ) {
    u32 * st = (u32 *)(ws + L.st);
    st[i] = act ? nit : 0u; st[N + i] = nha; st[2*N + i] = nhb;
  }
  if( !act ) return;
  fe RX, RY;
  {
    i32 const * Rw = (i32 const *)(ws + L.R);
    _Pragma("unroll") for( int k=0; k<10; k++ ) { RX.v[k] = Rw[(size_t)k*N + ii]; RY.v[k] = Rw[(size_t)(10+k)*N + ii]; }
  }
  fe xZ = fe_mul( Z, RX );
  fe yZ = fe_mul( Z, RY );
  bool eq = true;
  _Pragma("unroll") for( int k=0; k<8; k++ ) eq = eq && (xZ.v[k] == X.v[k]) && (yZ.v[k] == Y.v[k]);   /* limbs 0..7 (user.c:424-425) */
  err[i] = (i8)(eq ? 0 : -3);
}

/* ------------------------------------------------------------------ */
/* launch                                                               */

int
fd_amd_launch_verify( u32 n, u8 const * d_pub, u8 const * d_sig, u32 const * d_off, u32 const * d_sz,
                      u8 const * d_blob, i8 * d_err, void * d_ws, hipStream_t stream, int want_stats,
                      hipEvent_t const * ev ) {
  if( !n ) return 0;
  ws_layout_t L = fd_amd_ws_layout( n );
  u8 * ws = (u8 *)d_ws;
  u32 nb = (n + 63u) / 64u;
  if( ev ) (void)hipEventRecord( ev[0], stream );
  hipLaunchKernelGGL( k_prep,   dim3(nb),      dim3(64), 0, stream, n, d_pub, d_sig, d_off, d_sz, d_blob, d_err, ws, L );
  if( ev ) (void)hipEventRecord( ev[1], stream );
  hipLaunchKernelGGL( k_decomp, dim3(2u*nb),   dim3(64), 0, stream, n, d_pub, d_sig, d_err, ws, L );
  if( ev ) (void)hipEventRecord( ev[2], stream );
  hipLaunchKernelGGL( k_dsm,    dim3(nb),      dim3(64), 0, stream, n, d_err, ws, L, want_stats );
  if( ev ) (void)hipEventRecord( ev[3], stream );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
