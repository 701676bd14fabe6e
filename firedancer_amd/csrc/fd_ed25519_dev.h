/* firedancer_amd/csrc/fd_ed25519_dev.h
 *
 * CDNA4 (gfx950) device arithmetic for the ed25519 verify engine: one
 * signature per lane, every value in VGPRs.
 *
 * Field elements are the reference's representation (10 x int32 signed
 * limbs, radix 2^25.5) and every field op reproduces the reference's AVX
 * build limb for limb (src/ballet/ed25519/avx/
 * fd_ed25519_fe_avx_inl.h:484-674): int32 pre-multiples with wrap-around,
 * exact int64 column sums built from v_mad_i64_i32 chains, then the
 * reference carry chain.  Limbs are never canonicalised except where the
 * reference calls fe_tobytes (isnonzero / isnegative).
 */
#ifndef FD_ED25519_DEV_H
#define FD_ED25519_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fd_ed25519_consts.h"

#define FD_DEV static __device__ __forceinline__

typedef int32_t  i32;
typedef uint32_t u32;
typedef int64_t  i64;
typedef uint64_t u64;
typedef uint8_t  u8;

struct fe { i32 v[10]; };

FD_DEV fe fe_zero() { fe r; _Pragma("unroll") for( int i=0; i<10; i++ ) r.v[i] = 0; return r; }
FD_DEV fe fe_one () { fe r = fe_zero(); r.v[0] = 1; return r; }

FD_DEV i32 wmul( i32 a, i32 k ) { return (i32)((u32)a * (u32)k); }   /* int32 wrap: the low 32 bits the AVX mul sees */
FD_DEV i64 mll ( i32 a, i32 b ) { return (i64)a * (i64)b; }            /* v_mad_i64_i32 */

/* Column sums as explicit v_mad_i64_i32 chains.  fd_pin is an empty asm
   (no instruction) that only makes its value opaque: LLVM can then neither
   reassociate a chain nor move its accumulator input (a column bias, or a
   carry) to a trailing 64-bit add. */
FD_DEV i64 fd_pin( i64 x ) { asm( "" : "+v"(x) ); return x; }
FD_DEV i64 mac( i32 a, i32 b, i64 c ) { return fd_pin( (i64)a * (i64)b + c ); }

/* a + b + c (mod 2^32) as one v_add3_u32: LLVM otherwise reassociates a
   chain of adds around its operands; c may be a wave-uniform SGPR value
   (gfx9 VOP3 takes no literal, so a constant offset goes through an SGPR). */
FD_DEV i32 fd_add3( i32 a, i32 b, i32 c ) {
  i32 r; asm( "v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c) ); return r;
}
FD_DEV i32 fd_add3s( i32 a, i32 b, i32 c ) {
  i32 r; asm( "v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c) ); return r;
}
/* (a ^ b) + c as one v_xad_u32 (with b = 0 / -1 and c = 0 / 1: a or -a) */
FD_DEV i32 fd_xad( i32 a, i32 b, i32 c ) {
  i32 r; asm( "v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c) ); return r;
}

FD_DEV fe fe_add( fe const & f, fe const & g ) { fe h; _Pragma("unroll") for( int i=0; i<10; i++ ) h.v[i] = (i32)((u32)f.v[i] + (u32)g.v[i]); return h; }
FD_DEV fe fe_sub( fe const & f, fe const & g ) { fe h; _Pragma("unroll") for( int i=0; i<10; i++ ) h.v[i] = (i32)((u32)f.v[i] - (u32)g.v[i]); return h; }
FD_DEV fe fe_neg( fe const & f )               { fe h; _Pragma("unroll") for( int i=0; i<10; i++ ) h.v[i] = (i32)(0u - (u32)f.v[i]); return h; }

/* Reference carry chain (avx/fd_ed25519_fe_avx_inl.h:570-584):
   0,4 | 1,5 | 2,6 | 3,7 | 4,8 | 9(x19) | 0, rounding carries
   c = (h + 2^(w-1)) >> w with an arithmetic shift. */
FD_DEV fe fe_carry( i64 h0, i64 h1, i64 h2, i64 h3, i64 h4, i64 h5, i64 h6, i64 h7, i64 h8, i64 h9 ) {
  i64 c;
  c = (h0 + (1L<<25)) >> 26; h1 += c; h0 -= c << 26;
  c = (h4 + (1L<<25)) >> 26; h5 += c; h4 -= c << 26;
  c = (h1 + (1L<<24)) >> 25; h2 += c; h1 -= c << 25;
  c = (h5 + (1L<<24)) >> 25; h6 += c; h5 -= c << 25;
  c = (h2 + (1L<<25)) >> 26; h3 += c; h2 -= c << 26;
  c = (h6 + (1L<<25)) >> 26; h7 += c; h6 -= c << 26;
  c = (h3 + (1L<<24)) >> 25; h4 += c; h3 -= c << 25;
  c = (h7 + (1L<<24)) >> 25; h8 += c; h7 -= c << 25;
  c = (h4 + (1L<<25)) >> 26; h5 += c; h4 -= c << 26;
  c = (h8 + (1L<<25)) >> 26; h9 += c; h8 -= c << 26;
  c = (h9 + (1L<<24)) >> 25; h0 += c * 19; h9 -= c << 25;
  c = (h0 + (1L<<25)) >> 26; h1 += c; h0 -= c << 26;
  fe r;
  r.v[0] = (i32)h0; r.v[1] = (i32)h1; r.v[2] = (i32)h2; r.v[3] = (i32)h3; r.v[4] = (i32)h4;
  r.v[5] = (i32)h5; r.v[6] = (i32)h6; r.v[7] = (i32)h7; r.v[8] = (i32)h8; r.v[9] = (i32)h9;
  return r;
}

/* The same carry chain on PRE-BIASED column sums h_k' = h_k + 2^(w_k-1)
   (2^25 for even k, 2^24 for odd k), the bias being folded into the first
   v_mad_i64_i32 of each column for free.  Each rounding carry is then a
   plain arithmetic shift c = h' >> w, the bias cancels in the second carry
   of limbs 4 and 0, and every output limb is (h' mod 2^w) - 2^(w-1) in
   32-bit arithmetic.  Identical limbs to fe_carry on the unbiased sums. */
FD_DEV fe fe_carry_b( i64 h0, i64 h1, i64 h2, i64 h3, i64 h4, i64 h5, i64 h6, i64 h7, i64 h8, i64 h9 ) {
  i64 const M26 = (1L<<26) - 1, M25 = (1L<<25) - 1;
  h1 += h0 >> 26;
  h5 += h4 >> 26;
  h2 += h1 >> 25;
  h6 += h5 >> 25;
  h3 += h2 >> 26;
  h7 += h6 >> 26;
  i64 t4 = (h4 & M26) + (h3 >> 25);
  h8 += h7 >> 25;
  i32 c4b = (i32)(t4 >> 26);
  h9 += h8 >> 26;
  i64 t0 = (h0 & M26) + (h9 >> 25) * 19;
  i32 c0b = (i32)(t0 >> 26);
  fe r;
  r.v[0] = (i32)((u32)t0 & (u32)M26) - (1<<25);
  r.v[1] = (i32)((u32)h1 & (u32)M25) - (1<<24) + c0b;
  r.v[2] = (i32)((u32)h2 & (u32)M26) - (1<<25);
  r.v[3] = (i32)((u32)h3 & (u32)M25) - (1<<24);
  r.v[4] = (i32)((u32)t4 & (u32)M26) - (1<<25);
  r.v[5] = (i32)((u32)h5 & (u32)M25) - (1<<24) + c4b;
  r.v[6] = (i32)((u32)h6 & (u32)M26) - (1<<25);
  r.v[7] = (i32)((u32)h7 & (u32)M25) - (1<<24);
  r.v[8] = (i32)((u32)h8 & (u32)M26) - (1<<25);
  r.v[9] = (i32)((u32)h9 & (u32)M25) - (1<<24);
  return r;
}

/* Carry-folded chain (used where MAC chains are pinned, fd_pin): the
   rounding carry out of columns 0,2,4,6,8 is the accumulator INPUT of the
   chains of columns 1,3,5,7,9, so five 64-bit adds vanish.  Even columns
   start from K = 2^25 + 2^50: their own rounding bias plus the next odd
   column's 2^24 pre-shifted by 26 ((h + 2^50) >> 26 == (h >> 26) + 2^24,
   low 26 bits untouched); odd columns carry no bias of their own.  This
   finishes the chain once columns 1..9 hold their carries-in.  Same limbs
   as fe_carry / fe_carry_b.  BIAS: return every limb plus its rounding
   offset (2^25 even, 2^24 odd limbs), for a consumer that folds the offset
   into an operation it does anyway (the k_dsm mix), saving the subtract. */
template<bool BIAS = false>
FD_DEV fe fe_carry_fold_out( i64 h0, i64 h1, i64 h2, i64 h3, i64 h4, i64 h5, i64 h6, i64 h7, i64 h8, i64 h9 ) {
  i64 const M26 = (1L<<26) - 1;
  i64 t4 = (h4 & M26) + (h3 >> 25);
  i32 c4b = (i32)(t4 >> 26);
  i64 t0 = (h0 & M26) + (h9 >> 25) * 19;
  i32 c0b = (i32)(t0 >> 26);
  u32 const m26 = (1u<<26) - 1u, m25 = (1u<<25) - 1u;
  i32 const o26 = BIAS ? 0 : (1<<25), o25 = BIAS ? 0 : (1<<24);
  fe r;
  r.v[0] = (i32)((u32)t0 & m26) - o26;
  r.v[1] = (i32)((u32)h1 & m25) - o25 + c0b;
  r.v[2] = (i32)((u32)h2 & m26) - o26;
  r.v[3] = (i32)((u32)h3 & m25) - o25;
  r.v[4] = (i32)((u32)t4 & m26) - o26;
  r.v[5] = (i32)((u32)h5 & m25) - o25 + c4b;
  r.v[6] = (i32)((u32)h6 & m26) - o26;
  r.v[7] = (i32)((u32)h7 & m25) - o25;
  r.v[8] = (i32)((u32)h8 & m26) - o26;
  r.v[9] = (i32)((u32)h9 & m25) - o25;
  return r;
}

/* The column biases as OPAQUE wave-uniform values: LLVM canonicalises an
   integer constant to the end of an add chain, which would cost one extra
   64-bit add per column; an opaque SGPR value stays first and becomes the
   src2 of the column's first v_mad_i64_i32. */
FD_DEV i64 fd_opaque( i64 x ) { asm( "" : "+s"(x) ); return x; }
#define FD_B26 b26
#define FD_B25 b25
#define FD_BIAS_DECL i64 const b26 = fd_opaque( 1L<<25 ), b25 = fd_opaque( 1L<<24 )

/* f * 1 through the reference multiplier: the column sums are the limbs
   themselves, so it is exactly the carry chain ("x1" renormalisation of
   the AVX flow, avx/fd_ed25519_ge.c:440-446 and the madd lane 0). */
FD_DEV fe fe_mul_one( fe const & f ) {
  return fe_carry( f.v[0], f.v[1], f.v[2], f.v[3], f.v[4], f.v[5], f.v[6], f.v[7], f.v[8], f.v[9] );
}

/* FE_AVX_INL_MUL, one lane (avx/fd_ed25519_fe_avx_inl.h:484-585) */
FD_DEV fe fe_mul( fe const & F, fe const & G ) {
  i32 const * f = F.v; i32 const * g = G.v;
  FD_BIAS_DECL;
  i32 g1_19 = wmul( g[1], 19 ), g2_19 = wmul( g[2], 19 ), g3_19 = wmul( g[3], 19 );
  i32 g4_19 = wmul( g[4], 19 ), g5_19 = wmul( g[5], 19 ), g6_19 = wmul( g[6], 19 );
  i32 g7_19 = wmul( g[7], 19 ), g8_19 = wmul( g[8], 19 ), g9_19 = wmul( g[9], 19 );
  i32 f1_2 = wmul( f[1], 2 ), f3_2 = wmul( f[3], 2 ), f5_2 = wmul( f[5], 2 );
  i32 f7_2 = wmul( f[7], 2 ), f9_2 = wmul( f[9], 2 );
  i64 h0 = FD_B26 + mll(f[0],g[0]) + mll(f1_2,g9_19) + mll(f[2],g8_19) + mll(f3_2,g7_19) + mll(f[4],g6_19) + mll(f5_2,g5_19) + mll(f[6],g4_19) + mll(f7_2,g3_19) + mll(f[8],g2_19) + mll(f9_2,g1_19);
  i64 h1 = FD_B25 + mll(f[0],g[1]) + mll(f[1],g[0]) + mll(f[2],g9_19) + mll(f[3],g8_19) + mll(f[4],g7_19) + mll(f[5],g6_19) + mll(f[6],g5_19) + mll(f[7],g4_19) + mll(f[8],g3_19) + mll(f[9],g2_19);
  i64 h2 = FD_B26 + mll(f[0],g[2]) + mll(f1_2,g[1]) + mll(f[2],g[0]) + mll(f3_2,g9_19) + mll(f[4],g8_19) + mll(f5_2,g7_19) + mll(f[6],g6_19) + mll(f7_2,g5_19) + mll(f[8],g4_19) + mll(f9_2,g3_19);
  i64 h3 = FD_B25 + mll(f[0],g[3]) + mll(f[1],g[2]) + mll(f[2],g[1]) + mll(f[3],g[0]) + mll(f[4],g9_19) + mll(f[5],g8_19) + mll(f[6],g7_19) + mll(f[7],g6_19) + mll(f[8],g5_19) + mll(f[9],g4_19);
  i64 h4 = FD_B26 + mll(f[0],g[4]) + mll(f1_2,g[3]) + mll(f[2],g[2]) + mll(f3_2,g[1]) + mll(f[4],g[0]) + mll(f5_2,g9_19) + mll(f[6],g8_19) + mll(f7_2,g7_19) + mll(f[8],g6_19) + mll(f9_2,g5_19);
  i64 h5 = FD_B25 + mll(f[0],g[5]) + mll(f[1],g[4]) + mll(f[2],g[3]) + mll(f[3],g[2]) + mll(f[4],g[1]) + mll(f[5],g[0]) + mll(f[6],g9_19) + mll(f[7],g8_19) + mll(f[8],g7_19) + mll(f[9],g6_19);
  i64 h6 = FD_B26 + mll(f[0],g[6]) + mll(f1_2,g[5]) + mll(f[2],g[4]) + mll(f3_2,g[3]) + mll(f[4],g[2]) + mll(f5_2,g[1]) + mll(f[6],g[0]) + mll(f7_2,g9_19) + mll(f[8],g8_19) + mll(f9_2,g7_19);
  i64 h7 = FD_B25 + mll(f[0],g[7]) + mll(f[1],g[6]) + mll(f[2],g[5]) + mll(f[3],g[4]) + mll(f[4],g[3]) + mll(f[5],g[2]) + mll(f[6],g[1]) + mll(f[7],g[0]) + mll(f[8],g9_19) + mll(f[9],g8_19);
  i64 h8 = FD_B26 + mll(f[0],g[8]) + mll(f1_2,g[7]) + mll(f[2],g[6]) + mll(f3_2,g[5]) + mll(f[4],g[4]) + mll(f5_2,g[3]) + mll(f[6],g[2]) + mll(f7_2,g[1]) + mll(f[8],g[0]) + mll(f9_2,g9_19);
  i64 h9 = FD_B25 + mll(f[0],g[9]) + mll(f[1],g[8]) + mll(f[2],g[7]) + mll(f[3],g[6]) + mll(f[4],g[5]) + mll(f[5],g[4]) + mll(f[6],g[3]) + mll(f[7],g[2]) + mll(f[8],g[1]) + mll(f[9],g[0]);
  return fe_carry_b( h0, h1, h2, h3, h4, h5, h6, h7, h8, h9 );
}

/* Two fe_muls with the carry fold of fe_sq_fold (even columns start from
   K = 2^25 + 2^50, odd columns start from the previous column's carry), every
   independent pinned MAC chain interleaved term by term: the ten even columns
   of both products, then columns 1,5 (four chains), 3,7 (four), 9 (two), so
   each chain's dependent v_mad_i64_i32 is separated by the others' and no
   hazard wait remains.  Term (i, j = K-i mod 10) of column K: f_i doubled
   when i and j are both odd, g_j x19 when i+j >= 10 (the pre-multiples of
   fe_mul); the sum is exact, so the term order does not change it.  Same
   limbs as fe_mul. */
template<int K>
FD_DEV void fe_term( int i, i32 const * f, i32 const * f_2, i32 const * g, i32 const * g_19, i64 & a );
template<bool BIAS1 = false, bool BIAS2 = false>   /* per product: limbs + rounding offset (fe_carry_fold_out) */
FD_DEV void fe_mul_fold2w( fe & R1, fe const & F1, fe const & G1, fe & R2, fe const & F2, fe const & G2 ) {
  i64 const kb = fd_opaque( (1L<<25) + (1L<<50) );
  i32 f1_2[10], g1_19[10], f2_2[10], g2_19[10];
  _Pragma("unroll") for( int k=0; k<10; k++ ) {
    f1_2[k] = wmul( F1.v[k], 2 ); g1_19[k] = wmul( G1.v[k], 19 );
    f2_2[k] = wmul( F2.v[k], 2 ); g2_19[k] = wmul( G2.v[k], 19 );
  }
  i32 const * f1 = F1.v; i32 const * g1 = G1.v; i32 const * f2 = F2.v; i32 const * g2 = G2.v;
# define FD_TA( K_, A_ ) fe_term<K_>( i, f1, f1_2, g1, g1_19, A_ )
# define FD_TB( K_, B_ ) fe_term<K_>( i, f2, f2_2, g2, g2_19, B_ )
  i64 a0 = kb, b0 = kb, a4 = kb, b4 = kb, a2 = kb, b2 = kb, a6 = kb, b6 = kb, a8 = kb, b8 = kb;
  _Pragma("unroll") for( int i=0; i<10; i++ ) {
    FD_TA( 0, a0 ); FD_TB( 0, b0 ); FD_TA( 4, a4 ); FD_TB( 4, b4 ); FD_TA( 2, a2 ); FD_TB( 2, b2 );
    FD_TA( 6, a6 ); FD_TB( 6, b6 ); FD_TA( 8, a8 ); FD_TB( 8, b8 );
  }
  i64 a1 = a0 >> 26, b1 = b0 >> 26, a5 = a4 >> 26, b5 = b4 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { FD_TA( 1, a1 ); FD_TB( 1, b1 ); FD_TA( 5, a5 ); FD_TB( 5, b5 ); }
  a2 += a1 >> 25; b2 += b1 >> 25; a6 += a5 >> 25; b6 += b5 >> 25;
  i64 a3 = a2 >> 26, b3 = b2 >> 26, a7 = a6 >> 26, b7 = b6 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { FD_TA( 3, a3 ); FD_TB( 3, b3 ); FD_TA( 7, a7 ); FD_TB( 7, b7 ); }
  a8 += a7 >> 25; b8 += b7 >> 25;
  i64 a9 = a8 >> 26, b9 = b8 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { FD_TA( 9, a9 ); FD_TB( 9, b9 ); }
# undef FD_TA
# undef FD_TB
  R1 = fe_carry_fold_out<BIAS1>( a0, a1, a2, a3, a4, a5, a6, a7, a8, a9 );
  R2 = fe_carry_fold_out<BIAS2>( b0, b1, b2, b3, b4, b5, b6, b7, b8, b9 );
}

/* Term i of column K of one fe_mul (the rule above fe_mul_fold2w). */
template<int K>
FD_DEV void fe_term( int i, i32 const * f, i32 const * f_2, i32 const * g, i32 const * g_19, i64 & a ) {
  int const j = (K - i + 10) % 10;
  bool const dbl = (i & 1) && (j & 1), x19 = (i + j) >= 10;
  a = mac( dbl ? f_2[i] : f[i], x19 ? g_19[j] : g[j], a );
}

/* One fe_mul with the carry fold for a lane that has no second product to
   interleave with: the independent columns of the product are interleaved
   instead (0,4,2,6,8 | 1,5 | 3,7,9).  Columns 1,3,5,7 start from the
   previous column's carry; column 9 runs beside 3 and 7 from its own bias
   and takes column 8's carry with an add.  Same limbs as fe_mul. */
FD_DEV fe fe_mul_fold1( fe const & F, fe const & G ) {
  i64 const kb = fd_opaque( (1L<<25) + (1L<<50) );
  i64 const k8 = fd_opaque( 1L<<25 ), k9 = fd_opaque( 1L<<24 );   /* column 8 carries no bias for 9 */
  i32 f_2[10], g_19[10];
  _Pragma("unroll") for( int k=0; k<10; k++ ) { f_2[k] = wmul( F.v[k], 2 ); g_19[k] = wmul( G.v[k], 19 ); }
  i32 const * f = F.v; i32 const * g = G.v;
  i64 h0 = kb, h4 = kb, h2 = kb, h6 = kb, h8 = k8;
  _Pragma("unroll") for( int i=0; i<10; i++ ) {
    fe_term<0>( i, f, f_2, g, g_19, h0 ); fe_term<4>( i, f, f_2, g, g_19, h4 );
    fe_term<2>( i, f, f_2, g, g_19, h2 ); fe_term<6>( i, f, f_2, g, g_19, h6 );
    fe_term<8>( i, f, f_2, g, g_19, h8 );
  }
  i64 h1 = h0 >> 26, h5 = h4 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { fe_term<1>( i, f, f_2, g, g_19, h1 ); fe_term<5>( i, f, f_2, g, g_19, h5 ); }
  h2 += h1 >> 25; h6 += h5 >> 25;
  i64 h3 = h2 >> 26, h7 = h6 >> 26, h9 = k9;
  _Pragma("unroll") for( int i=0; i<10; i++ ) {
    fe_term<3>( i, f, f_2, g, g_19, h3 ); fe_term<7>( i, f, f_2, g, g_19, h7 );
    fe_term<9>( i, f, f_2, g, g_19, h9 );
  }
  h8 += h7 >> 25;
  h9 += h8 >> 26;
  return fe_carry_fold_out( h0, h1, h2, h3, h4, h5, h6, h7, h8, h9 );
}

/* FE_AVX_INL_SQN, one lane, n in {1,2} (avx/fd_ed25519_fe_avx_inl.h:592-674):
   55 products; the column sums are doubled before the carry when n==2. */
template<int N>
FD_DEV fe fe_sqn( fe const & F ) {
  i32 const * f = F.v;
  FD_BIAS_DECL;
  i32 f0_2 = wmul( f[0], 2 ), f1_2 = wmul( f[1], 2 ), f2_2 = wmul( f[2], 2 ), f3_2 = wmul( f[3], 2 );
  i32 f4_2 = wmul( f[4], 2 ), f5_2 = wmul( f[5], 2 ), f6_2 = wmul( f[6], 2 ), f7_2 = wmul( f[7], 2 );
  i32 f5_38 = wmul( f[5], 38 ), f6_19 = wmul( f[6], 19 ), f7_38 = wmul( f[7], 38 );
  i32 f8_19 = wmul( f[8], 19 ), f9_38 = wmul( f[9], 38 );
  i64 h0 = mac( f[5], f5_38, mac( f4_2, f6_19, mac( f3_2, f7_38, mac( f2_2, f8_19, mac( f1_2, f9_38, mac( f[0], f[0], (N==1 ? FD_B26 : 0L) ) ) ) ) ) );
  i64 h1 = mac( f5_2, f6_19, mac( f[4], f7_38, mac( f3_2, f8_19, mac( f[2], f9_38, mac( f0_2, f[1], (N==1 ? FD_B25 : 0L) ) ) ) ) );
  i64 h2 = mac( f[6], f6_19, mac( f5_2, f7_38, mac( f4_2, f8_19, mac( f3_2, f9_38, mac( f1_2, f[1], mac( f0_2, f[2], (N==1 ? FD_B26 : 0L) ) ) ) ) ) );
  i64 h3 = mac( f[6], f7_38, mac( f5_2, f8_19, mac( f[4], f9_38, mac( f1_2, f[2], mac( f0_2, f[3], (N==1 ? FD_B25 : 0L) ) ) ) ) );
  i64 h4 = mac( f[7], f7_38, mac( f6_2, f8_19, mac( f5_2, f9_38, mac( f[2], f[2], mac( f1_2, f3_2, mac( f0_2, f[4], (N==1 ? FD_B26 : 0L) ) ) ) ) ) );
  i64 h5 = mac( f7_2, f8_19, mac( f[6], f9_38, mac( f2_2, f[3], mac( f1_2, f[4], mac( f0_2, f[5], (N==1 ? FD_B25 : 0L) ) ) ) ) );
  i64 h6 = mac( f[8], f8_19, mac( f7_2, f9_38, mac( f3_2, f[3], mac( f2_2, f[4], mac( f1_2, f5_2, mac( f0_2, f[6], (N==1 ? FD_B26 : 0L) ) ) ) ) ) );
  i64 h7 = mac( f[8], f9_38, mac( f3_2, f[4], mac( f2_2, f[5], mac( f1_2, f[6], mac( f0_2, f[7], (N==1 ? FD_B25 : 0L) ) ) ) ) );
  i64 h8 = mac( f[9], f9_38, mac( f[4], f[4], mac( f3_2, f5_2, mac( f2_2, f[6], mac( f1_2, f7_2, mac( f0_2, f[8], (N==1 ? FD_B26 : 0L) ) ) ) ) ) );
  i64 h9 = mac( f4_2, f[5], mac( f3_2, f[6], mac( f2_2, f[7], mac( f1_2, f[8], mac( f0_2, f[9], (N==1 ? FD_B25 : 0L) ) ) ) ) );
  if( N==2 ) {
    h0 += h0; h1 += h1; h2 += h2; h3 += h3; h4 += h4; h5 += h5; h6 += h6; h7 += h7; h8 += h8; h9 += h9;
    return fe_carry( h0, h1, h2, h3, h4, h5, h6, h7, h8, h9 );
  }
  return fe_carry_b( h0, h1, h2, h3, h4, h5, h6, h7, h8, h9 );
}

/* fe_sqn<1> with the carry fold (same limbs) */
FD_DEV fe fe_sq_fold( fe const & F ) {
  i32 const * f = F.v;
  i64 const kb = fd_opaque( (1L<<25) + (1L<<50) );
  i32 f0_2 = wmul( f[0], 2 ), f1_2 = wmul( f[1], 2 ), f2_2 = wmul( f[2], 2 ), f3_2 = wmul( f[3], 2 );
  i32 f4_2 = wmul( f[4], 2 ), f5_2 = wmul( f[5], 2 ), f6_2 = wmul( f[6], 2 ), f7_2 = wmul( f[7], 2 );
  i32 f5_38 = wmul( f[5], 38 ), f6_19 = wmul( f[6], 19 ), f7_38 = wmul( f[7], 38 );
  i32 f8_19 = wmul( f[8], 19 ), f9_38 = wmul( f[9], 38 );
  i64 h0 = mac( f[5], f5_38, mac( f4_2, f6_19, mac( f3_2, f7_38, mac( f2_2, f8_19, mac( f1_2, f9_38, mac( f[0], f[0], kb ) ) ) ) ) );
  i64 h4 = mac( f[7], f7_38, mac( f6_2, f8_19, mac( f5_2, f9_38, mac( f[2], f[2], mac( f1_2, f3_2, mac( f0_2, f[4], kb ) ) ) ) ) );
  i64 h2 = mac( f[6], f6_19, mac( f5_2, f7_38, mac( f4_2, f8_19, mac( f3_2, f9_38, mac( f1_2, f[1], mac( f0_2, f[2], kb ) ) ) ) ) );
  i64 h6 = mac( f[8], f8_19, mac( f7_2, f9_38, mac( f3_2, f[3], mac( f2_2, f[4], mac( f1_2, f5_2, mac( f0_2, f[6], kb ) ) ) ) ) );
  i64 h8 = mac( f[9], f9_38, mac( f[4], f[4], mac( f3_2, f5_2, mac( f2_2, f[6], mac( f1_2, f7_2, mac( f0_2, f[8], kb ) ) ) ) ) );
  i64 h1 = mac( f5_2, f6_19, mac( f[4], f7_38, mac( f3_2, f8_19, mac( f[2], f9_38, mac( f0_2, f[1], h0 >> 26 ) ) ) ) );
  i64 h5 = mac( f7_2, f8_19, mac( f[6], f9_38, mac( f2_2, f[3], mac( f1_2, f[4], mac( f0_2, f[5], h4 >> 26 ) ) ) ) );
  h2 += h1 >> 25;
  h6 += h5 >> 25;
  i64 h3 = mac( f[6], f7_38, mac( f5_2, f8_19, mac( f[4], f9_38, mac( f1_2, f[2], mac( f0_2, f[3], h2 >> 26 ) ) ) ) );
  i64 h7 = mac( f[8], f9_38, mac( f3_2, f[4], mac( f2_2, f[5], mac( f1_2, f[6], mac( f0_2, f[7], h6 >> 26 ) ) ) ) );
  h8 += h7 >> 25;
  i64 h9 = mac( f4_2, f[5], mac( f3_2, f[6], mac( f2_2, f[7], mac( f1_2, f[8], mac( f0_2, f[9], h8 >> 26 ) ) ) ) );
  return fe_carry_fold_out( h0, h1, h2, h3, h4, h5, h6, h7, h8, h9 );
}

FD_DEV fe fe_sq( fe const & f ) { return fe_sq_fold( f ); }

/* Term (i, j = K-i mod 10), i <= j, of column K of a square: the pair's
   coefficient is 2 (i != j) x 2 (i, j both odd) x 19 (i + j >= 10) x 2 (D2,
   the reference's sq2), its power of two applied to f_i as a shift, the 19
   taken from f19[j] (j >= 5 whenever i + j >= 10).  For |f| <= 2^26 no
   operand wraps (f << 3 <= 2^29, 19 f <= 2^30.25), so the column sums are
   the exact integers sum_{i+j=K} c_ij f_i f_j -- the sums of fe_mul( f, f )
   (resp. fe_mul( f, f+f )) -- and the carry gives the same limbs. */
template<int K, bool D2>
FD_DEV void sq_term( int i, i32 const * f, i32 const * f19, i64 & a ) {
  int const j = (K - i + 10) % 10;
  if( i > j ) return;
  int const c2 = (i != j) + ((i & 1) && (j & 1)) + (D2 ? 1 : 0);
  bool const x19 = (i + j) >= 10;
  i32 const lhs = c2 ? (i32)((u32)f[i] << c2) : f[i];
  a = mac( lhs, x19 ? f19[j] : f[j], a );
}

/* Two squares (55 products each) with fe_mul_fold2w's column order and
   carry fold.  D2: the column sums of f * (f + f) (the AVX sq2). */
template<bool D2A, bool D2B>
FD_DEV void fe_sq_fold2w( fe & R1, fe const & F1, fe & R2, fe const & F2 ) {
  i64 const kb = fd_opaque( (1L<<25) + (1L<<50) );
  i32 f1_19[10], f2_19[10];
  _Pragma("unroll") for( int k=0; k<10; k++ ) { f1_19[k] = wmul( F1.v[k], 19 ); f2_19[k] = wmul( F2.v[k], 19 ); }
  i32 const * f1 = F1.v; i32 const * f2 = F2.v;
# define FD_SA( K_, A_ ) sq_term<K_, D2A>( i, f1, f1_19, A_ )
# define FD_SB( K_, B_ ) sq_term<K_, D2B>( i, f2, f2_19, B_ )
  i64 a0 = kb, b0 = kb, a4 = kb, b4 = kb, a2 = kb, b2 = kb, a6 = kb, b6 = kb, a8 = kb, b8 = kb;
  _Pragma("unroll") for( int i=0; i<10; i++ ) {
    FD_SA( 0, a0 ); FD_SB( 0, b0 ); FD_SA( 4, a4 ); FD_SB( 4, b4 ); FD_SA( 2, a2 ); FD_SB( 2, b2 );
    FD_SA( 6, a6 ); FD_SB( 6, b6 ); FD_SA( 8, a8 ); FD_SB( 8, b8 );
  }
  i64 a1 = a0 >> 26, b1 = b0 >> 26, a5 = a4 >> 26, b5 = b4 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { FD_SA( 1, a1 ); FD_SB( 1, b1 ); FD_SA( 5, a5 ); FD_SB( 5, b5 ); }
  a2 += a1 >> 25; b2 += b1 >> 25; a6 += a5 >> 25; b6 += b5 >> 25;
  i64 a3 = a2 >> 26, b3 = b2 >> 26, a7 = a6 >> 26, b7 = b6 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { FD_SA( 3, a3 ); FD_SB( 3, b3 ); FD_SA( 7, a7 ); FD_SB( 7, b7 ); }
  a8 += a7 >> 25; b8 += b7 >> 25;
  i64 a9 = a8 >> 26, b9 = b8 >> 26;
  _Pragma("unroll") for( int i=0; i<10; i++ ) { FD_SA( 9, a9 ); FD_SB( 9, b9 ); }
# undef FD_SA
# undef FD_SB
  R1 = fe_carry_fold_out( a0, a1, a2, a3, a4, a5, a6, a7, a8, a9 );
  R2 = fe_carry_fold_out( b0, b1, b2, b3, b4, b5, b6, b7, b8, b9 );
}

FD_DEV fe fe_sq_iter( fe h, int n ) {
  _Pragma("unroll 1")
  for( int i=0; i<n; i++ ) h = fe_sq( h );
  return h;
}

/* fe_avx_pow22523, avx/fd_ed25519_fe_avx.h:246-275: z^(2^252-3) */
FD_DEV fe fe_pow22523( fe const & z ) {
  fe t0, t1, t2;
  t0 = fe_sq( z );
  t1 = fe_sq_iter( t0, 2 );
  t1 = fe_mul( z, t1 );
  t0 = fe_mul( t0, t1 );
  t0 = fe_sq( t0 );
  t0 = fe_mul( t1, t0 );
  t1 = fe_sq_iter( t0, 5 );
  t0 = fe_mul( t1, t0 );
  t1 = fe_sq_iter( t0, 10 );
  t1 = fe_mul( t1, t0 );
  t2 = fe_sq_iter( t1, 20 );
  t1 = fe_mul( t2, t1 );
  t1 = fe_sq_iter( t1, 10 );
  t0 = fe_mul( t1, t0 );
  t1 = fe_sq_iter( t0, 50 );
  t1 = fe_mul( t1, t0 );
  t2 = fe_sq_iter( t1, 100 );
  t1 = fe_mul( t2, t1 );
  t1 = fe_sq_iter( t1, 50 );
  t0 = fe_mul( t1, t0 );
  t0 = fe_sq_iter( t0, 2 );
  return fe_mul( t0, z );
}

/* fd_ed25519_fe_frombytes (avx/fd_ed25519_fe.c:4-46).  s = 8 LE words. */
FD_DEV fe fe_frombytes( u32 const w[8] ) {
  /* byte-granular loads of the reference expressed on 32-bit words */
  auto B = [&]( int k ) -> u64 { return (u64)((w[k>>2] >> (8*(k&3))) & 0xffu); };
  auto L3 = [&]( int k ) -> u64 { return B(k) | (B(k+1)<<8) | (B(k+2)<<16); };
  auto L4 = [&]( int k ) -> u64 { return L3(k) | (B(k+3)<<24); };
  i64 h0 = (i64) L4(0);
  i64 h1 = (i64) L3(4) << 6;
  i64 h2 = (i64) L3(7) << 5;
  i64 h3 = (i64) L3(10) << 3;
  i64 h4 = (i64) L3(13) << 2;
  i64 h5 = (i64) L4(16);
  i64 h6 = (i64) L3(20) << 7;
  i64 h7 = (i64) L3(23) << 5;
  i64 h8 = (i64) L3(26) << 4;
  i64 h9 = (i64)((L3(29) & 0x7fffffUL) << 2);
  i64 c;
  c = (h9 + (1L<<24)) >> 25; h0 += c*19; h9 -= c<<25;
  c = (h1 + (1L<<24)) >> 25; h2 += c;    h1 -= c<<25;
  c = (h3 + (1L<<24)) >> 25; h4 += c;    h3 -= c<<25;
  c = (h5 + (1L<<24)) >> 25; h6 += c;    h5 -= c<<25;
  c = (h7 + (1L<<24)) >> 25; h8 += c;    h7 -= c<<25;
  c = (h0 + (1L<<25)) >> 26; h1 += c;    h0 -= c<<26;
  c = (h2 + (1L<<25)) >> 26; h3 += c;    h2 -= c<<26;
  c = (h4 + (1L<<25)) >> 26; h5 += c;    h4 -= c<<26;
  c = (h6 + (1L<<25)) >> 26; h7 += c;    h6 -= c<<26;
  c = (h8 + (1L<<25)) >> 26; h9 += c;    h8 -= c<<26;
  fe r;
  r.v[0]=(i32)h0; r.v[1]=(i32)h1; r.v[2]=(i32)h2; r.v[3]=(i32)h3; r.v[4]=(i32)h4;
  r.v[5]=(i32)h5; r.v[6]=(i32)h6; r.v[7]=(i32)h7; r.v[8]=(i32)h8; r.v[9]=(i32)h9;
  return r;
}

/* fd_ed25519_fe_tobytes canonicalisation (avx/fd_ed25519_fe.c:48-110),
   returning the 10 reduced limbs (packing is only needed for the two
   predicates below, which read bit 0 and "all zero"). */
FD_DEV void fe_reduce( i32 h[10], fe const & f ) {
  _Pragma("unroll") for( int i=0; i<10; i++ ) h[i] = f.v[i];
  i32 q = (wmul( h[9], 19 ) + (1<<24)) >> 25;
  _Pragma("unroll") for( int i=0; i<10; i++ ) q = (h[i] + q) >> ((i&1) ? 25 : 26);
  h[0] += wmul( q, 19 );
  _Pragma("unroll") for( int i=0; i<9; i++ ) {
    int w = (i&1) ? 25 : 26;
    h[i+1] += h[i] >> w; h[i] &= (i32)((1u<<w)-1u);
  }
  h[9] &= (i32)((1u<<25)-1u);
}

/* fd_ed25519_fe_isnonzero / isnegative (avx/fd_ed25519_fe.h:118-129) */
FD_DEV bool fe_isnonzero( fe const & f ) {
  i32 h[10]; fe_reduce( h, f );
  i32 o = 0; _Pragma("unroll") for( int i=0; i<10; i++ ) o |= h[i];
  return o != 0;
}
FD_DEV int fe_isnegative( fe const & f ) { i32 h[10]; fe_reduce( h, f ); return h[0] & 1; }

/* ------------------------------------------------------------------ */
/* SHA-512 (FIPS 180-4) of R || A || M, one message per lane.
   Reference: src/ballet/sha512/fd_sha512.c:264-399. */

__constant__ static u64 const SHA512_K[80] = FD_AMD_SHA512_K;

/* 64-bit rotate / shift on the two 32-bit halves with v_alignbit_b32 (two
   instructions; the generic form costs two 64-bit shifts and two ORs).  n is
   a compile-time constant at every call site. */
FD_DEV u64 rotr64( u64 x, int n ) {
  u32 lo = (u32)x, hi = (u32)(x >> 32);
  if( n >= 32 ) { u32 t = lo; lo = hi; hi = t; n -= 32; }
  if( !n ) return ((u64)hi << 32) | lo;
  return ((u64)__builtin_amdgcn_alignbit( lo, hi, (u32)n ) << 32) | __builtin_amdgcn_alignbit( hi, lo, (u32)n );
}
FD_DEV u64 shr64( u64 x, int n ) {
  u32 lo = (u32)x, hi = (u32)(x >> 32);
  return ((u64)(hi >> n) << 32) | __builtin_amdgcn_alignbit( hi, lo, (u32)n );
}

/* 3-input bitwise ops as one v_bitop3_b32 per half (gfx950): 0x96 = x^y^z,
   0xE8 = majority (both symmetric in their inputs) */
#define FD_BITOP3_64( x, y, z, LUT ) \
  ( ((u64)(u32)__builtin_amdgcn_bitop3_b32( (u32)((x) >> 32), (u32)((y) >> 32), (u32)((z) >> 32), LUT ) << 32) | \
    (u64)(u32)__builtin_amdgcn_bitop3_b32( (u32)(x), (u32)(y), (u32)(z), LUT ) )

/* One SHA-512 round on renamed state (FIPS 180-4 s6.4.2): the caller
   rotates the argument order instead of moving a..h, so every index is
   static and the state never moves between registers. */
FD_DEV void
sha512_round( u64 a, u64 b, u64 c, u64 & d, u64 e, u64 f, u64 g, u64 & h, u64 k, u64 w ) {
  u64 S1 = FD_BITOP3_64( rotr64( e, 14 ), rotr64( e, 18 ), rotr64( e, 41 ), 0x96 );
  u64 ch = (e & f) ^ (~e & g);
  u64 t1 = h + S1 + ch + k + w;
  u64 S0 = FD_BITOP3_64( rotr64( a, 28 ), rotr64( a, 34 ), rotr64( a, 39 ), 0x96 );
  u64 mj = FD_BITOP3_64( a, b, c, 0xE8 );
  d += t1;
  h  = t1 + S0 + mj;
}

/* 8 rounds starting at round r (r % 8 == 0), message words w[j0 .. j0+7] */
FD_DEV void
sha512_round8( u64 & a, u64 & b, u64 & c, u64 & d, u64 & e, u64 & f, u64 & g, u64 & h, int r, u64 const * w ) {
  sha512_round( a, b, c, d, e, f, g, h, SHA512_K[r+0], w[0] );
  sha512_round( h, a, b, c, d, e, f, g, SHA512_K[r+1], w[1] );
  sha512_round( g, h, a, b, c, d, e, f, SHA512_K[r+2], w[2] );
  sha512_round( f, g, h, a, b, c, d, e, SHA512_K[r+3], w[3] );
  sha512_round( e, f, g, h, a, b, c, d, SHA512_K[r+4], w[4] );
  sha512_round( d, e, f, g, h, a, b, c, SHA512_K[r+5], w[5] );
  sha512_round( c, d, e, f, g, h, a, b, SHA512_K[r+6], w[6] );
  sha512_round( b, c, d, e, f, g, h, a, SHA512_K[r+7], w[7] );
}

FD_DEV void sha512_compress( u64 st[8], u64 w[16] ) {
  u64 a=st[0], b=st[1], c=st[2], d=st[3], e=st[4], f=st[5], g=st[6], h=st[7];
  sha512_round8( a, b, c, d, e, f, g, h, 0, w     );
  sha512_round8( a, b, c, d, e, f, g, h, 8, w + 8 );
  _Pragma("unroll 1")
  for( int r=16; r<80; r+=16 ) {
    /* message schedule for rounds r .. r+15 in place: w[k] <- W[r+k] */
    _Pragma("unroll") for( int k=0; k<16; k++ ) {
      u64 w15 = w[(k+1) & 15], w2 = w[(k+14) & 15];
      u64 s0 = FD_BITOP3_64( rotr64( w15, 1 ), rotr64( w15, 8 ), shr64( w15, 7 ), 0x96 );
      u64 s1 = FD_BITOP3_64( rotr64( w2, 19 ), rotr64( w2, 61 ), shr64( w2, 6 ), 0x96 );
      w[k] = w[k] + s0 + w[(k+9) & 15] + s1;
    }
    sha512_round8( a, b, c, d, e, f, g, h, r,     w     );
    sha512_round8( a, b, c, d, e, f, g, h, r + 8, w + 8 );
  }
  st[0]+=a; st[1]+=b; st[2]+=c; st[3]+=d; st[4]+=e; st[5]+=f; st[6]+=g; st[7]+=h;
}

/* 8 bytes of the padded message starting at message offset o (multiple of
   8), little-endian: message bytes, the 0x80 terminator at offset sz, zeros
   after.  Only dwords that intersect [0, sz) are loaded. */
FD_DEV u64
msg_word( u8 const * __restrict__ m, u32 sz, u32 o ) {
  uintptr_t a  = (uintptr_t)(m + o);
  u32 sh = (u32)(a & 3u);
  u32 const * p = (u32 const *)(a - sh);   /* dword j covers message bytes [o-sh+4j, o-sh+4j+4) */
  u32 d0 = (o       < sz + sh)         ? p[0] : 0u;
  u32 d1 = (o + 4u  < sz + sh)         ? p[1] : 0u;
  u32 d2 = (sh && o + 8u < sz + sh)    ? p[2] : 0u;
  u32 lo = __builtin_amdgcn_alignbyte( d1, d0, sh );
  u32 hi = __builtin_amdgcn_alignbyte( d2, d1, sh );
  u64 w = ((u64)hi << 32) | lo;
  if( sz >= o + 8u ) return w;                                /* 8 message bytes */
  if( sz <  o      ) return 0UL;                              /* past the terminator */
  u32 nv = sz - o;                                            /* 0..7 message bytes, then 0x80 */
  return (w & ((1UL << (8u*nv)) - 1UL)) | (0x80UL << (8u*nv));
}

FD_DEV u64 bswap64( u64 x ) {
  return ((u64)__builtin_bswap32( (u32)x ) << 32) | (u64)__builtin_bswap32( (u32)(x >> 32) );
}

/* ------------------------------------------------------------------ */
/* x mod L for a 512-bit x (fd_ed25519_sc_reduce, fd_ed25519_user.c:3-110:
   canonical result, so any exact reduction is bit-identical). 32-bit word
   serial Horner: r <- (2^32 r + w) mod L, r kept in 9 x 32-bit limbs. */

FD_DEV void sc_reduce( u32 out[8], u32 const in[16] ) {
  u32 const Lw[8] = { 0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u };
  u32 r[9] = { 0,0,0,0,0,0,0,0,0 };
  for( int k=15; k>=0; k-- ) {
    /* r = r*2^32 + in[k]   (r < L < 2^253 -> r*2^32 < 2^285: 9 limbs) */
    _Pragma("unroll") for( int i=8; i>0; i-- ) r[i] = r[i-1];
    r[0] = in[k];
    /* q ~= floor(r / 2^252) <= 2^33: estimate from the top limbs; it may
       overshoot floor(r/L) by at most 1 (r/2^252 - r/L < 2^-120 r/2^252). */
    u64 q = ((u64)r[8] << 4) | (r[7] >> 28);
    /* r -= q*L */
    i64 br = 0; u64 carry = 0;
    _Pragma("unroll") for( int i=0; i<9; i++ ) {
      u64 lw = (i < 8) ? (u64)Lw[i] : 0u;
      /* q*L word i: 64x32 -> up to 97 bits; split q */
      u64 plo = (q & 0xffffffffu) * lw;
      u64 phi = (q >> 32) * lw;
      u64 t = plo + carry;
      u64 c2 = (t < plo) ? 1u : 0u;
      u32 pw = (u32)t;
      carry = (t >> 32) + (phi) + (c2 << 32);
      i64 d = (i64)(u64)r[i] - (i64)(u64)pw + br;
      r[i] = (u32)d; br = d >> 32;
    }
    if( br < 0 ) {   /* overshoot: add L back once */
      u64 c = 0;
      _Pragma("unroll") for( int i=0; i<9; i++ ) {
        u64 s = (u64)r[i] + (i < 8 ? (u64)Lw[i] : 0u) + c; r[i] = (u32)s; c = s >> 32;
      }
    }
  }
  /* final: r < 2L possible -> conditional subtract */
  {
    bool ge = true;
    _Pragma("unroll") for( int i=7; i>=0; i-- ) { /* lexicographic compare, r[8]==0 here */
      if( r[i] != Lw[i] ) { ge = r[i] > Lw[i]; break; }
    }
    if( r[8] ) ge = true;
    if( ge ) {
      i64 br = 0;
      _Pragma("unroll") for( int i=0; i<8; i++ ) { i64 d = (i64)(u64)r[i] - (i64)(u64)Lw[i] + br; r[i] = (u32)d; br = d >> 32; }
    }
  }
  _Pragma("unroll") for( int i=0; i<8; i++ ) out[i] = r[i];
}

#endif /* FD_ED25519_DEV_H */
