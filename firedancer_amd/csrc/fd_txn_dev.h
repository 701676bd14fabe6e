/* firedancer_amd/csrc/fd_txn_dev.h -- device-side fd_txn_parse, shared by
   the transaction front end (fd_txn_kernels.hip: k_txn_parse) and the
   streaming tile's persistent kernel (fd_ed25519_kernels.hip:
   k_tile_persist, TXN framing).  One lane parses one untrusted wire
   transaction with the exact accept/reject behaviour and descriptor bytes of
   the reference's fd_txn_parse (src/ballet/txn/fd_txn_parse.c:6-217;
   compact-u16 rules of fd_compact_u16.h:35-87). */
#ifndef FD_TXN_DEV_H
#define FD_TXN_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fd_txn_dev {

typedef uint8_t  u8;
typedef uint16_t u16;
typedef uint32_t u32;

#define TXN_SIG_MAX        127u
#define TXN_ACCT_ADDR_MAX  256u
#define TXN_LUT_MAX        254u
#define TXN_ERR_PARSE      (-4)    /* FD_TXN_AMD_ERR_PARSE */

/* fd_txn_t / fd_txn_instr_t / fd_txn_acct_addr_lut_t byte offsets
   (fd_txn.h:107-139,146-272,281-318; include/fd_txn_amd.h) */
enum { TX_VER = 0, TX_NSIG = 1, TX_SIGOFF = 2, TX_MSGOFF = 4, TX_ROS = 6, TX_ROU = 7, TX_NACCT = 8,
       TX_ACCTOFF = 10, TX_BHOFF = 12, TX_NLUT = 14, TX_ADTLW = 15, TX_ADTL = 16, TX_PAD = 17,
       TX_NINSTR = 18, TX_HDR = 20, IX_SZ = 10, LUT_SZ = 8 };

/* cursor over one untrusted payload in HBM (byte loads hit L1/L2 after the
   first touch of each line; payloads are <= a few KB) */
struct cur_t {
  u8 const * p;
  u32        sz;
  u32        at;
  __device__ bool room( u32 n ) const { return n <= sz - at; }      /* CHECK_LEFT, no overflow */
  __device__ u8   b( u32 k ) const { return p[k]; }
  /* READ_CHECKED_COMPACT_U16: false on truncated / non-minimal / > 16 bit */
  __device__ bool cu16( u32 * out ) {
    u32 avail = sz - at;
    u32 b0 = avail >= 1u ? p[at] : 0u;
    if( avail >= 1u && !(b0 & 0x80u) ) { *out = b0; at += 1u; return true; }
    u32 b1 = avail >= 2u ? p[at+1u] : 0u;
    if( avail >= 2u && !(b1 & 0x80u) ) {
      if( !b1 ) return false;
      *out = (b0 & 0x7fu) + (b1 << 7); at += 2u; return true;
    }
    u32 b2 = avail >= 3u ? p[at+2u] : 0u;
    if( avail >= 3u && !(b2 & 0xfcu) ) {
      if( !b2 ) return false;
      *out = (b0 & 0x7fu) + ((b1 & 0x7fu) << 7) + (b2 << 14); at += 3u; return true;
    }
    return false;
  }
};

__device__ __forceinline__ void st16( u8 * o, u32 off, u32 v ) { *(u16 *)(o + off) = (u16)v; }

/* The parse proper.  Writes descriptor fields to o (may be NULL: validate
   only; instruction records are then kept in a tiny local ring for the
   final index checks, re-read from the payload).  Returns the footprint or
   0, and the three offsets the verify layout needs. */
__device__ inline u32
txn_parse( u8 const * payload, u32 sz, u8 * o, u32 * nsig_out, u32 * sigoff_out, u32 * acctoff_out, u32 * msgoff_out ) {
  cur_t c = { payload, sz, 0u };
  if( sz > 0xffffu ) return 0u;                                        /* :73 */
  if( !c.room( 1u ) ) return 0u;                                       /* :79 */
  u32 nsig = c.b( c.at++ );
  if( nsig < 1u || nsig > TXN_SIG_MAX ) return 0u;                     /* :81 */
  if( !c.room( 64u*nsig ) ) return 0u;                                 /* :82 */
  u32 sig_off = c.at; c.at += 64u*nsig;
  u32 msg_off = c.at;
  if( !c.room( 1u ) ) return 0u;                                       /* :85 */
  u32 b0 = c.b( c.at++ );
  u32 ver;
  if( b0 & 0x80u ) {
    ver = b0 & 0x7fu;
    if( ver != 0u ) return 0u;                                         /* :91 */
    if( !c.room( 1u ) || c.b( c.at ) != nsig ) return 0u;              /* :93 */
    c.at++;
  } else {
    ver = 0xffu;
    if( b0 != nsig ) return 0u;                                        /* :96 */
  }
  if( !c.room( 1u ) ) return 0u;                                       /* :98 */
  u32 ros = c.b( c.at++ );
  if( ros >= nsig ) return 0u;                                         /* :100 */
  if( !c.room( 1u ) ) return 0u;                                       /* :102 */
  u32 rou = c.b( c.at++ );
  u32 nacct;
  if( !c.cu16( &nacct ) ) return 0u;                                   /* :105 */
  if( nsig > nacct || nacct > TXN_ACCT_ADDR_MAX ) return 0u;           /* :106 */
  if( nsig + rou > nacct ) return 0u;                                  /* :107 */
  if( !c.room( 32u*nacct ) ) return 0u;                                /* :109 */
  u32 acct_off = c.at; c.at += 32u*nacct;
  if( !c.room( 32u ) ) return 0u;                                      /* :110 */
  u32 bh_off = c.at; c.at += 32u;
  u32 ninstr;
  if( !c.cu16( &ninstr ) ) return 0u;                                  /* :113 */
  if( !c.room( 3u*ninstr ) ) return 0u;                                /* :115 */

  u32 ix_start = c.at;                                                 /* instructions are re-walked below */
  for( u32 j=0u; j<ninstr; j++ ) {
    if( !c.room( 3u ) ) return 0u;                                     /* :136 */
    u32 prog = c.b( c.at++ );
    u32 nacc, ndata;
    if( !c.cu16( &nacc ) ) return 0u;                                  /* :137 */
    if( !c.room( nacc ) ) return 0u;                                   /* :138 */
    u32 a_off = c.at; c.at += nacc;
    if( !c.cu16( &ndata ) ) return 0u;                                 /* :139 */
    if( !c.room( ndata ) ) return 0u;                                  /* :140 */
    u32 d_off = c.at; c.at += ndata;
    if( o ) {
      u8 * ix = o + TX_HDR + IX_SZ*j;
      ix[0] = (u8)prog; ix[1] = 0u;
      st16( ix, 2, nacc ); st16( ix, 4, ndata ); st16( ix, 6, a_off ); st16( ix, 8, d_off );
    }
  }

  u32 nlut = 0u, adtl_w = 0u, adtl = 0u;
  if( ver == 0u ) {
    if( !c.cu16( &nlut ) ) return 0u;                                  /* :161 */
    if( nlut > TXN_LUT_MAX ) return 0u;                                /* :162 */
    if( !c.room( 34u*nlut ) ) return 0u;                               /* :163 */
    for( u32 j=0u; j<nlut; j++ ) {
      if( !c.room( 32u ) ) return 0u;                                  /* :166 */
      u32 addr = c.at; c.at += 32u;
      u32 nw, nr;
      if( !c.cu16( &nw ) ) return 0u;                                  /* :170 */
      if( !c.room( nw ) ) return 0u;                                   /* :171 */
      u32 w_off = c.at; c.at += nw;
      if( !c.cu16( &nr ) ) return 0u;                                  /* :172 */
      if( !c.room( nr ) ) return 0u;                                   /* :173 */
      u32 r_off = c.at; c.at += nr;
      if( nw > TXN_ACCT_ADDR_MAX - nacct ) return 0u;                  /* :175 */
      if( nr > TXN_ACCT_ADDR_MAX - nacct ) return 0u;                  /* :176 */
      if( o ) {
        u8 * l = o + TX_HDR + IX_SZ*ninstr + LUT_SZ*j;
        st16( l, 0, addr ); l[2] = (u8)nw; l[3] = (u8)nr; st16( l, 4, w_off ); st16( l, 6, r_off );
      }
      adtl_w += nw; adtl += nw + nr;
    }
  }
  if( c.at != sz ) return 0u;                                          /* :189 */
  if( nacct + adtl > TXN_ACCT_ADDR_MAX ) return 0u;                    /* :191 */

  /* account index range checks (:196-204), re-walking the (already
     validated) instruction records from the payload */
  u32 total = nacct + adtl;
  c.at = ix_start;
  for( u32 j=0u; j<ninstr; j++ ) {
    u32 prog = c.b( c.at++ );
    u32 nacc, ndata;
    c.cu16( &nacc );
    if( !(prog > 0u && prog < total) ) return 0u;                      /* :200 */
    for( u32 k=0u; k<nacc; k++ ) if( c.b( c.at + k ) >= total ) return 0u;   /* :202 */
    c.at += nacc;
    c.cu16( &ndata );
    c.at += ndata;
  }

  if( o ) {
    o[TX_VER] = (u8)ver; o[TX_NSIG] = (u8)nsig; st16( o, TX_SIGOFF, sig_off ); st16( o, TX_MSGOFF, msg_off );
    o[TX_ROS] = (u8)ros; o[TX_ROU] = (u8)rou; st16( o, TX_NACCT, nacct ); st16( o, TX_ACCTOFF, acct_off );
    st16( o, TX_BHOFF, bh_off ); o[TX_NLUT] = (u8)nlut; o[TX_ADTLW] = (u8)adtl_w; o[TX_ADTL] = (u8)adtl;
    o[TX_PAD] = 0u; st16( o, TX_NINSTR, ninstr );
  }
  *nsig_out = nsig; *sigoff_out = sig_off; *acctoff_out = acct_off; *msgoff_out = msg_off;
  return (u32)TX_HDR + IX_SZ*ninstr + LUT_SZ*nlut;                     /* fd_txn_footprint */
}

} /* namespace fd_txn_dev */

#endif /* FD_TXN_DEV_H */
