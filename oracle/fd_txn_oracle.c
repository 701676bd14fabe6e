/* oracle/fd_txn_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the reference's transaction parser,
 * fd_txn_parse (src/ballet/txn/fd_txn_parse.c:6-217, compact-u16 rules of
 * src/ballet/txn/fd_compact_u16.h:35-87), and of the multi-signer verify
 * rule the GPU transaction front end applies on top of it (signature i is
 * checked against account address i over payload[message_off, sz),
 * src/ballet/txn/fd_txn.h:159-217).  It is the checker for k_txn_parse /
 * fd_ed25519_amd_verify_txns; it is never linked into the product.
 *
 * Parity pin: oracle/gen_txn_golden.c runs this restatement and the
 * reference's own fd_txn_parse (compiled from its sources into
 * oracle/_ref/libfdref.so) over the reference's fixtures and the
 * reference test's byte-mutation sweep (test_txn_parse.c:124-214), and
 * aborts on any difference in return value, output bytes or failure line.
 *
 * Failure bookkeeping follows the reference: a failed check records the
 * source line of the reference check that failed (fd_txn_parse.c) in the
 * counters' ring, so "why did it fail" is comparable too.
 */
#include <stdint.h>
#include <string.h>
#include <stddef.h>
#include <pthread.h>

typedef unsigned char  uchar;
typedef unsigned short ushort;
typedef unsigned long  ulong;
typedef unsigned int   uint;
typedef signed char    schar;

#include "../include/fd_txn_amd.h"

/* compact-u16 length (fd_compact_u16.h:69-87): 1..3 on success, 0 if the
   encoding is truncated, non-minimal or exceeds 16 bits. */
static ulong
cu16_len( uchar const * p, ulong avail ) {
  if( avail >= 1UL && !(p[0] & 0x80) ) return 1UL;
  if( avail >= 2UL && !(p[1] & 0x80) ) return p[1] ? 2UL : 0UL;
  if( avail >= 3UL && !(p[2] & 0xFC) ) return p[2] ? 3UL : 0UL;
  return 0UL;
}

/* compact-u16 value for a known length (fd_compact_u16.h:35-52) */
static ushort
cu16_val( uchar const * p, ulong len ) {
  ulong v = (ulong)(p[0] & 0x7F);
  if( len == 1UL ) return (ushort)p[0];
  v += (ulong)(p[1] & (len == 2UL ? 0xFF : 0x7F)) << 7;
  if( len == 3UL ) v += (ulong)p[2] << 14;
  return (ushort)v;
}

/* Reader over the untrusted payload.  Every accessor reports the reference
   line number of the check it stands for. */
typedef struct {
  uchar const * p;
  ulong         sz;
  ulong         at;
  ulong         fail_line;
} rd_t;

static int
rd_room( rd_t * r, ulong n, ulong line ) {           /* CHECK_LEFT: n <= sz-at */
  if( n <= r->sz - r->at ) return 1;
  r->fail_line = line; return 0;
}

static int
rd_test( rd_t * r, int ok, ulong line ) {             /* CHECK */
  if( ok ) return 1;
  r->fail_line = line; return 0;
}

static int
rd_cu16( rd_t * r, ushort * out, ulong line ) {       /* READ_CHECKED_COMPACT_U16 */
  ulong len = cu16_len( r->p + r->at, r->sz - r->at );
  if( !len ) { r->fail_line = line; return 0; }
  *out = cu16_val( r->p + r->at, len );
  r->at += len;
  return 1;
}

static ulong
parse( uchar const * payload, ulong sz, void * out_buf, ulong * fail_line ) {
  rd_t r = { payload, sz, 0UL, 0UL };
  fd_txn_t * t = (fd_txn_t *)out_buf;
# define NEED( c ) do { if( !(c) ) { *fail_line = r.fail_line; return 0UL; } } while(0)

  NEED( rd_test( &r, sz <= 0xFFFFUL, 73 ) );

  /* signatures */
  NEED( rd_room( &r, 1UL, 79 ) );
  ulong nsig = payload[ r.at++ ];
  NEED( rd_test( &r, nsig >= 1UL && nsig <= FD_TXN_SIG_MAX, 81 ) );
  NEED( rd_room( &r, FD_TXN_SIGNATURE_SZ*nsig, 82 ) );
  ulong sig_off = r.at; r.at += FD_TXN_SIGNATURE_SZ*nsig;

  /* message header: optional version prefix, then the three counts */
  ulong msg_off = r.at;
  NEED( rd_room( &r, 1UL, 85 ) );
  uchar b0 = payload[ r.at++ ];
  uchar ver;
  if( b0 & 0x80 ) {
    ver = (uchar)(b0 & 0x7F);
    NEED( rd_test( &r, ver == FD_TXN_V0, 91 ) );
    NEED( rd_room( &r, 1UL, 93 ) );
    NEED( rd_test( &r, payload[ r.at ] == nsig, 93 ) );
    r.at++;
  } else {
    ver = FD_TXN_VLEGACY;
    NEED( rd_test( &r, b0 == nsig, 96 ) );
  }
  NEED( rd_room( &r, 1UL, 98 ) );
  ulong ro_signed = payload[ r.at++ ];
  NEED( rd_test( &r, ro_signed < nsig, 100 ) );
  NEED( rd_room( &r, 1UL, 102 ) );
  ulong ro_unsigned = payload[ r.at++ ];

  /* static account addresses and the blockhash */
  ushort nacct;
  NEED( rd_cu16( &r, &nacct, 105 ) );
  NEED( rd_test( &r, nsig <= nacct && nacct <= FD_TXN_ACCT_ADDR_MAX, 106 ) );
  NEED( rd_test( &r, nsig + ro_unsigned <= (ulong)nacct, 107 ) );
  NEED( rd_room( &r, FD_TXN_ACCT_ADDR_SZ*nacct, 109 ) );
  ulong acct_off = r.at; r.at += FD_TXN_ACCT_ADDR_SZ*nacct;
  NEED( rd_room( &r, FD_TXN_BLOCKHASH_SZ, 110 ) );
  ulong bh_off = r.at; r.at += FD_TXN_BLOCKHASH_SZ;

  /* instructions: 1 B program index, cu16 account count + indices,
     cu16 data size + data; at least 3 bytes each */
  ushort ninstr;
  NEED( rd_cu16( &r, &ninstr, 113 ) );
  NEED( rd_room( &r, 3UL*ninstr, 115 ) );

  t->transaction_version   = ver;
  t->signature_cnt         = (uchar)nsig;
  t->signature_off         = (ushort)sig_off;
  t->message_off           = (ushort)msg_off;
  t->readonly_signed_cnt   = (uchar)ro_signed;
  t->readonly_unsigned_cnt = (uchar)ro_unsigned;
  t->acct_addr_cnt         = nacct;
  t->acct_addr_off         = (ushort)acct_off;
  t->recent_blockhash_off  = (ushort)bh_off;
  t->instr_cnt             = ninstr;

  for( ulong j=0UL; j<ninstr; j++ ) {
    fd_txn_instr_t * ix = &t->instr[ j ];
    NEED( rd_room( &r, 3UL, 136 ) );
    uchar prog = payload[ r.at++ ];
    ushort nacc, ndata;
    NEED( rd_cu16( &r, &nacc, 137 ) );
    NEED( rd_room( &r, nacc, 138 ) );
    ulong a_off = r.at; r.at += nacc;
    NEED( rd_cu16( &r, &ndata, 139 ) );
    NEED( rd_room( &r, ndata, 140 ) );
    ulong d_off = r.at; r.at += ndata;
    ix->program_id          = prog;
    ix->_padding_reserved_1 = 0;
    ix->acct_cnt            = nacc;
    ix->data_sz             = ndata;
    ix->acct_off            = (ushort)a_off;
    ix->data_off            = (ushort)d_off;
  }

  /* v0 address lookup tables (absent for legacy transactions) */
  ulong nlut = 0UL, adtl_w = 0UL, adtl = 0UL;
  fd_txn_acct_addr_lut_t * lut = (fd_txn_acct_addr_lut_t *)(t->instr + ninstr);
  if( ver == FD_TXN_V0 ) {
    ushort cnt;
    NEED( rd_cu16( &r, &cnt, 161 ) );
    nlut = cnt;
    NEED( rd_test( &r, nlut <= FD_TXN_ADDR_TABLE_LOOKUP_MAX, 162 ) );
    NEED( rd_room( &r, 34UL*nlut, 163 ) );
    for( ulong j=0UL; j<nlut; j++ ) {
      NEED( rd_room( &r, FD_TXN_ACCT_ADDR_SZ, 166 ) );
      ulong addr = r.at; r.at += FD_TXN_ACCT_ADDR_SZ;
      ushort nw, nr;
      NEED( rd_cu16( &r, &nw, 170 ) );
      NEED( rd_room( &r, nw, 171 ) );
      ulong w_off = r.at; r.at += nw;
      NEED( rd_cu16( &r, &nr, 172 ) );
      NEED( rd_room( &r, nr, 173 ) );
      ulong r_off = r.at; r.at += nr;
      NEED( rd_test( &r, nw <= FD_TXN_ACCT_ADDR_MAX - nacct, 175 ) );
      NEED( rd_test( &r, nr <= FD_TXN_ACCT_ADDR_MAX - nacct, 176 ) );
      lut[ j ].addr_off     = (ushort)addr;
      lut[ j ].writable_cnt = (uchar)nw;
      lut[ j ].readonly_cnt = (uchar)nr;
      lut[ j ].writable_off = (ushort)w_off;
      lut[ j ].readonly_off = (ushort)r_off;
      adtl_w += nw;
      adtl   += (ulong)nw + (ulong)nr;
    }
  }

  NEED( rd_test( &r, r.at == sz, 189 ) );
  NEED( rd_test( &r, nacct + adtl <= FD_TXN_ACCT_ADDR_MAX, 191 ) );

  /* every referenced account index must exist; the program is never the
     fee payer (index 0) */
  ulong total = nacct + adtl;
  for( ulong j=0UL; j<ninstr; j++ ) {
    fd_txn_instr_t const * ix = &t->instr[ j ];
    NEED( rd_test( &r, ix->program_id > 0 && ix->program_id < total, 200 ) );
    for( ulong k=0UL; k<ix->acct_cnt; k++ ) NEED( rd_test( &r, payload[ ix->acct_off + k ] < total, 202 ) );
  }

  t->addr_table_lookup_cnt        = (uchar)nlut;
  t->addr_table_adtl_writable_cnt = (uchar)adtl_w;
  t->addr_table_adtl_cnt          = (uchar)adtl;
  t->_padding_reserved_1          = 0;
  *fail_line = 0UL;
  return fd_txn_footprint( ninstr, nlut );
# undef NEED
}

/* Same contract as fd_txn_parse (fd_txn.h:377-389). */
ulong
oracle_txn_parse( uchar const *             payload,
                  ulong                     payload_sz,
                  void *                    out_buf,
                  fd_txn_parse_counters_t * counters_opt ) {
  ulong line = 0UL;
  ulong fp = parse( payload, payload_sz, out_buf, &line );
  if( counters_opt ) {
    if( fp ) counters_opt->success_cnt++;
    else     counters_opt->failure_ring[ (counters_opt->failure_cnt++) % FD_TXN_PARSE_COUNTERS_RING_SZ ] = line;
  }
  return fp;
}

/* Line of the reference check that rejects the payload (0 if it parses). */
ulong
oracle_txn_parse_fail_line( uchar const * payload, ulong payload_sz ) {
  static __thread uchar buf[ FD_TXN_MAX_SZ ] __attribute__((aligned(8)));
  ulong line = 0UL;
  (void)parse( payload, payload_sz, buf, &line );
  return line;
}

/* Multi-signer batch verdicts (the rule fd_ed25519_amd_verify_txns
   implements), for the tests: txn t is payload[txn_off[t] .. +txn_sz[t]).
   txn_err[t]: FD_TXN_AMD_ERR_PARSE if the payload does not parse, else
   the first nonzero per-signature code in signature order, else 0.
   Signature numbering (sig_base, txn_cnt+1 entries) follows the engine's
   slot rule: a payload reserves payload[0] slots when that byte is a
   plausible signature count (1..127 with room for the signatures,
   fd_txn_parse.c:79-82), else none -- exact for every payload that parses;
   the slots of a payload that fails to parse read FD_TXN_AMD_ERR_PARSE. */
static ulong
txn_slots( uchar const * p, ulong sz ) {
  if( !sz ) return 0UL;
  ulong k = p[0];
  return ( k >= 1UL && k <= FD_TXN_SIG_MAX && 64UL*k <= sz - 1UL ) ? k : 0UL;
}

int oracle_ed25519_verify( void const * msg, ulong sz, void const * sig, void const * pub );

typedef struct {
  ulong lo, hi;
  uchar const * payload; uint const * off; uint const * sz;
  schar * txn_err; uint const * base; schar * sig_err;
} txn_job_t;

static void *
txn_worker( void * arg ) {
  txn_job_t * j = (txn_job_t *)arg;
  uchar buf[ FD_TXN_MAX_SZ ] __attribute__((aligned(8)));
  for( ulong t=j->lo; t<j->hi; t++ ) {
    uchar const * p = j->payload + j->off[ t ];
    ulong line;
    ulong fp = parse( p, j->sz[ t ], buf, &line );
    if( !fp ) {
      j->txn_err[ t ] = (schar)FD_TXN_AMD_ERR_PARSE;
      if( j->sig_err ) for( uint s=j->base[ t ]; s<j->base[ t+1 ]; s++ ) j->sig_err[ s ] = (schar)FD_TXN_AMD_ERR_PARSE;
      continue;
    }
    fd_txn_t const * x = (fd_txn_t const *)buf;
    int first = 0;
    for( ulong i=0UL; i<x->signature_cnt; i++ ) {
      int e = oracle_ed25519_verify( p + x->message_off, j->sz[ t ] - x->message_off,
                                     p + x->signature_off + 64UL*i, p + x->acct_addr_off + 32UL*i );
      if( j->sig_err ) j->sig_err[ j->base[ t ] + i ] = (schar)e;
      if( e && !first ) first = e;
    }
    j->txn_err[ t ] = (schar)first;
  }
  return NULL;
}

/* sig_base is always filled (needs txn_cnt+1 entries); sig_err optional. */
int
oracle_txn_verify_batch( ulong txn_cnt, uchar const * payload, uint const * txn_off, uint const * txn_sz,
                         schar * txn_err, uint * sig_base, schar * sig_err, int nthread ) {
  uint acc = 0U;
  for( ulong t=0UL; t<txn_cnt; t++ ) {
    sig_base[ t ] = acc;
    acc += (uint)txn_slots( payload + txn_off[ t ], txn_sz[ t ] );
  }
  sig_base[ txn_cnt ] = acc;
  if( nthread < 1 ) nthread = 1;
  if( nthread > 64 ) nthread = 64;
  pthread_t th[ 64 ]; txn_job_t jb[ 64 ];
  for( int k=0; k<nthread; k++ ) {
    jb[ k ] = (txn_job_t){ txn_cnt*(ulong)k/(ulong)nthread, txn_cnt*(ulong)(k+1)/(ulong)nthread,
                           payload, txn_off, txn_sz, txn_err, sig_base, sig_err };
    pthread_create( &th[ k ], NULL, txn_worker, &jb[ k ] );
  }
  for( int k=0; k<nthread; k++ ) pthread_join( th[ k ], NULL );
  return 0;
}
