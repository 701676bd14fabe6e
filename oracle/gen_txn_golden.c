/* oracle/gen_txn_golden.c -- TEST INFRASTRUCTURE ONLY (build container).
 *
 * Pins the transaction-parser restatement (oracle/fd_txn_oracle.c) against
 * the reference's own fd_txn_parse (src/ballet/txn/fd_txn_parse.c, compiled
 * from its sources into oracle/_ref/libfdref.so) and writes the committed
 * fixture tests/golden/txn_mutations.bin.
 *
 *   gen_txn_golden <out.bin> <fixture.bin>...     (the reference's txn fixtures)
 *   gen_txn_golden fuzz <seed> <count>             (synthetic txns + mutations)
 *
 * For every fixture payload it runs, on both parsers:
 *   - the exhaustive single-byte sweep (every position x all 255 other
 *     values) and every truncation, as the reference test does
 *     (test_txn_parse.c:124-214);
 *   - compares return value, output bytes (footprint) and the failure line
 *     recorded in the counters ring; any difference aborts.
 * The fixture file keeps a reduced, deterministic mutation list per payload
 * (tests/_txn.py: mutation_list) with the expected footprint and failure
 * line of each mutation and an FNV-1a digest of all successful outputs, so
 * the GPU parser can be checked on the box without the reference.
 *
 * fixture file (little endian):
 *   magic[16] "FDTXNGOLDEN1\0\0\0\0", u32 nfix, u32 0,
 *   nfix x { u32 sz, u32 nmut, u64 out_digest, payload[sz],
 *            nmut x { u16 footprint, u16 fail_line } }
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned char  uchar;
typedef unsigned short ushort;
typedef unsigned long  ulong;
typedef unsigned int   uint;
typedef signed char    schar;
#include "../include/fd_txn_amd.h"

/* reference (oracle/_ref/libfdref.so) and restatement (liboracle.so) */
ulong fd_txn_parse( uchar const * payload, ulong payload_sz, void * out_buf, fd_txn_parse_counters_t * counters_opt );
ulong oracle_txn_parse( uchar const * payload, ulong payload_sz, void * out_buf, fd_txn_parse_counters_t * counters_opt );

static uint64_t fnv( uint64_t h, void const * p, ulong n ) {
  uchar const * b = (uchar const *)p;
  for( ulong i=0; i<n; i++ ) { h ^= b[i]; h *= 0x100000001b3UL; }
  return h;
}

static ulong g_cmp, g_ok;

/* one payload on both parsers; returns footprint, *line = failure line */
static ulong
both( uchar const * p, ulong sz, ulong * line, uint64_t * dig ) {
  static uchar a[ FD_TXN_MAX_SZ + 64 ] __attribute__((aligned(8))), b[ FD_TXN_MAX_SZ + 64 ] __attribute__((aligned(8)));
  fd_txn_parse_counters_t ca, cb; memset( &ca, 0, sizeof ca ); memset( &cb, 0, sizeof cb );
  ulong fa = fd_txn_parse( p, sz, a, &ca );
  ulong fb = oracle_txn_parse( p, sz, b, &cb );
  ulong la = fa ? 0UL : ca.failure_ring[ 0 ];
  ulong lb = fb ? 0UL : cb.failure_ring[ 0 ];
  g_cmp++;
  if( fa != fb || la != lb || (fa && memcmp( a, b, fa )) ) {
    fprintf( stderr, "PARSE MISMATCH sz=%lu ref=(%lu,line %lu) oracle=(%lu,line %lu)\n", sz, fa, la, fb, lb );
    exit( 1 );
  }
  if( fa ) { g_ok++; if( dig ) *dig = fnv( *dig, a, fa ); }
  *line = la;
  return fa;
}

/* the reduced mutation list (mirrored by tests/_txn.py: mutation_list):
   per position i the values orig^1, orig^0x80, orig+1, 0x00, 0xff (those
   that differ from orig), then every truncation length 0..sz-1 */
static ulong
mutations( uchar const * orig, ulong sz, FILE * out, uint64_t * dig ) {
  uchar * p = (uchar *)malloc( sz ? sz : 1 );
  memcpy( p, orig, sz );
  ulong n = 0, line;
  for( ulong i=0; i<sz; i++ ) {
    uchar o = orig[ i ];
    uchar vs[5] = { (uchar)(o ^ 1), (uchar)(o ^ 0x80), (uchar)(o + 1), 0x00, 0xff };
    for( int k=0; k<5; k++ ) {
      if( vs[k] == o ) continue;
      p[ i ] = vs[k];
      ulong fp = both( p, sz, &line, dig );
      if( out ) { ushort r[2] = { (ushort)fp, (ushort)line }; fwrite( r, 2, 2, out ); }
      n++;
    }
    p[ i ] = o;
  }
  for( ulong L=0; L<sz; L++ ) {
    ulong fp = both( p, L, &line, dig );
    if( out ) { ushort r[2] = { (ushort)fp, (ushort)line }; fwrite( r, 2, 2, out ); }
    n++;
  }
  free( p );
  return n;
}

/* exhaustive: every position x all 255 other values (not stored) */
static void
exhaustive( uchar const * orig, ulong sz ) {
  uchar * p = (uchar *)malloc( sz ? sz : 1 );
  memcpy( p, orig, sz );
  ulong line;
  for( ulong i=0; i<sz; i++ ) {
    for( int v=1; v<256; v++ ) { p[ i ] = (uchar)(orig[ i ] + v); both( p, sz, &line, NULL ); }
    p[ i ] = orig[ i ];
  }
  free( p );
}

/* ---- synthetic transactions for the fuzz mode ---- */
static uint64_t sm64( uint64_t * s ) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15UL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9UL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebUL;
  return z ^ (z >> 31);
}
static ulong put_cu16( uchar * p, ulong v ) {
  if( v < 0x80 ) { p[0] = (uchar)v; return 1; }
  if( v < 0x4000 ) { p[0] = (uchar)(0x80 | (v & 0x7f)); p[1] = (uchar)(v >> 7); return 2; }
  p[0] = (uchar)(0x80 | (v & 0x7f)); p[1] = (uchar)(0x80 | ((v >> 7) & 0x7f)); p[2] = (uchar)(v >> 14); return 3;
}
/* a well-formed legacy or v0 transaction with random counts */
static ulong
synth( uint64_t * s, uchar * p ) {
  ulong at = 0;
  int v0 = (int)(sm64( s ) & 1);
  ulong nsig = 1 + sm64( s ) % 4, nacct = nsig + sm64( s ) % 6, ninstr = sm64( s ) % 4, nlut = v0 ? sm64( s ) % 3 : 0;
  p[ at++ ] = (uchar)nsig;
  for( ulong i=0; i<64*nsig; i++ ) p[ at++ ] = (uchar)sm64( s );
  if( v0 ) p[ at++ ] = 0x80;
  p[ at++ ] = (uchar)nsig;
  p[ at++ ] = (uchar)(sm64( s ) % nsig);
  p[ at++ ] = (uchar)(sm64( s ) % (nacct - nsig + 1));
  at += put_cu16( p + at, nacct );
  for( ulong i=0; i<32*nacct + 32; i++ ) p[ at++ ] = (uchar)sm64( s );
  at += put_cu16( p + at, ninstr );
  ulong adtl = 0; ulong lw[3], lr[3];
  for( ulong j=0; j<nlut; j++ ) { lw[j] = sm64( s ) % 3; lr[j] = sm64( s ) % 3; adtl += lw[j] + lr[j]; }
  ulong total = nacct + adtl;
  for( ulong j=0; j<ninstr; j++ ) {
    p[ at++ ] = (uchar)(1 + sm64( s ) % (total - 1 ? total - 1 : 1));
    ulong na = sm64( s ) % 4, nd = sm64( s ) % 20;
    at += put_cu16( p + at, na );
    for( ulong k=0; k<na; k++ ) p[ at++ ] = (uchar)(sm64( s ) % total);
    at += put_cu16( p + at, nd );
    for( ulong k=0; k<nd; k++ ) p[ at++ ] = (uchar)sm64( s );
  }
  if( v0 ) {
    at += put_cu16( p + at, nlut );
    for( ulong j=0; j<nlut; j++ ) {
      for( int k=0; k<32; k++ ) p[ at++ ] = (uchar)sm64( s );
      at += put_cu16( p + at, lw[j] ); for( ulong k=0; k<lw[j]; k++ ) p[ at++ ] = (uchar)sm64( s );
      at += put_cu16( p + at, lr[j] ); for( ulong k=0; k<lr[j]; k++ ) p[ at++ ] = (uchar)sm64( s );
    }
  }
  return at;
}

int
main( int argc, char ** argv ) {
  if( argc >= 4 && !strcmp( argv[1], "fuzz" ) ) {
    uint64_t s = strtoull( argv[2], NULL, 0 ) * 0x2545F4914F6CDD1DUL + 7;
    ulong cnt = strtoul( argv[3], NULL, 0 ), line;
    uchar p[ 4096 ];
    for( ulong c=0; c<cnt; c++ ) {
      ulong sz = synth( &s, p );
      both( p, sz, &line, NULL );
      for( int m=0; m<32; m++ ) {                 /* random single/double byte edits + truncation */
        ulong i = sm64( &s ) % sz; uchar o = p[ i ];
        p[ i ] = (uchar)sm64( &s );
        both( p, sz, &line, NULL );
        both( p, sm64( &s ) % (sz + 1), &line, NULL );
        p[ i ] = o;
      }
    }
    printf( "fuzz seed=%s txns=%lu parses=%lu accepted=%lu mismatches=0\n", argv[2], cnt, g_cmp, g_ok );
    return 0;
  }
  if( argc < 3 ) { fprintf( stderr, "usage: %s out.bin fixture.bin... | fuzz seed count\n", argv[0] ); return 2; }
  FILE * out = fopen( argv[1], "wb" );
  char magic[16] = "FDTXNGOLDEN1";
  uint hdr[2] = { (uint)(argc - 2), 0 };
  fwrite( magic, 1, 16, out ); fwrite( hdr, 4, 2, out );
  for( int f=2; f<argc; f++ ) {
    FILE * in = fopen( argv[f], "rb" );
    if( !in ) { perror( argv[f] ); return 1; }
    static uchar buf[ 70000 ];
    ulong sz = fread( buf, 1, sizeof buf, in ); fclose( in );
    exhaustive( buf, sz );
    /* count + digest pass, then the stored pass */
    uint64_t dig = 0xcbf29ce484222325UL;
    ulong nmut = mutations( buf, sz, NULL, &dig );
    uint rec[2] = { (uint)sz, (uint)nmut };
    fwrite( rec, 4, 2, out ); fwrite( &dig, 8, 1, out ); fwrite( buf, 1, sz, out );
    mutations( buf, sz, out, NULL );
    ulong line; ulong fp = both( buf, sz, &line, NULL );
    printf( "%s: sz=%lu footprint=%lu mutations=%lu digest=%016lx\n", argv[f], sz, fp, nmut, (unsigned long)dig );
  }
  fclose( out );
  printf( "compared %lu parses (%lu accepted), 0 mismatches\n", g_cmp, g_ok );
  return 0;
}
