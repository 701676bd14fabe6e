/* oracle/check_vs_ref.c -- TEST INFRASTRUCTURE ONLY (build container).
 *
 * Pins the clean-room restatement (liboracle.so) against the compiled
 * reference (oracle/_ref/libfdref.so = the reference's own sources, default
 * AVX build) on a seeded stream of signatures:
 *
 *   check_vs_ref <seed> <count> <szlo> <szhi> [falsereject_out.txt]
 *
 * Every vector is a fresh keypair + message signed by the reference signer;
 * 10 % get one flipped bit in sig, msg or pub (SURVEY s8 d, config 3).
 * Prints the number of verdict/error-code disagreements (must be 0) and the
 * per-code histogram.  Valid (unflipped) signatures that the reference
 * rejects (the AVX limb-compare false rejects) are appended to
 * the optional output file as "pub sig msg" hex lines so gen_golden can pin
 * them as fixtures.
 */
#include "vecgen.h"

int
main( int argc, char ** argv ) {
  if( argc < 5 ) { fprintf( stderr, "usage: %s seed count szlo szhi [fr_out]\n", argv[0] ); return 2; }
  uint64_t rs   = strtoull( argv[1], NULL, 0 ) * 0x2545F4914F6CDD1DUL + 1;
  uint64_t cnt  = strtoull( argv[2], NULL, 0 );
  uint32_t szlo = (uint32_t)strtoul( argv[3], NULL, 0 );
  uint32_t szhi = (uint32_t)strtoul( argv[4], NULL, 0 );
  FILE * fr = argc > 5 ? fopen( argv[5], "a" ) : NULL;
  uint64_t mism = 0, hist[4] = {0,0,0,0}, fr_cnt = 0;
  vec_t v;
  for( uint64_t i=0; i<cnt; i++ ) {
    vg_mixed( &v, &rs, szlo, szhi );
    int e_ref = fd_ed25519_verify( v.msg, v.sz, v.sig, v.pub, vg_sha() );
    int e_orc = oracle_ed25519_verify( v.msg, v.sz, v.sig, v.pub );
    if( e_ref != e_orc ) {
      mism++;
      fprintf( stderr, "MISMATCH idx=%lu cls=%u ref=%d oracle=%d\n", (unsigned long)i, v.cls, e_ref, e_orc );
    }
    if( e_ref >= -3 && e_ref <= 0 ) hist[-e_ref]++;
    if( v.cls == CLS_VALID && e_ref != 0 ) {
      fr_cnt++;
      if( fr ) {
        for( int k=0; k<32; k++ ) fprintf( fr, "%02x", v.pub[k] );
        fputc( ' ', fr );
        for( int k=0; k<64; k++ ) fprintf( fr, "%02x", v.sig[k] );
        fputc( ' ', fr );
        for( uint32_t k=0; k<v.sz; k++ ) fprintf( fr, "%02x", v.msg[k] );
        fputc( '\n', fr ); fflush( fr );
      }
    }
    if( (i & 0xFFFFF) == 0xFFFFF ) {
      fprintf( stderr, "progress %lu/%lu mism=%lu fr=%lu\n", (unsigned long)(i+1), (unsigned long)cnt,
               (unsigned long)mism, (unsigned long)fr_cnt );
    }
  }
  printf( "seed=%s count=%lu mismatches=%lu codes[0,-1,-2,-3]=%lu,%lu,%lu,%lu valid_rejected=%lu\n",
          argv[1], (unsigned long)cnt, (unsigned long)mism,
          (unsigned long)hist[0], (unsigned long)hist[1], (unsigned long)hist[2], (unsigned long)hist[3],
          (unsigned long)fr_cnt );
  if( fr ) fclose( fr );
  return mism ? 1 : 0;
}
