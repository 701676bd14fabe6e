/* oracle/gen_golden.c -- TEST INFRASTRUCTURE ONLY (build container).
 *
 * Writes the committed golden fixtures of tests/golden/ from the COMPILED
 * REFERENCE (oracle/_ref/libfdref.so, built from the reference's own sources
 * by oracle/Makefile).  Expected codes are the reference's
 * fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:345-431) on the
 * exact bytes stored; the clean-room oracle is run on every vector too and
 * generation aborts on any disagreement.
 *
 *   gen_golden vectors <out.bin> <mainnet_dir> [falsereject.txt ...]
 *   gen_golden stream  <seed> <count> <szlo> <szhi> <mixed:0|1>
 *
 * vectors: binary file, little endian
 *   magic[16] "FDED25519GOLD1\0\0", u32 count, u32 reserved,
 *   count x { pub[32], sig[64], u32 sz, i8 expect, u8 cls, u16 0, msg[sz] }
 * stream:  prints one JSON line with the verdict histogram and the FNV-1a
 *   64 digest of the int8 code array of a seeded stream (vecgen.h vg_valid /
 *   vg_mixed), so the GPU box can regenerate the same stream with the
 *   product signer and check codes at scale without the reference.
 */
#include "vecgen.h"
#include <dirent.h>

static FILE * g_out; static uint32_t g_cnt; static uint64_t g_bad;

static void
emit( vec_t const * v ) {
  int e_ref = fd_ed25519_verify( v->msg, v->sz, v->sig, v->pub, vg_sha() );
  int e_orc = oracle_ed25519_verify( v->msg, v->sz, v->sig, v->pub );
  if( e_ref != e_orc ) { fprintf( stderr, "ORACLE MISMATCH cls=%u ref=%d oracle=%d\n", v->cls, e_ref, e_orc ); g_bad++; }
  int8_t  e  = (int8_t)e_ref;
  uint8_t hdr[8];
  memcpy( hdr, &v->sz, 4 ); hdr[4] = (uint8_t)e; hdr[5] = v->cls; hdr[6] = 0; hdr[7] = 0;
  fwrite( v->pub, 1, 32, g_out ); fwrite( v->sig, 1, 64, g_out ); fwrite( hdr, 1, 8, g_out );
  fwrite( v->msg, 1, v->sz, g_out );
  g_cnt++;
}

static int ref_code( vec_t const * v ) { return fd_ed25519_verify( v->msg, v->sz, v->sig, v->pub, vg_sha() ); }

/* minimal Solana txn walk (src/ballet/txn/fd_txn.h:154-217): compact-u16 sig
   count, sigs, then the message; v0 messages start with 0x80|version.
   Signature i verifies account address i over payload[message_off:]. */
static uint32_t cu16( uint8_t const * p, uint32_t * off ) {
  uint32_t v = 0, sh = 0;
  for( ;; ) { uint8_t b = p[(*off)++]; v |= (uint32_t)(b & 0x7f) << sh; if( !(b & 0x80) ) break; sh += 7; }
  return v;
}

static void
mainnet( char const * dir ) {
  char const * names[3] = { "transaction1.bin", "transaction2.bin", "transaction3.bin" };
  for( int t=0; t<3; t++ ) {
    char path[4096]; snprintf( path, sizeof(path), "%s/%s", dir, names[t] );
    FILE * f = fopen( path, "rb" ); if( !f ) { fprintf( stderr, "skip %s\n", path ); continue; }
    uint8_t buf[2048]; uint32_t n = (uint32_t)fread( buf, 1, sizeof(buf), f ); fclose( f );
    uint32_t off = 0; uint32_t nsig = cu16( buf, &off );
    uint32_t sig_off = off; uint32_t msg_off = sig_off + 64*nsig;
    uint32_t o = msg_off;
    if( buf[o] & 0x80 ) o++;            /* v0 prefix */
    o += 3;                              /* message header */
    uint32_t nacct = cu16( buf, &o );
    if( nacct < nsig ) { fprintf( stderr, "bad txn %s\n", path ); continue; }
    for( uint32_t i=0; i<nsig; i++ ) {
      vec_t v; memset( &v, 0, sizeof(v) );
      memcpy( v.sig, buf + sig_off + 64*i, 64 );
      memcpy( v.pub, buf + o + 32*i, 32 );
      v.sz = n - msg_off; memcpy( v.msg, buf + msg_off, v.sz );
      v.cls = CLS_MAINNET;
      emit( &v );
    }
  }
}

static void
vectors( char const * out, char const * mainnet_dir, int nfr, char ** frfiles ) {
  g_out = fopen( out, "wb" );
  uint8_t hdr[24] = "FDED25519GOLD1";
  fwrite( hdr, 1, 24, g_out );                 /* count patched at the end */
  uint64_t rs = 0x5eed0001UL;
  vec_t v;

  /* mixed stream, msg sizes 0..300 */
  for( int i=0; i<768; i++ ) { vg_mixed( &v, &rs, 0, 300 ); emit( &v ); }
  /* zero-length and MTU-length messages */
  for( int i=0; i<16; i++ ) { vg_valid( &v, &rs, 0, 0 ); v.cls = CLS_ZERO_MSG; emit( &v ); }
  for( int i=0; i<8;  i++ ) { vg_valid( &v, &rs, 1232, 1232 ); v.cls = CLS_MAX_MSG; emit( &v ); }
  for( int i=0; i<8;  i++ ) { vg_valid( &v, &rs, 1232, 1232 ); v.msg[i*100] ^= 1; v.cls = CLS_MAX_MSG; emit( &v ); }
  /* every SHA-512 block-boundary length around the 128-B block (64 + sz + 17 padding) */
  for( uint32_t sz=40; sz<=200; sz++ ) { vg_valid( &v, &rs, sz, sz ); emit( &v ); }

  /* RFC 8032 s7.1 TEST 1..3 (secret, message) -- signed by the reference */
  {
    char const * sec[3] = { "9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
                            "4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
                            "c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7" };
    char const * msg[3] = { "", "72", "af82" };
    for( int k=0; k<3; k++ ) {
      uint8_t prv[32]; vg_hex( prv, sec[k] );
      v.sz = (uint32_t)vg_hex( v.msg, msg[k] );
      vg_sign( &v, prv ); v.cls = CLS_RFC8032; emit( &v );
    }
  }

  /* s-range classes on top of valid signatures */
  for( int i=0; i<32; i++ ) {
    vg_valid( &v, &rs, 0, 200 );
    v.sig[63] = 0x10; v.sig[32 + 16 + (i % 15)] = (uint8_t)(1 + (sm64( &rs ) % 255));   /* window -> 0 */
    v.cls = CLS_S_WINDOW; emit( &v );
  }
  for( int i=0; i<32; i++ ) {
    vg_valid( &v, &rs, 0, 200 );
    switch( i % 4 ) {
    case 0: v.sig[63] = (uint8_t)(0x11 + (sm64( &rs ) % 0xEF)); break;            /* top byte > 0x10 */
    case 1: memcpy( v.sig + 32, VG_L, 32 ); break;                                /* s == L */
    case 2: memcpy( v.sig + 32, VG_L, 32 ); v.sig[32] = (uint8_t)(VG_L[0] - 1); break;  /* s == L-1 */
    case 3: memcpy( v.sig + 32, VG_L, 32 ); v.sig[32 + (i/4)%16] += 1; break;       /* L < s < 2^252+2^128 */
    }
    v.cls = CLS_S_RANGE; emit( &v );
  }
  /* malleation s' = s + L */
  for( int i=0; i<96; i++ ) { vg_valid( &v, &rs, 0, 200 ); vg_add256( v.sig + 32, VG_L ); v.cls = CLS_MALLEATE; emit( &v ); }

  /* off-curve A and R: y = 2,3,... encodings that fail decompression */
  {
    int na = 0, nr = 0;
    for( uint32_t y=2; y<400 && (na<16 || nr<16); y++ ) {
      vg_valid( &v, &rs, 0, 64 );
      vec_t w = v; memset( w.pub, 0, 32 ); w.pub[0] = (uint8_t)y; w.pub[1] = (uint8_t)(y>>8);
      if( (y & 1) ) w.pub[31] |= 0x80;
      if( ref_code( &w ) == -2 && na < 16 ) { w.cls = CLS_OFFCURVE_A; emit( &w ); na++; }
      vec_t x = v; memset( x.sig, 0, 32 ); x.sig[0] = (uint8_t)y; x.sig[1] = (uint8_t)(y>>8);
      if( ref_code( &x ) == -2 && nr < 16 ) { x.cls = CLS_OFFCURVE_R; emit( &x ); nr++; }
    }
  }

  /* small-order A and R (the 8 torsion points), s = 0, 4-byte messages */
  for( int a=0; a<8; a++ ) for( int r=0; r<8; r++ ) for( int m=0; m<4; m++ ) {
    memset( &v, 0, sizeof(v) );
    vg_hex( v.pub, VG_TORSION[a] ); vg_hex( v.sig, VG_TORSION[r] );
    v.sz = 4; sm_bytes( &rs, v.msg, 4 );
    v.cls = CLS_SMALL_ORDER; emit( &v );
  }
  /* small-order A, R = identity, s = 0: the message-dependent acceptance of App. D */
  for( int a=0; a<8; a++ ) for( int m=0; m<24; m++ ) {
    memset( &v, 0, sizeof(v) );
    vg_hex( v.pub, VG_TORSION[a] ); vg_hex( v.sig, VG_TORSION[0] );
    v.sz = 4; v.msg[0] = (uint8_t)m; v.msg[1] = (uint8_t)a;
    v.cls = CLS_SMALL_ORDER; emit( &v );
  }
  /* non-canonical encodings for A and R (with s = 0, and with a real s) */
  for( int a=0; a<6; a++ ) for( int r=0; r<6; r++ ) {
    memset( &v, 0, sizeof(v) );
    vg_hex( v.pub, VG_NONCANON[a] ); vg_hex( v.sig, VG_NONCANON[r] );
    v.sz = 8; sm_bytes( &rs, v.msg, 8 );
    v.cls = CLS_NONCANON; emit( &v );
    vg_valid( &v, &rs, 0, 64 ); vg_hex( v.sig, VG_NONCANON[r] ); v.cls = CLS_NONCANON; emit( &v );
    vg_valid( &v, &rs, 0, 64 ); vg_hex( v.pub, VG_NONCANON[a] ); v.cls = CLS_NONCANON; emit( &v );
  }
  /* the identity A=O, R=O, s=0 also with A/R "-0" (table V) */
  for( int i=0; i<3; i++ ) for( int m=0; m<4; m++ ) {
    memset( &v, 0, sizeof(v) );
    vg_hex( v.pub, i==1 ? VG_NONCANON[2] : VG_TORSION[0] );
    vg_hex( v.sig, i==2 ? VG_NONCANON[2] : VG_TORSION[0] );
    v.sz = (uint32_t)m; v.cls = CLS_NONCANON; emit( &v );
  }

  /* uniformly random bytes */
  for( int i=0; i<128; i++ ) {
    memset( &v, 0, sizeof(v) );
    sm_bytes( &rs, v.pub, 32 ); sm_bytes( &rs, v.sig, 64 ); v.sig[63] &= 0x0f;   /* pass the s check mostly */
    v.sz = (uint32_t)(sm64( &rs ) % 64); sm_bytes( &rs, v.msg, v.sz );
    v.cls = CLS_RANDOM; emit( &v );
  }
  for( int i=0; i<32; i++ ) {
    vg_valid( &v, &rs, 0, 64 ); sm_bytes( &rs, v.sig, 32 );                       /* random R, real s */
    v.cls = CLS_RANDOM; emit( &v );
  }

  /* AVX limb-compare false rejects: SURVEY App. B (4 cases, 128-B msgs) + sweep finds */
  {
    static char const * const APPB[4][3] = {
      { "28451dedf9cb5f473320afe09e3215c0c392a754413b98aa57be06bef40545be",
        "9e4c899c5e1a7d43edba66e0f27c59536d6f10242d34b7f9009ecea002fc1f806efda8e7c36655b9039943d12d2e167e26446be9826abe65d8090a64e7b5eb0f",
        "b68313cb88bbd4be9a990767bef03e822ac01ef57f829ba5cd8308f4298afb36caa6a58049f42e59eab02eeedad6567dc4886ab416e801b4c5418a36ac5201e7700353cdf7a449842957204070c1d9f0d0f16afa9eb1c58e8f3707b1a4fd2df0afcd677423dc136f4b7914cabb255f65b4489c15df9292cda02b743f3ae7b820" },
      { "a6120c3bd695893f6f6eac45aa657a89653131a7561cf830d8ad20bda3e39a91",
        "bc3ce0c8481bbe82e769c2777dd1fb7f45a55d76470c531b3ae52c89468315d9cc4732422414cea938b2b4765097a70d9c2962a5dbb7b3be5ed210549ae31606",
        "56129fc9f26a32c1f5743d366a612f672ecb620ea3eaf255654579475d83a94487d62f4bfb9c80b9e3385b195083a0d78074cb8a3a4f29effc8079982b2b56d01aa0894419448b875660528b0c32d8818a6a80346cfe58e6c589e4ae0444823e076cc4d353236f0633e48b9122fee1682ef6f6e7fe4a2fdc454bf9021a3d2f48" },
      { "0508686b2c7423a02e929010cc60545c13b4f2c3e6924cccbd401a4527582766",
        "a9df1658493fb8e5ca2be3099da30d9ffef6b7b035fccf16c0d1c7023997b7892655c8de038a2bb52a2045f2df642eaa93631d8974357f2d6d1ef0c1dd611b06",
        "9af0acba7cf8d3aa26368c602f127facb6604d50bf0d5273e2924374b5e30fafeebd570047ecf0d370971a4b3f2e789f8553bb685f4ab88f4b3c45f9002d801cb07317b4c4d99b668faca62355b8422e2f3a317cad21fc22cb425a2a2a8e4d0a6cd2995a3577986fd7b33eb363d93b6fe2f505a9b980761eb5288b44ea38961e" },
      { "01319283a49eb79e596f9c5ecd4693a295ef7030be0ab1d8dee14a2007401a7b",
        "82c5c9f0f9bfa6d5a1c328ad9f9accf6d1b385e99ffc026fd515eef07f5ba3d4f324866d3070a2f29dae883124e66fe7aaf492a2f4c13a56e867f8ccba82c30c",
        "50f610c9b5ed71cdbe28ea80999e56aa2567d798295a801dbfff705a6cfa84d07fc9205b48279fe33bdf070a983db9fa5896c1520b3574b2f1f0fe7543876d0f9d86ec59070b918c29abe3e12ebe15e57e60641c6554156970ab5ee32593636e3973bab89e68cec49321af853ff00ed2e46b025b452aba97dc8b07fda0afc01f" } };
    for( int k=0; k<4; k++ ) {
      memset( &v, 0, sizeof(v) );
      vg_hex( v.pub, APPB[k][0] ); vg_hex( v.sig, APPB[k][1] ); v.sz = (uint32_t)vg_hex( v.msg, APPB[k][2] );
      v.cls = CLS_FALSE_REJECT; emit( &v );
    }
    for( int f=0; f<nfr; f++ ) {
      FILE * fp = fopen( frfiles[f], "r" ); if( !fp ) continue;
      static char line[8192];
      while( fgets( line, sizeof(line), fp ) ) {
        char p[128], s[256], m[4096];
        if( sscanf( line, "%127s %255s %4095s", p, s, m ) < 2 ) continue;
        memset( &v, 0, sizeof(v) );
        vg_hex( v.pub, p ); vg_hex( v.sig, s );
        v.sz = (strlen( line ) > 2*32+2*64+2 && sscanf( line, "%127s %255s %4095s", p, s, m )==3) ? (uint32_t)vg_hex( v.msg, m ) : 0;
        v.cls = CLS_FALSE_REJECT; emit( &v );
      }
      fclose( fp );
    }
  }

  if( mainnet_dir ) mainnet( mainnet_dir );

  fseek( g_out, 16, SEEK_SET ); fwrite( &g_cnt, 4, 1, g_out ); fclose( g_out );
  fprintf( stderr, "wrote %u vectors to %s (oracle mismatches: %lu)\n", g_cnt, out, (unsigned long)g_bad );
}

static void
stream( uint64_t seed, uint64_t cnt, uint32_t szlo, uint32_t szhi, int mixed ) {
  uint64_t rs = seed;
  uint64_t hist[4] = {0,0,0,0}, h = 0xcbf29ce484222325UL, bad = 0;
  vec_t v;
  for( uint64_t i=0; i<cnt; i++ ) {
    if( mixed ) vg_mixed( &v, &rs, szlo, szhi ); else vg_valid( &v, &rs, szlo, szhi );
    int e = ref_code( &v );
    if( e != oracle_ed25519_verify( v.msg, v.sz, v.sig, v.pub ) ) bad++;
    hist[-e]++;
    h = (h ^ (uint8_t)(int8_t)e) * 0x100000001b3UL;
  }
  printf( "{\"seed\": %lu, \"count\": %lu, \"szlo\": %u, \"szhi\": %u, \"mixed\": %d, "
          "\"codes\": [%lu, %lu, %lu, %lu], \"fnv1a64\": \"%016lx\", \"oracle_mismatch\": %lu}\n",
          (unsigned long)seed, (unsigned long)cnt, szlo, szhi, mixed,
          (unsigned long)hist[0], (unsigned long)hist[1], (unsigned long)hist[2], (unsigned long)hist[3],
          (unsigned long)h, (unsigned long)bad );
}

int
main( int argc, char ** argv ) {
  if( argc >= 4 && !strcmp( argv[1], "vectors" ) ) {
    vectors( argv[2], argc > 3 ? argv[3] : NULL, argc - 4, argv + 4 );
    return g_bad ? 1 : 0;
  }
  if( argc == 7 && !strcmp( argv[1], "stream" ) ) {
    stream( strtoull( argv[2], NULL, 0 ), strtoull( argv[3], NULL, 0 ),
            (uint32_t)strtoul( argv[4], NULL, 0 ), (uint32_t)strtoul( argv[5], NULL, 0 ), atoi( argv[6] ) );
    return 0;
  }
  fprintf( stderr, "usage: gen_golden vectors <out.bin> <mainnet_dir> [fr.txt...] | stream seed count szlo szhi mixed\n" );
  return 2;
}
