// debug: dump SHA words / digest of k_prep's construction for one message
#include "../../firedancer_amd/csrc/fd_ed25519_kernels.hip"
#include <stdio.h>
__global__ void k_dbg( u8 const * sig, u8 const * pub, u8 const * blob, u32 sz, u64 * out ) {
  uint4 const * S4 = (uint4 const *)(sig);
  uint4 const * P4 = (uint4 const *)(pub);
  uint4 r0 = S4[0], r1 = S4[1], a0 = P4[0], a1 = P4[1];
  u64 const ra[8] = { ((u64)r0.y << 32) | r0.x, ((u64)r0.w << 32) | r0.z, ((u64)r1.y << 32) | r1.x, ((u64)r1.w << 32) | r1.z,
                      ((u64)a0.y << 32) | a0.x, ((u64)a0.w << 32) | a0.z, ((u64)a1.y << 32) | a1.x, ((u64)a1.w << 32) | a1.z };
  u64 bitlen = (u64)(64u + sz) << 3;
  u32 nblk = (64u + sz + 17u + 127u) / 128u;
  u64 st[8] = FD_AMD_SHA512_H0;
  for( u32 blk=0; blk<nblk; blk++ ) {
    u64 w[16];
    _Pragma("unroll") for( int k=0; k<16; k++ ) {
      u32 kk = blk*16u + (u32)k;
      u64 v;
      if( kk < 8u ) v = ra[k & 7];
      else          v = msg_word( blob, sz, 8u*(kk - 8u) );
      v = bswap64( v );
      if( blk == nblk-1u && k == 15 ) v |= bitlen;
      w[k] = v;
      if( blk == 0 ) out[k] = v;
    }
    sha512_compress( st, w );
  }
  for( int a=0; a<8; a++ ) out[16+a] = st[a];
}
int main() {
  u8 h_sig[64], h_pub[32], h_msg[64];
  for( int i=0; i<64; i++ ) { h_sig[i] = (u8)i; h_msg[i] = (u8)(0xa0 + i); }
  for( int i=0; i<32; i++ ) h_pub[i] = (u8)(0x40 + i);
  u8 *d_sig, *d_pub, *d_msg; u64 * d_out;
  hipMalloc( &d_sig, 64 ); hipMalloc( &d_pub, 32 ); hipMalloc( &d_msg, 64 ); hipMalloc( &d_out, 24*8 );
  hipMemcpy( d_sig, h_sig, 64, hipMemcpyHostToDevice ); hipMemcpy( d_pub, h_pub, 32, hipMemcpyHostToDevice );
  hipMemcpy( d_msg, h_msg, 64, hipMemcpyHostToDevice );
  hipLaunchKernelGGL( k_dbg, dim3(1), dim3(1), 0, 0, d_sig, d_pub, d_msg, 7u, d_out );
  u64 out[24]; hipMemcpy( out, d_out, 24*8, hipMemcpyDeviceToHost );
  for( int k=0; k<16; k++ ) printf( "w%02d %016lx\n", k, (unsigned long)out[k] );
  for( int a=0; a<8; a++ ) printf( "st%d %016lx\n", a, (unsigned long)out[16+a] );
  return 0;
}
