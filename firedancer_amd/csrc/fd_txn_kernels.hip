/* firedancer_amd/csrc/fd_txn_kernels.hip
 *
 * GPU transaction front end of the verify engine: parse a
 * batch of wire-format Solana transactions, one transaction per lane, with
 * the exact accept/reject behaviour and descriptor bytes of the reference's
 * fd_txn_parse (src/ballet/txn/fd_txn_parse.c:6-217; compact-u16 rules of
 * fd_compact_u16.h:35-87), and lay every signature of every well-formed
 * transaction out for the verify kernels: signature i of transaction t is
 * checked with account address i over the message payload[message_off, sz)
 * (fd_txn.h:159-217).  The message bytes are NOT copied: every signature of
 * a transaction points at the same bytes of the payload blob in HBM.
 *
 *   k_txn_parse   parse + signature layout (one lane per transaction)
 *   k_txn_reduce  per-transaction verdict: parse failure, else the first
 *                 failing signature's code in signature order, else 0
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "fd_ed25519_kernels.h"

typedef uint8_t  u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef int8_t   i8;

#include "fd_txn_dev.h"

using namespace fd_txn_dev;

namespace {

/* n bytes from an unaligned source as little-endian dwords */
__device__ __forceinline__ void
copy_dw( u32 * dst, u8 const * src, u32 ndw ) {
  for( u32 k=0u; k<ndw; k++ )
    dst[k] = (u32)src[4u*k] | ((u32)src[4u*k+1u] << 8) | ((u32)src[4u*k+2u] << 16) | ((u32)src[4u*k+3u] << 24);
}

} /* namespace */

__global__ void __launch_bounds__(64)
k_txn_parse( u32 txn_cnt, u8 const * __restrict__ payload, u32 const * __restrict__ toff, u32 const * __restrict__ tsz,
             u32 * __restrict__ fp_out, u8 * __restrict__ out, size_t out_stride, u32 const * __restrict__ tbase,
             u8 * __restrict__ pub, u8 * __restrict__ sig, u32 * __restrict__ moff, u32 * __restrict__ msz,
             i8 * __restrict__ skip ) {
  u32 t = blockIdx.x * 64u + threadIdx.x;
  if( t >= txn_cnt ) return;
  u8 const * p = payload + toff[t];
  u32 sz = tsz[t];
  u32 nsig = 0u, sig_off = 0u, acct_off = 0u, msg_off = 0u;
  u32 fp = txn_parse( p, sz, out ? out + (size_t)t*out_stride : (u8 *)0, &nsig, &sig_off, &acct_off, &msg_off );
  if( fp_out ) fp_out[t] = fp;
  if( !tbase ) return;
  u32 b = tbase[t], e = tbase[t+1u];
  if( !fp ) {                                 /* reserved slots of a rejected payload */
    for( u32 s=b; s<e; s++ ) skip[s] = (i8)TXN_ERR_PARSE;
    return;
  }
  /* host reserved payload[0] slots; a parsed transaction has exactly that
     many.  A caller-supplied tbase that reserved a different count (device
     API) rejects the transaction instead of verifying a subset: fail closed */
  if( e - b != nsig ) {
    if( fp_out ) fp_out[t] = 0u;
    for( u32 s=b; s<e; s++ ) skip[s] = (i8)TXN_ERR_PARSE;
    return;
  }
  for( u32 i=0u; i<nsig; i++ ) {
    u32 s = b + i;
    copy_dw( (u32 *)(pub + 32UL*s), p + acct_off + 32u*i,  8u );
    copy_dw( (u32 *)(sig + 64UL*s), p + sig_off  + 64u*i, 16u );
    moff[s] = toff[t] + msg_off;
    msz[s]  = sz - msg_off;
    skip[s] = 0;
  }
}

__global__ void __launch_bounds__(64)
k_txn_reduce( u32 txn_cnt, u32 const * __restrict__ fp, u32 const * __restrict__ tbase,
              i8 const * __restrict__ err, i8 * __restrict__ terr ) {
  u32 t = blockIdx.x * 64u + threadIdx.x;
  if( t >= txn_cnt ) return;
  if( !fp[t] ) { terr[t] = (i8)TXN_ERR_PARSE; return; }
  i8 r = 0;
  for( u32 s=tbase[t]; s<tbase[t+1u]; s++ ) { i8 e = err[s]; if( e ) { r = e; break; } }
  terr[t] = r;
}

int
fd_amd_launch_txn_parse( uint32_t txn_cnt, uint8_t const * d_payload, uint32_t const * d_toff,
                         uint32_t const * d_tsz, uint32_t * d_fp, uint8_t * d_out, size_t out_stride,
                         uint32_t const * d_tbase, uint8_t * d_pub, uint8_t * d_sig, uint32_t * d_off,
                         uint32_t * d_sz, int8_t * d_skip, hipStream_t stream ) {
  if( !txn_cnt ) return 0;
  hipLaunchKernelGGL( k_txn_parse, dim3((txn_cnt + 63u)/64u), dim3(64), 0, stream, txn_cnt, d_payload, d_toff, d_tsz,
                      d_fp, d_out, out_stride, d_tbase, d_pub, d_sig, d_off, d_sz, d_skip );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int
fd_amd_launch_txn_reduce( uint32_t txn_cnt, uint32_t const * d_fp, uint32_t const * d_tbase,
                          int8_t const * d_err, int8_t * d_terr, hipStream_t stream ) {
  if( !txn_cnt ) return 0;
  hipLaunchKernelGGL( k_txn_reduce, dim3((txn_cnt + 63u)/64u), dim3(64), 0, stream, txn_cnt, d_fp, d_tbase, d_err, d_terr );
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
