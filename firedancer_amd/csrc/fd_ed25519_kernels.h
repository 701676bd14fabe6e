/* firedancer_amd/csrc/fd_ed25519_kernels.h -- internal interface between
   the host engine (fd_ed25519_engine.cpp) and the HIP kernels. */
#ifndef FD_ED25519_KERNELS_H
#define FD_ED25519_KERNELS_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

typedef struct {
  size_t N;      /* n rounded up to 64 */
  size_t dig, top, A, R, Ai, st;   /* byte offsets of the workspace planes */
  size_t total;  /* footprint in bytes */
} ws_layout_t;

ws_layout_t fd_amd_ws_layout( size_t n );

/* Enqueue k_prep -> k_decomp -> k_dsm on `stream`; when ev != NULL record
   ev[0..3] before/between/after the three kernels.  0 on success. */
int fd_amd_launch_verify( uint32_t n, uint8_t const * d_pub, uint8_t const * d_sig, uint32_t const * d_off,
                          uint32_t const * d_sz, uint8_t const * d_blob, int8_t * d_err, void * d_ws,
                          hipStream_t stream, int want_stats, hipEvent_t const * ev /* 4 or NULL */ );

#endif
