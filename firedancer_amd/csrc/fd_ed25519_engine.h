/* firedancer_amd/csrc/fd_ed25519_engine.h -- internal: the batch engine's
   double-buffered slots, shared by the C-ABI (fd_ed25519_engine.cpp) and
   the streaming verify tile (fd_verify_tile.cpp). */
#ifndef FD_ED25519_ENGINE_H
#define FD_ED25519_ENGINE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/fd_ed25519_amd.h"

struct slot_t {
  /* device */
  uint8_t  * d_pub;  uint8_t * d_sig; uint8_t * d_blob;
  uint32_t * d_off;  uint32_t * d_sz; int8_t * d_err; void * d_ws;
  /* pinned host staging */
  uint8_t  * h_pub;  uint8_t * h_sig; uint8_t * h_blob;
  uint32_t * h_off;  uint32_t * h_sz; int8_t * h_err;
  hipStream_t stream;
  hipEvent_t  done;
  uint8_t  * d_pack; uint8_t * h_pack;   /* packed [pub|sig|off|sz|blob] for n: one H2D per chunk */
  uint8_t  * m_pack;                     /* device address of the mapped h_pack (latency path reads it in place) */
  void * m_err, * m_terr, * m_tag;   /* device addresses of the mapped h_err / h_terr / h_tag */
  uint64_t * h_tag;      /* dedup tags (pinned, allocated with the txn buffers) */
  int        want_tag;
  int        dsm_mode;   /* kernel path for the next launch (fd_amd_launch_verify dsm_mode) */
  /* the chunk in flight: where its verdicts go */
  schar *    out;
  ulong      n;
  int        busy;
  ulong      chk_err, chk_terr;   /* verdict bytes the launch writes to h_err / h_terr (checked for FD_AMD_VERDICT_DEVICE) */
  /* transaction front end (allocated on first use): per-transaction
     payload offset/size, footprint, signature-slot base, verdict; per-slot
     skip plane */
  uint32_t * d_toff; uint32_t * d_tsz; uint32_t * d_fp; uint32_t * d_tbase; int8_t * d_terr; int8_t * d_skip;
  uint32_t * h_toff; uint32_t * h_tsz; uint32_t * h_tbase; int8_t * h_terr;
  /* transaction chunk in flight */
  schar *    t_out;      /* per-transaction verdicts */
  ulong      t_n;
  schar *    s_out;      /* per-signature verdicts (optional) */
  ulong      s_n;
};

#define FD_AMD_SLOT_MAX (16)

struct fd_ed25519_amd {
  int    device;
  ulong  cap;        /* signatures per chunk */
  ulong  blob_cap;   /* message bytes per chunk */
  int    nslot;      /* 2 for the batch API (double buffering); the tile uses more */
  slot_t slot[FD_AMD_SLOT_MAX];
};

/* NUMA placement (fd_numa.cpp): bind the calling thread to the device's
   node (CPUs + preferred memory), or prefer it only while allocating. */
int  fd_amd_numa_bind_thread( int device );
int  fd_amd_numa_prefer_begin( int device, int * saved_mode, unsigned long * saved_mask /* 16 words */ );
void fd_amd_numa_prefer_end( int saved_mode, unsigned long const * saved_mask );

/* An engine with `nslot` in-flight slots (2..FD_AMD_SLOT_MAX). */
fd_ed25519_amd_t * fd_amd_engine_new( int device, ulong batch_max, ulong blob_max, int nslot );


/* n bytes of device results -> the mapped host buffer h_dst (one of the
   slot's h_err / h_terr / h_tag) by a kernel on the slot's stream. */
int  fd_amd_slot_out( slot_t * s, void * h_dst, void const * d_src, ulong n );
/* Chunk of n signatures staged in s->h_pack as [pub 32n | sig 64n | off 4n | sz 4n | blob]. */
int  fd_amd_slot_launch_packed( slot_t * s, ulong n, ulong blob_sz, schar * out );
/* 1 if the slot's chunk finished (or nothing is in flight), 0 if still
   running, negative on a HIP error.  Non-blocking. */
int  fd_amd_slot_ready( slot_t * s );
/* Block until the slot's chunk finished; deliver verdicts to `out`. */
int  fd_amd_slot_drain( slot_t * s );
int  fd_amd_slot_alloc_aux( slot_t * s, ulong cap );
/* Transaction chunk: c payloads staged in h_blob / h_toff / h_tsz with
   signature-slot bases h_tbase[0..c] (nslot = h_tbase[c]); per-transaction
   verdicts land in h_terr, slot tags in h_tag when want_tag. */
int  fd_amd_slot_launch_txn( slot_t * s, ulong c, ulong nslot, ulong blob_sz, schar * t_out, schar * s_out, int want_tag,
                             uint8_t const * d_payload );   /* d_payload != NULL: payloads read in place (h_toff index it), no blob H2D */
/* signature slots reserved for a payload (fd_txn_parse.c:79-82 rule) */
ulong fd_amd_txn_slots1( uchar const * p, ulong sz );

#endif
