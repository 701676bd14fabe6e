/* firedancer_amd/csrc/fd_ed25519_kernels.h -- internal interface between
   the host engine (fd_ed25519_engine.cpp) and the HIP kernels. */
#ifndef FD_ED25519_KERNELS_H
#define FD_ED25519_KERNELS_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

typedef struct {
  size_t N;      /* n rounded up to 64 */
  size_t dig, evn, top, A, R, Ai, st, tag, ds, init, ctr;   /* byte offsets of the workspace planes */
  size_t total;  /* footprint in bytes */
} ws_layout_t;

ws_layout_t fd_amd_ws_layout( size_t n );

/* Enqueue k_prep -> k_decomp -> k_dsm on `stream`; when ev != NULL record
   ev[0..3] before/between/after the three kernels.  d_skip (NULL = none):
   per-signature int8, nonzero = do not verify, the verdict is that value
   (transaction slots whose payload failed to parse).  0 on success. */
int fd_amd_launch_verify( uint32_t n, uint8_t const * d_pub, uint8_t const * d_sig, uint32_t const * d_off,
                          uint32_t const * d_sz, uint8_t const * d_blob, int8_t * d_err, void * d_ws,
                          hipStream_t stream, int want_stats, hipEvent_t const * ev /* 4 or NULL */,
                          int8_t const * d_skip = NULL, int dsm_mode = 0, int8_t * d_out = NULL );
/* d_out (NULL = none): on the latency path (fd_amd_uses_latency_path) the
   last kernel also writes every verdict to d_out, e.g. mapped host memory,
   so the caller needs no copy kernel; the throughput path ignores it. */
/* Verdict byte that marks every signature of a launch whose k_dsmp hang
   guard tripped (never a reference code): the host calls turn it into
   FD_ED25519_AMD_ERR_DEVICE. */
#define FD_AMD_VERDICT_DEVICE (-128)
/* dsm_mode: 0 = by batch size (fd_ed25519_amd_set_latency_batch_max,
   fd_ed25519_amd_set_small_batch_max), 1 = the throughput path (k_prep,
   k_decomp, k_dsm), 2 = k_front + k_dsm4, 3 = k_front + k_dsm8. */

/* Transaction front end (fd_txn_kernels.hip).
   k_txn_parse: one lane per transaction t = d_payload[d_toff[t] .. +d_tsz[t]).
     d_fp[t] = fd_txn_parse return value; d_out (optional) + t*out_stride gets
     the fd_txn_t descriptor.  When d_tbase != NULL it also lays out the
     transaction's signatures for the verify kernels at slots
     [d_tbase[t], d_tbase[t+1]): pub/sig copied from the payload, msg_off/msg_sz
     pointing at the shared message inside d_payload, skip = 0; a payload that
     fails to parse marks its slots skip = FD_TXN_AMD_ERR_PARSE.
   k_txn_reduce: d_terr[t] = parse failure code, or the first nonzero
     verdict among the transaction's slots, or 0. */
int fd_amd_launch_txn_parse( uint32_t txn_cnt, uint8_t const * d_payload, uint32_t const * d_toff,
                             uint32_t const * d_tsz, uint32_t * d_fp, uint8_t * d_out, size_t out_stride,
                             uint32_t const * d_tbase, uint8_t * d_pub, uint8_t * d_sig, uint32_t * d_off,
                             uint32_t * d_sz, int8_t * d_skip, hipStream_t stream );
int fd_amd_launch_txn_reduce( uint32_t txn_cnt, uint32_t const * d_fp, uint32_t const * d_tbase,
                              int8_t const * d_err, int8_t * d_terr, hipStream_t stream );

/* GPU keygen + sign (fd_ed25519_sign.hip): prv[n][32] seeds, messages
   blob[off[i] .. +sz[i]) -> pub[n][32], sig[n][64].  0 on success. */
int fd_amd_launch_sign( uint32_t n, uint8_t const * d_prv, uint32_t const * d_off, uint32_t const * d_sz,
                        uint8_t const * d_blob, uint8_t * d_pub, uint8_t * d_sig, hipStream_t stream );

/* Streaming tile, persistent consumer (k_tile_persist).  One launch per
   tile run; its waves take chunk descriptors the tile's host thread
   publishes in mapped host memory and verify them, so the GPU never drains
   between hand-offs and the tile needs one stream (one hardware queue).

   ring entry (host -> GPU): the frag's chunk in the source region, its
   output frame's chunk (zero-copy: the GPU writes the verified bytes
   there), its size, and (TXN framing) its signature slots
   (fd_amd_txn_slots1).  Entry of ring index j at ent[j & mask]. */
typedef struct { uint32_t src_chunk, out_chunk, sz, slots; } fd_amd_tile_ent_t;
/* chunk descriptor (host -> GPU): ring entries [first, first + count),
   count <= 64 | FD_AMD_TILE_LAT (8 lanes per signature) or FD_AMD_TILE_QUAD
   (4 lanes per signature); the entries' signature slots total <= 64 (<= 8
   in a latency chunk, <= 16 in a quad chunk) */
typedef struct { uint64_t first; uint32_t count; uint32_t pad; } fd_amd_tile_desc_t;   /* pad: pair sub | seq << 1 */
#define FD_AMD_TILE_LAT  (0x80000000u)
#define FD_AMD_TILE_QUAD (0x40000000u)
/* a quad PAIR (PUB_SIG_MSG): two descriptors over the same 17..32 entries,
   pad = sub | pair_seq << 1.  Sub 0 hashes and decompresses all of them
   into pair workspace pair_seq & pair_mask, raises its flag, and verifies
   entries 0..15; sub 1 waits for the flag and verifies entries 16.. -- one
   front pass (all lanes busy) serves two quad chunks */
#define FD_AMD_TILE_PAIR (0x20000000u)
#define FD_AMD_TILE_COUNT(c) ((c) & 0x1fffffffu)
/* result of ring index j (GPU -> host), two arrays of R words: tag[j & mask]
   and word[j & mask] = (j + 1) << 8 | (uint8_t)verdict, the word stored
   after the tag and after the frag's output bytes (system-scope release),
   so a host that sees word's index also sees the rest.  Arrays, not
   {tag, word} records: a chunk's 64 lanes then store 512 contiguous bytes
   per instruction (whole lines) -- interleaved 8-B stores into mapped host
   memory held the L2 so long that every wave of the GPU slowed ~5x
   (tools/tile_synth.py, profiles/r03_tile_persist_ab.txt). */
/* control words in mapped host memory, each on its own 64-B line: the
   first three are written by the host, the last by the GPU's scout */
typedef struct {
  uint64_t head;  uint64_t pad0[7];   /* chunk descriptors [.., head) are published to the GPU */
  uint64_t beat;  uint64_t pad1[7];   /* host heartbeat: the kernel's watchdog */
  uint32_t stop;  uint32_t kerr;  uint64_t pad2[7];   /* stop: exit once drained; kerr: set by the kernel on a watchdog exit */
  uint64_t gclock;                    /* scout: its s_memrealtime (100 MHz), every ~10 us; nonzero = the kernel started */
  uint64_t gdone;                     /* scout: chunks the waves finished (mirror of dctl->done) */
  uint64_t pad3[6];
} fd_amd_tile_hctl_t;
/* device control block (zeroed by the host before each launch) */
#define FD_AMD_TILE_MIRRORS (8)
typedef struct { uint64_t w; uint64_t pad[7]; } fd_amd_tile_mirror_t;
typedef struct {
  uint64_t             ticket;  uint64_t pad0[7];   /* next chunk ticket (one atomic add per chunk) */
  fd_amd_tile_mirror_t mw[FD_AMD_TILE_MIRRORS];     /* per XCD: descriptor head | heartbeat << 48 | err << 62 | stop << 63 */
  uint64_t             done;    uint64_t pad1[7];   /* chunks finished (one atomic add per chunk; the scout mirrors it) */
  uint64_t             stat[6];                     /* chunks in latency mode, in throughput mode; frags in each; quad chunks, their frags */
  uint64_t             prof[8];                     /* diagnostics build (FD_AMD_DIAG, args.prof): summed ticks gather, decomp, DSM, results, wait, fence, prep */
} fd_amd_tile_dctl_t;
typedef struct {
  fd_amd_tile_hctl_t *       hctl;     /* device address of the mapped control words */
  fd_amd_tile_ent_t const *  ent;      /* device address of the mapped ring */
  fd_amd_tile_desc_t const * desc;     /* device address of the mapped chunk descriptors (same size as the ring) */
  uint64_t *                 res_tag;  /* device address of the mapped results: tags */
  uint64_t *                 res_word; /*   and verdict words */
  uint64_t *                 res_time; /*   and (NULL = none) per frag: claim | done << 32, low 32 bits of the
                                            s_memrealtime ticks when its wave took the chunk and stored its results */
  uint64_t                   mask;     /* ring size - 1 (power of 2) */
  uint8_t const *            src;      /* frag source region (mapped): input dcache (zero-copy) or the output frames */
  uint8_t *                  out;      /* output frames (mapped) to fill, or NULL (copy mode: the host filled them) */
  fd_amd_tile_dctl_t *       dctl;
  uint8_t *                  scratch;  /* per-wave scratch, fd_amd_tile_scratch_stride() bytes apart */
  uint64_t                   watchdog; /* s_memrealtime ticks (100 MHz) without a host heartbeat before the kernel gives up */
  uint32_t                   prof;     /* diagnostics build only: sum per-phase time stamps into dctl->prof */
  uint32_t                   txn;      /* TXN framing: entries are wire transactions, results per transaction */
  uint8_t *                  pair_ws;  /* quad pairs: pair_mask + 1 workspaces, fd_amd_tile_scratch_stride() apart */
  uint32_t *                 pair_flag;/*   and their flags (pair_seq + 1 once a pair's front is done) */
  uint32_t                   pair_mask;
  uint32_t                   pad_;
} fd_amd_tile_args_t;
size_t fd_amd_tile_scratch_stride( void );
/* waves: grid size (wave 0 is the scout that mirrors the host words) */
int fd_amd_launch_tile_persist( fd_amd_tile_args_t const * a, uint32_t waves, hipStream_t stream );   /* 0, -1 (waves), or a hipError_t */

#ifdef FD_AMD_DIAG
/* diagnostics build: the chunk pipeline alone, every argument in device memory */
int fd_amd_launch_tile_synth( fd_amd_tile_args_t const * a, uint32_t waves, uint32_t iters, int eight, hipStream_t stream );
#endif

/* Dense slide digits of the last call on workspace d_ws (debug): u16
   [n][256] (low byte h digit, high byte s digit) rebuilt from the event
   lists k_prep writes. */
int fd_amd_launch_digits_dense( uint32_t n, void const * d_ws, uint16_t * d_dig, hipStream_t stream );

/* 1 when a batch of n takes the latency kernels (k_front + k_dsm8/k_dsm4). */
int fd_amd_uses_latency_path( uint32_t n, int dsm_mode );
/* dsm_mode for one of several concurrent batches (the streaming tile, up to
   4 in flight): k_dsm8 while four of its largest batches fit one wave per
   SIMD (cap at most a quarter of fd_ed25519_amd_set_latency_batch_max), k_dsm4 up to
   fd_ed25519_amd_set_small_batch_max, else k_dsm.  cap: the largest batch
   the caller will have in flight. */
int fd_amd_batch_dsm_mode( uint32_t n, uint32_t cap );

/* d_off[i] -= lo for every nonempty message (0 for empty ones). */
int fd_amd_launch_rebase_off( uint32_t n, uint32_t * d_off, uint32_t const * d_sz, uint32_t lo, hipStream_t stream );

/* n bytes device -> mapped host memory by a kernel (no DMA engine). */
int fd_amd_launch_copy_out( void * d_dst_mapped, void const * d_src, size_t n, hipStream_t stream );

#endif
