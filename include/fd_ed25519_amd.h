#ifndef HEADER_fd_ed25519_amd_h
#define HEADER_fd_ed25519_amd_h

/* MI355X ed25519 batch-verification engine -- the C-ABI drop-in boundary.
 *
 * Library: firedancer_amd/libfd_ed25519_amd.so (hipcc, gfx950).
 *
 * Part 1 reproduces the reference's public API for the verify path
 * (lijunwangs/firedancer src/ballet/ed25519/fd_ed25519.h), same names,
 * same argument meaning, same return codes, so an existing caller (the
 * verify tile, the Rust re-export ffi/rust/firedancer-sys/src/ballet/
 * ed25519.rs:1-10) relinks against this library unchanged.  Verdicts are
 * bit-exact with the reference's DEFAULT x86_64 (AVX) build, including its
 * documented non-strict behaviours.
 *
 * Part 2 is new: batch entry points (the reference only verifies one
 * signature per call).  Every verdict they return equals what Part 1's
 * fd_ed25519_verify returns for the same inputs.
 *
 * All verify work runs on the GPU.  There is no CPU fallback: without a
 * usable HIP device every verify entry point returns FD_ED25519_AMD_ERR_DEVICE
 * (batch API) or aborts with a message (drop-in API, which has no error code
 * for "no device").
 */

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned char uchar;
typedef unsigned long ulong;
typedef unsigned int  uint;
typedef signed char   schar;

/* ===== Part 1: reference API (src/ballet/ed25519/fd_ed25519.h) ===== */

/* fd_ed25519.h:11-14 */
#define FD_ED25519_SUCCESS    ( 0) /* Operation was succesful */
#define FD_ED25519_ERR_SIG    (-1) /* signature obviously invalid (s check) */
#define FD_ED25519_ERR_PUBKEY (-2) /* public key (or R) failed to decompress */
#define FD_ED25519_ERR_MSG    (-3) /* message didn't match the signature */

/* fd_ed25519.h:17-20 */
#define FD_ED25519_SIG_SZ (64UL)
typedef uchar fd_ed25519_sig_t[ FD_ED25519_SIG_SZ ];

/* The reference passes a caller-owned SHA-512 calculator as scratch
   (fd_ed25519.h:81-95; src/ballet/sha512/fd_sha512.h:15-16,56-77: 256 B,
   128-aligned).  This library hashes on the GPU and only takes the
   reference's write interest in it; it never dereferences it.  A caller
   that already includes the reference's fd_sha512.h keeps its definition. */
#ifndef FD_SHA512_ALIGN
#define FD_SHA512_ALIGN     (128UL)
#define FD_SHA512_FOOTPRINT (256UL)
typedef struct fd_sha512_private fd_sha512_t;
#endif

/* fd_ed25519_verify -- replaces fd_ed25519.h:96-101 (impl
   fd_ed25519_user.c:345-431).  Returns FD_ED25519_SUCCESS or an
   FD_ED25519_ERR_* code, bit-exact with the reference.  Reentrant; runs as
   a batch of one on the calling thread's own engine, on the thread's
   device (fd_ed25519_amd_dropin_set_device below).  msg==NULL fine when
   sz==0. */
int
fd_ed25519_verify( void const *  msg,
                   ulong         sz,
                   void const *  sig,
                   void const *  public_key,
                   fd_sha512_t * sha );

/* Device routing of the drop-in call.  The reference runs N verify tiles
   as threads of one process (src/app/frank/fd_frank_main.c:118-143), each
   calling fd_ed25519_verify (fd_frank_verify_synth_load.c:380), so the
   device is chosen per calling thread:
   - fd_ed25519_amd_dropin_set_device( d ) (d >= 0) from the thread (e.g. at
     its tile's boot) pins the thread's calls to HIP device d; its next call
     moves its engine there.  FD_ED25519_AMD_DROPIN_AUTO returns the thread
     to the default.  0, ERR_INVAL (d < -1 or not a device) or ERR_DEVICE
     (no HIP).
   - default (picked once, at the thread's first call):
     FD_ED25519_AMD_DEVICE when set; else round robin over the GPUs on the
     NUMA node of the CPU the thread runs on (a tile pinned to a core gets a
     GPU of its own socket), over all GPUs when none is local: the rule of
     fd_ed25519_amd_dropin_pick, with ordinal = the threads of that node that
     took a default before it.
   fd_ed25519_amd_dropin_device: the device of the calling thread's engine
   (-1 before its first call).  fd_ed25519_amd_dropin_pick (pure): of
   dev_cnt devices on NUMA nodes dev_node[] (-1 unknown), the device for
   the ordinal-th thread on node cpu_node (-1 unknown). */
#define FD_ED25519_AMD_DROPIN_AUTO    (-1)
#define FD_ED25519_AMD_DROPIN_DEV_MAX (64)
int
fd_ed25519_amd_dropin_set_device( int device );

int
fd_ed25519_amd_dropin_device( void );

int
fd_ed25519_amd_dropin_pick( int const * dev_node, int dev_cnt, int cpu_node, ulong ordinal );

/* fd_ed25519_strerror -- replaces fd_ed25519.h:108-109 (impl
   fd_ed25519_user.c:433-443): same strings. */
char const *
fd_ed25519_strerror( int err );

/* fd_ed25519_public_from_private / fd_ed25519_sign -- replace
   fd_ed25519.h:40-78 (impl fd_ed25519_user.c:279-343).  Host-side (not
   the verify hot path); deterministic RFC 8032 signing, so the bytes equal
   the reference's. */
void *
fd_ed25519_public_from_private( void *        public_key,
                                void const *  private_key,
                                fd_sha512_t * sha );

void *
fd_ed25519_sign( void *        sig,
                 void const *  msg,
                 ulong         sz,
                 void const *  public_key,
                 void const *  private_key,
                 fd_sha512_t * sha );

/* ===== Part 2: batch engine (new) ===== */

#define FD_ED25519_AMD_OK          ( 0)
#define FD_ED25519_AMD_ERR_INVAL   (-10) /* bad argument (NULL, n too large, a message larger than the engine's blob_max) */
#define FD_ED25519_AMD_ERR_DEVICE  (-11) /* HIP error / no device */

/* Solana MTU: the message size the staging is dimensioned
   for.  Longer messages verify too, as long as each fits the engine's
   blob_max (the drop-in fd_ed25519_verify grows its engine as needed). */
#define FD_ED25519_AMD_MSG_MAX     (1232UL)

typedef struct fd_ed25519_amd fd_ed25519_amd_t;

/* Create an engine bound to HIP device `device`, able to verify up to
   batch_max signatures whose messages total at most blob_max bytes per
   call (larger calls are split internally).  Owns its HIP stream, device
   buffers and pinned, double-buffered host staging.  NULL on failure.
   One engine per host thread; engines on different devices run
   independently (multi-GPU = one engine per device).  Chunks in flight:
   2, or FD_ED25519_AMD_NSLOT (2..6) from the environment. */
fd_ed25519_amd_t *
fd_ed25519_amd_new( int device, ulong batch_max, ulong blob_max );

void
fd_ed25519_amd_delete( fd_ed25519_amd_t * eng );

/* Pointer-array batch (the shape of n independent fd_ed25519_verify
   calls): msg[i] (sz[i] bytes), sig[i] (64 B), pub[i] (32 B) -> err[i]
   in {0,-1,-2,-3}.  Host memory, caller-owned, read-only except err.
   Returns FD_ED25519_AMD_OK or a negative FD_ED25519_AMD_ERR_*. */
int
fd_ed25519_amd_verify_batch( fd_ed25519_amd_t *   eng,
                             ulong                n,
                             void const * const * msg,
                             ulong const *        sz,
                             void const * const * sig,
                             void const * const * pub,
                             schar *              err );

/* SoA host batch: pub[n][32], sig[n][64], message i is
   blob[msg_off[i] .. msg_off[i]+msg_sz[i]).  Staged through pinned memory
   (double-buffered, copies overlap the previous chunk's kernels). */
int
fd_ed25519_amd_verify_soa( fd_ed25519_amd_t * eng,
                           ulong              n,
                           uchar const *      pub,
                           uchar const *      sig,
                           uint const *       msg_off,
                           uint const *       msg_sz,
                           uchar const *      blob,
                           ulong              blob_sz,
                           schar *            err );

/* Zero-copy host batch.  fd_ed25519_amd_host_register pins [base,
   base+sz) of caller memory once (hipHostRegister, portable to every
   device; FD_ED25519_AMD_ERR_DEVICE if the runtime refuses).  When pub,
   sig, msg_off, msg_sz and blob all lie in registered memory,
   fd_ed25519_amd_verify_soa_registered moves each chunk's planes and its
   message window from the caller's memory to the device by DMA, with no
   host-side copy (fd_ed25519_amd_verify_soa copies into pinned staging
   first); a batch small enough for the latency kernels (the
   fd_ed25519_amd_set_small_batch_max cap, default 16384, and at most
   batch_max) is read in place by the GPU over PCIe, with no copy at all.
   Same arguments, verdicts and errors as
   fd_ed25519_amd_verify_soa; FD_ED25519_AMD_ERR_INVAL if a plane is not
   registered.  A chunk whose messages are scattered over much more than
   their total size is gathered through the staging instead. */
int
fd_ed25519_amd_host_register( void * base, ulong sz );

int
fd_ed25519_amd_host_unregister( void * base );

int
fd_ed25519_amd_verify_soa_registered( fd_ed25519_amd_t * eng,
                                      ulong              n,
                                      uchar const *      pub,
                                      uchar const *      sig,
                                      uint const *       msg_off,
                                      uint const *       msg_sz,
                                      uchar const *      blob,
                                      ulong              blob_sz,
                                      schar *            err );

/* Multi-device engine (SURVEY s8 e: signatures are independent, so a batch
   shards with no exchange step).  One engine and one persistent host thread
   per entry of devices[0..ndev) (a device may be listed more than once:
   several engines share it); a batch is split into contiguous shards, one
   per engine, verified concurrently, and the call returns when every shard
   is done.  No collective, no peer traffic: each shard's inputs go host ->
   its device, its verdicts device -> host.  The reference scales the same
   way, as N independent verify tiles each with its own input
   (src/app/frank/fd_frank_init:67-80).  batch_max / blob_max are per
   engine.  One call at a time per multi engine (its worker threads serve
   one batch at a time); independent multi engines may run concurrently.
   NULL on failure (any device unusable). */
typedef struct fd_ed25519_amd_multi fd_ed25519_amd_multi_t;

fd_ed25519_amd_multi_t *
fd_ed25519_amd_multi_new( int const * devices, ulong ndev, ulong batch_max, ulong blob_max );

void
fd_ed25519_amd_multi_delete( fd_ed25519_amd_multi_t * multi );

ulong
fd_ed25519_amd_multi_ndev( fd_ed25519_amd_multi_t const * multi );

/* Shard [lo, hi) of n items that engine r of ndev verifies: lo = n*r/ndev. */
void
fd_ed25519_amd_shard_range( ulong n, ulong ndev, ulong r, ulong * lo, ulong * hi );

/* NUMA placement.  Each multi-engine thread binds itself to its device's
   NUMA node (the node's CPUs it may use, and the node as its preferred
   memory) before creating its engine, so the pinned staging it fills is
   node-local; a single engine prefers the device's node while it allocates
   its staging and leaves the caller's thread as it was.
   FD_ED25519_AMD_NUMA=0 turns both off.  The node of a device:
   hipDeviceGetPCIBusId -> /sys/bus/pci/devices/<bdf>/numa_node (-1 when
   unknown).  fd_ed25519_amd_sysfs_numa reads that file and the node's
   cpulist under any sysfs root: node (-1 if unknown) and up to cpus_max
   CPUs; returns the CPU count, -1 on an unreadable or malformed tree. */
int
fd_ed25519_amd_device_numa_node( int device );

int
fd_ed25519_amd_sysfs_numa( char const * sysfs_root, char const * pci_bdf, int * node, int * cpus, int cpus_max );

/* fd_ed25519_amd_verify_soa over the engines (same arguments and
   verdicts; err[i] for every i).  Returns the first engine error, if any. */
int
fd_ed25519_amd_multi_verify_soa( fd_ed25519_amd_multi_t * multi,
                                 ulong                    n,
                                 uchar const *            pub,
                                 uchar const *            sig,
                                 uint const *             msg_off,
                                 uint const *             msg_sz,
                                 uchar const *            blob,
                                 ulong                    blob_sz,
                                 schar *                  err );

/* Device-resident batch: every pointer is HIP device memory, already
   resident (the layout of fd_ed25519_amd_verify_soa).  Enqueues the
   verify kernels on `stream` (hipStream_t, NULL = default stream) and
   returns without synchronising.  `ws` is device scratch of at least
   fd_ed25519_amd_workspace_footprint(n) bytes, 256-aligned. */
ulong
fd_ed25519_amd_workspace_footprint( ulong n );

int
fd_ed25519_amd_verify_dev( ulong         n,
                           uchar const * d_pub,
                           uchar const * d_sig,
                           uint const *  d_msg_off,
                           uint const *  d_msg_sz,
                           uchar const * d_blob,
                           schar *       d_err,
                           void *        d_ws,
                           void *        stream );

/* Same as fd_ed25519_amd_verify_dev; when ev != NULL it points to 4
   hipEvent_t that are recorded on `stream` before k_prep, between the
   stages and after k_dsm (per-stage kernel timing for the bench). */
int
fd_ed25519_amd_verify_dev_ev( ulong         n,
                              uchar const * d_pub,
                              uchar const * d_sig,
                              uint const *  d_msg_off,
                              uint const *  d_msg_sz,
                              uchar const * d_blob,
                              schar *       d_err,
                              void *        d_ws,
                              void *        stream,
                              void * const * ev );

/* Optional per-signature work statistics of the last device-resident call
   on the same workspace: d_stats is planar [3][n] uint (double-scalar-
   multiply loop iterations, nonzero h digits, nonzero s digits; zeros for
   signatures decided before the multiply) -- used to report the
   algorithmic multiply count.  Enqueued on `stream`. */
int
fd_ed25519_amd_work_stats_dev( ulong n, void const * d_ws, uint * d_stats, void * stream );

/* Debug: copy the signed sliding-window digits (u16 [n][256], low byte =
   digit of h = SHA-512(R||A||M) mod L, high byte = digit of s; recoding of
   avx/fd_ed25519_ge.c:378-400) and the top digit position (int [n]) that
   the last device-resident call left in workspace `d_ws`. */
int
fd_ed25519_amd_debug_digits_dev( ulong n, void const * d_ws, unsigned short * d_dig, int * d_top, void * stream );

/* Host-side batch keygen + sign over the SoA layout (workload synthesis;
   not the verify path): prv[n][32] -> pub[n][32], sig[n][64] over
   blob[msg_off[i] .. +msg_sz[i]), on nthread host threads.  Returns 0. */
int
fd_ed25519_amd_sign_batch( ulong         n,
                           uchar const * prv,
                           uchar const * blob,
                           uint const *  msg_off,
                           uint const *  msg_sz,
                           uchar *       pub,
                           uchar *       sig,
                           int           nthread );

/* GPU batch keygen + sign (workload synthesis): device
   buffers prv[n][32] (32-aligned records), messages d_blob[d_msg_off[i] ..
   +d_msg_sz[i]) -> d_pub[n][32], d_sig[n][64]; the bytes equal
   fd_ed25519_public_from_private / fd_ed25519_sign (deterministic RFC 8032).
   Not constant time: never for real keys.  Enqueued on `stream`. */
int
fd_ed25519_amd_sign_dev( ulong         n,
                         uchar const * d_prv,
                         uint const *  d_msg_off,
                         uint const *  d_msg_sz,
                         uchar const * d_blob,
                         uchar *       d_pub,
                         uchar *       d_sig,
                         void *        stream );

/* Kernel choice for the double-scalar multiply, by batch size.  Batches
   of at most fd_ed25519_amd_set_latency_batch_max signatures (default 8192)
   run k_dsm8 (eight lanes per signature: the shortest per-batch latency
   while its waves fit one per SIMD); batches of at most
   fd_ed25519_amd_set_small_batch_max (default 16384) run k_dsm4 (four lanes
   per signature); larger ones the throughput kernel k_dsm (one lane per
   signature, its own op per lane), or k_dsmp (one lane per signature,
   signatures pooled per wave so that a wave runs one op class at a time)
   for batches of at least fd_ed25519_amd_set_pool_batch_min signatures
   (default 2^19; ~0UL disables it).  All give identical verdicts; 0
   disables a latency kernel.  Process-wide. */
void
fd_ed25519_amd_set_small_batch_max( ulong n );

void
fd_ed25519_amd_set_latency_batch_max( ulong n );

void
fd_ed25519_amd_set_pool_batch_min( ulong n );

/* k_dsmp bounds its step loop (a hang guard: every step advances at least
   one op of a signature's bounded op stream).  If a launch ever reaches the
   bound, every verdict of that launch is set to FD_ED25519_AMD_VERDICT_DEVICE
   (never a reference code) and the host batch calls return
   FD_ED25519_AMD_ERR_DEVICE instead of verdicts; device-resident callers
   (fd_ed25519_amd_verify_dev) see the marker in d_err.  Debug: cap the
   bound at `cap` steps per wave (0 restores it), to exercise that path. */
#define FD_ED25519_AMD_VERDICT_DEVICE (-128)
void
fd_ed25519_amd_debug_set_pool_iter_cap( ulong cap );

/* Library version / build string. */
char const *
fd_ed25519_amd_version( void );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_ed25519_amd_h */
