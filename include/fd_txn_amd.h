#ifndef HEADER_fd_txn_amd_h
#define HEADER_fd_txn_amd_h

/* Solana transaction descriptor types and the GPU transaction front end of
 * the MI355X verify engine.
 *
 * Part 1 is the reference's parsed-transaction layout
 * (src/ballet/txn/fd_txn.h:1-393), reproduced byte for byte so that a
 * descriptor written by the GPU parser (k_txn_parse) is memcmp-equal to the
 * one the reference's fd_txn_parse (src/ballet/txn/fd_txn_parse.c:6-217)
 * writes for the same payload.  When the reference's own fd_txn.h has been
 * included first its definitions are used instead.
 *
 * Part 2 declares the batch entry points: device-side parsing of a batch of
 * wire-format transactions and multi-signer verification of every signature
 * (signature i is checked with public key acct_addr[i] over the message
 * payload[message_off, payload_sz), fd_txn.h:159-217).
 */

#include "fd_ed25519_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ===== Part 1: reference layout (src/ballet/txn/fd_txn.h) ===== */

#ifndef HEADER_fd_src_ballet_txn_fd_txn_h

typedef unsigned short ushort;

#define FD_TXN_VLEGACY               ((uchar)0xFF)   /* fd_txn.h:36 */
#define FD_TXN_V0                    ((uchar)0x00)   /* fd_txn.h:40 */
#define FD_TXN_SIGNATURE_SZ          (64UL)
#define FD_TXN_PUBKEY_SZ             (32UL)
#define FD_TXN_ACCT_ADDR_SZ          (32UL)
#define FD_TXN_BLOCKHASH_SZ          (32UL)
#define FD_TXN_SIG_MAX               (127UL)         /* fd_txn.h:70 */
#define FD_TXN_ACCT_ADDR_MAX         (256UL)
#define FD_TXN_ADDR_TABLE_LOOKUP_MAX (254UL)
#define FD_TXN_INSTR_MAX             (65535UL)
#define FD_TXN_MAX_SZ                (3570UL)        /* fd_txn.h:95 */

struct fd_txn_instr {                                /* fd_txn.h:107-139 */
  uchar  program_id;
  uchar  _padding_reserved_1;
  ushort acct_cnt;
  ushort data_sz;
  ushort acct_off;
  ushort data_off;
};
typedef struct fd_txn_instr fd_txn_instr_t;

struct fd_txn {                                      /* fd_txn.h:146-272 */
  uchar          transaction_version;
  uchar          signature_cnt;
  ushort         signature_off;
  ushort         message_off;
  uchar          readonly_signed_cnt;
  uchar          readonly_unsigned_cnt;
  ushort         acct_addr_cnt;
  ushort         acct_addr_off;
  ushort         recent_blockhash_off;
  uchar          addr_table_lookup_cnt;
  uchar          addr_table_adtl_writable_cnt;
  uchar          addr_table_adtl_cnt;
  uchar          _padding_reserved_1;
  ushort         instr_cnt;
  fd_txn_instr_t instr[];
};
typedef struct fd_txn fd_txn_t;

struct fd_txn_acct_addr_lut {                        /* fd_txn.h:281-318 */
  ushort addr_off;
  uchar  writable_cnt;
  uchar  readonly_cnt;
  ushort writable_off;
  ushort readonly_off;
};
typedef struct fd_txn_acct_addr_lut fd_txn_acct_addr_lut_t;

#define FD_TXN_PARSE_COUNTERS_RING_SZ (32UL)         /* fd_txn.h:322-341 */
struct fd_txn_parse_counters {
  ulong success_cnt;
  ulong failure_cnt;
  ulong failure_ring[ FD_TXN_PARSE_COUNTERS_RING_SZ ];
};
typedef struct fd_txn_parse_counters fd_txn_parse_counters_t;

/* fd_txn.h:369-375 */
static inline ulong
fd_txn_footprint( ulong instr_cnt, ulong addr_table_lookup_cnt ) {
  return sizeof(fd_txn_t) + instr_cnt*sizeof(fd_txn_instr_t) + addr_table_lookup_cnt*sizeof(fd_txn_acct_addr_lut_t);
}

/* fd_txn.h:351-354 */
static inline fd_txn_acct_addr_lut_t *
fd_txn_get_address_tables( fd_txn_t * txn ) {
  return (fd_txn_acct_addr_lut_t *)(txn->instr + txn->instr_cnt);
}

#endif /* HEADER_fd_src_ballet_txn_fd_txn_h */

/* ===== Part 2: GPU transaction batch (new) ===== */

/* Transaction verdict codes.  0 and the FD_ED25519_ERR_* codes keep their
   meaning (the code of the FIRST signature, in signature order, that failed);
   a payload that fd_txn_parse rejects gets FD_TXN_AMD_ERR_PARSE and none of
   its signatures is checked. */
#define FD_TXN_AMD_ERR_PARSE (-4)

/* Device-side batch parse: transaction t is d_payload[d_txn_off[t] ..
   +d_txn_sz[t]).  Writes d_footprint[t] = what fd_txn_parse returns (0 on
   failure, else fd_txn_footprint) and, when d_out != NULL, the fd_txn_t
   descriptor to d_out + t*out_stride (out_stride >= FD_TXN_MAX_SZ, multiple
   of 2).  Enqueued on `stream`; returns 0 or FD_ED25519_AMD_ERR_*. */
int
fd_txn_amd_parse_dev( ulong         txn_cnt,
                      uchar const * d_payload,
                      uint const *  d_txn_off,
                      uint const *  d_txn_sz,
                      uint *        d_footprint,
                      uchar *       d_out,
                      ulong         out_stride,
                      void *        stream );

/* Host batch of wire-format transactions (same layout, host memory):
   parse on the GPU, verify every signature of every well-formed
   transaction with the multi-signer rule, reduce to one verdict per
   transaction.  txn_err[t] in {0, -1, -2, -3, FD_TXN_AMD_ERR_PARSE}.
   Optional outputs (NULL to skip): sig_base[t] = index of transaction t's
   first signature in sig_err (sig_base[txn_cnt] = total signatures) and
   sig_err[...] = per-signature fd_ed25519_verify codes (capacity: the
   total that fd_ed25519_amd_txn_slots returns for the same batch).  Every
   payload must be at most FD_TXN_AMD_MTU bytes (the wire limit), fit the
   engine's blob_max, and reserve at most batch_max signature slots
   (FD_ED25519_AMD_ERR_INVAL otherwise, checked before anything is
   launched; batch_max >= 19 admits every payload).  Returns
   FD_ED25519_AMD_OK or a negative FD_ED25519_AMD_ERR_*. */
#define FD_TXN_AMD_MTU (1232UL)
int
fd_ed25519_amd_verify_txns( fd_ed25519_amd_t * eng,
                            ulong              txn_cnt,
                            uchar const *      payload,
                            uint const *       txn_off,
                            uint const *       txn_sz,
                            ulong              payload_sz,
                            schar *            txn_err,
                            uint *             sig_base,
                            schar *            sig_err );

/* Multi-device form (fd_ed25519_amd_multi_new): the transactions are split
   into contiguous shards, one per device, verified concurrently, each by
   its own engine and host thread; outputs as fd_ed25519_amd_verify_txns,
   sig_base numbered over the whole batch. */
int
fd_ed25519_amd_multi_verify_txns( fd_ed25519_amd_multi_t * multi,
                                  ulong                    txn_cnt,
                                  uchar const *            payload,
                                  uint const *             txn_off,
                                  uint const *             txn_sz,
                                  ulong                    payload_sz,
                                  schar *                  txn_err,
                                  uint *                   sig_base,
                                  schar *                  sig_err );

/* Device-resident form (inputs already in HBM, caller's stream, no sync).
   Signature slots follow the same rule as fd_ed25519_amd_verify_txns:
   d_tbase[t] (txn_cnt+1 entries, slot_cnt = d_tbase[txn_cnt]) is what
   fd_ed25519_amd_txn_slots computes on the host.  d_sig_err (optional,
   slot_cnt entries) receives the per-signature codes.  d_ws: at least
   fd_ed25519_amd_txn_workspace_footprint(txn_cnt, slot_cnt) bytes,
   256-aligned; it begins with the signature verify's workspace, so
   fd_ed25519_amd_work_stats_dev( slot_cnt, d_ws, ... ) reads the call's
   per-signature work statistics. */
ulong
fd_ed25519_amd_txn_workspace_footprint( ulong txn_cnt, ulong slot_cnt );

ulong
fd_ed25519_amd_txn_slots( ulong         txn_cnt,
                          uchar const * payload,
                          uint const *  txn_off,
                          uint const *  txn_sz,
                          uint *        tbase );

int
fd_ed25519_amd_verify_txns_dev( ulong         txn_cnt,
                                ulong         slot_cnt,
                                uchar const * d_payload,
                                uint const *  d_txn_off,
                                uint const *  d_txn_sz,
                                uint const *  d_tbase,
                                schar *       d_txn_err,
                                schar *       d_sig_err,
                                void *        d_ws,
                                void *        stream );

/* Workload synthesis (config 4): txn_cnt well-formed legacy / v0
   transactions with nsig_lo..nsig_hi signers (account addresses = the
   next public keys of pub[]) and ~msg_lo..msg_hi-byte messages, capped at
   the MTU; signature fields zero.  Per signature: its message range in
   payload (sig_msg_off, sig_msg_sz) and where its 64 bytes go (sig_at).
   Returns the signature count, 0 if payload_cap / pub_cnt is too small. */
ulong
fd_ed25519_amd_synth_txns( ulong         seed,
                           ulong         txn_cnt,
                           uint          nsig_lo,
                           uint          nsig_hi,
                           uint          msg_lo,
                           uint          msg_hi,
                           uchar const * pub,
                           ulong         pub_cnt,
                           uchar *       payload,
                           ulong         payload_cap,
                           uint *        txn_off,
                           uint *        txn_sz,
                           uint *        sig_msg_off,
                           uint *        sig_msg_sz,
                           uint *        sig_at );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_txn_amd_h */
