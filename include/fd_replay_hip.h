#ifndef HEADER_fd_replay_hip_h
#define HEADER_fd_replay_hip_h

/* fd_replay_hip.h -- C ABI of the bulk verify callers outside the verify
   tile, batched onto the MI355X engine:

     replay   fd_executor_txn_verify  src/flamenco/runtime/fd_executor.c:1607-1623
              called once per transaction by the exec tile
              (src/discof/exec/fd_exec_tile.c:161, FD_EXEC_TT_TXN_SIGVERIFY):
              fd_ed25519_verify_batch_single_msg over the transaction's
              signatures and the first signature_cnt account addresses, with
              message = payload[ message_off, payload_sz ).  Result
              FD_RUNTIME_EXECUTE_SUCCESS, or FD_RUNTIME_TXN_ERR_SIGNATURE_FAILURE
              on any verify error (fd_runtime_err.h:4,19).
     shred    FEC-set root check      src/disco/shred/fd_fec_resolver.c:476
              fd_ed25519_verify( root, 32, shred->signature, leader_pubkey ):
              the resolver rejects the set on anything but FD_ED25519_SUCCESS.
     precompile  ed25519 program      src/flamenco/runtime/program/
              instructions            fd_precompiles.c:114-211
              fd_precompile_ed25519_verify, run by the executor for every
              instruction addressed to the ed25519 program: signature /
              pubkey / message spans named by 14-byte offset records, possibly
              inside other instructions of the same transaction.

   Replay hands the engine every transaction of a block (or of a batch of
   exec-tile tasks) at once instead of one fd_executor_txn_verify call per
   transaction; the shred tile hands it the roots of every FEC set it
   received in one poll.  Results equal the reference's per-call results.

   Library: firedancer_amd/libfd_ed25519_hip.so (same library as
   fd_ed25519_hip.h).  No torch or HIP types in any signature. */

#include "fd_ed25519_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned short ushort;

/* fd_runtime_err.h:4,19 */
#define FD_RUNTIME_HIP_EXECUTE_SUCCESS            ( 0)
#define FD_RUNTIME_HIP_TXN_ERR_SIGNATURE_FAILURE  (-13)

/* One parsed transaction as the exec tile holds it: the fd_txn_p_t payload
   (src/disco/fd_txn_p.h:6-42, payload = pool + payload_off, payload_sz) and
   the fd_txn_t fields fd_executor_txn_verify reads (fd_txn.h:186-249). */
typedef struct {
  uint   payload_off;
  ushort payload_sz;      /* fd_txn_p_t.payload_sz            */
  ushort signature_off;   /* fd_txn_t.signature_off           */
  ushort message_off;     /* fd_txn_t.message_off             */
  ushort acct_addr_off;   /* fd_txn_t.acct_addr_off           */
  uchar  signature_cnt;   /* fd_txn_t.signature_cnt           */
  uchar  _pad[ 3 ];
} fd_txn_hip_desc_t;      /* 16 bytes */

/* ---- replay ----------------------------------------------------------------

   A replay verifier owns device scratch for up to max_txn transactions per
   call (their signature records included) and runs on ctx's device. */

typedef struct fd_replay_hip fd_replay_hip_t;

fd_replay_hip_t * fd_replay_hip_new   ( fd_ed25519_hip_ctx_t * ctx, ulong max_txn );
void              fd_replay_hip_delete( fd_replay_hip_t * r );

/* fd_executor_txn_verify for n transactions: d_result[j] (int) is
   FD_RUNTIME_HIP_EXECUTE_SUCCESS or FD_RUNTIME_HIP_TXN_ERR_SIGNATURE_FAILURE,
   as the reference returns for transaction j.  signature_cnt 0 or > 16
   fails without reading any signature (fd_ed25519_user.c:238-241).
   d_pool / d_desc / d_result are device pointers; d_pool readable 16 bytes
   past its last payload.  Asynchronous on stream (NULL: ctx's stream): the
   signature-record count stays on the device.  Returns 0, or -1 if
   n > max_txn. */
int
fd_replay_hip_txn_verify_dev( fd_replay_hip_t *         r,
                              ulong                     n,
                              uchar const *             d_pool,
                              fd_txn_hip_desc_t const * d_desc,
                              int *                     d_result,
                              void *                    stream );

/* The same for a caller that holds the transactions in host memory (the
   replay tile: fd_txn_p_t payloads it packs into h_pool, descriptors into
   h_desc; integration/fd_replay_hip.patch).  Copies h_pool[0,pool_sz) and
   h_desc[0,n) into device staging owned by r (pool_sz up to
   FD_REPLAY_HIP_TXN_MTU * max_txn), verifies, and copies the n results into
   h_result.  Asynchronous on stream (NULL: ctx's stream): h_pool, h_desc and
   h_result must stay untouched until fd_replay_hip_poll returns 1 or
   fd_replay_hip_wait returns; pinned host memory
   (fd_ed25519_hip_host_alloc / _host_register) makes the copies DMA.
   Returns 0, or -1 (nothing launched) if n > max_txn, pool_sz is over the
   staging, or a descriptor's payload runs past pool_sz. */
#define FD_REPLAY_HIP_TXN_MTU (1232UL)   /* FD_TXN_MTU, fd_txn.h:65 */

int
fd_replay_hip_txn_verify_host( fd_replay_hip_t *         r,
                               ulong                     n,
                               uchar const *             h_pool,
                               ulong                     pool_sz,
                               fd_txn_hip_desc_t const * h_desc,
                               int *                     h_result,
                               void *                    stream );

/* Non-blocking completion check of the last fd_replay_hip_txn_verify_dev /
   _host call (its results are in place once this says so): 1 done, 0 still
   running, -1 no call yet.  For a caller that polls from its run loop (the
   replay tile's after_credit). */
int
fd_replay_hip_poll( fd_replay_hip_t const * r );

/* Blocks until the last call is done.  Returns 0. */
int
fd_replay_hip_wait( fd_replay_hip_t * r );

/* ---- shred FEC-set roots ----------------------------------------------------

   d_codes[i] = fd_ed25519_verify( d_roots + 32*i, 32, d_sigs + 64*i,
   d_pubs + 32*i ) for n FEC sets (FD_ED25519_* codes).  Device pointers,
   d_roots readable 16 bytes past its end; asynchronous on stream. */
int
fd_fec_hip_verify_roots_dev( fd_ed25519_hip_ctx_t * ctx,
                             ulong                  n,
                             uchar const *          d_roots,
                             uchar const *          d_sigs,
                             uchar const *          d_pubs,
                             signed char *          d_codes,
                             void *                 stream );

/* ---- ed25519 program (precompile) instructions -----------------------------

   fd_precompile_ed25519_verify (fd_precompiles.c:114-211, data fetch
   fd_precompile_get_instr_data :76-107) for n instructions at once, e.g.
   every ed25519-program instruction of a block.  Instruction j is described
   by d_desc[j]; the data of every instruction of its transaction (for
   offset records that name another instruction by index) by the table
   entries d_instr_tab[ instr_base, instr_base + instr_cnt ).  All data
   spans live in d_pool (e.g. the block's txn payloads), readable 16 bytes
   past the last one. */

/* fd_executor_err.h:14,40 and fd_precompiles.h:16-18 */
#define FD_PRECOMPILE_HIP_INSTR_SUCCESS          (  0)
#define FD_PRECOMPILE_HIP_INSTR_ERR_CUSTOM_ERR   (-26)
#define FD_PRECOMPILE_HIP_ERR_SIGNATURE          (  2)
#define FD_PRECOMPILE_HIP_ERR_DATA_OFFSET        (  3)
#define FD_PRECOMPILE_HIP_ERR_INSTR_DATA_SIZE    (  4)
/* a descriptor the reference cannot produce (data_sz above the 1232-byte
   transaction MTU, fd_txn.h:65): d_err -1, d_custom_err 0xFFFFFFFF */
#define FD_PRECOMPILE_HIP_ERR_DESC               ( -1)
#define FD_PRECOMPILE_HIP_DATA_MAX               (1232)
/* signatures one instruction can name: (1232 - 2) / 14 */
#define FD_PRECOMPILE_HIP_SIG_MAX                (  87)

typedef struct {
  uint   data_off;        /* this instruction's data: d_pool[ data_off, +data_sz )  */
  ushort data_sz;         /* fd_instr_info_t.data_sz                                 */
  ushort instr_cnt;       /* TXN( txn )->instr_cnt                                   */
  uint   instr_base;      /* its transaction's first entry in d_instr_tab            */
  uint   _pad;
} fd_precompile_hip_desc_t;   /* 16 bytes */

typedef struct {
  uint data_off;          /* instruction k of the transaction: d_pool[ data_off, +data_sz ) */
  uint data_sz;
} fd_precompile_hip_instr_t;  /* 8 bytes */

typedef struct fd_precompile_hip fd_precompile_hip_t;

/* device scratch for up to max_instr instructions per call (and their
   FD_PRECOMPILE_HIP_SIG_MAX signatures each) on ctx's device */
fd_precompile_hip_t * fd_precompile_hip_new   ( fd_ed25519_hip_ctx_t * ctx, ulong max_instr );
void                  fd_precompile_hip_delete( fd_precompile_hip_t * pc );

/* d_err[j] = the reference's return for instruction j
   (FD_PRECOMPILE_HIP_INSTR_SUCCESS or _INSTR_ERR_CUSTOM_ERR) and
   d_custom_err[j] the txn_out->err.custom_err it sets (0 on success): the
   first failing signature in offset-record order decides, its span checks
   (signature, public key, message) before its verify.  Device pointers,
   asynchronous on stream (NULL: ctx's stream).  Returns 0, or -1 if
   n > max_instr. */
int
fd_precompile_hip_ed25519_verify_dev( fd_precompile_hip_t *             pc,
                                      ulong                             n,
                                      uchar const *                     d_pool,
                                      fd_precompile_hip_desc_t const *  d_desc,
                                      fd_precompile_hip_instr_t const * d_instr_tab,
                                      int *                             d_err,
                                      uint *                            d_custom_err,
                                      void *                            stream );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_replay_hip_h */
