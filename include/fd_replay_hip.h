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

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_replay_hip_h */
