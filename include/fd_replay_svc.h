#ifndef HEADER_fd_replay_svc_h
#define HEADER_fd_replay_svc_h

/* fd_replay_svc.h -- a replay block's sigverify through the GPU tile's
   service (include/fd_verify_svc.h "clients"): the replay tile stays a
   single-threaded process with no HIP context and no device fd, and keeps
   the reference's sandbox, while its transactions' signatures ride the
   GPU tile's launches beside the verify tiles' frags.

   What it computes, per transaction: fd_executor_txn_verify
   (src/flamenco/runtime/fd_executor.c:1607-1623):
   fd_ed25519_verify_batch_single_msg( payload + message_off,
   payload_sz - message_off, payload + signature_off,
   payload + acct_addr_off, signature_cnt ) == SUCCESS ?
   FD_RUNTIME_EXECUTE_SUCCESS : FD_RUNTIME_TXN_ERR_SIGNATURE_FAILURE
   (fd_runtime_err.h:4,19).  batch_single_msg fails a signature_cnt of 0
   or over 16 without verifying (fd_ed25519_user.c:238-241), else succeeds
   iff every fd_ed25519_verify( msg, sig_k, pub_k ) does: so a transaction
   is one service record per signature (the message is the same for all of
   them), and its result is the AND of its records' verdicts.

   Use (integration/fd_replay_hip.patch FD_HAS_HIP_SVC,
   integration/sched_run.c svc mode): join once; per claimed batch
   fd_replay_svc_start( r, cnt, txns, result ) with each transaction's
   payload pointer and fd_txn_t spans (they must stay in place until the
   batch is done); then fd_replay_svc_step( r ) from the run loop until it
   returns 1: it adds records while the client's slots allow, posts them,
   and collects answered requests -- never blocks, no syscall.  result[ j ]
   is then the reference's return for transaction j. */

#include "fd_verify_svc.h"

#define FD_REPLAY_SVC_EXECUTE_SUCCESS            ( 0)   /* FD_RUNTIME_EXECUTE_SUCCESS           */
#define FD_REPLAY_SVC_TXN_ERR_SIGNATURE_FAILURE  (-13)  /* FD_RUNTIME_TXN_ERR_SIGNATURE_FAILURE */
#define FD_REPLAY_SVC_BATCH_SIG_MAX              (16UL) /* fd_ed25519_user.c:238-241            */

typedef struct {
  uchar const * payload;
  ushort        payload_sz, signature_off, message_off, acct_addr_off;
  uchar         signature_cnt;
} fd_replay_svc_txn_t;

typedef struct {
  fd_verify_svc_client_t      c[1];
  fd_replay_svc_txn_t const * txn;
  int *                       result;
  ulong                       cnt;        /* transactions of the batch in flight (0: none) */
  ulong                       next_txn;   /* the next record to add: transaction, signature */
  ulong                       next_sig;
  ulong                       recs;       /* records of the batch */
  ulong                       recs_done;
  ulong                       batches, sigs;
} fd_replay_svc_t;

static inline fd_replay_svc_t *
fd_replay_svc_join( fd_replay_svc_t * r, fd_verify_svc_seg_t * seg, ulong t ) {
  if( !r || !fd_verify_svc_client_join( r->c, seg, t ) ) return (fd_replay_svc_t *)0;
  r->txn = 0; r->result = 0; r->cnt = 0UL; r->next_txn = 0UL; r->next_sig = 0UL; r->recs = 0UL; r->recs_done = 0UL;
  r->batches = 0UL; r->sigs = 0UL;
  return r;
}

/* records are made for a transaction with 1..16 signatures whose message
   fits a record (every transaction does: payload_sz <= FD_TXN_MTU 1232,
   fd_txn.h:65, against FD_VERIFY_SVC_SIG_MSG_MAX 1952); any other fails
   without a record, as batch_single_msg fails a count outside 1..16 */
static inline int
fd_replay_svc_txn_ok( fd_replay_svc_txn_t const * x ) {
  return x->signature_cnt>=1 && (ulong)x->signature_cnt<=FD_REPLAY_SVC_BATCH_SIG_MAX && x->message_off<=x->payload_sz &&
         (ulong)( x->payload_sz - x->message_off )<=FD_VERIFY_SVC_SIG_MSG_MAX;
}

static inline void
fd_replay_svc_start( fd_replay_svc_t * r, ulong cnt, fd_replay_svc_txn_t const * txn, int * result ) {
  r->txn = txn; r->result = result; r->cnt = cnt; r->next_txn = 0UL; r->next_sig = 0UL; r->recs = 0UL; r->recs_done = 0UL;
  for( ulong j=0UL; j<cnt; j++ ) {
    ulong k = txn[ j ].signature_cnt;
    int   ok = fd_replay_svc_txn_ok( txn + j );
    result[ j ] = ok ? FD_REPLAY_SVC_EXECUTE_SUCCESS : FD_REPLAY_SVC_TXN_ERR_SIGNATURE_FAILURE;
    if( ok ) r->recs += k;
  }
  r->batches++; r->sigs += r->recs;
}

static inline void
fd_replay_svc_verdict( void * ctx, uint tag, int code ) {
  fd_replay_svc_t * r = (fd_replay_svc_t *)ctx;
  if( code ) r->result[ tag ] = FD_REPLAY_SVC_TXN_ERR_SIGNATURE_FAILURE;
}

/* 1 once every record of the batch is answered (result[] final, the
   batch closed), else 0 */
static inline int
fd_replay_svc_step( fd_replay_svc_t * r, long now ) {
  if( !r->cnt ) return 1;
  while( r->next_txn<r->cnt ) {
    fd_replay_svc_txn_t const * x = r->txn + r->next_txn;
    ulong k = x->signature_cnt;
    if( !fd_replay_svc_txn_ok( x ) ) { r->next_txn++; r->next_sig = 0UL; continue; }
    int rc = fd_verify_svc_client_add( r->c, x->payload + x->signature_off + 64UL*r->next_sig,
                                       x->payload + x->acct_addr_off + 32UL*r->next_sig, x->payload + x->message_off,
                                       (ulong)x->payload_sz - x->message_off, (uint)r->next_txn, now );
    if( rc<=0 ) break;                                             /* no free slot: collect first */
    if( ++r->next_sig==k ) { r->next_txn++; r->next_sig = 0UL; }
  }
  if( r->next_txn==r->cnt ) (void)fd_verify_svc_client_flush( r->c, now );
  r->recs_done += fd_verify_svc_client_poll( r->c, fd_replay_svc_verdict, r );
  if( r->next_txn<r->cnt || r->recs_done<r->recs ) return 0;
  r->cnt = 0UL;
  return 1;
}

#endif /* HEADER_fd_replay_svc_h */
