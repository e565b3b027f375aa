/* fd_txn_hip_int.h -- private: the frag-batch core of fd_txn_hip.hip, shared
   with the verify service (fd_verify_svc.hip).  Not part of the C ABI. */
#ifndef HEADER_fd_txn_hip_int_h
#define HEADER_fd_txn_hip_int_h

#include "../../include/fd_ed25519_hip.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

/* a staging frag: FD_TPU_PARSED_MTU (2168 B) in 64-B chunks */
#define FD_TXN_HIP_STAGE_CHUNKS 34ul

/* records the core needs for n frags: 12 x (n + slack) */
extern "C" __attribute__((visibility("hidden"))) ulong fd_txn_hip_record_cap( ulong n );
/* bytes of the misc block (counters, corrupt flag, record segments) */
extern "C" __attribute__((visibility("hidden"))) ulong fd_txn_hip_misc_bytes( void );

/* One frag batch on stream st: k_txnm_batch<16> (during_frag's copy of
   in frag j, at in + 64 in_chunk[j], into the frag at out + 64
   out_chunk[j]; after_frag's parse; fd_hash( seedv[j], sig0 ); the
   signature records), the verify of every record
   (fd_ed25519_hip_verify_segs) and the per-txn reduce (tcode[j] =
   fd_ed25519_verify_batch_single_msg).  fdesc[j] as k_out_flush reads it
   (copy end, payload_sz, txn_t_sz, gossip, corrupt).  Record buffers hold
   fd_txn_hip_record_cap( n ) records; ctx's scratch as many.  Asynchronous;
   aborts on a refused layout. */
extern "C" __attribute__((visibility("hidden"))) void
fd_txn_hip_batch_core( fd_ed25519_hip_ctx_t * ctx, hipStream_t st, ulong n,
                       uint8_t const * in, uint32_t const * in_chunk, uint16_t const * in_sz,
                       uint8_t const * in_kind, uint8_t * out, uint32_t const * out_chunk,
                       uint64_t const * seedv, uint16_t * tsz, uint64_t * tag, uint64_t * bid,
                       uint32_t * first, uint8_t * cnt, uint32_t * misc, uint8_t * rsig, uint8_t * rpub,
                       uint32_t * rmoff, uint32_t * rmsz, ulong rcap, signed char * rcode,
                       signed char * tcode, uint64_t * fdesc );

#endif /* HEADER_fd_txn_hip_int_h */
