/* fd_hip_order.h -- internal to libfd_ed25519_hip.so (not part of the C ABI).

   1. The SHA-512 block-count key that orders records for k_verify_prep on
      the variable-size message paths.  Shared by the producers of the
      histogram (k_txnm_batch in fd_txn_hip.hip, k_msg_hist) and its
      consumer (k_msg_order, fd_ed25519_hip.hip): the bucket bases
      k_msg_order takes from the histogram are only a permutation of the
      records if both sides key every record's message size identically.
      A prefixed message R||A||M of sz bytes is (sz + 64 + 17 + 127) / 128
      SHA-512 blocks (64 bytes of R||A, 17 of padding and length); keys are
      clamped to 15.

   2. Segmented record arrays.  One device-scope atomic word serves about
      88 returning atomics per microsecond (MI355X_MICROARCH.md, dequeue),
      so a kernel in which each of 65536 workgroups claims its record range
      on one counter spends ~0.75 ms on that counter alone.  k_txnm_batch
      instead gives workgroup b the segment b % n_seg: records
      [s*seg_cap, s*seg_cap + count_s) with count_s on its own 128-B line,
      and the segment's block-count histogram on another.  The verify reads
      such a layout through fd_ed25519_hip_verify_segs: one workgroup sums
      the segments (total record count, histogram), k_msg_order maps prep's
      dense processing slots onto the segments' records, and codes land at
      the records' own indices. */
#ifndef HEADER_fd_hip_order_h
#define HEADER_fd_hip_order_h

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fd_ed25519_hip.h"

#define FD_HIP_ORD_KEYS      16u    /* histogram bins */

__device__ __forceinline__ uint32_t fd_hip_msg_key( uint32_t sz ) {
  uint32_t b = (sz + 81u + 127u) >> 7;
  return b < 15u ? b : 15u;
}

#define FD_HIP_SEG_MAX     256u     /* segments at most */
#define FD_HIP_SEG_STRIDE   64u     /* words per segment: its counter line, then its histogram line */
#define FD_HIP_SEG_CNT_W     0u     /* record count (u32) */
#define FD_HIP_SEG_HIST_W   32u     /* FD_HIP_ORD_KEYS u32 histogram words */

typedef struct {
  uint32_t const * seg;     /* segment s's words at seg[ s*FD_HIP_SEG_STRIDE ] */
  uint32_t         n_seg;   /* <= FD_HIP_SEG_MAX */
  unsigned long    seg_cap; /* records per segment: record index = s*seg_cap + local */
  uint32_t *       total;   /* written by the verify: the total record count (device) */
} fd_hip_segs_t;

/* Verify every record of the segments (n_seg*seg_cap <= the context's
   chunk_sigs; variable-size messages, block-count order).  Asynchronous on
   stream; -1 on a bad layout.  Hidden: called from fd_txn_hip.hip only. */
extern "C" __attribute__((visibility("hidden"))) int
fd_ed25519_hip_verify_segs( fd_ed25519_hip_ctx_t * ctx, fd_hip_segs_t segs, uchar const * d_sigs,
                            uchar const * d_pubs, uchar const * d_pool, uint const * d_msg_off,
                            uint const * d_msg_sz, signed char * d_codes, void * stream );

#endif /* HEADER_fd_hip_order_h */
