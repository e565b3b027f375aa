#ifndef HEADER_fd_sha512_hip_h
#define HEADER_fd_sha512_hip_h

/* Batched SHA-512 on the GPU ("multi-message SHA-512",
   the GPU counterpart of the reference's batching API,
   src/ballet/sha512/fd_sha512.h:232-419 and fd_sha512_batch_avx512.c).

   The hash core is the one k_verify_prep runs for SHA-512(R||A||M): one
   message per lane, the wave's 128-byte message blocks loaded cooperatively
   (16-B pieces, coalesced) through LDS (fd_ed25519_dev.h
   sha512_prefixed_coop); digests are bit-exact against the reference's
   fd_sha512_hash (tests/test_sha512_cavp.py: the reference's CAVP vectors).
   A wave runs as many blocks as its longest message: a caller with mixed
   sizes gets the best rate by adding messages of similar size next to each
   other.

   Two entry points:
   - fd_sha512_hip_batch_dev: messages resident in HBM, asynchronous;
   - fd_sha512_hip_batch_{init,add,fini,abort}: the reference's batching API
     shape (fd_sha512.h:306-341) over host memory, with a larger batch. */

#include "fd_ed25519_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* n messages d_pool[ d_off[i], +d_sz[i] ) -> 64-byte digests at
   d_hash + 64*i (d_hash 16-byte aligned).  d_pool must be readable up to the
   16-byte boundary after each message's last byte (as for the verify
   entries).  Device pointers, asynchronous on stream (NULL: the context's
   stream).  Returns 0. */
int fd_sha512_hip_batch_dev( fd_ed25519_hip_ctx_t * ctx,
                             ulong                  n,
                             uchar const *          d_pool,
                             uint const *           d_off,
                             uint const *           d_sz,
                             uchar *                d_hash,
                             void *                 stream );

/* Host batching API.  Semantics follow fd_sha512_batch_* (fd_sha512.h:
   306-341): add records (data, sz, hash); the hash is written no later than
   fini, which hashes what is still pending and returns the batch memory;
   data must stay readable and unchanged until then; abort drops pending
   records without hashing them.  When FD_SHA512_HIP_BATCH_MAX records are
   pending, add hashes them before returning (the reference flushes at its
   own FD_SHA512_BATCH_MAX, 8 for AVX-512).  Each flush copies the pending
   messages into a pinned staging block, runs one kernel launch on the
   context's stream and waits for it.  ctx NULL: the process-wide context the
   fd_ed25519_verify drop-in uses (FD_ED25519_HIP_DEVICE).  A message longer
   than FD_SHA512_HIP_MSG_MAX aborts the process (32-bit offsets; never a
   silent wrong digest).  Not thread-safe per batch; distinct batches may be
   used from distinct threads. */

#define FD_SHA512_HIP_BATCH_ALIGN (128UL)
#define FD_SHA512_HIP_BATCH_MAX   (4096UL)
#define FD_SHA512_HIP_MSG_MAX     (2147483648UL)

typedef struct fd_sha512_hip_batch fd_sha512_hip_batch_t;

ulong                   fd_sha512_hip_batch_align    ( void );
ulong                   fd_sha512_hip_batch_footprint( void );
fd_sha512_hip_batch_t * fd_sha512_hip_batch_init     ( void * mem, fd_ed25519_hip_ctx_t * ctx );
fd_sha512_hip_batch_t * fd_sha512_hip_batch_add      ( fd_sha512_hip_batch_t * batch, void const * data, ulong sz,
                                                       void * hash );
void *                  fd_sha512_hip_batch_fini     ( fd_sha512_hip_batch_t * batch );
void *                  fd_sha512_hip_batch_abort    ( fd_sha512_hip_batch_t * batch );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_sha512_hip_h */
