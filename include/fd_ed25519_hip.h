#ifndef HEADER_fd_ed25519_hip_h
#define HEADER_fd_ed25519_hip_h

/* fd_ed25519_hip.h -- C ABI of the MI355X (gfx950) ed25519 verify engine.

   Drop-in boundary for the reference's verify path
   (anoushk1234/firedancer, src/ballet/ed25519/fd_ed25519.h).  Part 1 is
   link-compatible with the reference declarations it replaces; part 2 is the
   GPU-native bulk interface the verify tile's batches go through (the
   reference has no such entry; the precedent is the async wiredancer offload,
   src/wiredancer/c/wd_f1.h:71-112).  No torch or HIP types appear in any
   signature: plain pointers and sizes only.

   Library: firedancer_amd/libfd_ed25519_hip.so (built by __graft_entry__.build()).
   The reference-side bindings a maintainer would add are in INTEGRATION.md. */

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned char uchar;
typedef unsigned long ulong;
typedef unsigned int  uint;

/* Result codes: fd_ed25519.h:11-14 */
#define FD_ED25519_SUCCESS    ( 0)
#define FD_ED25519_ERR_SIG    (-1)
#define FD_ED25519_ERR_PUBKEY (-2)
#define FD_ED25519_ERR_MSG    (-3)

/* ---- Part 1: reference API (link-compatible) ----------------------------

   fd_sha512_t is opaque here (footprint 256, align 128: fd_sha512.h:56-77);
   the GPU engine takes no interest in it (the reference uses it as scratch).
   Semantics, including the order of the checks and the error code of every
   reject, are those of the reference's AVX-512 build (fd_ed25519_user.c with
   avx512/fd_r43x6_ge.c decode); fd_ed25519_hip_set_errmode() switches the
   error codes to the portable build's (the accept/reject bit is the same).
   Each call is synchronous on process-wide contexts (device
   FD_ED25519_HIP_DEVICE, default 0, or fd_ed25519_hip_dropin_init's) and
   re-entrant: concurrent calls from different threads are combined into
   staged batches, and up to 4 batches run at once, each on its own context
   and stream (FD_ED25519_HIP_DROPIN_SLOTS, 1..16; a caller that finds a slot
   free runs the open batch for all in it).  msg_sz above about 2^32-27K aborts
   the process (the engine's message offsets are 32-bit; hashing a prefix
   would silently diverge).

   Sandboxed callers (a tile's unprivileged_init installs seccomp and closes
   fds) must call fd_ed25519_hip_dropin_init() from privileged_init, so that
   the HIP runtime opens /dev/kfd and /dev/dri and maps its memory before
   the sandbox is up; INTEGRATION.md lists the fds and syscalls to allow. */

struct fd_sha512_private;

/* replaces fd_ed25519_verify, fd_ed25519.h:96-101 (fd_ed25519_user.c:135-230) */
int
fd_ed25519_verify( uchar const                msg[], /* msg_sz */
                   ulong                      msg_sz,
                   uchar const                sig[ 64 ],
                   uchar const                public_key[ 32 ],
                   struct fd_sha512_private * sha );

/* replaces fd_ed25519_verify_batch_single_msg, fd_ed25519.h:124-130
   (fd_ed25519_user.c:232-310): batch_sz 0 or >16 -> ERR_SIG; otherwise the
   first pre-check failure in signature order, else ERR_MSG if any equation
   fails, else SUCCESS. */
int
fd_ed25519_verify_batch_single_msg( uchar const                msg[], /* msg_sz */
                                    ulong const                msg_sz,
                                    uchar const                signatures[ 64 ], /* 64*batch_sz */
                                    uchar const                pubkeys[ 32 ],    /* 32*batch_sz */
                                    struct fd_sha512_private * shas[ 1 ],        /* batch_sz, ignored */
                                    uchar const                batch_sz );

/* replaces fd_ed25519_strerror, fd_ed25519.h:137-138 (fd_ed25519_user.c:312-322) */
char const *
fd_ed25519_strerror( int err );

/* Create the drop-in's process-wide contexts (one per batch slot) on
   `device` now, with their pinned staging, instead of lazily at the first
   verify.  Returns 0, or -1
   if the context already exists on another device.  Call it once from a
   tile's privileged_init (the HIP context must exist before
   the sandbox). */
int
fd_ed25519_hip_dropin_init( int device );

/* Drop-in combining statistics: out[0] = launches (batches run),
   out[1] = calls they served (>= out[0]; the ratio is the mean number of
   concurrent calls combined per launch). */
void
fd_ed25519_hip_dropin_stats( ulong out[ 2 ] );

/* ---- Part 2: GPU-native bulk interface -----------------------------------

   A context owns one HIP device, one stream, the base-point tables and the
   scratch for up to chunk_sigs signatures in flight per launch
   (larger requests are processed in chunks of chunk_sigs).  Contexts are not
   thread-safe; use one per host thread (one per verify tile).  Calls on one
   context may name different streams: each verify waits (hipStreamWaitEvent)
   for the context's previous verify before it touches the shared scratch, so
   they run in call order; calls on different contexts run concurrently.

   Record layout (all pointers are device pointers for *_dev, host pointers
   otherwise):
     sigs     64*n bytes   sig i = R||S  (fd_ed25519_sig_t, fd_ed25519.h:17-20)
     pubs     32*n bytes
     pool     message bytes; message i = pool[ msg_off[i], msg_off[i]+msg_sz[i] )
              (several signatures may share one message, as in a txn)
     codes    n int8 results (FD_ED25519_* codes, fd_ed25519_verify semantics)
     bitmap   ceil(n/64) ulong: bit i%64 of word i/64 set iff codes[i]==0; the
              bits of the last word past n are zero (device-count calls:
              left as they were, see verify_dev_count)
   Device buffers for *_dev must be 16-byte aligned and the pool must stay
   readable 16 bytes past its last message byte.

   Any HIP failure aborts the process with a message on stderr (the tile
   restarts) -- a device error is never reported as a rejected signature. */

typedef struct fd_ed25519_hip_ctx fd_ed25519_hip_ctx_t;

#define FD_ED25519_HIP_ERRMODE_AVX512 0   /* error codes of the AVX-512 build (default) */
#define FD_ED25519_HIP_ERRMODE_REF    1   /* error codes of the portable build */

fd_ed25519_hip_ctx_t * fd_ed25519_hip_ctx_new   ( int device, ulong chunk_sigs );
void                   fd_ed25519_hip_ctx_delete( fd_ed25519_hip_ctx_t * ctx );
int                    fd_ed25519_hip_ctx_device( fd_ed25519_hip_ctx_t const * ctx );
/* HIP devices visible to the process (0 if none or the runtime fails);
   a verify tile binds kind_id % this */
int                    fd_ed25519_hip_device_cnt( void );
/* Grow the per-launch scratch to at least chunk_sigs signatures (2.3 KB of
   HBM each); waits for the device to go idle first.  A caller whose record
   count is only known on the device (verify_dev_count) reserves its upper
   bound so one launch pair covers it. */
void                   fd_ed25519_hip_ctx_reserve( fd_ed25519_hip_ctx_t * ctx, ulong chunk_sigs );
void *                 fd_ed25519_hip_ctx_stream( fd_ed25519_hip_ctx_t const * ctx ); /* hipStream_t */
void                   fd_ed25519_hip_set_errmode( fd_ed25519_hip_ctx_t * ctx, int errmode );

/* The double-scalar multiplication checks [k2*S mod L]B - [k1]A - [k2]R == O
   with k1 == k*k2 (mod 8L), k2 odd, both ~2^128 (half-size scalars, ~128
   doublings); the verdict equals the reference's [S]B - [k]A == R bit for
   bit.  set_halfsize(ctx, 0) runs every signature with the full-length pair
   (k, 1) instead (252 doublings): an A/B and test switch, same results. */
void                   fd_ed25519_hip_set_halfsize( fd_ed25519_hip_ctx_t * ctx, int on );

/* Calls of at most max_n records (default 32, at most 256) whose count is
   known on the host run on the latency path: one workgroup of three waves per
   signature (the A and R decodes, the hash, and the [k1]A, [k2]R and B terms
   run side by side; each signature races copies on other CUs, up to 16 and
   one workgroup per CU over the call, as far as the context's budget,
   fd_ed25519_hip_set_lat_cus, allows), instead of one lane per signature
   through k_verify_prep / k_verify_dsm.  Same verdicts and
   codes; 0 sends every call to the bulk kernels.  The drop-in entry points
   run on their own batch-slot contexts.  A latency call's n x copies
   workgroups each hold a quarter of a CU until they end (a 32-record call
   with 8 copies: 256 workgroups for ~0.5 ms), so a context whose small calls
   share the GPU with throughput work on other streams should lower the
   limit or set 0. */
void                   fd_ed25519_hip_set_small_batch( fd_ed25519_hip_ctx_t * ctx, ulong max_n );

/* k_verify_lat workgroup slots a latency-path call may fill with racing
   copies (default: all of them, 4 per CU; the drop-in's batch slots each get
   1/slots, and take calls of up to that many records, at most 256, on the
   latency path): a call of n records runs min(cus / n, 16, CUs / n) copies
   of each signature, at least one. */
void                   fd_ed25519_hip_set_lat_cus( fd_ed25519_hip_ctx_t * ctx, ulong cus );

/* Recreates the context's stream restricted to the CUs whose bits are set in
   mask[0..words) (hipExtStreamCreateWithCUMask numbering; words 0: all CUs
   again).  Work already queued on the old stream is drained first.  Returns
   0, or -1 if the runtime refused the mask.  A masked stream is a BLOCKING
   stream (hipExtStreamCreateWithCUMask takes no flags): unlike the default
   non-blocking context stream it synchronises with work on the null stream
   (e.g. torch's legacy default stream), so keep such work off the null
   stream while a masked context is busy. */
int                    fd_ed25519_hip_ctx_set_cu_mask( fd_ed25519_hip_ctx_t * ctx, uint const * mask, uint words );

/* k_verify_dsm runs a persistent grid sized to every resident workgroup
   slot of the GPU.  share > 1 sizes it to 1/share of them, so that that
   many contexts' DSM launches (verify tiles on other streams) run side by
   side and fill each other's tails instead of queueing whole-GPU grids.
   Default 1; same verdicts. */
void                   fd_ed25519_hip_set_dsm_share( fd_ed25519_hip_ctx_t * ctx, ulong share );

/* Leave `reserve` of the GPU's resident k_verify_dsm workgroup slots free
   while this context's DSM runs (room for other streams' kernels beside
   it: the verify service's IO kernels).  At most half
   the slots are reserved; a larger value is clamped, said once on stderr,
   and 1 is returned (0 otherwise, -1 for a NULL ctx).  The environment's
   FD_ED25519_HIP_DSM_RESERVE, if set, is applied to every new context. */
int                    fd_ed25519_hip_ctx_set_dsm_reserve( fd_ed25519_hip_ctx_t * ctx, ulong reserve );

/* Test hook: the device half-size reduction of n scalars k < L (d_k: 8 LE
   u32 words each) into d_out (18 words each: |k1| (8), k2 (8), k1 < 0 ? ~0 :
   0, max bit length).  Asynchronous on stream. */
int fd_ed25519_hip_test_halfsize( fd_ed25519_hip_ctx_t * ctx, ulong n, uint const * d_k, uint * d_out,
                                  void * stream );

/* Test hook: one device primitive over n items; d_in and d_out hold 32 u32
   words per item.  Field elements are 9 limbs, value = sum v[i]*2^(29 i),
   at words 0..8 (a) and 9..17 (b) of the input.  Ops and outputs:
     FE_MUL a*b, FE_SQ a^2 (tight limbs, 0..8); FE_MUL2 a*b, b*a and FE_SQ2
     a^2, b^2 (two products run interleaved, 0..8 and 9..17); FE_CANON a
     canonical (limbs < 2^32-8); FE_FROMWORDS of input words 0..7 (32 LE
     bytes, bit 255 masked); FE_SUB a-b canonical (b tight); FE_POW22523
     a^(2^252-3) and FE_INVERT a^(p-2), canonical (fd_f25519.c:25-74);
     GE_DECODE of input words 0..7 (fd_ed25519_point_frombytes with the
     AVX-512 failure split): word 0 flags (bit 0 not on the curve, bit 1
     x==0 with the sign bit set), word 1 small order
     (fd_ed25519_affine_is_small_order), words 2..9 x, 10..17 y (canonical
     LE); SC_REDUCE of 16 input words mod L (fd_curve25519_scalar_reduce);
     SC_CANONICAL word 0 = input words 0..7 < L (scalar_validate).
   Returns -1 for an unknown op.  Asynchronous on stream. */
#define FD_ED25519_HIP_PRIM_FE_MUL        0
#define FD_ED25519_HIP_PRIM_FE_SQ         1
#define FD_ED25519_HIP_PRIM_FE_MUL2       2
#define FD_ED25519_HIP_PRIM_FE_SQ2        3
#define FD_ED25519_HIP_PRIM_FE_CANON      4
#define FD_ED25519_HIP_PRIM_FE_FROMWORDS  5
#define FD_ED25519_HIP_PRIM_FE_SUB        6
#define FD_ED25519_HIP_PRIM_FE_POW22523   7
#define FD_ED25519_HIP_PRIM_FE_INVERT     8
#define FD_ED25519_HIP_PRIM_GE_DECODE     9
#define FD_ED25519_HIP_PRIM_SC_REDUCE    10
#define FD_ED25519_HIP_PRIM_SC_CANONICAL 11
int fd_ed25519_hip_test_prim( fd_ed25519_hip_ctx_t * ctx, int op, ulong n, uint const * d_in, uint * d_out,
                              void * stream );

/* Test hook: plain SHA-512 (fd_sha512_init/append/fini, fd_sha512.c:264-399)
   of n messages d_pool[ d_msg_off[i], +d_msg_sz[i] ) with both device hash
   paths: the per-lane one (sha512_prefixed: signing) writes 64-byte digests
   to d_out + 64*i, the wave-cooperative LDS-staged one k_verify_prep uses
   (sha512_prefixed_coop) to d_out + 64*(n+i).  d_out holds 128*n bytes,
   16-byte aligned.  Asynchronous on stream. */
int fd_ed25519_hip_test_sha512( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_pool, uint const * d_msg_off,
                                uint const * d_msg_sz, uchar * d_out, void * stream );

/* Kernel timing for measurement legs: when on, every verify chunk brackets
   k_verify_prep and k_verify_dsm with HIP events on the launch stream and
   accumulates their durations (this serialises the host per chunk).
   set_timing also resets the accumulators. */
void fd_ed25519_hip_set_timing( fd_ed25519_hip_ctx_t * ctx, int on );
void fd_ed25519_hip_get_timing( fd_ed25519_hip_ctx_t const * ctx, double * prep_ms, double * dsm_ms,
                                ulong * launches );
/* signatures that passed every pre-check and ran through k_verify_dsm,
   accumulated while timing is on (the unit of the DSM roofline) */
ulong fd_ed25519_hip_get_dsm_units( fd_ed25519_hip_ctx_t const * ctx );

/* Per-signature verify, inputs resident in HBM, asynchronous on `stream`
   (NULL: the context's stream).  bitmap may be NULL.  Returns 0. */
int
fd_ed25519_hip_verify_dev( fd_ed25519_hip_ctx_t * ctx,
                           ulong                  n,
                           uchar const *          d_sigs,
                           uchar const *          d_pubs,
                           uchar const *          d_pool,
                           uint const *           d_msg_off,
                           uint const *           d_msg_sz,
                           signed char *          d_codes,
                           ulong *                d_bitmap,
                           void *                 stream );

/* Same with the record count in device memory (e.g. written by a preceding
   kernel): verifies records [0, min(n_max, *d_n)) without a host round trip;
   codes (and bitmap bits) at or past *d_n are left untouched.  The launch
   covers n_max records (ceil(n_max/chunk_sigs) chunk launches; threads past
   the count exit at once). */
int
fd_ed25519_hip_verify_dev_count( fd_ed25519_hip_ctx_t * ctx,
                                 ulong                  n_max,
                                 uint const *           d_n,
                                 uchar const *          d_sigs,
                                 uchar const *          d_pubs,
                                 uchar const *          d_pool,
                                 uint const *           d_msg_off,
                                 uint const *           d_msg_sz,
                                 signed char *          d_codes,
                                 ulong *                d_bitmap,
                                 void *                 stream );

/* Fixed-size messages laid out back to back: message i = d_msgs[ i*msg_sz,
   (i+1)*msg_sz ) (e.g. 32-byte shred Merkle roots, fd_fec_resolver.c:476).
   Same semantics and requirements as fd_ed25519_hip_verify_dev (d_msgs
   readable 16 bytes past its end). */
int
fd_ed25519_hip_verify_fixed_dev( fd_ed25519_hip_ctx_t * ctx,
                                 ulong                  n,
                                 uchar const *          d_sigs,
                                 uchar const *          d_pubs,
                                 uchar const *          d_msgs,
                                 uint                   msg_sz,
                                 signed char *          d_codes,
                                 ulong *                d_bitmap,
                                 void *                 stream );

/* Same from host memory, synchronous (copies in/out over PCIe).  Returns 0,
   or -1 without touching the GPU if a message lies outside [0, pool_sz). */
int
fd_ed25519_hip_verify_host( fd_ed25519_hip_ctx_t * ctx,
                            ulong                  n,
                            uchar const *          sigs,
                            uchar const *          pubs,
                            uchar const *          pool,
                            ulong                  pool_sz,
                            uint const *           msg_off,
                            uint const *           msg_sz,
                            signed char *          codes,
                            ulong *                bitmap );

/* Group reduction with fd_ed25519_verify_batch_single_msg semantics: group g
   covers signatures [first[g], first[g]+cnt[g]) of a preceding verify; its
   code is ERR_SIG if cnt is 0 or >16, else the first ERR_SIG/ERR_PUBKEY in
   order, else ERR_MSG if any signature failed its equation, else SUCCESS.
   Device pointers, asynchronous on `stream`. */
int
fd_ed25519_hip_group_reduce_dev( fd_ed25519_hip_ctx_t * ctx,
                                 ulong                  n_groups,
                                 uint const *           d_first,
                                 uchar const *          d_cnt,
                                 signed char const *    d_sig_codes,
                                 signed char *          d_group_codes,
                                 void *                 stream );

/* Key generation + signing on the GPU (synthetic workloads, fd_ed25519_user.c
   :4-133 semantics; NOT hardened against side channels: do not use with
   secrets you care about).  prvs 32*n, writes pubs 32*n and sigs 64*n.
   Device pointers, asynchronous on `stream`. */
int
fd_ed25519_hip_sign_dev( fd_ed25519_hip_ctx_t * ctx,
                         ulong                  n,
                         uchar const *          d_prvs,
                         uchar const *          d_pool,
                         uint const *           d_msg_off,
                         uint const *           d_msg_sz,
                         uchar *                d_pubs,
                         uchar *                d_sigs,
                         void *                 stream );

/* Pinned host memory mapped into every device's address space (hipHostMalloc
   mapped|portable): kernels read and write it in place over PCIe at the same
   address, so a verify tile's in-link dcache placed here is ingested by the
   GPU with no copy (fd_verify_hip_tile_submit_frags).  Aborts on failure. */
void * fd_ed25519_hip_host_alloc( ulong sz );
void   fd_ed25519_hip_host_free ( void * p );

/* Map existing host memory (e.g. a tile's out-link dcache in its
   workspace) for device access: page-locks [p, p+sz) and returns the
   address kernels use for it (NULL for a NULL or empty range).  Call it
   before the sandbox is up (privileged_init).  Aborts on failure. */
void * fd_ed25519_hip_host_register  ( void * p, ulong sz );
void   fd_ed25519_hip_host_unregister( void * p );

/* Enqueue a host->device copy of sz bytes on stream (NULL: the context's
   stream), e.g. a verify tile's in-link dcache region staged into HBM ahead
   of fd_verify_hip_tile_submit_frags.  With h_src from
   fd_ed25519_hip_host_alloc the copy is a DMA transfer that returns at once;
   the caller keeps h_src unchanged until the stream has passed the copy. */
int fd_ed25519_hip_stage_async( fd_ed25519_hip_ctx_t * ctx, void * d_dst, void const * h_src, ulong sz,
                                void * stream );

/* Blocks until all work queued on the context's stream is done. */
int fd_ed25519_hip_sync( fd_ed25519_hip_ctx_t * ctx );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_ed25519_hip_h */
