#ifndef HEADER_fd_verify_hip_h
#define HEADER_fd_verify_hip_h

/* fd_verify_hip.h -- C ABI of the verify-tile layer of the MI355X engine
   (verify-tile integration and GPU txn parse).

   It takes the verify tile's raw frags (UDP payloads, fd_txn_m_payload) in
   device memory and reproduces, for a batch of frags in arrival order, what
   the reference verify tile does per frag:

     after_frag     src/disco/verify/fd_verify_tile.c:101-161
                    fd_txn_parse -> bundle bookkeeping -> fd_txn_verify ->
                    publish / count the failure
     fd_txn_verify  src/disco/verify/fd_verify_tile.h:61-111
                    tag = fd_hash(seed, sig0, 64); tcache query (dedup);
                    fd_ed25519_verify_batch_single_msg over the txn's
                    signatures; tcache insert

   Work split (MI355X-first):
     GPU  k_txn_parse   one lane per frag: fd_txn_parse_core restated
                        (fd_txn_parse.c:7-254), fd_txn_t written out, sig0
                        tag (fd_hash, util/fd_hash.c:14-72)
          k_txn_expand  wave-aggregated slot allocation, txn -> signature
                        records (sig, pubkey, message span)
          verify        fd_ed25519_hip_verify_dev over all records
          group reduce  fd_ed25519_verify_batch_single_msg per txn
     host the order-dependent part: the tcache (dedup) and the bundle state
          machine, over 11 bytes per frag, in arrival order.  The tcache is
          the reference's own memory layout (fd_tcache.h), so a verify tile
          can hand its ctx->tcache_{sync,ring,map} to the engine.

   Every verdict equals the reference's sequential per-frag result: a frag
   the reference would drop before verifying (dedup hit, failed bundle peer)
   is verified here too and the extra verdict discarded.

   Library: firedancer_amd/libfd_ed25519_hip.so (same library as
   fd_ed25519_hip.h).  No torch or HIP types in any signature. */

#include "fd_ed25519_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned short ushort;

/* fd_txn.h:60,65 */
#define FD_TXN_HIP_MAX_SZ  852UL    /* FD_TXN_MAX_SZ: out stride of the parse */
#define FD_TXN_HIP_MTU     1232UL   /* FD_TXN_MTU */

/* fd_verify_tile.h:9-11 */
#define FD_TXN_VERIFY_SUCCESS  0
#define FD_TXN_VERIFY_FAILED  -1
#define FD_TXN_VERIFY_DEDUP   -2

/* Per-frag outcome of after_frag.  PUBLISH / FAILED / DEDUP are
   fd_txn_verify's codes; the two others are the early returns of
   after_frag (fd_verify_tile.c:125-134), each with its metric. */
#define FD_VERIFY_HIP_FRAG_PUBLISH      ( 0)
#define FD_VERIFY_HIP_FRAG_VERIFY_FAIL  (-1)   /* metrics.verify_fail_cnt      */
#define FD_VERIFY_HIP_FRAG_DEDUP        (-2)   /* metrics.dedup_fail_cnt       */
#define FD_VERIFY_HIP_FRAG_PARSE_FAIL   (-3)   /* metrics.parse_fail_cnt       */
#define FD_VERIFY_HIP_FRAG_BUNDLE_PEER  (-4)   /* metrics.bundle_peer_fail_cnt */
#define FD_VERIFY_HIP_FRAG_OVERRUN      (-5)   /* skipped by complete_skip: the stem's overrun (no after_frag) */

/* ---- verify-tile frag formats (x86-64 layouts of the reference structs;
   tests/test_ref_layout.py checks every offset against the reference headers
   with offsetof) -------------------------------------------------------- */

/* fd_txn_m_t (src/disco/fd_txn_m.h:15-61): 80-byte header, then payload[],
   then the fd_txn_t at fd_txn_m_txn_t (:101-104) */
#define FD_VERIFY_HIP_TXNM_SZ               80u   /* sizeof(fd_txn_m_t)              */
#define FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF    8u   /* ushort payload_sz               */
#define FD_VERIFY_HIP_TXNM_TXN_T_SZ_OFF     10u   /* ushort txn_t_sz                 */
#define FD_VERIFY_HIP_TXNM_SRC_IPV4_OFF     12u   /* uint   source_ipv4              */
#define FD_VERIFY_HIP_TXNM_SRC_TPU_OFF      16u   /* uchar  source_tpu               */
#define FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF    24u   /* ulong  block_engine.bundle_id   */
#define FD_VERIFY_HIP_TXN_ALIGN              2u   /* alignof(fd_txn_t)               */
#define FD_VERIFY_HIP_TPU_RAW_MTU         1312u   /* FD_TPU_RAW_MTU (fd_txn_m.h:139) */
#define FD_VERIFY_HIP_TPU_SOURCE_GOSSIP      3u   /* FD_TXN_M_TPU_SOURCE_GOSSIP      */

/* fd_gossip_update_message_t carrying a vote (src/flamenco/gossip/
   fd_gossip_types.h:136-141,191-212) */
#define FD_VERIFY_HIP_GOSSIP_UPDATE_TAG_VOTE  3u  /* FD_GOSSIP_UPDATE_TAG_VOTE       */
#define FD_VERIFY_HIP_GOSSIP_VOTE_ADDR_OFF   56u  /* vote.socket.addr (uint)         */
#define FD_VERIFY_HIP_GOSSIP_VOTE_TXN_SZ_OFF 72u  /* vote.txn_sz (ulong)             */
#define FD_VERIFY_HIP_GOSSIP_VOTE_TXN_OFF    80u  /* vote.txn[1232]                  */

/* in-link kinds (fd_verify_tile.c:7-10) */
#define FD_VERIFY_HIP_IN_QUIC   0u
#define FD_VERIFY_HIP_IN_BUNDLE 1u
#define FD_VERIFY_HIP_IN_GOSSIP 2u
#define FD_VERIFY_HIP_IN_SEND   3u
/* or'd into a QUIC / BUNDLE / SEND kind: the host tile did during_frag's
   copy into the frag's out chunk itself (a frag of a link the GPU does not
   map); d_in_chunk[j] is ignored and the frag is parsed in place (GOSSIP |
   HOSTCOPY: the host converted the vote into an fd_txn_m_t already; it
   still counts as a gossiped vote). */
#define FD_VERIFY_HIP_IN_HOSTCOPY 0x80u

/* before_frag (fd_verify_tile.c:37-58) on the host: 1 = this tile skips
   the frag (round robin over verify tiles by seq; bundles to tile 0;
   gossip frags other than votes), 0 = it takes it. */
int
fd_verify_hip_before_frag( uint in_kind, ulong seq, ulong sig, ulong round_robin_cnt, ulong round_robin_idx );

/* ---- GPU txn parse ------------------------------------------------------

   Parses n payloads: payload j = d_pool[ d_txn_off[j], +d_txn_sz[j] ).
   d_txn_t_sz[j] = fd_txn_parse( payload, sz, out, NULL ) (the fd_txn_t
   footprint 20+10*instr_cnt+8*lut_cnt, or 0 on a parse failure);
   replaces fd_txn_parse / fd_txn_parse_core with instr_max =
   FD_TXN_INSTR_MAX (fd_txn.h:712-715, fd_txn_parse.c:7-254).
   d_txn_out (may be NULL) receives each fd_txn_t at stride
   FD_TXN_HIP_MAX_SZ, bytes identical to the reference's output (only the
   first d_txn_t_sz[j] bytes are defined).  Async on stream (NULL: the
   ctx's stream). */
int
fd_txn_hip_parse_dev( fd_ed25519_hip_ctx_t * ctx,
                      ulong                  n,
                      uchar const *          d_pool,
                      uint const *           d_txn_off,
                      ushort const *         d_txn_sz,
                      uchar *                d_txn_out,
                      ushort *               d_txn_t_sz,
                      void *                 stream );

/* fd_hash (util/fd_hash.c:14-72) on the host, for callers that need the
   same tag the engine computes on the GPU. */
ulong
fd_verify_hip_hash( ulong seed, void const * buf, ulong sz );

/* ---- tcache on the reference layout (fd_tcache.h:115-410) ---------------

   ring[depth], map[map_cnt] (power of 2, >= depth+2), oldest in [0,depth).
   Same memory effects as fd_tcache_reset / FD_TCACHE_QUERY /
   FD_TCACHE_INSERT, so the arrays stay interchangeable with the
   reference's.  Tag 0 is the null tag (a query for it always "finds"). */
ulong fd_verify_hip_tcache_map_cnt_default( ulong depth );
ulong fd_verify_hip_tcache_reset ( ulong * ring, ulong depth, ulong * map, ulong map_cnt );
int   fd_verify_hip_tcache_query ( ulong const * map, ulong map_cnt, ulong tag );
int   fd_verify_hip_tcache_insert( ulong * oldest, ulong * ring, ulong depth,
                                   ulong * map, ulong map_cnt, ulong tag );

/* ---- verify tile engine --------------------------------------------------

   A tile owns device scratch for up to max_txn frags per batch (two batches
   in flight), a tcache (internal, or joined from the caller), the bundle
   state and the metrics.  It runs on ctx's device and stream.

     submit(k)   enqueues parse, expand, verify and per-txn reduce of batch k
                 and returns without waiting on the GPU (the signature count
                 stays on the device and sizes the verify there);
     complete(k) waits for batch k and runs the ordered host pass, writing
                 result[j] (FD_VERIFY_HIP_FRAG_*), tag[j] (opt_sig on
                 publish, else 0) and txn_t_sz[j] (parse footprint).

   Pipelined use: submit(0); for k: submit(k+1); complete(k).  The host pass
   of batch k then overlaps the GPU work of batch k+1.  Batches must be
   completed in submission order; at most two may be outstanding.
   Payload memory (d_pool, offsets, sizes, d_txn_out) must stay valid until
   the batch completes.  bundle_id (host, NULL: none) is given at completion,
   it only affects the ordered pass. */

typedef struct fd_verify_hip_tile fd_verify_hip_tile_t;

fd_verify_hip_tile_t *
fd_verify_hip_tile_new( fd_ed25519_hip_ctx_t * ctx,
                        ulong                  max_txn,
                        ulong                  hashmap_seed,   /* fd_verify_ctx_t.hashmap_seed */
                        ulong                  tcache_depth,   /* tile->verify.tcache_depth    */
                        ulong                  tcache_map_cnt );/* 0: fd_tcache_map_cnt_default */

/* Use the caller's tcache (fd_verify_ctx_t tcache_sync/ring/depth/map/map_cnt,
   fd_verify_tile.c:196-200) instead of the tile's own from now on. */
void
fd_verify_hip_tile_join_tcache( fd_verify_hip_tile_t * tile, ulong * sync, ulong * ring, ulong depth,
                                ulong * map, ulong map_cnt );

void fd_verify_hip_tile_tcache_reset( fd_verify_hip_tile_t * tile );

/* Replace hashmap_seed for batches submitted from now on (the reference
   draws it once per tile boot, fd_verify_tile.c:170; a new seed gives the
   same traffic fresh tags, which the bench uses to replay one batch). */
void fd_verify_hip_tile_set_seed( fd_verify_hip_tile_t * tile, ulong hashmap_seed );
void fd_verify_hip_tile_delete( fd_verify_hip_tile_t * tile );

int
fd_verify_hip_tile_submit( fd_verify_hip_tile_t * tile,
                           ulong                  n,
                           uchar const *          d_pool,
                           uint const *           d_txn_off,
                           ushort const *         d_txn_sz,
                           uchar *                d_txn_out );   /* NULL or n*FD_TXN_HIP_MAX_SZ */

/* The verify tile's own frag format: n frags (those before_frag kept, in
   arrival order) in the in-link dcache, frag j's sz bytes at
   d_in + 64*d_in_chunk[j] (fd_chunk_to_laddr), kind d_in_kind[j]
   (FD_VERIFY_HIP_IN_*).  Per frag the GPU does during_frag
   (fd_verify_tile.c:64-99) into the out dcache at d_out + 64*d_out_chunk[j]
   -- the copy of a QUIC/BUNDLE/SEND fd_txn_m_t frag, or the conversion of a
   gossip vote message into one -- then after_frag's parse (:118-120): the
   fd_txn_t at fd_txn_m_txn_t and txn_t_sz into the header.  bundle_id comes
   from each header (complete's bundle_id argument is ignored for such a
   batch) and GOSSIP/SEND frags count into gossiped_votes_cnt (:112).
   A QUIC/BUNDLE/SEND frag whose in and out addresses are the same, or whose
   kind carries FD_VERIFY_HIP_IN_HOSTCOPY, is parsed in place (no copy): a
   host tile that keeps during_frag's copy into its out dcache passes in =
   out, or the flag for the frags it copied while the GPU copies the others
   from d_in (integration/fd_verify_tile_hip.patch, FD_VERIFY_HIP_GPU_COPY).
   A corrupt frag (sz > FD_TPU_RAW_MTU, or > 2048 for gossip; payload_sz >
   FD_TPU_MTU) aborts the process in complete(), as the reference's
   FD_LOG_ERR ends the tile.  All pointers are device-visible (HBM, or
   pinned host memory mapped to the device); chunks are 64-byte units, so
   an out chunk must hold FD_TPU_PARSED_MTU bytes. */
int
fd_verify_hip_tile_submit_frags( fd_verify_hip_tile_t * tile,
                                 ulong                  n,
                                 uchar const *          d_in,
                                 uint const *           d_in_chunk,
                                 ushort const *         d_in_sz,
                                 uchar const *          d_in_kind,
                                 uchar *                d_out,
                                 uint const *           d_out_chunk );

/* mcache range mode: the tile reads an unpolled quic_verify link
   (FD_TOPOB_UNPOLLED; integration/fd_verify_topo_hip.patch) by whole
   published seq ranges instead of one stem frag at a time.  The GPU reads
   the link's mcache lines [seq0, seq0+seq_cnt) (fd_frag_meta_t, 32 B:
   seq, sig, chunk, sz, ctl, tsorig, tspub), keeps before_frag's round
   robin share (seq % rr_cnt == rr_idx, fd_verify_tile.c:37-58), checks
   each as the stem and during_frag do (the line still holds seq; chunk in
   [chunk0, wmark]; sz <= FD_TPU_RAW_MTU, :74-76) and ingests the kept
   frags as submit_frags does, from d_in + 64*(chunk - chunk_off).  Kept
   frag j (seq first + j*rr_cnt) goes to out chunk d_out_chunk[j]
   (fd_verify_hip_range_frag_cnt of them).

   The caller submits only seqs it saw published (the line of the range's
   last seq holding that seq), and after the batch does the stem's overrun
   check: if the line of the range's first kept seq no longer holds it,
   each kept frag whose line was reused is skipped (complete_range's skip).
   A line the GPU found reused or corrupt flags the batch corrupt; with no
   frag skipped that aborts in complete, as during_frag's FD_LOG_ERR ends
   the tile.  mcache and d_in are device-visible (the link's mcache and
   dcache registered with fd_ed25519_hip_host_register).  -1 for a bad
   range (depth not a power of 2, seq_cnt > depth, rr_idx >= rr_cnt,
   chunk0 outside [chunk_off, wmark]), -2 while every slot is busy, -1 if
   the share exceeds the tile's max_txn. */
typedef struct {
  void const * mcache;          /* device address of line 0 */
  ulong        depth;           /* lines (power of 2) */
  ulong        seq0, seq_cnt;   /* the range */
  ulong        rr_cnt, rr_idx;  /* before_frag's round robin */
  ulong        chunk_off;       /* link chunk of d_in's first byte (64-byte units from the link's wksp) */
  ulong        chunk0, wmark;   /* during_frag's chunk range (fd_dcache_compact_chunk0 / _wmark) */
} fd_verify_hip_range_t;

/* kept seqs of [seq0, seq0+seq_cnt): seq % rr_cnt == rr_idx */
static inline ulong
fd_verify_hip_range_frag_cnt( ulong seq0, ulong seq_cnt, ulong rr_cnt, ulong rr_idx ) {
  if( !seq_cnt || !rr_cnt || rr_idx>=rr_cnt ) return 0UL;
  ulong first = seq0 + ( rr_idx + rr_cnt - seq0 % rr_cnt ) % rr_cnt;
  ulong end   = seq0 + seq_cnt;
  return first<end ? ( end - 1UL - first )/rr_cnt + 1UL : 0UL;
}

int
fd_verify_hip_tile_submit_range( fd_verify_hip_tile_t *        tile,
                                 fd_verify_hip_range_t const * range,
                                 uchar const *                 d_in,
                                 uchar *                       d_out,
                                 uint const *                  d_out_chunk );

/* complete_skip for any frag batch, and for a range batch each kept
   frag's mcache tsorig (NULL: not wanted; -1 if wanted from a batch that
   is not a range).  txn_t_sz / payload_sz as in complete_skip (NULL: not
   wanted). */
int
fd_verify_hip_tile_complete_range( fd_verify_hip_tile_t * tile,
                                   uchar const *          skip,         /* host, n (NULL: none skipped) */
                                   signed char *          result,       /* host, n */
                                   ushort *               txn_t_sz,     /* host, n or NULL */
                                   ushort *               payload_sz,   /* host, n or NULL */
                                   uint *                 tsorig );     /* host, n or NULL */

/* Non-blocking: 1 if the oldest outstanding batch has finished on the GPU
   (complete() will not wait), 0 if it is still running, -1 if no batch is
   outstanding.  A stem loop polls from after_credit and calls complete()
   only on 1, so its in-links keep draining while the GPU works
   (integration/fd_verify_tile_hip.patch). */
int
fd_verify_hip_tile_poll( fd_verify_hip_tile_t const * tile );

/* batches submitted and not yet completed (at most the in-flight limit) */
ulong
fd_verify_hip_tile_inflight( fd_verify_hip_tile_t const * tile );

/* Batches the tile keeps on the GPU at once (1..FD_VERIFY_HIP_INFLIGHT_MAX;
   2 for a new tile, both on ctx's stream, run back to back): submit returns
   -2 while that many are outstanding.  After set_inflight every slot past
   the first runs on a verify context (stream and scratch) of its own, on
   ctx's device, so the batches in flight run concurrently: a batch's GPU
   time is nearly independent of its size until it fills the GPU.
   Allocates and warms the slots (call from privileged_init: device memory
   for 12 records per frag of max_txn in each).  -1 if k is out of range or
   batches are outstanding.  Results still complete in submission order. */
#define FD_VERIFY_HIP_INFLIGHT_MAX 8
int
fd_verify_hip_tile_set_inflight( fd_verify_hip_tile_t * tile, ulong k );

/* Out staging, for an out dcache in pinned host memory (the tile's
   verify_dedup link).  With it on, a frag batch's kernels work on staging
   frags in HBM -- during_frag's copy, the fd_txn_t, the messages the verify
   hashes -- and one kernel then writes the out dcache with coalesced
   stores, exactly the bytes the reference writes there (the copy,
   txn_t_sz and the fd_txn_t; for a gossip vote its header fields and
   payload); every other out byte keeps its value.  Without it the kernels
   read and write the out dcache in place: over PCIe that is a small write
   per fd_txn_t field and a small read per message piece.  Allocates
   max_txn x 2176 B of HBM per slot (call from privileged_init).  -1 with
   batches outstanding, or to turn it on under FD_VERIFY_HIP_INGEST=split. */
int
fd_verify_hip_tile_set_staging( fd_verify_hip_tile_t * tile, int on );

/* fd_ed25519_hip_ctx_set_cu_mask on every slot context of the tile: its
   batches run on the CUs the mask names (words = 0: all of them again).
   For tiles that share a GPU, each on its own CUs.  -1 with batches
   outstanding or if the runtime refuses the mask.  A masked stream is a
   blocking stream (fd_ed25519_hip.h). */
int
fd_verify_hip_tile_set_cu_mask( fd_verify_hip_tile_t * tile, uint const * mask, uint words );

int
fd_verify_hip_tile_complete( fd_verify_hip_tile_t * tile,
                             ulong const *          bundle_id,   /* host, n entries or NULL */
                             signed char *          result,      /* host, n */
                             ulong *                tag,         /* host, n or NULL */
                             ushort *               txn_t_sz );  /* host, n or NULL */

/* complete() for a frag batch of which the caller found some frags overrun
   after the GPU read them (skip[j] != 0: the in-link's mcache line of the
   frag's seq was overwritten by then, so its bytes may be a later frag's --
   the GPU-copy form of the stem's overrun check after during_frag,
   integration/fd_verify_tile_hip.patch FD_VERIFY_HIP_GPU_COPY).  A skipped
   frag gets FD_VERIFY_HIP_FRAG_OVERRUN and is invisible to the ordered pass
   (no tcache query or insert, no bundle state, no metric), as a frag the
   stem drops never reaches after_frag.  A batch with a skipped frag does
   not abort on the corrupt-frag flag (the corrupt bytes may be the
   overrun's; a corrupt frag that is not skipped parses as a parse failure
   and is not published).  payload_sz[j] is the frag's out header
   payload_sz after the GPU's during_frag (for fd_txn_m_realized_footprint
   without reading the header back).  Frag batches only: -1 for a
   fd_verify_hip_tile_submit batch. */
int
fd_verify_hip_tile_complete_skip( fd_verify_hip_tile_t * tile,
                                  uchar const *          skip,         /* host, n (NULL: none skipped) */
                                  signed char *          result,       /* host, n */
                                  ulong *                tag,          /* host, n or NULL */
                                  ushort *               txn_t_sz,     /* host, n or NULL */
                                  ushort *               payload_sz ); /* host, n or NULL */

/* metrics (cumulative): out[0..3] = parse_fail, verify_fail, dedup_fail,
   bundle_peer_fail (fd_verify_tile.h:51-57); out[4] = published,
   out[5] = signatures sent to the GPU verify.  metrics2 adds out[6] =
   gossiped_votes (GOSSIP/SEND frags, fd_verify_tile.c:33,112); the 6-slot
   form keeps the layout of ABI version 1. */
#define FD_VERIFY_HIP_ABI_VERSION 2
void fd_verify_hip_tile_metrics ( fd_verify_hip_tile_t const * tile, ulong out[ 6 ] );
void fd_verify_hip_tile_metrics2( fd_verify_hip_tile_t const * tile, ulong out[ 7 ] );

/* timing of the last completed batch (ms): out[0] = GPU (first kernel to
   results on host, HIP events), out[1] = host ordered pass, out[2] =
   signatures in the batch */
void fd_verify_hip_tile_last_timing( fd_verify_hip_tile_t const * tile, double out[ 3 ] );

/* Frag-ingest kernel accounting (submit_frags batches; the north star's
   "achieved HBM GB/s on packet ingest").  set_ingest_timing( tile, 1 )
   brackets each batch's ingest kernel (k_txnm_batch: copy, parse, record
   expansion) with HIP events on the tile's stream; ingest_stats then
   reports, for the last completed batch:
     out[0] kernel time (ms; 0 when timing is off)
     out[1] frags
     out[2] algorithmic bytes: in-frag bytes read + out-frag bytes written
            (during_frag's copy) + fd_txn_t and txn_t_sz written (after_frag)
            + signature records written (96 B + 8 B of message span each)
            + per-frag results (23 B)
     out[3] signature records */
void fd_verify_hip_tile_set_ingest_timing( fd_verify_hip_tile_t * tile, int on );
void fd_verify_hip_tile_ingest_stats     ( fd_verify_hip_tile_t const * tile, double out[ 4 ] );

/* Batch latency histograms (SURVEY: the tile's counters plus GPU batch
   latency), laid out as the reference's fd_histf (src/util/hist/fd_histf.h:
   16 buckets: [0,min), roughly geometric integer edges from min to max, and
   [max,inf)), in nanoseconds, one sample per completed batch:
     which = 0: GPU time (first kernel to results on the host, HIP events);
     which = 1: the host ordered pass.
   hist_init resets both with the edges fd_histf_new( min_ns, max_ns ) would
   give (-1 if max_ns <= min_ns); a new tile starts at 10 us .. 1 s.
   hist copies out counts, left edges and the sum of the samples (NULL: skip);
   -1 for another which.  hist_edges is the edge rule alone. */
#define FD_VERIFY_HIP_HIST_BUCKET_CNT 16
int fd_verify_hip_hist_edges    ( ulong min_v, ulong max_v, ulong edge[ 16 ] );
int fd_verify_hip_tile_hist_init( fd_verify_hip_tile_t * tile, ulong min_ns, ulong max_ns );
int fd_verify_hip_tile_hist     ( fd_verify_hip_tile_t const * tile, int which, ulong counts[ 16 ],
                                  ulong left_edge_ns[ 16 ], ulong * sum_ns );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_verify_hip_h */
