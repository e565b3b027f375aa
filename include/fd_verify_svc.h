#ifndef HEADER_fd_verify_svc_h
#define HEADER_fd_verify_svc_h

/* fd_verify_svc.h -- the per-GPU verify service: sandboxed verify tiles
   without HIP, one GPU-owner process per GPU.

   Why.  A verify tile that creates a HIP context in privileged_init
   (integration/fd_verify_tile_hip.patch, the direct form) is multithreaded
   from then on, so fd_sandbox_enter's unshare( CLONE_NEWUSER )
   (src/util/sandbox/fd_sandbox.c:649) fails and seccomp covers only the
   tile thread; and each tile's batches are tile-sized (~55 K signatures),
   too small to fill the GPU.  Here the tiles keep
   the reference's process model -- one thread, the reference's seccomp
   policy (fd_verify_tile.seccomppolicy: write and fsync only), no device
   fds -- and one GPU tile per GPU owns the context and merges the requests
   of every tile it serves into large launches.

   Processes.
     verify tile   src/disco/verify/fd_verify_tile.c with
                   integration/fd_verify_tile_svc.patch.  Posts requests,
                   runs the order-dependent part of after_frag (the tcache
                   dedup and the bundle state, fd_verify_tile.c:101-161,
                   fd_verify_tile.h:61-111) on the results, assigns out
                   chunks exactly as after_frag does (fd_dcache_compact_next
                   by realized size, on publish only), asks the service to
                   write the published frags, publishes them.  Everything
                   here is loads and stores on shared memory: no syscall.
     GPU tile      integration/fd_verify_gpu_tile.c around fd_verify_svc_*
                   (libfd_ed25519_hip.so): the HIP context, the
                   quic_verify links' mcache and dcache and the tiles'
                   verify_dedup dcaches registered for the GPU.

   Per request (one tile's batch) the GPU does what the reference tile does
   per frag up to the tcache: before_frag's round robin and during_frag's
   checks and copy (range requests read the unpolled quic_verify link's
   mcache lines), after_frag's fd_txn_parse, fd_txn_verify's tag
   (fd_hash( seed, sig0, 64 )) and fd_ed25519_verify_batch_single_msg.
   The out frags wait in HBM (staging) until the tile has decided which are
   published; a flush then writes exactly those, at the chunks the tile
   assigned, with one kernel storing into the registered out dcache.

   Shared memory (one segment per GPU, in the topology a workspace object
   both tile kinds join):
     header                    fd_verify_svc_seg_t
     per verify tile t         fd_verify_svc_tile_t, then req_depth
                               request slots, then per slot:
                                 res [slot_cap]   fd_verify_svc_res_t (service writes)
                                 out [slot_cap]   fd_verify_svc_out_t (tile writes)
                                 frag area (frag_cap > 0): frag_cap frags of
                                   FD_VERIFY_SVC_FRAG_STRIDE bytes, their
                                   sizes and kinds (tile writes; polled links)
   Protocol, per tile, single producer / single consumer, no locks:
     slot state  FREE -(tile posts)-> POSTED -(service: the GPU has read
                 the request's frags into HBM)-> INGESTED -(service, results
                 written)-> RESULTS -(tile, once every published frag of the
                 slot is out)-> FREE.  Slots are posted and consumed in ring
                 order.  INGESTED is when a range request's link lines and
                 bytes may be reused: the tile runs the stem's overrun check
                 and moves its fseq then, not after the verify, so the link
                 holds a frag only for the copy (a service may go straight to
                 RESULTS, which implies INGESTED).
     flush ring  the tile appends { slot, lo, hi } (out entries [lo, hi) of
                 the slot) and advances flush_post; the service completes
                 flushes in order and advances flush_done.
   A state or counter is stored with release and loaded with acquire
   semantics; everything it covers is written before it.

   Credits (the reference's out dcache sizing, fd_dcache_req_data_sz with
   burst 1): the tile posts a flush of k frags only while the stem's
   credits less the frags already flushed but not published cover k, and
   publishes a flush's frags as soon as it completes, so at most credit
   many frags' data are written ahead of their publish -- the invariant
   after_frag keeps with burst 1.  Dropped frags take no chunk (ADVICE r04
   high: chunks were taken per frag, published or not).

   Plain C (gcc and hipcc), no HIP types.  Library (service side only):
   firedancer_amd/libfd_ed25519_hip.so. */

#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned char  uchar;
typedef unsigned short ushort;
typedef unsigned int   uint;
typedef unsigned long  ulong;

#define FD_VERIFY_SVC_MAGIC        (0xfd7e51f5e1c0de02UL)
#define FD_VERIFY_SVC_TILE_MAX     (32UL)      /* verify tiles and clients per GPU */
#define FD_VERIFY_SVC_LINK_MAX     (16UL)
#define FD_VERIFY_SVC_FLUSH_DEPTH  (256UL)     /* flush ring entries per tile (power of 2) */
#define FD_VERIFY_SVC_FRAG_STRIDE  (2048UL)    /* a polled frag's bytes in the frag area: <= 2048 (gossip, fd_verify_tile.c:89) */
#define FD_VERIFY_SVC_ALIGN        (4096UL)

/* request kinds */
#define FD_VERIFY_SVC_REQ_RANGE    (1UL)   /* seq range of an unpolled quic_verify link (range mode) */
#define FD_VERIFY_SVC_REQ_FRAGS    (2UL)   /* frags the tile copied into the slot's frag area (polled links) */
#define FD_VERIFY_SVC_REQ_SIGS     (3UL)   /* signature records a client wrote into the slot's frag area: one
                                              fd_ed25519_verify each (the shred tile's FEC-set roots,
                                              fd_fec_resolver.c:476; the replay tile's transactions,
                                              fd_executor.c:1607-1623); see "clients" below */

/* slot states */
#define FD_VERIFY_SVC_FREE         (0UL)
#define FD_VERIFY_SVC_POSTED       (1UL)
#define FD_VERIFY_SVC_RESULTS      (2UL)
#define FD_VERIFY_SVC_INGESTED     (3UL)

static inline int fd_verify_svc_state_ingested( unsigned long state ) { return state==3UL || state==2UL; }

/* service states (fd_verify_svc_seg_t.svc_state) */
#define FD_VERIFY_SVC_SVC_NONE     (0UL)
#define FD_VERIFY_SVC_SVC_RUNNING  (1UL)
#define FD_VERIFY_SVC_SVC_STOPPED  (2UL)

/* fd_verify_svc_res_t.flags */
#define FD_VERIFY_SVC_RES_BAD      (1)   /* during_frag's FD_LOG_ERR (fd_verify_tile.c:75-85): chunk outside
                                            [chunk0, wmark], sz > FD_TPU_RAW_MTU (2048 gossip), payload_sz >
                                            FD_TPU_MTU -- or, for a range frag, a line that no longer held its
                                            seq when the GPU read it (the tile's overrun check tells the two
                                            apart: an overrun frag is dropped, a corrupt one ends the tile) */
#define FD_VERIFY_SVC_RES_HOST     (2)   /* after_frag's parse read bytes during_frag did not copy (sz below
                                            80 + payload_sz): those are the out dcache's own bytes at the chunk
                                            the frag gets, which the GPU cannot know; the tile redoes the frag
                                            as after_frag does, on its core.  No producer of the reference
                                            makes such a frag (fd_tpu_reasm.c:278 publishes sz = 80 +
                                            payload_sz). */

/* The GPU's per-frag result (32 bytes). */
typedef struct {
  ulong  tag;          /* fd_hash( seed, sig0, 64 ) (fd_verify_tile.h:83); 0 if the parse failed */
  ulong  bundle_id;    /* the out frag's block_engine.bundle_id (fd_verify_tile.c:122) */
  ushort txn_t_sz;     /* fd_txn_parse's footprint; 0: parse failure (:120,130) */
  ushort payload_sz;   /* the out frag's payload_sz after during_frag */
  signed char code;    /* fd_ed25519_verify_batch_single_msg over the txn's signatures (FD_ED25519_*) */
  uchar  flags;        /* FD_VERIFY_SVC_RES_* */
  uchar  sig_cnt;      /* signatures verified for this frag */
  uchar  rsv0;
  uint   tsorig;       /* range requests: the mcache line's tsorig; frag requests: 0 */
  uint   rsv1;
} fd_verify_svc_res_t;

/* A published frag (16 bytes), in publish order: the tile's after_frag
   decision and out chunk. */
#define FD_VERIFY_SVC_OUT_HOSTWRITTEN (1)   /* the tile wrote this frag's out bytes itself */
typedef struct {
  uint   idx;          /* frag index in the slot's request */
  uint   chunk;        /* out chunk (ctx->out_chunk when after_frag published it) */
  ushort sz;           /* fd_txn_m_realized_footprint( txnm, 1, 0 ) */
  ushort flags;        /* FD_VERIFY_SVC_OUT_* */
  uint   tsorig;       /* the frag's tsorig, for the publish (the service ignores it) */
} fd_verify_svc_out_t;

/* A request slot (128 bytes).  The tile writes every field but state,
   sig_cnt and batch_frags before posting; the service writes sig_cnt and
   batch_frags before RESULTS. */
typedef struct {
  ulong state;                          /* FD_VERIFY_SVC_{FREE,POSTED,INGESTED,RESULTS}: atomics only */
  ulong kind;                           /* FD_VERIFY_SVC_REQ_* */
  ulong link;                           /* RANGE: index into the service's link table */
  ulong seq0, seq_cnt, rr_cnt, rr_idx;  /* RANGE: lines [seq0, seq0+seq_cnt), kept seq % rr_cnt == rr_idx */
  ulong n;                              /* frags of the request (RANGE: fd_verify_svc_range_cnt) */
  ulong seed;                           /* the tile's hashmap_seed (fd_verify_tile.c:170) */
  ulong id;                             /* the tile's request counter: slot = id % req_depth */
  long  t_post;                         /* the tile's tickcount at post (diagnostics) */
  ulong sig_cnt;                        /* service: signatures verified */
  ulong batch_frags;                    /* service: frags of the merged launch the request rode in */
  ulong rsv[ 3 ];
} fd_verify_svc_req_t;

typedef struct { ulong slot, lo, hi, rsv; } fd_verify_svc_flush_t;

/* A tile's block (followed by its slots and their arrays). */
typedef struct {
  ulong flush_post;                     /* tile: flushes posted (atomics) */
  ulong rsv0[ 15 ];
  ulong flush_done;                     /* service: flushes completed (atomics) */
  ulong rsv1[ 15 ];
  fd_verify_svc_flush_t flush[ FD_VERIFY_SVC_FLUSH_DEPTH ];
} fd_verify_svc_tile_t;

typedef struct {
  ulong magic;
  ulong tile_cnt, req_depth, slot_cap, frag_cap;
  ulong tile_sz;                        /* bytes per tile block */
  ulong slot_sz;                        /* bytes of a slot's arrays */
  ulong svc_state;                      /* FD_VERIFY_SVC_SVC_*: atomics */
  ulong svc_heartbeat;                  /* service loop iterations (diagnostics) */
  ulong shutdown;                       /* set by whoever ends the run: the service stops */
  ulong rsv[ 6 ];
} fd_verify_svc_seg_t;

/* ---- layout --------------------------------------------------------------- */

static inline ulong fd_verify_svc_align_up( ulong x, ulong a ) { return ( x + a - 1UL ) & ~( a - 1UL ); }

static inline ulong
fd_verify_svc_slot_sz( ulong slot_cap, ulong frag_cap ) {
  return fd_verify_svc_align_up( slot_cap*sizeof(fd_verify_svc_res_t), 4096UL ) +
         fd_verify_svc_align_up( slot_cap*sizeof(fd_verify_svc_out_t), 4096UL ) +
         fd_verify_svc_align_up( frag_cap*( FD_VERIFY_SVC_FRAG_STRIDE + 2UL + 1UL + 4UL ) + 8UL, 4096UL );
}

static inline ulong
fd_verify_svc_tile_sz( ulong req_depth, ulong slot_cap, ulong frag_cap ) {
  return fd_verify_svc_align_up( sizeof(fd_verify_svc_tile_t) + req_depth*sizeof(fd_verify_svc_req_t), 4096UL ) +
         req_depth*fd_verify_svc_slot_sz( slot_cap, frag_cap );
}

/* 0 on bad parameters: tile_cnt in [1, TILE_MAX], req_depth a power of 2 in
   [2, 256], slot_cap in [1, 2^20], frag_cap <= slot_cap */
static inline ulong
fd_verify_svc_footprint( ulong tile_cnt, ulong req_depth, ulong slot_cap, ulong frag_cap ) {
  if( !tile_cnt || tile_cnt>FD_VERIFY_SVC_TILE_MAX || req_depth<2UL || req_depth>256UL ||
      ( req_depth & ( req_depth-1UL ) ) || !slot_cap || slot_cap>(1UL<<20) || frag_cap>slot_cap ) return 0UL;
  return FD_VERIFY_SVC_ALIGN + tile_cnt*fd_verify_svc_tile_sz( req_depth, slot_cap, frag_cap );
}

static inline fd_verify_svc_seg_t *
fd_verify_svc_new( void * mem, ulong tile_cnt, ulong req_depth, ulong slot_cap, ulong frag_cap ) {
  ulong fp = fd_verify_svc_footprint( tile_cnt, req_depth, slot_cap, frag_cap );
  if( !mem || !fp || ( (ulong)mem & ( FD_VERIFY_SVC_ALIGN-1UL ) ) ) return (fd_verify_svc_seg_t *)0;
  uchar * p = (uchar *)mem;
  for( ulong i=0UL; i<FD_VERIFY_SVC_ALIGN; i++ ) p[ i ] = 0;
  fd_verify_svc_seg_t * s = (fd_verify_svc_seg_t *)mem;
  s->tile_cnt = tile_cnt; s->req_depth = req_depth; s->slot_cap = slot_cap; s->frag_cap = frag_cap;
  s->tile_sz  = fd_verify_svc_tile_sz( req_depth, slot_cap, frag_cap );
  s->slot_sz  = fd_verify_svc_slot_sz( slot_cap, frag_cap );
  for( ulong t=0UL; t<tile_cnt; t++ ) {                       /* headers and slots; the arrays need no init */
    uchar * b = p + FD_VERIFY_SVC_ALIGN + t*s->tile_sz;
    ulong hsz = sizeof(fd_verify_svc_tile_t) + req_depth*sizeof(fd_verify_svc_req_t);
    for( ulong i=0UL; i<hsz; i++ ) b[ i ] = 0;
  }
  __atomic_store_n( &s->magic, FD_VERIFY_SVC_MAGIC, __ATOMIC_RELEASE );
  return s;
}

static inline fd_verify_svc_seg_t *
fd_verify_svc_join( void * mem ) {
  fd_verify_svc_seg_t * s = (fd_verify_svc_seg_t *)mem;
  if( !s || __atomic_load_n( &s->magic, __ATOMIC_ACQUIRE )!=FD_VERIFY_SVC_MAGIC ) return (fd_verify_svc_seg_t *)0;
  return s;
}

static inline fd_verify_svc_tile_t *
fd_verify_svc_tile( fd_verify_svc_seg_t * s, ulong t ) {
  return (fd_verify_svc_tile_t *)( (uchar *)s + FD_VERIFY_SVC_ALIGN + t*s->tile_sz );
}
static inline fd_verify_svc_req_t *
fd_verify_svc_req( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (fd_verify_svc_req_t *)( fd_verify_svc_tile( s, t ) + 1 ) + slot;
}
static inline uchar *
fd_verify_svc_slot_base( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (uchar *)fd_verify_svc_tile( s, t ) +
         fd_verify_svc_align_up( sizeof(fd_verify_svc_tile_t) + s->req_depth*sizeof(fd_verify_svc_req_t), 4096UL ) +
         slot*s->slot_sz;
}
static inline fd_verify_svc_res_t *
fd_verify_svc_res( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (fd_verify_svc_res_t *)fd_verify_svc_slot_base( s, t, slot );
}
static inline fd_verify_svc_out_t *
fd_verify_svc_out( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (fd_verify_svc_out_t *)( fd_verify_svc_slot_base( s, t, slot ) +
                                  fd_verify_svc_align_up( s->slot_cap*sizeof(fd_verify_svc_res_t), 4096UL ) );
}
/* the frag area: frag i's bytes, then the sizes (ushort), kinds (uchar,
   FD_VERIFY_HIP_IN_*) and tsorigs (uint, the stem's, for the publish) */
static inline uchar *
fd_verify_svc_frag( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (uchar *)fd_verify_svc_out( s, t, slot ) +
         fd_verify_svc_align_up( s->slot_cap*sizeof(fd_verify_svc_out_t), 4096UL );
}
static inline ushort * fd_verify_svc_frag_sz  ( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (ushort *)( fd_verify_svc_frag( s, t, slot ) + s->frag_cap*FD_VERIFY_SVC_FRAG_STRIDE );
}
static inline uchar *  fd_verify_svc_frag_kind( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (uchar *)( fd_verify_svc_frag_sz( s, t, slot ) + s->frag_cap );
}
static inline uint *   fd_verify_svc_frag_tso ( fd_verify_svc_seg_t * s, ulong t, ulong slot ) {
  return (uint *)fd_verify_svc_align_up( (ulong)( fd_verify_svc_frag_kind( s, t, slot ) + s->frag_cap ), 4UL );
}

/* ---- atomics --------------------------------------------------------------- */

static inline ulong fd_verify_svc_ld( ulong const * p )      { return __atomic_load_n( p, __ATOMIC_ACQUIRE ); }
static inline void  fd_verify_svc_st( ulong * p, ulong v )   { __atomic_store_n( p, v, __ATOMIC_RELEASE ); }

/* ---- tile side -------------------------------------------------------------- */

/* kept seqs of [seq0, seq0+seq_cnt): seq % rr_cnt == rr_idx (before_frag,
   fd_verify_tile.c:37-58) */
static inline ulong
fd_verify_svc_range_cnt( ulong seq0, ulong seq_cnt, ulong rr_cnt, ulong rr_idx ) {
  if( !seq_cnt || !rr_cnt || rr_idx>=rr_cnt ) return 0UL;
  ulong first = seq0 + ( rr_idx + rr_cnt - seq0 % rr_cnt ) % rr_cnt;
  ulong end   = seq0 + seq_cnt;
  return first<end ? ( end - 1UL - first )/rr_cnt + 1UL : 0UL;
}

/* the first kept seq of a range */
static inline ulong
fd_verify_svc_range_first( ulong seq0, ulong rr_cnt, ulong rr_idx ) {
  return seq0 + ( rr_idx + rr_cnt - seq0 % rr_cnt ) % rr_cnt;
}

/* Post a request in slot id % req_depth (which must be FREE).  Returns 0,
   or -1 if the slot is not free or n exceeds the slot's capacity. */
static inline int
fd_verify_svc_post_range( fd_verify_svc_seg_t * s, ulong t, ulong id, ulong link, ulong seq0, ulong seq_cnt,
                          ulong rr_cnt, ulong rr_idx, ulong seed, long now ) {
  fd_verify_svc_req_t * r = fd_verify_svc_req( s, t, id & ( s->req_depth-1UL ) );
  ulong n = fd_verify_svc_range_cnt( seq0, seq_cnt, rr_cnt, rr_idx );
  if( fd_verify_svc_ld( &r->state )!=FD_VERIFY_SVC_FREE || n>s->slot_cap ) return -1;
  r->kind = FD_VERIFY_SVC_REQ_RANGE; r->link = link; r->seq0 = seq0; r->seq_cnt = seq_cnt;
  r->rr_cnt = rr_cnt; r->rr_idx = rr_idx; r->n = n; r->seed = seed; r->id = id; r->t_post = now;
  r->sig_cnt = 0UL; r->batch_frags = 0UL;
  fd_verify_svc_st( &r->state, FD_VERIFY_SVC_POSTED );
  return 0;
}

/* frags [0, n) already in the slot's frag area (bytes, sizes, kinds) */
static inline int
fd_verify_svc_post_frags( fd_verify_svc_seg_t * s, ulong t, ulong id, ulong n, ulong seed, long now ) {
  fd_verify_svc_req_t * r = fd_verify_svc_req( s, t, id & ( s->req_depth-1UL ) );
  if( fd_verify_svc_ld( &r->state )!=FD_VERIFY_SVC_FREE || n>s->frag_cap ) return -1;
  r->kind = FD_VERIFY_SVC_REQ_FRAGS; r->link = 0UL; r->seq0 = 0UL; r->seq_cnt = 0UL; r->rr_cnt = 1UL; r->rr_idx = 0UL;
  r->n = n; r->seed = seed; r->id = id; r->t_post = now; r->sig_cnt = 0UL; r->batch_frags = 0UL;
  fd_verify_svc_st( &r->state, FD_VERIFY_SVC_POSTED );
  return 0;
}

/* Out entries [lo, hi) of slot to be written; -1 if the ring is full. */
static inline int
fd_verify_svc_post_flush( fd_verify_svc_seg_t * s, ulong t, ulong slot, ulong lo, ulong hi ) {
  fd_verify_svc_tile_t * b = fd_verify_svc_tile( s, t );
  ulong post = b->flush_post;                                   /* only this tile writes it */
  if( post - fd_verify_svc_ld( &b->flush_done )>=FD_VERIFY_SVC_FLUSH_DEPTH ) return -1;
  fd_verify_svc_flush_t * f = &b->flush[ post & ( FD_VERIFY_SVC_FLUSH_DEPTH-1UL ) ];
  f->slot = slot; f->lo = lo; f->hi = hi;
  fd_verify_svc_st( &b->flush_post, post+1UL );
  return 0;
}

/* ---- clients ----------------------------------------------------------------

   A client is a segment tile that posts FD_VERIFY_SVC_REQ_SIGS requests
   only: the shred tile (FEC-set roots) and the replay tile (its block's
   transaction signatures) stay single-threaded and without a device fd,
   as the verify tiles do, and their verifies ride the GPU tile's launches
   (fd_verify_svc_set_client on the service side; a client has no out
   dcache and posts no flush).  Record i of a request is frag i of the
   slot's frag area: the signature (64 B), the public key (32 B), then the
   message; frag_sz[ i ] = 96 + the message's size.  The service writes
   res[ i ].code = fd_ed25519_verify( msg, msg_sz, sig, pub ) (FD_ED25519_*
   in the service contexts' error mode), sig_cnt 1 and payload_sz the
   message size; a record shorter than 96 B or over the frag stride gets
   FD_VERIFY_SVC_RES_BAD and code FD_ED25519_ERR_SIG.  The slot goes from
   POSTED to RESULTS; the client reads the codes and stores FREE.

   fd_verify_svc_client_t keeps one client's request ring: records are
   added into the open request (the next slot, when FREE), a request is
   posted when full or on flush, and poll hands every finished record's
   code back with the caller's 32-bit tag (kept in the slot's out array,
   which a client does not otherwise use), oldest request first.  No
   syscall, no allocation: it runs inside the reference's seccomp
   policies. */

#define FD_VERIFY_SVC_SIG_HDR_SZ   (96UL)
#define FD_VERIFY_SVC_SIG_MSG_MAX  (FD_VERIFY_SVC_FRAG_STRIDE - FD_VERIFY_SVC_SIG_HDR_SZ)

typedef struct {
  fd_verify_svc_seg_t * seg;
  ulong t;                 /* the client's tile index in the segment */
  ulong id_post;           /* next request id to post (the open request, if open_n) */
  ulong id_done;           /* oldest posted request not yet collected */
  ulong open_n;            /* records in the open request */
  ulong recs_posted, recs_done, reqs_posted;
} fd_verify_svc_client_t;

static inline fd_verify_svc_client_t *
fd_verify_svc_client_join( fd_verify_svc_client_t * c, fd_verify_svc_seg_t * seg, ulong t ) {
  if( !c || !seg || t>=seg->tile_cnt || !seg->frag_cap ) return (fd_verify_svc_client_t *)0;
  c->seg = seg; c->t = t; c->id_post = 0UL; c->id_done = 0UL; c->open_n = 0UL;
  c->recs_posted = 0UL; c->recs_done = 0UL; c->reqs_posted = 0UL;
  return c;
}

/* requests posted and not yet collected */
static inline ulong fd_verify_svc_client_busy( fd_verify_svc_client_t const * c ) { return c->id_post - c->id_done; }

/* post the open request (nothing if it is empty); 0, or -1 on a protocol error */
static inline int
fd_verify_svc_client_flush( fd_verify_svc_client_t * c, long now ) {
  if( !c->open_n ) return 0;
  fd_verify_svc_seg_t * s = c->seg;
  fd_verify_svc_req_t * r = fd_verify_svc_req( s, c->t, c->id_post & ( s->req_depth-1UL ) );
  r->kind = FD_VERIFY_SVC_REQ_SIGS; r->link = 0UL; r->seq0 = 0UL; r->seq_cnt = 0UL; r->rr_cnt = 1UL; r->rr_idx = 0UL;
  r->n = c->open_n; r->seed = 0UL; r->id = c->id_post; r->t_post = now; r->sig_cnt = 0UL; r->batch_frags = 0UL;
  fd_verify_svc_st( &r->state, FD_VERIFY_SVC_POSTED );
  c->recs_posted += c->open_n; c->reqs_posted++;
  c->id_post++; c->open_n = 0UL;
  return 0;
}

/* add one record (tag: the caller's, handed back by poll).  Returns 1 if
   added, 0 if no slot is free (poll, then retry), -1 if msg_sz is over
   FD_VERIFY_SVC_SIG_MSG_MAX.  A full request is posted at once. */
static inline int
fd_verify_svc_client_add( fd_verify_svc_client_t * c, uchar const * sig, uchar const * pub, uchar const * msg,
                          ulong msg_sz, uint tag, long now ) {
  if( msg_sz>FD_VERIFY_SVC_SIG_MSG_MAX ) return -1;
  fd_verify_svc_seg_t * s = c->seg;
  ulong slot = c->id_post & ( s->req_depth-1UL );
  if( !c->open_n ) {                                            /* opening a request: its slot must be free */
    if( c->id_post - c->id_done>=s->req_depth ||
        fd_verify_svc_ld( &fd_verify_svc_req( s, c->t, slot )->state )!=FD_VERIFY_SVC_FREE ) return 0;
  }
  ulong i = c->open_n;
  uchar * f = fd_verify_svc_frag( s, c->t, slot ) + i*FD_VERIFY_SVC_FRAG_STRIDE;
  memcpy( f, sig, 64UL ); memcpy( f+64UL, pub, 32UL ); memcpy( f+96UL, msg, msg_sz );
  fd_verify_svc_frag_sz  ( s, c->t, slot )[ i ] = (ushort)( FD_VERIFY_SVC_SIG_HDR_SZ + msg_sz );
  fd_verify_svc_frag_kind( s, c->t, slot )[ i ] = 0;
  fd_verify_svc_out( s, c->t, slot )[ i ].idx = tag;
  c->open_n = i+1UL;
  if( c->open_n==s->frag_cap ) (void)fd_verify_svc_client_flush( c, now );
  return 1;
}

/* collect finished requests, oldest first: cb( ctx, tag, code ) per record
   (code FD_ED25519_*, or FD_ED25519_ERR_SIG for a record the service
   found malformed); stops at the first request still on the GPU.  Returns
   the records collected. */
typedef void (*fd_verify_svc_client_cb_t)( void * ctx, uint tag, int code );

static inline ulong
fd_verify_svc_client_poll( fd_verify_svc_client_t * c, fd_verify_svc_client_cb_t cb, void * ctx ) {
  fd_verify_svc_seg_t * s = c->seg;
  ulong got = 0UL;
  while( c->id_done!=c->id_post ) {
    ulong slot = c->id_done & ( s->req_depth-1UL );
    fd_verify_svc_req_t * r = fd_verify_svc_req( s, c->t, slot );
    if( fd_verify_svc_ld( &r->state )!=FD_VERIFY_SVC_RESULTS ) break;
    fd_verify_svc_res_t const * res = fd_verify_svc_res( s, c->t, slot );
    fd_verify_svc_out_t const * out = fd_verify_svc_out( s, c->t, slot );
    ulong n = r->n;
    for( ulong i=0UL; i<n; i++ ) cb( ctx, out[ i ].idx, ( res[ i ].flags & FD_VERIFY_SVC_RES_BAD ) ? -1 : (int)res[ i ].code );
    fd_verify_svc_st( &r->state, FD_VERIFY_SVC_FREE );
    c->id_done++; got += n;
  }
  c->recs_done += got;
  return got;
}

/* ---- sizing ----------------------------------------------------------------

   The service keeps every slot's out frags in HBM staging, tile_cnt x
   req_depth x slot_cap frags of FD_VERIFY_SVC_STAGE_FRAG_SZ bytes, and the
   verify addresses their messages with 32-bit byte offsets: the staging of
   one GPU stays below 4 GiB (fd_verify_svc_boot refuses a shape that does
   not fit).  fd_verify_svc_stage_ok checks a shape.

   fd_verify_svc_topo_shape is the shape the topologies give a GPU that
   serves tile_cnt verify tiles (integration/fd_verify_topo_hip.patch):
     req_depth  FD_VERIFY_SVC_TOPO_REQ_DEPTH: at the reference's quic_verify
                depth (16384, default.toml:1153) a range request spans
                depth / FD_VERIFY_SVC_RANGE_DIV seqs, and a tile holds a slot
                from its post to the publish of its frags (~2-5 ms): 128 slots
                keep up with > 50 M seqs/s
     slot_cap   the largest power of 2 up to FD_VERIFY_SVC_TOPO_SLOT_CAP whose
                staging fits (2 tiles: 4096; 6 tiles, the reference's default
                verify_tile_count: 2048; 16 tiles: 512)
     frag_cap   FD_VERIFY_SVC_TOPO_FRAG_CAP frags of the polled links (gossip
                votes, send, bundles) per request
   out[0..3] = tile_cnt, req_depth, slot_cap, frag_cap; returns 0, or -1 if
   tile_cnt is not in [1, FD_VERIFY_SVC_TILE_MAX]. */

#define FD_VERIFY_SVC_STAGE_FRAG_SZ   (2176UL)    /* FD_TXN_HIP_STAGE_CHUNKS (34) x 64 B: an out frag at its largest */
#define FD_VERIFY_SVC_TOPO_REQ_DEPTH  (128UL)
#define FD_VERIFY_SVC_TOPO_SLOT_CAP   (32768UL)
#define FD_VERIFY_SVC_TOPO_FRAG_CAP   (256UL)

static inline int
fd_verify_svc_stage_ok( ulong tile_cnt, ulong req_depth, ulong slot_cap ) {
  if( !tile_cnt || tile_cnt>FD_VERIFY_SVC_TILE_MAX || !req_depth || req_depth>256UL || !slot_cap || slot_cap>(1UL<<20) ) return 0;
  return tile_cnt*req_depth*slot_cap*FD_VERIFY_SVC_STAGE_FRAG_SZ + 4096UL < (1UL<<32);
}

/* every shape check fd_verify_svc_boot makes before it allocates: a
   segment footprint, 1..8 launches in flight of at least a slot each, the
   staging within 4 GiB, the ingest frags (FD_VERIFY_SVC_INGEST_CHUNKS
   64-B chunks each) addressed by 32-bit chunk indices */
#define FD_VERIFY_SVC_INGEST_CHUNKS   (32UL)
#define FD_VERIFY_SVC_INFLIGHT_MAX    (8UL)
static inline int
fd_verify_svc_boot_ok( ulong tile_cnt, ulong req_depth, ulong slot_cap, ulong frag_cap, ulong batch_max, ulong inflight ) {
  return fd_verify_svc_footprint( tile_cnt, req_depth, slot_cap, frag_cap )!=0UL &&
         inflight>=1UL && inflight<=FD_VERIFY_SVC_INFLIGHT_MAX && batch_max>=slot_cap &&
         fd_verify_svc_stage_ok( tile_cnt, req_depth, slot_cap ) &&
         FD_VERIFY_SVC_INGEST_CHUNKS*tile_cnt*req_depth*slot_cap < (1UL<<32);
}

static inline int
fd_verify_svc_topo_shape( ulong tile_cnt, ulong out[ 4 ] ) {
  if( !tile_cnt || tile_cnt>FD_VERIFY_SVC_TILE_MAX ) return -1;
  ulong cap = FD_VERIFY_SVC_TOPO_SLOT_CAP;
  while( cap>FD_VERIFY_SVC_TOPO_FRAG_CAP && !fd_verify_svc_stage_ok( tile_cnt, FD_VERIFY_SVC_TOPO_REQ_DEPTH, cap ) ) cap >>= 1;
  out[ 0 ] = tile_cnt; out[ 1 ] = FD_VERIFY_SVC_TOPO_REQ_DEPTH; out[ 2 ] = cap; out[ 3 ] = FD_VERIFY_SVC_TOPO_FRAG_CAP;
  return 0;
}

/* ---- multi-GPU assignment ---------------------------

   Verify tile kind_id is served by the GPU tile on device kind_id %
   gpu_cnt (the direct form's rule, fd_verify_tile_hip.patch
   privileged_init); within that GPU's segment it is tile
   kind_id / gpu_cnt.  Each verify tile keeps seq % verify_cnt == kind_id of
   every quic_verify link (before_frag), so the shares of the GPUs are
   disjoint and their union is every seq. */
static inline ulong fd_verify_svc_gpu_of ( ulong kind_id, ulong gpu_cnt ) { return kind_id % gpu_cnt; }
static inline ulong fd_verify_svc_slot_of( ulong kind_id, ulong gpu_cnt ) { return kind_id / gpu_cnt; }
static inline ulong fd_verify_svc_tiles_on( ulong gpu, ulong verify_cnt, ulong gpu_cnt ) {
  return gpu<verify_cnt%gpu_cnt ? verify_cnt/gpu_cnt + 1UL : verify_cnt/gpu_cnt;
}

/* ---- service side (libfd_ed25519_hip.so) -----------------------------------

   fd_verify_svc_boot( seg, device, batch_max, inflight ): the GPU tile's
     service on HIP device `device` over a segment made by fd_verify_svc_new
     (batch_max frags per merged launch at most, >= the segment's slot_cap;
     inflight launches at once, 1..8).  Allocates everything the steady state
     uses (HBM staging for req_depth x slot_cap frags per tile, one context
     and stream per launch slot).  NULL on failure.
   fd_verify_svc_map( svc, host, sz ): register host memory (a workspace: the
     segment, a link's mcache and dcache, a tile's out dcache) for the GPU;
     the addresses below must lie in mapped regions.  -1 on failure.
   fd_verify_svc_set_link( svc, link, mcache, depth, chunk_base, chunk0,
     wmark ): range link `link`: its mcache lines (fd_mcache_join's pointer),
     depth, the address chunk 0 is relative to (the link's workspace,
     fd_chunk_to_laddr), and during_frag's range (fd_dcache_compact_chunk0 /
     _wmark).
   fd_verify_svc_set_tile( svc, t, out_dcache, out_dcache_sz, out_chunk_base ):
     tile t's verify_dedup dcache (flush target) and its chunk base.
   fd_verify_svc_set_client( svc, t ): tile t is a client (see "clients");
     every tile of the segment is set one way or the other before run.
   fd_verify_svc_run( svc ): marks the service running; then
   fd_verify_svc_poll( svc ): one iteration of the service loop (retire
     finished launches, ingests and flushes, start flushes, copy newly
     posted requests' frags into HBM at once, merge ingested requests into a
     verify launch); 1 if it did anything.  Never blocks.
   fd_verify_svc_set_merge( svc, min_frags, wait_ns, idle_ns ): a verify
     launch starts once the ingested requests hold min_frags frags, or the
     oldest has waited wait_ns, or -- no launch in flight -- idle_ns
     (defaults batch_max / 2, 2 ms, 20 us; two launches in flight measure
     best on one MI355X).
   fd_verify_svc_stats( svc, out[ 16 ] ): launches, frags, requests,
     flushes, flushed frags, 0 (unused), flush kernels, GPU ns (summed over
     verify launches), host ns starting launches, host ns starting flushes,
     host ns polling events, polls, ingests, ingest GPU ns, host ns starting
     ingests, the largest launch's frags.
   fd_verify_svc_delete( svc ): waits for the GPU and frees everything. */

typedef struct fd_verify_svc fd_verify_svc_t;

fd_verify_svc_t * fd_verify_svc_boot    ( void * seg, int device, ulong batch_max, ulong inflight );
int               fd_verify_svc_map     ( fd_verify_svc_t * svc, void * host, ulong sz );
int               fd_verify_svc_set_link( fd_verify_svc_t * svc, ulong link, void const * mcache, ulong depth,
                                          void const * chunk_base, ulong chunk0, ulong wmark );
int               fd_verify_svc_set_tile( fd_verify_svc_t * svc, ulong t, void * out_dcache, ulong out_dcache_sz,
                                          void const * out_chunk_base );
/* tile t is a client (FD_VERIFY_SVC_REQ_SIGS requests only, no out dcache:
   a flush or a verify-tile request from it ends the service).  -1 on bad
   arguments or a tile already set. */
int               fd_verify_svc_set_client( fd_verify_svc_t * svc, ulong t );
void              fd_verify_svc_set_merge( fd_verify_svc_t * svc, ulong min_frags, ulong wait_ns, ulong idle_ns );
int               fd_verify_svc_run     ( fd_verify_svc_t * svc );
int               fd_verify_svc_poll    ( fd_verify_svc_t * svc );
void              fd_verify_svc_stats   ( fd_verify_svc_t const * svc, ulong out[ 16 ] );
/* where the slots are, sampled every 64th poll while any slot is in use:
   out[0] samples, then the summed slot counts posted (not yet ingested),
   ingested and waiting for a launch, in a launch, results (the tile's
   ordered pass, flushes and publish), free.  Divide by out[0] for the mean
   occupancy of each state. */
void              fd_verify_svc_occupancy( fd_verify_svc_t const * svc, ulong out[ 6 ] );
/* one line of the service's state (launches, request slots per tile, the
   IO engine's counters and leader state) into buf; the length written */
int               fd_verify_svc_debug   ( fd_verify_svc_t const * svc, char * buf, ulong sz );
void              fd_verify_svc_delete  ( fd_verify_svc_t * svc );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_verify_svc_h */
