/* fd_verify_svc.hip -- the per-GPU verify service (include/fd_verify_svc.h):
   the GPU tile's side of the shared-memory protocol.

   One process per GPU owns the HIP context.  Every verify tile it serves
   posts requests (a seq range of an unpolled quic_verify link, or frags it
   copied from a polled link) into its slots of the segment.  The service
   copies each newly posted request's frags into HBM at once, then merges
   the ingested requests of all tiles into one verify launch (up to
   batch_max frags), so a launch is C4-sized whatever the tile count:

     k_svc_gather   (the ingest, on its own stream, as soon as a request is
                    posted) one wave per frag: before_frag's share (range
                    requests name only the kept seqs: seq0 + i x rr_cnt),
                    the mcache line (seq still there, chunk in [chunk0,
                    wmark], sz <= FD_TPU_RAW_MTU: fd_stem.c and during_frag's
                    checks, fd_verify_tile.c:74-76), and the frag's bytes
                    from the link's dcache (pinned host memory) into the
                    request slot's HBM ingest frags.  Then the slot goes to
                    INGESTED: the tile checks for overruns and returns the
                    link's credits right away, so the link holds a frag for
                    the PCIe copy only, not for the merge and the verify
     k_svc_assemble the verify launch's per-frag arrays from its requests'
                    ingest frags
     fd_txn_hip_batch_core
                    k_txnm_batch<16> (during_frag's copy into the request's
                    HBM staging frags, fd_txn_parse, the sig0 tag with each
                    tile's seed, the signature records), the verify, the
                    per-txn fd_ed25519_verify_batch_single_msg reduce
     k_svc_results  32-B result records, written straight into each
                    request slot's result array in the segment (registered
                    host memory); then the slot goes to RESULTS

   The out frags stay in HBM.  After its ordered pass (tcache, bundles) the
   tile posts flushes: out entries (frag, chunk, realized size) of the frags
   it publishes, chunks assigned as after_frag assigns them.  A flush is one
   kernel (k_svc_compact) that writes those staging frags straight into the
   tile's out dcache (registered host memory) at their chunks: whole 64-B
   chunks in 16-B stores, each frag contiguous, so the PCIe writes are full
   lines.  Only published frags cross PCIe.

   Host work per step is a few HIP calls (the service thread is the one
   core that drives every tile's GPU work): descriptors live in mapped
   pinned memory the kernels read in place, and results and flushed frags
   are written by kernels, not copied -- no hipMemcpy on the steady-state
   path.  A flush costs one launch and one event, an ingest one launch and
   two events, a verify launch its kernels and two events.

   Flushes of a tile run in order on the tile's own stream; requests and
   flushes of different tiles are independent.  Every HIP failure aborts
   (the reference's FD_LOG_ERR ends a tile; a device error is never turned
   into a verdict). */

#include "../../include/fd_verify_svc.h"
#include "../../include/fd_verify_hip.h"
#include "fd_txn_hip_int.h"

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <pthread.h>
#include <sched.h>

#define SV_CHECK( x ) do {                                                            \
    hipError_t e_ = (x);                                                               \
    if( e_ != hipSuccess ) {                                                           \
      fprintf( stderr, "fd_verify_svc: %s failed at %s:%d: %s\n", #x, __FILE__,      \
               __LINE__, hipGetErrorString( e_ ) );                                    \
      abort();                                                                         \
    }                                                                                  \
  } while( 0 )

typedef uint8_t  u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

#define SVC_INGEST_CHUNKS 32ul   /* an ingest frag: 2048 B (a gossip message's bound, the RAW_MTU's 1312 below it) */
#define SVC_REQ_MAX       512u   /* requests per launch (small requests at shallow link depths: 512 x 1 K frags) */
#define SVC_LAUNCH_MAX    8ul
#define SVC_GATHER_WGS    256ul  /* the gather's default grid: 1024 waves, enough to keep PCIe busy (64: 2x slower) */
#define SVC_FLUSH_WGS     256ul  /* the flush kernel's default grid */
#define SVC_FLUSH_Q       64ul   /* flushes in flight per tile */
#define SVC_REGION_MAX    64ul
#define SVC_ING_MAX       8ul    /* ingest batches in flight */
#define SVC_FB_MAX        8ul    /* flush batches in flight */
#define SVC_FB_FLUSH_MAX  512u   /* flushes per flush batch */
#define SVC_DSM_RESERVE   128ul  /* DSM workgroup slots left free in the service's verify contexts */

/* the device current on the calling thread (the service runs on one
   thread; hipSetDevice only when it changes) */
static __thread int svc_cur_dev = -1;
static void svc_device( int dev ) {
  if( svc_cur_dev != dev ) { SV_CHECK( hipSetDevice( dev ) ); svc_cur_dev = dev; }
}

static long svc_now_ns( void ) {
  struct timespec ts;
  clock_gettime( CLOCK_MONOTONIC, &ts );
  return (long)ts.tv_sec * 1000000000L + (long)ts.tv_nsec;
}

/* one request of a launch, as the gather kernel reads it (128 B) */
struct __attribute__((aligned(16))) svc_desc {
  u64 base;        /* the request's first frag in the launch */
  u64 n;
  u64 kind;        /* FD_VERIFY_SVC_REQ_* */
  u64 src;         /* RANGE: the mcache's line 0; FRAGS: the frag area (device addresses) */
  u64 aux0;        /* RANGE: the link's chunk base; FRAGS: the sizes */
  u64 aux1;        /* FRAGS: the kinds */
  u64 first;       /* RANGE: the first kept seq */
  u64 stride;      /* RANGE: rr_cnt */
  u64 line_mask;   /* RANGE: depth - 1 */
  u64 chunk0, wmark;
  u64 seed;
  u64 stage0;      /* staging chunk of the request's frag 0 */
  u64 ibase;       /* ingest frag of the request's frag 0 (slot (t, s): (t x req_depth + s) x slot_cap) */
  u64 res;         /* the slot's result array in the segment (device address; verify launches) */
  u64 state;       /* the request slot's state word in the segment (device address; ingests: the kernel's last
                      workgroup stores INGESTED there itself) */
};
static_assert( sizeof(svc_desc) == 128, "svc_desc layout" );

/**********************************************************************/
/* kernels                                                             */

typedef u32 v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;     /* global memory: global_load / global_store, not flat */

__global__ __launch_bounds__(256)
void k_svc_gather( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u8 * __restrict__ ing,
                   u16 * __restrict__ ing_sz, u8 * __restrict__ ing_kind, u32 * __restrict__ ing_tso,
                   u8 * __restrict__ stage, u32 * __restrict__ done_ctr ) {
  /* the requests' descriptors into LDS first (dynamic, nreq x 128 B): they
     live in mapped host memory, and read in place every frag paid a chain of
     dependent PCIe round trips for its descriptor's fields */
  extern __shared__ uint4 sd4[];
  svc_desc const * sd = (svc_desc const *)sd4;
  for( u32 k = threadIdx.x; k < 8u * nreq; k += blockDim.x ) sd4[k] = ((uint4 const *)desc)[k];
  __syncthreads();
  /* a quarter wave (16 lanes) per frag, 16 frags per workgroup per trip,
     grid-stride: a grid of n/16 workgroups takes each frag once, a capped
     grid (gather_wgs) loops.  The loads are PCIe reads of host memory; a
     quarter issues its frag's line read, then every 256-B piece of the frag
     at once (up to 8, before any store), so a wave has 4 frags and all of
     their pieces in flight (one wave per frag, one piece per round trip
     after the line: 16 GB/s, 25 ns per frag at 3 tiles, profiles/r06/
     gather_mlp) */
  u32 const ql = threadIdx.x & 15u;
  for( ulong j = (ulong)blockIdx.x * 16ul + (threadIdx.x >> 4); j < n; j += 16ul * gridDim.x ) {
    u32 lo = 0u, hi = nreq;                                 /* sd[lo].base <= j < sd[hi].base */
    while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sd[mid].base <= j ) lo = mid; else hi = mid; }
    svc_desc const * d = sd + lo;
    ulong const i = j - d->base;
    u32 sz = 0u, kind = FD_VERIFY_HIP_IN_QUIC, tsv = 0u;
    bool ok;
    u8 const * src;
    if( d->kind == FD_VERIFY_SVC_REQ_RANGE ) {
      ulong const seq = d->first + i * d->stride;
      u8 const * line = (u8 const *)d->src + 32ul * (seq & d->line_mask);
      /* the quarter's lanes 0 and 1 read the line's two halves (seq, sig |
         chunk, sz, ctl, tsorig, tspub), every lane of the quarter takes them */
      uint4 v = make_uint4( 0u, 0u, 0u, 0u );
      if( ql < 2u ) v = *(uint4 const *)(line + 16u * ql);
      u64 const found = (u64)(u32)__shfl( (int)v.x, 0, 16 ) | ((u64)(u32)__shfl( (int)v.y, 0, 16 ) << 32);
      u32 const chunk = (u32)__shfl( (int)v.x, 1, 16 );
      sz  = (u32)__shfl( (int)v.y, 1, 16 ) & 0xffffu;
      tsv = (u32)__shfl( (int)v.z, 1, 16 );
      ok  = found == seq && (ulong)chunk >= d->chunk0 && (ulong)chunk <= d->wmark && sz <= FD_VERIFY_HIP_TPU_RAW_MTU;
      src = (u8 const *)d->aux0 + 64ul * chunk;
    } else {
      src  = (u8 const *)d->src + FD_VERIFY_SVC_FRAG_STRIDE * i;
      sz   = ((u16 const *)d->aux0)[i];
      bool const sigs = d->kind == FD_VERIFY_SVC_REQ_SIGS;   /* a client's signature records: no frag kind */
      kind = sigs ? FD_VERIFY_HIP_IN_QUIC : ((u8 const *)d->aux1)[i];
      ok   = sz <= FD_VERIFY_SVC_FRAG_STRIDE && ( !sigs || sz >= FD_VERIFY_SVC_SIG_HDR_SZ );
    }
    ulong const f = d->ibase + i;
    u8 * dst = ing + 64ul * SVC_INGEST_CHUNKS * f;
    u32 const m = ok ? sz : 0u;                             /* sz <= 2048: 8 pieces of 256 B */
    /* every piece load is made (a piece past the frag reads the destination,
       device memory, and is not stored), as global loads into named
       registers: predicated loads into an array went through scratch with a
       wait each */
    u32 const p0 = 16u * ql;
#define SVC_PIECE_LD( k ) v4u const v##k = *(gv4u const *)( p0 + 256u * k < m ? src + p0 + 256u * k : dst + p0 + 256u * k )
    SVC_PIECE_LD( 0 ); SVC_PIECE_LD( 1 ); SVC_PIECE_LD( 2 ); SVC_PIECE_LD( 3 );
    SVC_PIECE_LD( 4 ); SVC_PIECE_LD( 5 ); SVC_PIECE_LD( 6 ); SVC_PIECE_LD( 7 );
#undef SVC_PIECE_LD
#define SVC_PIECE_ST( k ) if( p0 + 256u * k < m ) *(gv4u *)( dst + p0 + 256u * k ) = v##k
    SVC_PIECE_ST( 0 ); SVC_PIECE_ST( 1 ); SVC_PIECE_ST( 2 ); SVC_PIECE_ST( 3 );
    SVC_PIECE_ST( 4 ); SVC_PIECE_ST( 5 ); SVC_PIECE_ST( 6 ); SVC_PIECE_ST( 7 );
#undef SVC_PIECE_ST
    /* a gossip vote's out header: the reference writes four fields into the
       out chunk's stale header (fd_verify_tile.c:90-93); here the rest is 0 */
    if( kind == FD_VERIFY_HIP_IN_GOSSIP && ql < 5u )
      *(uint4 *)(stage + 64ul * (d->stage0 + FD_TXN_HIP_STAGE_CHUNKS * i) + 16u * ql) = make_uint4( 0u, 0u, 0u, 0u );
    if( ql == 0u ) { ing_sz[f] = ok ? (u16)sz : (u16)0xffffu; ing_kind[f] = (u8)kind; ing_tso[f] = tsv; }
  }
  /* INGESTED from the GPU: once every workgroup has passed its loop (all of
     its loads from the links have returned), the last one stores INGESTED
     into each request's slot in the segment, so a tile may reuse its link
     without waiting for the service thread's turn (the service still
     retires the batch by its event before a verify launch reads the HBM
     frags).  done_ctr: this batch's counter, zero at launch; the last
     workgroup puts it back to zero for the next batch on the ingest stream */
  /* Only the links' reads must be over (their values were stored, so they
     have returned): no fence, and relaxed stores -- a system-scope release
     here would write the whole L2 back (the verify kernels' dirty lines
     included) once per request, which measured slower than the host's
     turn it saves */
  if( !done_ctr ) return;
  __syncthreads();
  __shared__ u32 last;
  if( threadIdx.x == 0u ) last = atomicAdd( done_ctr, 1u ) == gridDim.x - 1u;
  __syncthreads();
  if( !last ) return;
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x )
    if( sd[i].state )
      __hip_atomic_store( (u64 *)sd[i].state, (u64)FD_VERIFY_SVC_INGESTED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
  if( threadIdx.x == 0u ) *done_ctr = 0u;
}

/* the round-5 gather (the default; FD_VERIFY_SVC_GATHER=quarter selects
   k_svc_gather above): one wave per frag, descriptors read in place from
   mapped host memory */
__global__ __launch_bounds__(256)
void k_svc_gather_wave( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u8 * __restrict__ ing,
                   u16 * __restrict__ ing_sz, u8 * __restrict__ ing_kind, u32 * __restrict__ ing_tso,
                   u8 * __restrict__ stage, u32 * __restrict__ done_ctr ) {
  __shared__ u64 sbase[SVC_REQ_MAX];
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x ) sbase[i] = desc[i].base;
  __syncthreads();
  u32 const lane = threadIdx.x & 63u;
  /* one wave per frag, grid-stride: a grid of n/4 workgroups takes each frag
     once; a capped grid (gather_wgs) loops */
  for( ulong j = (ulong)blockIdx.x * 4ul + (threadIdx.x >> 6); j < n; j += 4ul * gridDim.x ) {
    u32 lo = 0u, hi = nreq;                                 /* sbase[lo] <= j < sbase[hi] */
    while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sbase[mid] <= j ) lo = mid; else hi = mid; }
    svc_desc const * d = desc + lo;
    ulong const i = j - d->base;
    u32 sz = 0u, kind = FD_VERIFY_HIP_IN_QUIC, tsv = 0u;
    bool ok;
    u8 const * src;
    if( d->kind == FD_VERIFY_SVC_REQ_RANGE ) {
      ulong const seq = d->first + i * d->stride;
      u8 const * line = (u8 const *)d->src + 32ul * (seq & d->line_mask);
      /* lanes 0 and 1 read the line's two halves (seq, sig | chunk, sz,
         ctl, tsorig, tspub) with vector loads, every lane takes them */
      uint4 v = make_uint4( 0u, 0u, 0u, 0u );
      if( lane < 2u ) v = *(uint4 const *)(line + 16u * lane);
      u64 const found = (u64)(u32)__shfl( (int)v.x, 0 ) | ((u64)(u32)__shfl( (int)v.y, 0 ) << 32);
      u32 const chunk = (u32)__shfl( (int)v.x, 1 );
      sz  = (u32)__shfl( (int)v.y, 1 ) & 0xffffu;
      tsv = (u32)__shfl( (int)v.z, 1 );
      ok  = found == seq && (ulong)chunk >= d->chunk0 && (ulong)chunk <= d->wmark && sz <= FD_VERIFY_HIP_TPU_RAW_MTU;
      src = (u8 const *)d->aux0 + 64ul * chunk;
    } else {
      src  = (u8 const *)d->src + FD_VERIFY_SVC_FRAG_STRIDE * i;
      sz   = ((u16 const *)d->aux0)[i];
      bool const sigs = d->kind == FD_VERIFY_SVC_REQ_SIGS;   /* a client's signature records: no frag kind */
      kind = sigs ? FD_VERIFY_HIP_IN_QUIC : ((u8 const *)d->aux1)[i];
      ok   = sz <= FD_VERIFY_SVC_FRAG_STRIDE && ( !sigs || sz >= FD_VERIFY_SVC_SIG_HDR_SZ );
    }
    ulong const f = d->ibase + i;
    u8 * dst = ing + 64ul * SVC_INGEST_CHUNKS * f;
    if( ok ) for( u32 p = 16u * lane; p < sz; p += 1024u ) *(uint4 *)(dst + p) = *(uint4 const *)(src + p);
    /* a gossip vote's out header: the reference writes four fields into the
       out chunk's stale header (fd_verify_tile.c:90-93); here the rest is 0 */
    if( kind == FD_VERIFY_HIP_IN_GOSSIP && lane < 5u )
      *(uint4 *)(stage + 64ul * (d->stage0 + FD_TXN_HIP_STAGE_CHUNKS * i) + 16u * lane) = make_uint4( 0u, 0u, 0u, 0u );
    if( lane == 0u ) { ing_sz[f] = ok ? (u16)sz : (u16)0xffffu; ing_kind[f] = (u8)kind; ing_tso[f] = tsv; }
  }
  /* INGESTED from the GPU: once every workgroup has passed its loop (all of
     its loads from the links have returned), the last one stores INGESTED
     into each request's slot in the segment, so a tile may reuse its link
     without waiting for the service thread's turn (the service still
     retires the batch by its event before a verify launch reads the HBM
     frags).  done_ctr: this batch's counter, zero at launch; the last
     workgroup puts it back to zero for the next batch on the ingest stream */
  /* Only the links' reads must be over (their values were stored, so they
     have returned): no fence, and relaxed stores -- a system-scope release
     here would write the whole L2 back (the verify kernels' dirty lines
     included) once per request, which measured slower than the host's
     turn it saves */
  if( !done_ctr ) return;
  __syncthreads();
  __shared__ u32 last;
  if( threadIdx.x == 0u ) last = atomicAdd( done_ctr, 1u ) == gridDim.x - 1u;
  __syncthreads();
  if( !last ) return;
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x )
    if( desc[i].state )
      __hip_atomic_store( (u64 *)desc[i].state, (u64)FD_VERIFY_SVC_INGESTED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
  if( threadIdx.x == 0u ) *done_ctr = 0u;
}

/* a verify launch's per-frag arrays (launch frag j = frag i of request d)
   from the requests' ingest frags: one thread per frag */
__global__ __launch_bounds__(256)
void k_svc_assemble( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u16 const * __restrict__ ing_sz,
                     u8 const * __restrict__ ing_kind, u32 const * __restrict__ ing_tso, u32 * __restrict__ in_chunk,
                     u16 * __restrict__ in_sz, u8 * __restrict__ in_kind, u32 * __restrict__ tso, u64 * __restrict__ seedv,
                     u32 * __restrict__ stage_chunk ) {
  __shared__ u64 sbase[SVC_REQ_MAX];
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x ) sbase[i] = desc[i].base;
  __syncthreads();
  ulong const j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  u32 lo = 0u, hi = nreq;
  while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sbase[mid] <= j ) lo = mid; else hi = mid; }
  svc_desc const * d = desc + lo;
  ulong const i = j - d->base, f = d->ibase + i;
  in_chunk[j] = (u32)(SVC_INGEST_CHUNKS * f); in_sz[j] = ing_sz[f]; in_kind[j] = ing_kind[f]; tso[j] = ing_tso[f];
  seedv[j] = d->seed; stage_chunk[j] = (u32)(d->stage0 + FD_TXN_HIP_STAGE_CHUNKS * i);
}

__global__ __launch_bounds__(256)
void k_svc_results( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u16 const * __restrict__ tsz,
                    u64 const * __restrict__ tag, u64 const * __restrict__ bid, u8 const * __restrict__ cnt,
                    signed char const * __restrict__ tcode, u64 const * __restrict__ fdesc, u32 const * __restrict__ tso ) {
  __shared__ u64 sbase[SVC_REQ_MAX];
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x ) sbase[i] = desc[i].base;
  __syncthreads();
  ulong const j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  u32 lo = 0u, hi = nreq;
  while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sbase[mid] <= j ) lo = mid; else hi = mid; }
  u64 const d = fdesc[j];
  u32 const cend = (u32)(d & 0xfffu), psz = (u32)((d >> 12) & 0x7ffu);
  bool const gossip = (d >> 33) & 1u, bad = (d >> 34) & 1u;
  fd_verify_svc_res_t r;
  r.tag = tag[j]; r.bundle_id = bid[j]; r.txn_t_sz = tsz[j]; r.payload_sz = (u16)psz; r.code = tcode[j];
  r.flags = bad ? (u8)FD_VERIFY_SVC_RES_BAD
                : (!gossip && cend < FD_VERIFY_HIP_TXNM_SZ + psz) ? (u8)FD_VERIFY_SVC_RES_HOST : (u8)0;
  r.sig_cnt = cnt[j]; r.rsv0 = 0u; r.tsorig = tso[j]; r.rsv1 = 0u;
  /* straight into the slot's result array in the (registered) segment: a
     wave writes 2 KB contiguous */
  ((fd_verify_svc_res_t *)desc[lo].res)[j - sbase[lo]] = r;
}

/* a signature launch (FD_VERIFY_SVC_REQ_SIGS, include/fd_verify_svc.h
   "clients"): record j of the launch (record i of request d) from its
   ingest frag -- signature, public key, message -- into the verify's
   inputs: the signature and key into the launch's record arrays, the
   message into the request slot's staging frag i (a client's slots are
   never flushed; staging offsets fit the verify's 32-bit msg_off).  One
   wave per record, grid-stride. */
__global__ __launch_bounds__(256)
void k_svc_sigrec( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u8 const * __restrict__ ing,
                   u16 const * __restrict__ ing_sz, u8 * __restrict__ stage, u8 * __restrict__ rsig,
                   u8 * __restrict__ rpub, u32 * __restrict__ rmoff, u32 * __restrict__ rmsz ) {
  __shared__ u64 sbase[SVC_REQ_MAX];
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x ) sbase[i] = desc[i].base;
  __syncthreads();
  u32 const lane = threadIdx.x & 63u;
  for( ulong j = (ulong)blockIdx.x * 4ul + (threadIdx.x >> 6); j < n; j += 4ul * gridDim.x ) {
    u32 lo = 0u, hi = nreq;
    while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sbase[mid] <= j ) lo = mid; else hi = mid; }
    svc_desc const * d = desc + lo;
    ulong const i = j - d->base, f = d->ibase + i;
    u32 const sz = ing_sz[f];
    bool const ok = sz != 0xffffu;                             /* the gather checked 96 <= sz <= the stride */
    u32 const msz = ok ? sz - (u32)FD_VERIFY_SVC_SIG_HDR_SZ : 0u;
    u8 const * src = ing + 64ul * SVC_INGEST_CHUNKS * f;
    ulong const moff = 64ul * (d->stage0 + FD_TXN_HIP_STAGE_CHUNKS * i);
    if( lane < 4u )      *(uint4 *)(rsig + 64ul * j + 16u * lane) = ok ? *(uint4 const *)(src + 16u * lane) : make_uint4( 0u, 0u, 0u, 0u );
    else if( lane < 6u ) *(uint4 *)(rpub + 32ul * j + 16u * (lane - 4u)) = ok ? *(uint4 const *)(src + 16u * lane) : make_uint4( 0u, 0u, 0u, 0u );
    /* the message: 16-B pieces from ingest byte 96 on (both 16-B aligned) */
    for( u32 p = 16u * lane; p < msz; p += 1024u )
      *(uint4 *)(stage + moff + p) = *(uint4 const *)(src + FD_VERIFY_SVC_SIG_HDR_SZ + p);
    if( lane == 0u ) { rmoff[j] = (u32)moff; rmsz[j] = msz; }
  }
}

/* a signature launch's results into the requests' result arrays */
__global__ __launch_bounds__(256)
void k_svc_sigres( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u16 const * __restrict__ ing_sz,
                   signed char const * __restrict__ rcode ) {
  __shared__ u64 sbase[SVC_REQ_MAX];
  for( u32 i = threadIdx.x; i < nreq; i += blockDim.x ) sbase[i] = desc[i].base;
  __syncthreads();
  ulong const j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  u32 lo = 0u, hi = nreq;
  while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sbase[mid] <= j ) lo = mid; else hi = mid; }
  svc_desc const * d = desc + lo;
  u32 const sz = ing_sz[d->ibase + (j - sbase[lo])];
  bool const ok = sz != 0xffffu;
  fd_verify_svc_res_t r;
  r.tag = 0ul; r.bundle_id = 0ul; r.txn_t_sz = 0u; r.payload_sz = ok ? (u16)(sz - FD_VERIFY_SVC_SIG_HDR_SZ) : (u16)0;
  r.code = ok ? rcode[j] : (signed char)-1;                     /* FD_ED25519_ERR_SIG */
  r.flags = ok ? (u8)0 : (u8)FD_VERIFY_SVC_RES_BAD;
  r.sig_cnt = ok ? (u8)1 : (u8)0; r.rsv0 = 0u; r.tsorig = 0u; r.rsv1 = 0u;
  ((fd_verify_svc_res_t *)d->res)[j - sbase[lo]] = r;
}

/* a flush: out entry e's staging frag (its realized bytes, in whole 64-B
   chunks) straight into the tile's out dcache (registered host memory) at the
   entry's chunk; one wave per entry, 16-B stores, a frag's bytes contiguous */
__global__ __launch_bounds__(256)
void k_svc_compact( fd_verify_svc_out_t const * __restrict__ out, ulong m, u8 const * __restrict__ stage,
                    ulong stage0, u8 * __restrict__ dcache, long delta, ulong out_sz, ulong slot_cap,
                    u32 * __restrict__ err ) {
  u32 const lane = threadIdx.x & 63u;
  /* one wave per entry, grid-stride (a capped grid, flush_wgs, loops) */
  for( ulong e = (ulong)blockIdx.x * 4ul + (threadIdx.x >> 6); e < m; e += 4ul * gridDim.x ) {
    fd_verify_svc_out_t const o = out[e];
    if( o.flags & FD_VERIFY_SVC_OUT_HOSTWRITTEN ) continue;
    u32 const len = ((u32)o.sz + 63u) & ~63u;
    long const at = (long)(64ul * (ulong)o.chunk) + delta;
    /* the entry comes from the tile, an untrusted peer: its frag must be one
       of the slot's staging frags (idx below slot_cap, at most a staging
       frag's bytes) and its chunk must lie inside its out dcache.  A bad
       entry is reported (the service aborts at the flush's retirement),
       never read or written (an idx past the slot read other
       tiles' staging or past the allocation) */
    if( (ulong)o.idx >= slot_cap || len > 64u * (u32)FD_TXN_HIP_STAGE_CHUNKS || at < 0 || at + (long)len > (long)out_sz ) {
      if( lane == 0u ) *(volatile u32 *)err = 1u;
      continue;
    }
    u8 const * src = stage + 64ul * (stage0 + FD_TXN_HIP_STAGE_CHUNKS * (ulong)o.idx);
    u8 *       dst = dcache + at;
    for( u32 p = 16u * lane; p < len; p += 1024u ) *(uint4 *)(dst + p) = *(uint4 const *)(src + p);
  }
}

/* one flush of a flush batch (64 B): k_svc_compact's arguments */
struct __attribute__((aligned(16))) svc_fdesc {
  u64 base;        /* the flush's first entry in the batch */
  u64 out;         /* its out entries (device address) */
  u64 stage0;
  u64 dcache;      /* the tile's out dcache (device address) */
  long delta;
  u64 out_sz;
  u64 err;         /* the tile's error flag (device address) */
  u64 rsv;
};
static_assert( sizeof(svc_fdesc) == 64, "svc_fdesc layout" );

/* a flush batch: the newly posted flushes of every tile in one launch
   (one wave per out entry, as k_svc_compact; entry j of the batch is entry
   j - base of the flush whose range holds it) */
__global__ __launch_bounds__(256)
void k_svc_compact_batch( svc_fdesc const * __restrict__ fd, u32 nf, ulong n, u8 const * __restrict__ stage,
                          ulong slot_cap ) {
  __shared__ u64 sbase[SVC_FB_FLUSH_MAX];
  for( u32 i = threadIdx.x; i < nf; i += blockDim.x ) sbase[i] = fd[i].base;
  __syncthreads();
  u32 const lane = threadIdx.x & 63u;
  for( ulong j = (ulong)blockIdx.x * 4ul + (threadIdx.x >> 6); j < n; j += 4ul * gridDim.x ) {
    u32 lo = 0u, hi = nf;
    while( hi - lo > 1u ) { u32 mid = (lo + hi) >> 1; if( sbase[mid] <= j ) lo = mid; else hi = mid; }
    svc_fdesc const * d = fd + lo;
    fd_verify_svc_out_t const o = ((fd_verify_svc_out_t const *)d->out)[j - sbase[lo]];
    if( o.flags & FD_VERIFY_SVC_OUT_HOSTWRITTEN ) continue;
    u32 const len = ((u32)o.sz + 63u) & ~63u;
    long const at = (long)(64ul * (ulong)o.chunk) + d->delta;
    /* the tile is an untrusted peer: k_svc_compact's checks */
    if( (ulong)o.idx >= slot_cap || len > 64u * (u32)FD_TXN_HIP_STAGE_CHUNKS || at < 0 || at + (long)len > (long)d->out_sz ) {
      if( lane == 0u ) *(volatile u32 *)d->err = 1u;
      continue;
    }
    u8 const * src = stage + 64ul * (d->stage0 + FD_TXN_HIP_STAGE_CHUNKS * (ulong)o.idx);
    u8 *       dst = (u8 *)d->dcache + at;
    for( u32 p = 16u * lane; p < len; p += 1024u ) *(uint4 *)(dst + p) = *(uint4 const *)(src + p);
  }
}

/**********************************************************************/
/* The IO engine: one persistent kernel (k_svc_io) that does the ingest
   and the flushes on the GPU, with no host call between a tile's post and
   the GPU's copy.

   Why.  A range request holds its quic_verify link until the GPU has read
   its frags.  With a kernel launched per ingest, the time from a tile's
   post to INGESTED was the service thread's turn, a launch and the kernel's
   dispatch beside 2-5 ms verify launches: ~0.5 ms on average at the
   reference's depth of 16384 (the flow-controlled stage ran 29.7 M frags/s
   there, one link lap per ~550 us), and a paced producer lapped the tiles
   above 6-12 M frags/s.  Here a leader wave polls
   the tiles' request and flush rings in the segment (mapped host memory,
   system-coherent loads) and splits each new request or flush into jobs of
   IO_JOB frags on a ring in HBM; the other waves take jobs, copy, and the
   wave that finishes a request's last job stores INGESTED into the segment
   itself.  The service thread only merges ingested requests into verify
   launches.

   Memory ordering (MI355X_MICROARCH.md, inter-workgroup visibility: the
   XCDs' L2s are not coherent and a CU's L1 is never refreshed by other
   CUs' stores):
   - host memory (the segment, the links, the out dcaches) is read with
     sc0 sc1 (system-coherent) loads and written with sc0 sc1 stores;
   - HBM shared between waves of this kernel (descriptors, job ring,
     counters) is written with sc1 stores or agent-scope atomics and read
     with sc1 loads, a flag or counter written only after the writing wave's
     s_waitcnt vmcnt(0);
   - the ingest frags (HBM) are stored sc1 and read by later verify kernel
     launches; the staging frags a flush reads were written by a verify
     kernel that ended before the tile saw RESULTS, and are read sc1.
   Every wave leaves when the host sets stop: the worker's job wait and
   the leader's loop both poll it, so the grid drains (teardown waits on an
   event recorded behind the kernel, with a deadline). */

#define IO_RING   16384ul   /* job ring entries (power of 2) */
#define IO_JOB    32ul      /* ingest frags per job */
#define IO_FJOB   64ul      /* flush entries per job */
#define IO_F      4u        /* frags a wave moves per step (their loads in flight together) */
#define IO_FQ     64ul      /* flushes taken and not retired, per tile */
#define IO_WGS    32ul      /* default grid: 127 worker waves, 4 workgroups per XCD */
#define IO_CONS   (1ull << 63)

typedef u32 io_v4 __attribute__((ext_vector_type(4)));

struct svc_io_link { u64 mcache, mask, base, chunk0, wmark, set; };
struct svc_io_tile { u64 out, out_sz; long delta; u64 rsv; };
struct svc_io_cfg {
  u64 seg, tile_cnt, req_depth, slot_cap, frag_cap, tile_sz, slot_sz, req_off, out_off, frag_off;
  u64 ing, ing_sz, ing_kind, ing_tso, stage;
  u64 ring, idesc, iremain, fdesc, fremain, fdone, dctl, hctl, hvd;
  u64 dbg;                    /* FD_VERIFY_SVC_IO_DBG: steps of the leader to leave out (diagnostics) */
  svc_io_link link[FD_VERIFY_SVC_LINK_MAX];
  svc_io_tile tile[FD_VERIFY_SVC_TILE_MAX];
};

/* host-mapped control block (coherent pinned memory) */
struct svc_io_hctl {
  u64 stop;                   /* host: 1 = every wave leaves */
  u64 err, err_a, err_b, err_c;   /* GPU: the first error (IO_ERR_*) and its details */
  u64 beat;                   /* leader loops / 256 */
  u64 st[8];                  /* the device counters (IO_ST_*), copied by the leader */
  u64 dbg[8];                 /* the leader's state, every 256 loops: ring tail, workers' claims, tile 0..3 takes,
                                 tile 0 flush takes, tile 0 flushes retired */
  u64 rsv[10];
};
/* device control block (HBM) */
struct svc_io_dctl {
  u64 claim; u64 rsv0[15];    /* job ring positions claimed by workers */
  u64 stop;  u64 rsv1[15];
  u64 err;   u64 rsv2[15];
  u64 st[8]; u64 rsv3[8];
};
struct svc_io_job { u64 tag; u64 pay; };            /* tag pos+1 when written, IO_CONS|pos once taken */
struct svc_io_fdesc { u64 out, m, stage0, tile, seq, rsv[3]; };

#define IO_ERR_RANGE  1ul   /* a: tile, b: slot, c: link */
#define IO_ERR_FRAGS  2ul   /* a: tile, b: slot, c: n */
#define IO_ERR_KIND   3ul   /* a: tile, b: slot, c: kind */
#define IO_ERR_ID     4ul   /* a: tile, b: slot, c: id */
#define IO_ERR_FLUSH  5ul   /* a: tile, b: flush, c: slot */
#define IO_ERR_ENTRY  6ul   /* a: tile, b: flush, c: entry */
#define IO_ERR_DESC   7ul   /* a: descriptor, b: job start, c: kind or frag count (a job whose descriptor was not
                               the leader's: never followed to memory) */

#define IO_ST_REQS    0     /* requests ingested */
#define IO_ST_FRAGS   1     /* frags ingested */
#define IO_ST_FLUSHES 2     /* flushes done */
#define IO_ST_FLFRAGS 3     /* frags flushed */
#define IO_ST_JOBS    4     /* jobs done */
#define IO_ST_EXITED  5     /* waves that left */
#define IO_ST_TAKEN   6     /* jobs taken off the ring */
#define IO_ST_LOADED  7     /* ingest jobs past their loads and stores */

/* global (not flat) accesses: the sc bits and the counters the visibility
   rules are stated for (MI355X_MICROARCH.md: never flat_ for these) */
typedef __attribute__((address_space(1))) u64 io_gu64;
#define IO_G( p ) ((io_gu64 *)(u64)(p))
/* a host-memory word the host writes while the engine runs (the rings, the
   stop flag): a system-scope load (sc0 sc1), which fine-grained host memory
   serves from the host's memory (the memory model's system coherence; an
   atomic add of zero over PCIe took ~50 us a read, profiles/r06g) */
static __device__ __forceinline__ u64 io_lds( u64 const * p ) { return __hip_atomic_load( IO_G( p ), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM ); }
static __device__ __forceinline__ void io_sts( u64 * p, u64 v ) { __hip_atomic_store( IO_G( p ), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM ); }
/* the engine's own HBM words (job ring, descriptors, counters) are read and
   written by atomics, which execute at the memory side and are never
   served from an XCD's L2 (MI355X_MICROARCH.md): a word written by a wave
   on one XCD is what a wave on another reads, whatever either L2 held */
static __device__ __forceinline__ u64 io_lda( u64 const * p ) {
  u64 r, z = 0ul;
  asm volatile( "global_atomic_add_x2 %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"( r ) : "v"( p ), "v"( z ) : "memory" );
  return r;
}
/* a poll's cheap form: an sc1 load (past this CU's L1, served by the XCD's
   L2); the worker's job wait polls with it and falls back to io_lda every
   16th read, so a copy its L2 may keep is never trusted for long */
static __device__ __forceinline__ u64 io_ldc( u64 const * p ) { return __hip_atomic_load( IO_G( p ), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
static __device__ __forceinline__ void io_sta( u64 * p, u64 v ) { (void)__hip_atomic_exchange( IO_G( p ), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
static __device__ __forceinline__ u64 io_adda( u64 * p, u64 v ) { return __hip_atomic_fetch_add( IO_G( p ), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ); }
/* FD_VERIFY_SVC_IO_DBG bit 64: the leader's host polls as system atomics (an A/B) */
static __device__ __forceinline__ u64 io_ldx( u64 const * p ) {
  u64 r, z = 0ul;
  asm volatile( "global_atomic_add_x2 %0, %1, %2, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"( r ) : "v"( p ), "v"( z ) : "memory" );
  return r;
}
#define IO_LDS( p ) ( (C.dbg & 64ul) ? io_ldx( p ) : io_lds( p ) )
static __device__ __forceinline__ void io_drain( void ) { asm volatile( "s_waitcnt vmcnt(0)" ::: "memory" ); }
/* a raw buffer over [p, p+n): accesses past n read 0 and write nothing */
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t io_rsrc( u64 p, u32 n ) {
  p = ((u64)(u32)__builtin_amdgcn_readfirstlane( (u32)(p >> 32) ) << 32) | (u64)(u32)__builtin_amdgcn_readfirstlane( (u32)p );
  return __builtin_amdgcn_make_buffer_rsrc( (void *)p, (short)0, (int)__builtin_amdgcn_readfirstlane( n ), 0x00020000 );
}
#define IO_SYS 17   /* sc0 sc1: system coherent (host memory) */
#define IO_SC1 16   /* sc1: past this CU's L1 (HBM shared with other CUs) */
static __device__ __forceinline__ u64 io_shfl64( u64 v, u32 l ) {
  return (u64)(u32)__shfl( (int)(u32)v, (int)l ) | ((u64)(u32)__shfl( (int)(u32)(v >> 32), (int)l ) << 32);
}
/* the first active lane's value, in SGPRs (readfirstlane returns an int:
   each half goes through u32 before it widens, or a low half with bit 31
   set would sign-extend over the high half -- a pointer so corrupted was
   the engine's first fault, profiles/r06h) */
static __device__ __forceinline__ u64 io_uni( u64 v ) {
  return ((u64)(u32)__builtin_amdgcn_readfirstlane( (u32)(v >> 32) ) << 32) | (u64)(u32)__builtin_amdgcn_readfirstlane( (u32)v );
}

/* the first error wins; the host aborts on it (the reference ends a tile
   with FD_LOG_ERR on a corrupt frag or a bad request) */
static __device__ void
io_err( svc_io_cfg const & C, u64 code, u64 a, u64 b, u64 c ) {
  svc_io_dctl * dc = (svc_io_dctl *)C.dctl;
  svc_io_hctl * hc = (svc_io_hctl *)C.hctl;
  u64 zero = 0;
  if( (threadIdx.x & 63u) == (u32)__builtin_ctzll( __ballot( 1 ) ) &&
      __hip_atomic_compare_exchange_strong( IO_G( &dc->err ), &zero, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT ) ) {
    io_sts( &hc->err_a, a ); io_sts( &hc->err_b, b ); io_sts( &hc->err_c, c );
    io_drain();
    io_sts( &hc->err, code );
  }
}

/* ingest job: frags [start, start+IO_JOB) of request r (its descriptor made
   by the leader): k_svc_gather's checks and copy, IO_F frags per step with
   their loads in flight together */
static __device__ __attribute__((noinline)) void
io_ingest( svc_io_cfg const & C, u32 r, u64 start ) {
  u32 const lane = threadIdx.x & 63u;
  u64 const dw = lane < 16u ? io_lda( (u64 const *)(C.idesc + 128ul * r) + lane ) : 0ul;
  u64 const n = io_uni( io_shfl64( dw, 1 ) ), kind = io_uni( io_shfl64( dw, 2 ) ), src = io_uni( io_shfl64( dw, 3 ) );
  u64 const aux0 = io_uni( io_shfl64( dw, 4 ) ), aux1 = io_uni( io_shfl64( dw, 5 ) );
  u64 const first = io_uni( io_shfl64( dw, 6 ) ), stride = io_uni( io_shfl64( dw, 7 ) );
  u64 const lmask = io_uni( io_shfl64( dw, 8 ) ), chunk0 = io_uni( io_shfl64( dw, 9 ) ), wmark = io_uni( io_shfl64( dw, 10 ) );
  u64 const stage0 = io_uni( io_shfl64( dw, 12 ) ), ibase = io_uni( io_shfl64( dw, 13 ) ), rq = io_uni( io_shfl64( dw, 15 ) );
  bool const range = kind == FD_VERIFY_SVC_REQ_RANGE;
  /* the descriptor is the leader's (written, drained, then the job's tag):
     one that is not -- a stale line -- is reported, never followed */
  bool const ok = start < n && ibase == (u64)r * C.slot_cap && rq && src &&
                  ( range ? ( n <= C.slot_cap && aux0 && lmask && stride ) : ( kind == FD_VERIFY_SVC_REQ_FRAGS &&
                                                                              n <= C.frag_cap && aux0 && aux1 ) );
  if( !ok ) { io_err( C, IO_ERR_DESC, r, start, range ? n : kind ); return; }
  u64 const end = start + IO_JOB < n ? start + IO_JOB : n;
  /* the request's lines and bytes (host memory, written by host cores
     before the tile posted it) are read with system-scope loads, which the
     host's memory serves; FD_VERIFY_SVC_IO_DBG bit 16 adds a system-scope
     acquire here (an A/B: it invalidates the XCD's L2) */
  if( C.dbg & 16ul ) __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "" );
  for( u64 i = start; i < end; i += IO_F ) {
    u32 const nf = (u32)(end - i < IO_F ? end - i : IO_F);
    /* lane f < nf: frag i+f's size, kind, tsorig, source, and whether it
       passes the stem's and during_frag's checks */
    u32 msz = 0u, mkind = FD_VERIFY_HIP_IN_QUIC, mtso = 0u; u64 msrc = 0ul; bool mok = false;
    if( range ) {
      /* lanes 2f, 2f+1 read frag f's mcache line halves (seq, sig | chunk,
         sz, ctl, tsorig, tspub) */
      __amdgpu_buffer_rsrc_t rm = io_rsrc( src, (u32)(32ul * (lmask + 1ul)) );
      u64 const lseq = first + (i + (lane >> 1)) * stride;
      io_v4 v = { 0u, 0u, 0u, 0u };
      if( lane < 2u * nf ) v = __builtin_amdgcn_raw_buffer_load_b128( rm, (u32)(32ul * (lseq & lmask)) + 16u * (lane & 1u), 0, IO_SYS );
      u32 const s0 = (u32)__shfl( (int)v.x, (int)(2u * lane) ), s1 = (u32)__shfl( (int)v.y, (int)(2u * lane) );
      u32 const ch = (u32)__shfl( (int)v.x, (int)(2u * lane + 1u) ), szc = (u32)__shfl( (int)v.y, (int)(2u * lane + 1u) );
      mtso = (u32)__shfl( (int)v.z, (int)(2u * lane + 1u) );
      u64 const seq = first + (i + lane) * stride;
      msz  = szc & 0xffffu;
      mok  = lane < nf && ((u64)s0 | ((u64)s1 << 32)) == seq && (u64)ch >= chunk0 && (u64)ch <= wmark &&
             msz <= FD_VERIFY_HIP_TPU_RAW_MTU;
      msrc = aux0 + 64ul * ch;
    } else {
      __amdgpu_buffer_rsrc_t rs = io_rsrc( aux0 + 2ul * i, 2u * nf );
      __amdgpu_buffer_rsrc_t rk = io_rsrc( aux1 + i, nf );
      msz   = __builtin_amdgcn_raw_buffer_load_b16( rs, 2u * lane, 0, IO_SYS );
      mkind = __builtin_amdgcn_raw_buffer_load_b8( rk, lane, 0, IO_SYS );
      mok   = lane < nf && msz <= FD_VERIFY_SVC_FRAG_STRIDE;
      msrc  = src + FD_VERIFY_SVC_FRAG_STRIDE * (i + lane);
    }
    u32 const mnb = mok ? (msz + 15u) & ~15u : 0u;
    io_v4 a[IO_F], b[IO_F];
#pragma unroll
    for( u32 f = 0; f < IO_F; f++ ) {
      __amdgpu_buffer_rsrc_t rs = io_rsrc( io_shfl64( msrc, f ), (u32)__shfl( (int)mnb, (int)f ) );
      a[f] = __builtin_amdgcn_raw_buffer_load_b128( rs, 16u * lane, 0, IO_SYS );
      b[f] = __builtin_amdgcn_raw_buffer_load_b128( rs, 16u * lane + 1024u, 0, IO_SYS );
    }
#pragma unroll
    for( u32 f = 0; f < IO_F; f++ ) {
      __amdgpu_buffer_rsrc_t rd = io_rsrc( C.ing + 64ul * SVC_INGEST_CHUNKS * (ibase + i + f), (u32)__shfl( (int)mnb, (int)f ) );
      __builtin_amdgcn_raw_buffer_store_b128( a[f], rd, 16u * lane, 0, IO_SC1 );
      __builtin_amdgcn_raw_buffer_store_b128( b[f], rd, 16u * lane + 1024u, 0, IO_SC1 );
      /* a gossip vote's out header: the reference writes four fields into
         the out chunk's stale header (fd_verify_tile.c:90-93); here the rest is 0 */
      if( f < nf && (u32)__shfl( (int)mkind, (int)f ) == FD_VERIFY_HIP_IN_GOSSIP ) {
        __amdgpu_buffer_rsrc_t rg = io_rsrc( C.stage + 64ul * (stage0 + FD_TXN_HIP_STAGE_CHUNKS * (i + f)), 80u );
        __builtin_amdgcn_raw_buffer_store_b128( io_v4{ 0u, 0u, 0u, 0u }, rg, 16u * lane, 0, IO_SC1 );
      }
    }
    __amdgpu_buffer_rsrc_t rz = io_rsrc( C.ing_sz + 2ul * (ibase + i), 2u * nf );
    __amdgpu_buffer_rsrc_t rk = io_rsrc( C.ing_kind + (ibase + i), nf );
    __amdgpu_buffer_rsrc_t rt = io_rsrc( C.ing_tso + 4ul * (ibase + i), 4u * nf );
    __builtin_amdgcn_raw_buffer_store_b16( (u16)(mok ? msz : 0xffffu), rz, 2u * lane, 0, IO_SC1 );
    __builtin_amdgcn_raw_buffer_store_b8( (u8)mkind, rk, lane, 0, IO_SC1 );
    __builtin_amdgcn_raw_buffer_store_b32( range ? mtso : 0u, rt, 4u * lane, 0, IO_SC1 );
  }
  svc_io_dctl * dc = (svc_io_dctl *)C.dctl;
  io_drain();
  if( lane == 0u ) io_adda( &dc->st[IO_ST_LOADED], 1ul );
  u64 const cnt = end - start;
  if( lane == 0u ) {
    u64 const left = io_adda( (u64 *)C.iremain + r, (u64)0 - cnt );
    io_adda( &dc->st[IO_ST_FRAGS], cnt ); io_adda( &dc->st[IO_ST_JOBS], 1ul );
    if( left == cnt ) {                                   /* the request's last job: its frags are in HBM */
      io_adda( &dc->st[IO_ST_REQS], 1ul );
      io_sts( (u64 *)rq, FD_VERIFY_SVC_INGESTED );
    }
  }
}

/* flush job: out entries [start, start+IO_FJOB) of flush fi, k_svc_compact's
   checks and copy (staging HBM -> the tile's out dcache in host memory) */
static __device__ __attribute__((noinline)) void
io_flush( svc_io_cfg const & C, u32 fi, u64 start ) {
  u32 const lane = threadIdx.x & 63u;
  u64 const fw = lane < 5u ? io_lda( (u64 const *)(C.fdesc + sizeof(svc_io_fdesc) * fi) + lane ) : 0ul;
  u64 const out = io_uni( io_shfl64( fw, 0 ) ), m = io_uni( io_shfl64( fw, 1 ) ), stage0 = io_uni( io_shfl64( fw, 2 ) );
  u64 const t = io_uni( io_shfl64( fw, 3 ) ), seq = io_uni( io_shfl64( fw, 4 ) );
  if( t >= C.tile_cnt || !out || start >= m || m > C.slot_cap || fi != t * IO_FQ + (seq & (IO_FQ - 1ul)) ) {
    io_err( C, IO_ERR_DESC, fi | (1ull << 31), start, m );
    return;
  }
  u64 const dc_out = C.tile[t].out, out_sz = C.tile[t].out_sz;
  long const delta = C.tile[t].delta;
  u64 const end = start + IO_FJOB < m ? start + IO_FJOB : m;
  /* the staging frags (HBM, written by a verify launch that ended before
     the tile saw RESULTS): an agent-scope acquire drops this CU's L1 copies
     of the slot's previous frags (the out entries are host memory, read with
     system-scope loads) */
  __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "agent" );
  for( u64 e = start; e < end; e += IO_F ) {
    u32 const nf = (u32)(end - e < IO_F ? end - e : IO_F);
    __amdgpu_buffer_rsrc_t ro = io_rsrc( out + 16ul * e, 16u * nf );
    io_v4 const o = __builtin_amdgcn_raw_buffer_load_b128( ro, 16u * lane, 0, IO_SYS );
    u32 const idx = o.x, len = ((o.z & 0xffffu) + 63u) & ~63u;
    bool const hw = ((o.z >> 16) & FD_VERIFY_SVC_OUT_HOSTWRITTEN) != 0u;
    long const at = (long)(64ul * (u64)o.y) + delta;
    bool const bad = lane < nf && !hw && ((u64)idx >= C.slot_cap || len > 64u * (u32)FD_TXN_HIP_STAGE_CHUNKS ||
                                          at < 0 || at + (long)len > (long)out_sz);
    u64 const bm = __ballot( bad );
    if( bm ) io_err( C, IO_ERR_ENTRY, t, seq, e + __builtin_ctzll( bm ) );
    u32 const mnb = lane < nf && !hw && !bad ? len : 0u;
    u64 const msrc = C.stage + 64ul * (stage0 + FD_TXN_HIP_STAGE_CHUNKS * (u64)idx);
    u64 const mdst = dc_out + (u64)at;
    io_v4 a[IO_F], b[IO_F], c[IO_F];
#pragma unroll
    for( u32 f = 0; f < IO_F; f++ ) {
      __amdgpu_buffer_rsrc_t rs = io_rsrc( io_shfl64( msrc, f ), (u32)__shfl( (int)mnb, (int)f ) );
      a[f] = __builtin_amdgcn_raw_buffer_load_b128( rs, 16u * lane, 0, IO_SC1 );
      b[f] = __builtin_amdgcn_raw_buffer_load_b128( rs, 16u * lane + 1024u, 0, IO_SC1 );
      c[f] = __builtin_amdgcn_raw_buffer_load_b128( rs, 16u * lane + 2048u, 0, IO_SC1 );
    }
#pragma unroll
    for( u32 f = 0; f < IO_F; f++ ) {
      __amdgpu_buffer_rsrc_t rd = io_rsrc( io_shfl64( mdst, f ), (u32)__shfl( (int)mnb, (int)f ) );
      __builtin_amdgcn_raw_buffer_store_b128( a[f], rd, 16u * lane, 0, IO_SYS );
      __builtin_amdgcn_raw_buffer_store_b128( b[f], rd, 16u * lane + 1024u, 0, IO_SYS );
      __builtin_amdgcn_raw_buffer_store_b128( c[f], rd, 16u * lane + 2048u, 0, IO_SYS );
    }
  }
  svc_io_dctl * dc = (svc_io_dctl *)C.dctl;
  io_drain();
  if( lane == 0u ) io_adda( &dc->st[IO_ST_LOADED], 1ul );
  u64 const cnt = end - start;
  if( lane == 0u ) {
    u64 const left = io_adda( (u64 *)C.fremain + fi, (u64)0 - cnt );
    io_adda( &dc->st[IO_ST_FLFRAGS], cnt ); io_adda( &dc->st[IO_ST_JOBS], 1ul );
    if( left == cnt ) io_sta( (u64 *)C.fdone + fi, seq + 1ul );   /* the leader retires flushes in order */
  }
}

/* push jobs [0, J) of descriptor idx (bit 31: a flush) at ring positions
   tail.. (each position's previous occupant must have been taken) */
static __device__ bool
io_push( svc_io_cfg const & C, u64 & tail, u32 idx, u64 J, u64 step ) {
  u32 const lane = threadIdx.x & 63u;
  svc_io_job * ring = (svc_io_job *)C.ring;
  svc_io_hctl * hc = (svc_io_hctl *)C.hctl;
  for( u64 k0 = 0; k0 < J; k0 += 64ul ) {
    u64 const k = k0 + lane, pos = tail + k;
    svc_io_job * j = ring + (pos & (IO_RING - 1ul));
    if( k < J ) {
      for( ;; ) {
        u64 const tg = io_lda( &j->tag );
        if( !tg || tg == (IO_CONS | (pos - IO_RING)) ) break;
        if( IO_LDS( &hc->stop ) ) break;
        __builtin_amdgcn_s_sleep( 4 );
      }
      io_sta( &j->pay, ((k * step) << 32) | (u64)idx );
    }
    io_drain();
    if( k < J ) io_sta( &j->tag, pos + 1ul );
  }
  tail += J;
  return true;
}

static __device__ void
io_leader( svc_io_cfg const & C ) {
  u32 const lane = threadIdx.x & 63u;
  svc_io_dctl * dc = (svc_io_dctl *)C.dctl;
  svc_io_hctl * hc = (svc_io_hctl *)C.hctl;
  u64 const T = C.tile_cnt, D = C.req_depth;
  bool const tl = lane < T;
  u64 const tb = C.seg + FD_VERIFY_SVC_ALIGN + (u64)lane * C.tile_sz;   /* this lane's tile block */
  u64 take = 0, ftake = 0, ffin = 0, tail = 0, beat = 0;
  bool dead = false;
  for( ;; ) {
    if( !(++beat & 255ul) ) {                               /* counters for the host, every 256th loop */
      if( lane < 8u ) io_sts( &hc->st[lane], io_lda( &dc->st[lane] ) );
      u64 dv = lane == 0u ? tail : lane == 1u ? io_lda( &dc->claim ) : 0ul;
      u64 const tk = io_shfl64( take, lane - 2u );
      if( lane >= 2u && lane < 6u ) dv = tk;
      u64 const f0 = io_shfl64( ftake, 0 ), r0 = io_shfl64( ffin, 0 );
      if( lane == 6u ) dv = f0;
      if( lane == 7u ) dv = r0;
      if( lane < 8u ) io_sts( &hc->dbg[lane], dv );
      if( lane == 0u ) io_sts( &hc->beat, beat >> 8 );
    }
    if( IO_LDS( &hc->stop ) ) { if( lane == 0u ) io_sta( &dc->stop, 1ul ); break; }
    bool active = false;

    /* 1. requests: each tile's next slot in ring order */
    u64 const slot = take & (D - 1ul);
    u64 const rq   = tb + sizeof(fd_verify_svc_tile_t) + slot * sizeof(fd_verify_svc_req_t);
    u64 const state = tl && !dead ? IO_LDS( (u64 const *)rq ) : 0ul;
    bool const posted = state == FD_VERIFY_SVC_POSTED;
    u64 const id = posted ? IO_LDS( (u64 const *)(rq + offsetof( fd_verify_svc_req_t, id )) ) : 0ul;
    bool const fresh = posted && id == take;
    bool const wrong = posted && id != take && id + D != take;
    if( __ballot( wrong ) ) {
      u64 const w = __ballot( wrong );
      u32 const t = __builtin_ctzll( w );
      io_err( C, IO_ERR_ID, t, io_shfl64( slot, t ), io_shfl64( id, t ) );
      if( wrong ) dead = true;
    }
    for( u64 fm = __ballot( fresh ); fm; fm &= fm - 1ul ) {
      u32 const t  = __builtin_ctzll( fm );
      u64 const rt = io_uni( io_shfl64( rq, t ) ), st = io_uni( io_shfl64( slot, t ) );
      u64 const w  = lane < 9u ? IO_LDS( (u64 const *)rt + lane ) : 0ul;      /* state kind link seq0 seq_cnt rr_cnt rr_idx n seed */
      u64 const kind = io_uni( io_shfl64( w, 1 ) ), link = io_uni( io_shfl64( w, 2 ) ), seq0 = io_uni( io_shfl64( w, 3 ) );
      u64 const seq_cnt = io_uni( io_shfl64( w, 4 ) ), rr_cnt = io_uni( io_shfl64( w, 5 ) ), rr_idx = io_uni( io_shfl64( w, 6 ) );
      u64 const n = io_uni( io_shfl64( w, 7 ) ), seed = io_uni( io_shfl64( w, 8 ) );
      u64 const r = (u64)t * D + st;
      u64 d[16] = { 0ul };                                 /* svc_desc */
      d[1] = n; d[2] = kind; d[11] = seed; d[12] = r * C.slot_cap * FD_TXN_HIP_STAGE_CHUNKS; d[13] = r * C.slot_cap;
      d[15] = rt;                                          /* the request (its state word) */
      u64 err = 0ul, ec = 0ul;
      if( kind == FD_VERIFY_SVC_REQ_RANGE ) {
        svc_io_link const * L = link < FD_VERIFY_SVC_LINK_MAX ? &C.link[link] : (svc_io_link const *)0;
        u64 cnt = 0ul, fst = 0ul;
        if( rr_cnt && rr_idx < rr_cnt && seq_cnt ) {
          fst = seq0 + (rr_idx + rr_cnt - seq0 % rr_cnt) % rr_cnt;
          cnt = fst < seq0 + seq_cnt ? (seq0 + seq_cnt - 1ul - fst) / rr_cnt + 1ul : 0ul;
        }
        if( !L || !L->set || !rr_cnt || rr_idx >= rr_cnt || seq_cnt > L->mask + 1ul || n != cnt || n > C.slot_cap ) {
          err = IO_ERR_RANGE; ec = link;
        } else {
          d[3] = L->mcache; d[4] = L->base; d[6] = fst; d[7] = rr_cnt; d[8] = L->mask; d[9] = L->chunk0; d[10] = L->wmark;
        }
      } else if( kind == FD_VERIFY_SVC_REQ_FRAGS ) {
        if( n > C.frag_cap ) { err = IO_ERR_FRAGS; ec = n; }
        u64 const fa = tb - (u64)lane * C.tile_sz + (u64)t * C.tile_sz + C.req_off + st * C.slot_sz + C.frag_off;
        d[3] = fa; d[4] = fa + C.frag_cap * FD_VERIFY_SVC_FRAG_STRIDE; d[5] = d[4] + 2ul * C.frag_cap;
      } else {
        err = IO_ERR_KIND; ec = kind;
      }
      if( err ) {
        io_err( C, err, t, st, ec );
        if( lane == t ) { dead = true; take++; }
        continue;
      }
      /* the descriptor (HBM, the workers') and the validated size and seed
         (host, the service thread's verify launch), then the jobs */
      u64 dv = 0ul;
#pragma unroll
      for( u32 k = 0; k < 16u; k++ ) if( lane == k ) dv = d[k];
      if( !(C.dbg & 1ul) && lane < 16u ) io_sta( (u64 *)(C.idesc + 128ul * r) + lane, dv );
      if( !(C.dbg & 2ul) && lane < 2u ) io_sts( (u64 *)C.hvd + 2ul * r + lane, lane ? seed : n );
      if( !(C.dbg & 4ul) && lane == 0u ) io_sta( (u64 *)C.iremain + r, n );
      io_drain();
      if( !n ) { if( !(C.dbg & 8ul) && lane == 0u ) io_sts( (u64 *)rt, FD_VERIFY_SVC_INGESTED ); }
      else io_push( C, tail, (u32)r, (n + IO_JOB - 1ul) / IO_JOB, IO_JOB );
      if( lane == t ) take++;
      active = true;
    }

    /* 2. flushes: each tile's newly posted flush ring entries */
    u64 const fpost = tl && !dead ? IO_LDS( (u64 const *)(tb + offsetof( fd_verify_svc_tile_t, flush_post )) ) : 0ul;
    bool const fnew = tl && !dead && ftake < fpost && ftake - ffin < IO_FQ;
    for( u64 fm = __ballot( fnew ); fm; fm &= fm - 1ul ) {
      u32 const t = __builtin_ctzll( fm );
      u64 const k = io_uni( io_shfl64( ftake, t ) );
      u64 const tbt = C.seg + FD_VERIFY_SVC_ALIGN + (u64)t * C.tile_sz;
      u64 const fe = tbt + offsetof( fd_verify_svc_tile_t, flush ) + (k & (FD_VERIFY_SVC_FLUSH_DEPTH - 1ul)) * sizeof(fd_verify_svc_flush_t);
      u64 const w = lane < 3u ? IO_LDS( (u64 const *)fe + lane ) : 0ul;
      u64 const fslot = io_uni( io_shfl64( w, 0 ) ), lo = io_uni( io_shfl64( w, 1 ) ), hi = io_uni( io_shfl64( w, 2 ) );
      if( fslot >= D || lo > hi || hi > C.slot_cap ) {
        io_err( C, IO_ERR_FLUSH, t, k, fslot );
        if( lane == t ) dead = true;
        continue;
      }
      u64 const fi = (u64)t * IO_FQ + (k & (IO_FQ - 1ul));
      u64 const r  = (u64)t * D + fslot;
      u64 fv = 0ul;
      if( lane == 0u ) fv = tbt + C.req_off + fslot * C.slot_sz + C.out_off + 16ul * lo;
      if( lane == 1u ) fv = hi - lo;
      if( lane == 2u ) fv = r * C.slot_cap * FD_TXN_HIP_STAGE_CHUNKS;
      if( lane == 3u ) fv = t;
      if( lane == 4u ) fv = k;
      if( lane < 5u ) io_sta( (u64 *)(C.fdesc + sizeof(svc_io_fdesc) * fi) + lane, fv );
      if( lane == 0u ) io_sta( (u64 *)C.fremain + fi, hi - lo );
      io_drain();
      if( hi == lo ) { if( lane == 0u ) io_sta( (u64 *)C.fdone + fi, k + 1ul ); }
      else io_push( C, tail, (u32)fi | 0x80000000u, (hi - lo + IO_FJOB - 1ul) / IO_FJOB, IO_FJOB );
      if( lane == t ) ftake++;
      active = true;
    }

    /* 3. finished flushes, in order per tile: flush_done */
    bool adv = false;
    for( ;; ) {
      bool const can = tl && ffin < ftake && io_lda( (u64 const *)C.fdone + (u64)lane * IO_FQ + (ffin & (IO_FQ - 1ul)) ) == ffin + 1ul;
      if( !__ballot( can ) ) break;
      if( can ) { ffin++; adv = true; }
    }
    if( __ballot( adv ) ) {
      __builtin_amdgcn_fence( __ATOMIC_RELEASE, "" );
      if( adv ) io_sts( (u64 *)(tb + offsetof( fd_verify_svc_tile_t, flush_done )), ffin );
      active = true;
    }
    if( !active ) __builtin_amdgcn_s_sleep( 8 );
  }
  if( lane == 0u ) io_adda( &dc->st[IO_ST_EXITED], 1ul );
}

static __device__ void
io_worker( svc_io_cfg const & C ) {
  u32 const lane = threadIdx.x & 63u;
  svc_io_dctl * dc = (svc_io_dctl *)C.dctl;
  svc_io_job * ring = (svc_io_job *)C.ring;
  for( ;; ) {
    u64 p = 0ul;
    if( lane == 0u ) p = io_adda( &dc->claim, 1ul );
    p = io_uni( io_shfl64( p, 0 ) );
    svc_io_job * j = ring + (p & (IO_RING - 1ul));
    u32 nap = 1u;
    bool stop = false;
    for( u32 it = 1u;; it++ ) {
      /* sc1 polls, an atomic read every 16th (and for the stop flag, every
         32nd): 127 waves' atomics on shared lines serialized at the memory
         side and slowed every atomic of the engine (the leader's loop ran
         ~90 us, profiles/r06i) */
      /* io_uni: every lane read the same word; the branches are the wave's
         (a compare on a VGPR value made the loop divergent to the compiler,
         and its per-lane loop exits left the engine's waves stuck) */
      u64 const tg = io_uni( (it & 15u) && !(C.dbg & 32ul) ? io_ldc( &j->tag ) : io_lda( &j->tag ) );
      if( tg == p + 1ul ) break;
      if( !(it & 31u) && io_uni( io_lda( &dc->stop ) ) ) { stop = true; break; }
      for( u32 q = 0; q < nap; q++ ) __builtin_amdgcn_s_sleep( 8 );
      nap = nap < 8u ? 2u * nap : 8u;
    }
    if( stop ) break;
    u64 const pay = io_uni( io_lda( &j->pay ) );
    if( lane == 0u ) { io_sta( &j->tag, IO_CONS | p ); io_adda( &dc->st[IO_ST_TAKEN], 1ul ); }
    u32 const idx = (u32)pay;
    if( idx & 0x80000000u ) io_flush( C, idx & 0x7fffffffu, pay >> 32 );
    else                    io_ingest( C, idx, pay >> 32 );
  }
  if( lane == 0u ) io_adda( &dc->st[IO_ST_EXITED], 1ul );
}

__global__ __launch_bounds__(256)
void k_svc_io( svc_io_cfg C ) {
  if( blockIdx.x == 0u && threadIdx.x < 64u ) io_leader( C );
  else                                        io_worker( C );
}

/**********************************************************************/
/* service                                                             */

struct svc_launch {
  int                    busy;
  int                    sig;            /* a signature launch (FD_VERIFY_SVC_REQ_SIGS requests) */
  fd_ed25519_hip_ctx_t * ctx;
  hipStream_t            st;
  hipEvent_t             ev0, ev1;
  u32 * d_in_chunk; u16 * d_in_sz; u8 * d_in_kind; u32 * d_tso; u64 * d_seed; u32 * d_stage_chunk;
  u16 * d_tsz; u64 * d_tag; u64 * d_bid; u32 * d_first; u8 * d_cnt; signed char * d_tcode; u32 * d_misc;
  u8 *  d_rsig; u8 * d_rpub; u32 * d_rmoff; u32 * d_rmsz; signed char * d_rcode; ulong rcap; u64 * d_fdesc;
  svc_desc * h_desc; svc_desc * d_desc;   /* mapped pinned memory: the kernels read h_desc at d_desc */
  ulong nreq, n;
  struct { ulong t, slot; } req[SVC_REQ_MAX];
};

struct svc_tile {
  int          set;
  int          client;         /* FD_VERIFY_SVC_REQ_SIGS only, no out dcache (fd_verify_svc_set_client) */
  u8 *         h_out;          /* the out dcache (host) */
  ulong        out_sz;
  u8 const *   chunk_base;     /* host address of out chunk 0 */
  u8 *         d_out;          /* the out dcache's device address (registered) */
  u32 *        h_err;          /* mapped pinned: a flush found an entry outside the out dcache */
  u32 *        d_err;
  hipStream_t  st;
  hipEvent_t   ev[SVC_FLUSH_Q];
  ulong        take;           /* next request id to take */
  ulong        flush_take;     /* next flush to start */
  ulong        flush_fin;      /* flushes retired */
};

struct svc_pend { ulong t, slot, n; long seen; ulong sig; };

/* a flush batch: every tile's newly posted flushes (up to
   SVC_FB_FLUSH_MAX) in one k_svc_compact_batch launch on the flush
   stream; retired in order, each flush's tile advancing flush_done */
struct svc_fbatch {
  int         busy;
  hipEvent_t  ev;
  svc_fdesc * h_desc; svc_fdesc * d_desc;   /* mapped pinned memory */
  u32         nf;
  ulong       n;
  u8          t[SVC_FB_FLUSH_MAX];          /* each flush's tile */
};

/* an ingest batch: the gather of newly posted requests, on the ingest stream */
struct svc_ingest {
  int         busy;
  hipEvent_t  ev0, ev1;
  svc_desc *  h_desc; svc_desc * d_desc;   /* mapped pinned memory */
  ulong       nreq, n;
  struct { ulong t, slot; } req[SVC_REQ_MAX];
};

struct fd_verify_svc {
  fd_verify_svc_seg_t * seg;
  int      dev;
  ulong    batch_max, inflight;
  ulong    merge_min; long merge_wait_ns;
  ulong    gather_wgs;   /* the gather's grid cap (0: one wave per frag); FD_VERIFY_SVC_GATHER_WGS, default
                            SVC_GATHER_WGS: a grid of one wave per frag fills the GPU with waves that wait on
                            PCIe reads, and the verify launches beside it ran ~12% slower (profiles/r05u,v) */
  ulong    flush_wgs;    /* the flush kernel's grid cap (0: one wave per entry); FD_VERIFY_SVC_FLUSH_WGS, default
                            SVC_FLUSH_WGS (profiles/r05w: 3 tiles 65-68 vs 61-64 M uncapped) */
  struct { u8 * h; ulong sz; u8 * d; } reg[SVC_REGION_MAX];
  ulong    nreg;
  struct { int set; u8 const * d_mcache; ulong depth; u8 const * d_base; ulong chunk0, wmark; } link[FD_VERIFY_SVC_LINK_MAX];
  svc_tile tile[FD_VERIFY_SVC_TILE_MAX];
  u8 *     d_stage;            /* staging: tile x slot x slot_cap frags of FD_TXN_HIP_STAGE_CHUNKS */
  u8 *     d_ing;              /* ingest: tile x slot x slot_cap frags of SVC_INGEST_CHUNKS */
  u16 *    d_ing_sz; u8 * d_ing_kind; u32 * d_ing_tso;   /* per ingest frag */
  hipStream_t st_ing;
  /* FD_VERIFY_SVC_ING_STREAMS=2: gathers alternate over two streams
     (st_ing, st_ing2).  One gather runs at ~24 GB/s of PCIe reads beside the
     verify kernels and gathers queue behind each other on one stream, but
     two did not win their A/B (profiles/r06/ing_streams: 24 M frags/s lost
     less, 28 M more, on the same box): default one */
  hipStream_t st_ing2;
  ulong    ing_nst;
  int      gather_wave;        /* k_svc_gather_wave (the round-5 kernel), the default; FD_VERIFY_SVC_GATHER=quarter:
                                  k_svc_gather (descriptors in LDS, a quarter wave per frag).  Same box, depth 16384,
                                  3 tiles, 9 paced runs each (profiles/r06/gather_ab): equal loss at 16-24 M except
                                  one run of the quarter form that collapsed (1.2 M frags lost, p99 16.8 ms; r06p
                                  had another at 32 M) -- its LDS grows with the requests in a gather (up to 64 KB),
                                  so a backlog makes its workgroups harder to place beside the DSM, a suspected
                                  feedback not yet proven */
  svc_ingest ING[SVC_ING_MAX];
  ulong    ing_take, ing_fin;  /* ingest batches started / retired (ring order) */
  u32 *    d_ing_ctr;          /* per ingest batch slot: k_svc_gather's workgroups done (HBM, zero between batches) */
  /* flushes: batched over tiles on one stream (default), or one launch per
     flush on each tile's stream (FD_VERIFY_SVC_FLUSH=tile, the round-5
     form, for an A/B) */
  int      flush_batch;
  hipStream_t st_flush;
  svc_fbatch FB[SVC_FB_MAX];
  ulong    fb_take, fb_fin;
  svc_desc * sdesc;            /* per (tile, slot): the request's descriptor, made at ingest */
  svc_launch L[SVC_LAUNCH_MAX];
  svc_pend * pend; ulong pend_cap, pend_head, pend_tail, pend_frags;
  svc_pend * spend; ulong spend_head, spend_tail;   /* ingested signature requests (clients), their own queue:
                                                       they ride signature launches, not the merge of txn frags */
  ulong    occ[6];             /* every 64th poll with a slot in use: samples, then the summed slot counts posted (not yet
                                  ingested), ingested and waiting for a launch, in a launch, results (the
                                  tile's ordered pass, flushes, publish), free */
  ulong    stat[16];           /* launches, frags, requests, flushes, flushed frags, flushed bytes, flush kernels, gpu ns;
                                  host ns starting launches, starting flushes, retiring, polls; ingests, ingest
                                  gpu ns, host ns starting ingests, the largest launch */
  long     merge_idle_ns;      /* a launch on an idle GPU once the oldest request has waited this long */
  int      running;
  /* the IO engine (k_svc_io), opt-in with FD_VERIFY_SVC_IO=io: a resident
     kernel that polls the tiles' rings itself.  The default is the
     per-ingest and per-flush kernel launches: post -> INGESTED 19.8 us
     median for 64 frags against the engine's 86.9 us (profiles/r06/probe_*),
     and the engine stalls svc_run under range traffic */
  int      io;
  ulong    io_wgs;
  u8 *     d_io;               /* job ring, descriptors, counters (HBM) */
  void *   h_ctl;              /* svc_io_hctl (coherent mapped pinned memory) */
  u8 *     d_ctl;
  u64 *    h_vd;               /* per request slot: the validated n and seed (coherent mapped pinned) */
  u8 *     d_vd;
  hipEvent_t io_ev;            /* recorded behind k_svc_io: the grid has drained */
  ulong    pend_take[FD_VERIFY_SVC_TILE_MAX];   /* next request id of each tile to merge */
  /* the ingest side (steps 1b and 2 of the poll: retire finished gathers,
     gather newly posted requests) on a thread of its own when the process
     may run on two or more CPUs (FD_VERIFY_SVC_INGEST_THREAD=0 keeps it on
     the service thread): a range request holds its link until its gather
     has read it, and on one thread a new request waited behind the flush
     and launch work of every other tile (profiles/r06/gpu_ingested: the
     service thread's ingest and flush turns filled the run).  Ingested
     requests reach the launch queues through ih, a single-producer
     single-consumer ring (ih_tail: stored by the ingest side with release;
     sdesc is written before it) */
  int      ithread;            /* the ingest thread runs */
  pthread_t ith;
  int      istop;
  int      iready;             /* the ingest thread has made its first HIP calls */
  int      iexited;            /* the ingest thread has left its loop */
  int      io_prio;            /* the ingest and flush streams' priority */
  svc_pend * ih; ulong ih_cap; ulong ih_tail, ih_head;
  long     launch_t0[SVC_LAUNCH_MAX];           /* a verify launch's start (the stuck-launch watchdog) */
};

static u8 * svc_dev( fd_verify_svc_t * s, void const * h, ulong sz ) {
  u8 const * p = (u8 const *)h;
  for( ulong k = 0; k < s->nreg; k++ )
    if( p >= s->reg[k].h && p + sz <= s->reg[k].h + s->reg[k].sz ) return s->reg[k].d + (p - s->reg[k].h);
  fprintf( stderr, "fd_verify_svc: %p (+%lu) is in no mapped region\n", h, sz );
  abort();
}

static ulong svc_stage0( fd_verify_svc_t const * s, ulong t, ulong slot ) {
  return (t * s->seg->req_depth + slot) * s->seg->slot_cap * FD_TXN_HIP_STAGE_CHUNKS;
}

static void launch_alloc( svc_launch & L, int dev, ulong nmax ) {
  memset( &L, 0, sizeof(L) );
  L.rcap = fd_txn_hip_record_cap( nmax );
  L.ctx  = fd_ed25519_hip_ctx_new( dev, L.rcap );
  if( !L.ctx ) { fprintf( stderr, "fd_verify_svc: context creation failed\n" ); abort(); }
  /* the verify contexts' DSM grids leave SVC_DSM_RESERVE workgroup slots
     free for the IO kernels beside a DSM pass (profiles/r05an: 3 tiles
     72.1 vs 69.0 M, 2 tiles 67.6 vs 66.9 M); per context, so that no other
     context of the process inherits it; the environment's value wins */
  if( !getenv( "FD_ED25519_HIP_DSM_RESERVE" ) ) (void)fd_ed25519_hip_ctx_set_dsm_reserve( L.ctx, SVC_DSM_RESERVE );
  /* FD_VERIFY_SVC_FREE_CUS=k: the verify launches' stream on all CUs but
     k (every (cus/k)-th), so that the ingest and flush kernels always find
     CUs no verify kernel holds -- a link's frags wait for the gather, and a
     one-shot verify kernel (prep, parse) fills every CU it may use for up to
     ~1 ms */
  {
    char const * e = getenv( "FD_VERIFY_SVC_FREE_CUS" );
    ulong k = e ? strtoul( e, 0, 0 ) : 0ul;
    if( k ) {
      hipDeviceProp_t prop;
      SV_CHECK( hipGetDeviceProperties( &prop, dev ) );
      ulong const cus = (ulong)prop.multiProcessorCount, step = k < cus ? cus / k : 1ul;
      uint mask[16]; memset( mask, 0, sizeof(mask) );
      ulong freed = 0;
      for( ulong c = 0; c < cus && c < 512ul; c++ ) {
        bool const keep = !( (c % step) == step - 1ul && freed < k );
        if( !keep ) freed++;
        if( keep ) mask[c >> 5] |= 1u << (c & 31ul);
      }
      if( fd_ed25519_hip_ctx_set_cu_mask( L.ctx, mask, (uint)((cus + 31ul) / 32ul) ) ) {
        fprintf( stderr, "fd_verify_svc: the verify stream's CU mask (%lu of %lu CUs free) failed\n", k, cus );
        abort();
      }
    }
  }
  L.st = (hipStream_t)fd_ed25519_hip_ctx_stream( L.ctx );
  SV_CHECK( hipMalloc( &L.d_in_chunk, 4ul * nmax ) ); SV_CHECK( hipMalloc( &L.d_in_sz, 2ul * nmax ) );
  SV_CHECK( hipMalloc( &L.d_in_kind, nmax ) );        SV_CHECK( hipMalloc( &L.d_tso, 4ul * nmax ) );
  SV_CHECK( hipMalloc( &L.d_seed, 8ul * nmax ) );     SV_CHECK( hipMalloc( &L.d_stage_chunk, 4ul * nmax ) );
  SV_CHECK( hipMalloc( &L.d_tsz, 2ul * nmax ) );      SV_CHECK( hipMalloc( &L.d_tag, 8ul * nmax ) );
  SV_CHECK( hipMalloc( &L.d_bid, 8ul * nmax ) );      SV_CHECK( hipMalloc( &L.d_first, 4ul * nmax ) );
  SV_CHECK( hipMalloc( &L.d_cnt, nmax ) );            SV_CHECK( hipMalloc( &L.d_tcode, nmax ) );
  SV_CHECK( hipMalloc( &L.d_misc, fd_txn_hip_misc_bytes() ) );
  SV_CHECK( hipMalloc( &L.d_rsig, 64ul * L.rcap ) );  SV_CHECK( hipMalloc( &L.d_rpub, 32ul * L.rcap ) );
  SV_CHECK( hipMalloc( &L.d_rmoff, 4ul * L.rcap ) );  SV_CHECK( hipMalloc( &L.d_rmsz, 4ul * L.rcap ) );
  SV_CHECK( hipMalloc( &L.d_rcode, L.rcap ) );        SV_CHECK( hipMalloc( &L.d_fdesc, 8ul * nmax ) );
  SV_CHECK( hipHostMalloc( &L.h_desc, sizeof(svc_desc) * SVC_REQ_MAX, hipHostMallocMapped ) );
  SV_CHECK( hipHostGetDevicePointer( (void **)&L.d_desc, L.h_desc, 0 ) );
  SV_CHECK( hipEventCreate( &L.ev0 ) ); SV_CHECK( hipEventCreate( &L.ev1 ) );
}

static void launch_free( svc_launch & L ) {
  if( !L.ctx ) return;
  (void)hipStreamSynchronize( L.st );
  (void)hipFree( L.d_in_chunk ); (void)hipFree( L.d_in_sz ); (void)hipFree( L.d_in_kind );
  (void)hipFree( L.d_tso ); (void)hipFree( L.d_seed ); (void)hipFree( L.d_stage_chunk ); (void)hipFree( L.d_tsz );
  (void)hipFree( L.d_tag ); (void)hipFree( L.d_bid ); (void)hipFree( L.d_first ); (void)hipFree( L.d_cnt );
  (void)hipFree( L.d_tcode ); (void)hipFree( L.d_misc ); (void)hipFree( L.d_rsig ); (void)hipFree( L.d_rpub );
  (void)hipFree( L.d_rmoff ); (void)hipFree( L.d_rmsz ); (void)hipFree( L.d_rcode ); (void)hipFree( L.d_fdesc );
  (void)hipHostFree( L.h_desc );
  (void)hipEventDestroy( L.ev0 ); (void)hipEventDestroy( L.ev1 );
  fd_ed25519_hip_ctx_delete( L.ctx );
  L.ctx = 0;
}

extern "C" fd_verify_svc_t *
fd_verify_svc_boot( void * seg_mem, int device, ulong batch_max, ulong inflight ) {
  fd_verify_svc_seg_t * seg = fd_verify_svc_join( seg_mem );
  static_assert( FD_TXN_HIP_STAGE_CHUNKS * 64ul == FD_VERIFY_SVC_STAGE_FRAG_SZ, "staging frag size" );
  static_assert( SVC_INGEST_CHUNKS == FD_VERIFY_SVC_INGEST_CHUNKS && SVC_LAUNCH_MAX == FD_VERIFY_SVC_INFLIGHT_MAX, "limits" );
  /* the shape checks (include/fd_verify_svc.h, the same function the
     topologies' sizing is tested against): staging messages are addressed
     by 32-bit byte offsets (the verify's msg_off), ingest frags by 32-bit
     chunk indices (the parse's in_chunk) */
  if( !seg ) return 0;
  if( !fd_verify_svc_boot_ok( seg->tile_cnt, seg->req_depth, seg->slot_cap, seg->frag_cap, batch_max, inflight ) ) {
    fprintf( stderr, "fd_verify_svc: segment shape %lu tiles x %lu slots x %lu frags (frag area %lu), batch_max %lu, "
             "%lu in flight: outside the service's limits (staging %lu B, 4 GiB at most)\n", seg->tile_cnt, seg->req_depth,
             seg->slot_cap, seg->frag_cap, batch_max, inflight,
             seg->tile_cnt * seg->req_depth * seg->slot_cap * FD_VERIFY_SVC_STAGE_FRAG_SZ );
    return 0;
  }
  ulong const stage_sz = seg->tile_cnt * seg->req_depth * seg->slot_cap * FD_TXN_HIP_STAGE_CHUNKS * 64ul;
  ulong const ing_cnt  = seg->tile_cnt * seg->req_depth * seg->slot_cap;
  SV_CHECK( hipSetDevice( device ) );
  fd_verify_svc_t * s = (fd_verify_svc_t *)calloc( 1, sizeof(fd_verify_svc_t) );
  s->seg = seg; s->dev = device; s->batch_max = batch_max; s->inflight = inflight;
  { char const * e = getenv( "FD_VERIFY_SVC_GATHER_WGS" ); s->gather_wgs = e ? strtoul( e, 0, 0 ) : SVC_GATHER_WGS; }
  { char const * e = getenv( "FD_VERIFY_SVC_FLUSH_WGS" );  s->flush_wgs  = e ? strtoul( e, 0, 0 ) : SVC_FLUSH_WGS; }
  s->merge_min = batch_max / 2ul; s->merge_wait_ns = 2000000L; s->merge_idle_ns = 20000L;
  SV_CHECK( hipMalloc( &s->d_stage, stage_sz + 4096ul ) );
  SV_CHECK( hipMalloc( &s->d_ing, 64ul * SVC_INGEST_CHUNKS * ing_cnt + 4096ul ) );
  SV_CHECK( hipMalloc( &s->d_ing_sz, 2ul * ing_cnt ) ); SV_CHECK( hipMalloc( &s->d_ing_kind, ing_cnt ) );
  SV_CHECK( hipMalloc( &s->d_ing_tso, 4ul * ing_cnt ) );
  SV_CHECK( hipMalloc( &s->d_ing_ctr, 4ul * SVC_ING_MAX ) ); SV_CHECK( hipMemset( s->d_ing_ctr, 0, 4ul * SVC_ING_MAX ) );
  /* FD_VERIFY_SVC_IO_PRIO=1: the ingest and flush streams at the device's
     greatest stream priority.  Opt-in: it lost its A/B (profiles/r06/
     io_prio, depth 16384, 3 tiles: 24 M frags/s runs lost 140-220 K frags
     with it, 0.5-2.4 K without) */
  {
    char const * e = getenv( "FD_VERIFY_SVC_IO_PRIO" );
    int lo = 0, hi = 0;
    SV_CHECK( hipDeviceGetStreamPriorityRange( &lo, &hi ) );
    s->io_prio = ( e && !strcmp( e, "1" ) ) ? hi : 0;
  }
  SV_CHECK( hipStreamCreateWithPriority( &s->st_ing, hipStreamNonBlocking, s->io_prio ) );
  {
    char const * e = getenv( "FD_VERIFY_SVC_ING_STREAMS" );
    s->ing_nst = ( e && !strcmp( e, "2" ) ) ? 2ul : 1ul;
    if( s->ing_nst == 2ul ) SV_CHECK( hipStreamCreateWithPriority( &s->st_ing2, hipStreamNonBlocking, s->io_prio ) );
  }
  { char const * e = getenv( "FD_VERIFY_SVC_GATHER" ); s->gather_wave = !( e && !strcmp( e, "quarter" ) ); }
  for( ulong k = 0; k < SVC_ING_MAX; k++ ) {
    svc_ingest & I = s->ING[k];
    SV_CHECK( hipHostMalloc( &I.h_desc, sizeof(svc_desc) * SVC_REQ_MAX, hipHostMallocMapped ) );
    SV_CHECK( hipHostGetDevicePointer( (void **)&I.d_desc, I.h_desc, 0 ) );
    SV_CHECK( hipEventCreate( &I.ev0 ) ); SV_CHECK( hipEventCreate( &I.ev1 ) );
  }
  {
    char const * e  = getenv( "FD_VERIFY_SVC_FLUSH" );
    char const * io = getenv( "FD_VERIFY_SVC_IO" );          /* the IO engine flushes on its own grid */
    s->flush_batch = !( e && !strcmp( e, "tile" ) ) && !( io && !strcmp( io, "io" ) );
  }
  if( s->flush_batch ) {
    SV_CHECK( hipStreamCreateWithPriority( &s->st_flush, hipStreamNonBlocking, s->io_prio ) );
    for( ulong k = 0; k < SVC_FB_MAX; k++ ) {
      svc_fbatch & F = s->FB[k];
      SV_CHECK( hipHostMalloc( &F.h_desc, sizeof(svc_fdesc) * SVC_FB_FLUSH_MAX, hipHostMallocMapped ) );
      SV_CHECK( hipHostGetDevicePointer( (void **)&F.d_desc, F.h_desc, 0 ) );
      SV_CHECK( hipEventCreateWithFlags( &F.ev, hipEventDisableTiming ) );
    }
  }
  s->sdesc = (svc_desc *)calloc( seg->tile_cnt * seg->req_depth, sizeof(svc_desc) );
  for( ulong k = 0; k < inflight; k++ ) launch_alloc( s->L[k], device, batch_max );
  s->pend_cap = seg->tile_cnt * seg->req_depth;
  s->pend = (svc_pend *)calloc( s->pend_cap, sizeof(svc_pend) );
  s->spend = (svc_pend *)calloc( s->pend_cap, sizeof(svc_pend) );
  s->ih_cap = s->pend_cap;                          /* a slot's request is in the handoff ring at most once */
  s->ih = (svc_pend *)calloc( s->ih_cap, sizeof(svc_pend) );
  { char const * e = getenv( "FD_VERIFY_SVC_IO" ); s->io = e && !strcmp( e, "io" ); }
  { char const * e = getenv( "FD_VERIFY_SVC_IO_WGS" ); s->io_wgs = e ? strtoul( e, 0, 0 ) : IO_WGS; }
  if( s->io_wgs < 2ul || s->io_wgs > 1024ul ) s->io_wgs = IO_WGS;
  if( s->io ) {
    ulong const nreq = seg->tile_cnt * seg->req_depth, nfl = seg->tile_cnt * IO_FQ;
    ulong const io_sz = IO_RING * sizeof(svc_io_job) + nreq * (128ul + 8ul) + nfl * (sizeof(svc_io_fdesc) + 16ul) +
                        sizeof(svc_io_dctl);
    SV_CHECK( hipMalloc( &s->d_io, io_sz ) );
    SV_CHECK( hipMemset( s->d_io, 0, io_sz ) );
    /* the control block and the validated sizes: coherent (fine-grained)
       host memory; the engine polls the stop flag with system atomics */
    SV_CHECK( hipHostMalloc( &s->h_ctl, 4096, hipHostMallocMapped | hipHostMallocCoherent ) );
    memset( s->h_ctl, 0, 4096 );
    SV_CHECK( hipHostGetDevicePointer( (void **)&s->d_ctl, s->h_ctl, 0 ) );
    SV_CHECK( hipHostMalloc( (void **)&s->h_vd, 16ul * nreq, hipHostMallocMapped | hipHostMallocCoherent ) );
    memset( s->h_vd, 0, 16ul * nreq );
    SV_CHECK( hipHostGetDevicePointer( (void **)&s->d_vd, s->h_vd, 0 ) );
    SV_CHECK( hipEventCreate( &s->io_ev ) );
  }
  SV_CHECK( hipDeviceSynchronize() );
  return s;
}

extern "C" int
fd_verify_svc_map( fd_verify_svc_t * s, void * host, ulong sz ) {
  if( !s || !host || !sz || s->nreg >= SVC_REGION_MAX ) return -1;
  ulong a = (ulong)host & ~4095ul, e = ((ulong)host + sz + 4095ul) & ~4095ul;
  SV_CHECK( hipSetDevice( s->dev ) );
  /* (with hipExtHostRegisterUncached the IO engine's first access to the
     segment faulted, profiles/r06d: registered as before; the engine reads
     what the host writes while it runs with system atomics and after
     system-scope acquires) */
  if( hipHostRegister( (void *)a, e - a, hipHostRegisterMapped | hipHostRegisterPortable ) != hipSuccess ) return -1;
  void * d = 0;
  SV_CHECK( hipHostGetDevicePointer( &d, (void *)a, 0 ) );
  s->reg[s->nreg].h = (u8 *)a; s->reg[s->nreg].sz = e - a; s->reg[s->nreg].d = (u8 *)d;
  s->nreg++;
  return 0;
}

extern "C" int
fd_verify_svc_set_link( fd_verify_svc_t * s, ulong link, void const * mcache, ulong depth, void const * chunk_base,
                        ulong chunk0, ulong wmark ) {
  if( !s || link >= FD_VERIFY_SVC_LINK_MAX || !mcache || !depth || (depth & (depth - 1ul)) || chunk0 > wmark ||
      wmark > 0xffffffffull ) return -1;
  s->link[link].d_mcache = svc_dev( s, mcache, 32ul * depth );
  s->link[link].depth    = depth;
  s->link[link].d_base   = svc_dev( s, (u8 const *)chunk_base + 64ul * chunk0, 64ul * (wmark - chunk0) + 2048ul ) -
                           64ul * chunk0;
  s->link[link].chunk0   = chunk0; s->link[link].wmark = wmark;
  s->link[link].set      = 1;
  return 0;
}

extern "C" int
fd_verify_svc_set_tile( fd_verify_svc_t * s, ulong t, void * out_dcache, ulong out_sz, void const * chunk_base ) {
  if( !s || t >= s->seg->tile_cnt || !out_dcache || !out_sz || s->tile[t].set ) return -1;
  svc_tile & T = s->tile[t];
  T.d_out = svc_dev( s, out_dcache, out_sz );               /* mapped: the flush kernel writes it */
  SV_CHECK( hipHostMalloc( &T.h_err, 64, hipHostMallocMapped ) );
  SV_CHECK( hipHostGetDevicePointer( (void **)&T.d_err, T.h_err, 0 ) );
  *T.h_err = 0u;
  (void)svc_dev( s, fd_verify_svc_tile( s->seg, t ), s->seg->tile_sz );   /* the tile's part of the segment */
  SV_CHECK( hipSetDevice( s->dev ) );
  T.h_out = (u8 *)out_dcache; T.out_sz = out_sz; T.chunk_base = (u8 const *)chunk_base;
  /* the IO engine flushes on its own grid: no stream per tile (one stream
     fewer per tile also keeps the process's streams within its hardware
     queues, so no stream ever shares a queue with the persistent kernel) */
  if( !s->io && !s->flush_batch ) {
    SV_CHECK( hipStreamCreateWithFlags( &T.st, hipStreamNonBlocking ) );
    for( ulong k = 0; k < SVC_FLUSH_Q; k++ ) SV_CHECK( hipEventCreateWithFlags( &T.ev[k], hipEventDisableTiming ) );
  }
  T.set = 1;
  return 0;
}

extern "C" int
fd_verify_svc_set_client( fd_verify_svc_t * s, ulong t ) {
  if( !s || t >= s->seg->tile_cnt || s->tile[t].set ) return -1;
  (void)svc_dev( s, fd_verify_svc_tile( s->seg, t ), s->seg->tile_sz );   /* the client's part of the segment is mapped */
  s->tile[t].client = 1;
  s->tile[t].set    = 1;
  return 0;
}

extern "C" void
fd_verify_svc_set_merge( fd_verify_svc_t * s, ulong min_frags, ulong wait_ns, ulong idle_ns ) {
  s->merge_min = min_frags; s->merge_wait_ns = (long)wait_ns; s->merge_idle_ns = (long)idle_ns;
}

static void * svc_ingest_main( void * arg );

extern "C" int
fd_verify_svc_run( fd_verify_svc_t * s ) {
  for( ulong t = 0; t < s->seg->tile_cnt; t++ ) if( !s->tile[t].set ) return -1;
  for( ulong t = 0; t < s->seg->tile_cnt && s->io; t++ )
    if( s->tile[t].client ) {
      fprintf( stderr, "fd_verify_svc: tile %lu is a client: the IO engine (FD_VERIFY_SVC_IO=io) serves verify tiles only\n", t );
      return -1;
    }
  svc_device( s->dev );
  /* the signature path (k_svc_sigrec, the verify's latency and bulk
     kernels, k_svc_sigres) once on zeroed records: its code objects load
     here, before the GPU tile's sandbox */
  for( ulong k = 0; k < s->inflight; k++ ) {
    svc_launch & L = s->L[k];
    SV_CHECK( hipMemsetAsync( L.d_rsig, 0, 64ul * 256ul, L.st ) ); SV_CHECK( hipMemsetAsync( L.d_rpub, 0, 32ul * 256ul, L.st ) );
    SV_CHECK( hipMemsetAsync( L.d_rmoff, 0, 4ul * 256ul, L.st ) ); SV_CHECK( hipMemsetAsync( L.d_rmsz, 0, 4ul * 256ul, L.st ) );
    hipLaunchKernelGGL( k_svc_sigrec, dim3( 1 ), dim3( 256 ), 0, L.st, L.d_desc, 0u, 0ul, (u8 const *)s->d_ing,
                        (u16 const *)s->d_ing_sz, s->d_stage, L.d_rsig, L.d_rpub, L.d_rmoff, L.d_rmsz );
    hipLaunchKernelGGL( k_svc_sigres, dim3( 1 ), dim3( 256 ), 0, L.st, L.d_desc, 0u, 0ul, (u16 const *)s->d_ing_sz,
                        (signed char const *)L.d_rcode );
    SV_CHECK( hipGetLastError() );
    if( fd_ed25519_hip_verify_dev( L.ctx, 1ul, L.d_rsig, L.d_rpub, s->d_stage, L.d_rmoff, L.d_rmsz, L.d_rcode, 0, L.st ) ||
        fd_ed25519_hip_verify_dev( L.ctx, 256ul, L.d_rsig, L.d_rpub, s->d_stage, L.d_rmoff, L.d_rmsz, L.d_rcode, 0, L.st ) ) {
      fprintf( stderr, "fd_verify_svc: signature path warm-up failed\n" );
      return -1;
    }
  }
  /* the kernels' code objects loaded and every buffer touched once before
     the first request (the steady state loads nothing) */
  for( ulong k = 0; k < s->inflight; k++ ) {
    svc_launch & L = s->L[k];
    hipLaunchKernelGGL( k_svc_assemble, dim3( 1 ), dim3( 256 ), 0, L.st, L.d_desc, 0u, 0ul, s->d_ing_sz, s->d_ing_kind,
                        s->d_ing_tso, L.d_in_chunk, L.d_in_sz, L.d_in_kind, L.d_tso, L.d_seed, L.d_stage_chunk );
    hipLaunchKernelGGL( k_svc_results, dim3( 1 ), dim3( 256 ), 0, L.st, L.d_desc, 0u, 0ul, L.d_tsz, L.d_tag, L.d_bid,
                        L.d_cnt, L.d_tcode, L.d_fdesc, L.d_tso );
    SV_CHECK( hipGetLastError() );
  }
  hipLaunchKernelGGL( k_svc_gather, dim3( 1 ), dim3( 256 ), 0, s->st_ing, s->ING[0].d_desc, 0u, 0ul, s->d_ing, s->d_ing_sz,
                      s->d_ing_kind, s->d_ing_tso, s->d_stage, (u32 *)0 );
  SV_CHECK( hipGetLastError() );
  if( s->flush_batch ) {
    hipLaunchKernelGGL( k_svc_compact_batch, dim3( 1 ), dim3( 256 ), 0, s->st_flush, s->FB[0].d_desc, 0u, 0ul,
                        (u8 const *)s->d_stage, s->seg->slot_cap );
    SV_CHECK( hipGetLastError() );
  }
  for( ulong t = 0; t < s->seg->tile_cnt && !s->io && !s->flush_batch; t++ ) {
    if( s->tile[t].client ) continue;
    hipLaunchKernelGGL( k_svc_compact, dim3( 1 ), dim3( 256 ), 0, s->tile[t].st, (fd_verify_svc_out_t const *)0, 0ul,
                        (u8 const *)s->d_stage, 0ul, s->tile[t].d_out, 0L, 0ul, s->seg->slot_cap, s->tile[t].d_err );
    SV_CHECK( hipGetLastError() );
  }
  SV_CHECK( hipDeviceSynchronize() );
  if( s->io ) {
    /* the IO engine: from here on nothing in this process may wait for the
       whole device (hipDeviceSynchronize, hipFree) until teardown has
       stopped it */
    fd_verify_svc_seg_t * g = s->seg;
    svc_io_cfg C;
    memset( &C, 0, sizeof(C) );
    C.seg = (u64)svc_dev( s, g, fd_verify_svc_footprint( g->tile_cnt, g->req_depth, g->slot_cap, g->frag_cap ) );
    C.tile_cnt = g->tile_cnt; C.req_depth = g->req_depth; C.slot_cap = g->slot_cap; C.frag_cap = g->frag_cap;
    C.tile_sz = g->tile_sz; C.slot_sz = g->slot_sz;
    C.req_off  = fd_verify_svc_align_up( sizeof(fd_verify_svc_tile_t) + g->req_depth * sizeof(fd_verify_svc_req_t), 4096ul );
    C.out_off  = fd_verify_svc_align_up( g->slot_cap * sizeof(fd_verify_svc_res_t), 4096ul );
    C.frag_off = C.out_off + fd_verify_svc_align_up( g->slot_cap * sizeof(fd_verify_svc_out_t), 4096ul );
    C.ing = (u64)s->d_ing; C.ing_sz = (u64)s->d_ing_sz; C.ing_kind = (u64)s->d_ing_kind; C.ing_tso = (u64)s->d_ing_tso;
    C.stage = (u64)s->d_stage;
    ulong const nreq = g->tile_cnt * g->req_depth, nfl = g->tile_cnt * IO_FQ;
    u8 * q = s->d_io;
    C.ring    = (u64)q; q += IO_RING * sizeof(svc_io_job);
    C.idesc   = (u64)q; q += nreq * 128ul;
    C.iremain = (u64)q; q += nreq * 8ul;
    C.fdesc   = (u64)q; q += nfl * sizeof(svc_io_fdesc);
    C.fremain = (u64)q; q += nfl * 8ul;
    C.fdone   = (u64)q; q += nfl * 8ul;
    C.dctl    = (u64)q;
    C.hctl = (u64)s->d_ctl; C.hvd = (u64)s->d_vd;
    { char const * e = getenv( "FD_VERIFY_SVC_IO_DBG" ); C.dbg = e ? strtoul( e, 0, 0 ) : 0ul; }
    if( getenv( "FD_VERIFY_SVC_IO_DBG" ) )
      fprintf( stderr, "fd_verify_svc: IO engine cfg seg %lx ring %lx idesc %lx iremain %lx dctl %lx hctl %lx hvd %lx dbg %lx\n",
               C.seg, C.ring, C.idesc, C.iremain, C.dctl, C.hctl, C.hvd, C.dbg );
    for( ulong l = 0; l < FD_VERIFY_SVC_LINK_MAX; l++ ) {
      if( !s->link[l].set ) continue;
      C.link[l].mcache = (u64)s->link[l].d_mcache; C.link[l].mask = s->link[l].depth - 1ul; C.link[l].base = (u64)s->link[l].d_base;
      C.link[l].chunk0 = s->link[l].chunk0; C.link[l].wmark = s->link[l].wmark; C.link[l].set = 1ul;
    }
    for( ulong t = 0; t < g->tile_cnt; t++ ) {
      C.tile[t].out = (u64)s->tile[t].d_out; C.tile[t].out_sz = s->tile[t].out_sz;
      C.tile[t].delta = (long)(s->tile[t].chunk_base - s->tile[t].h_out);
    }
    hipLaunchKernelGGL( k_svc_io, dim3( (unsigned)s->io_wgs ), dim3( 256 ), 0, s->st_ing, C );
    SV_CHECK( hipGetLastError() );
    SV_CHECK( hipEventRecord( s->io_ev, s->st_ing ) );
  }
  s->running = 1;
  /* the ingest thread: started here, before the GPU tile's sandbox, and
     only when the process may run on two CPUs or more (a thread sharing the
     service thread's one CPU would take turns with it, the opposite of the
     point); it inherits the process's CPU set */
  if( !s->io ) {
    char const * e = getenv( "FD_VERIFY_SVC_INGEST_THREAD" );
    cpu_set_t cs;
    CPU_ZERO( &cs );
    int const cpus = sched_getaffinity( 0, sizeof(cs), &cs ) ? 1 : CPU_COUNT( &cs );
    if( !( e && !strcmp( e, "0" ) ) && cpus >= 2 ) {
      if( pthread_create( &s->ith, 0, svc_ingest_main, s ) ) {
        fprintf( stderr, "fd_verify_svc: the ingest thread could not start\n" );
        return -1;
      }
      s->ithread = 1;
      while( !__atomic_load_n( &s->iready, __ATOMIC_ACQUIRE ) ) __builtin_ia32_pause();
    }
  }
  fd_verify_svc_st( &s->seg->svc_state, FD_VERIFY_SVC_SVC_RUNNING );
  return 0;
}

/* validate a posted request and write its launch descriptor */
static void
svc_desc_of( fd_verify_svc_t * s, ulong t, ulong slot, ulong base, svc_desc & d ) {
  fd_verify_svc_seg_t * g = s->seg;
  fd_verify_svc_req_t const * r = fd_verify_svc_req( g, t, slot );
  memset( &d, 0, sizeof(d) );
  d.base = base; d.n = r->n; d.kind = r->kind; d.seed = r->seed; d.stage0 = svc_stage0( s, t, slot );
  d.ibase = (t * g->req_depth + slot) * g->slot_cap;
  d.state = (u64)svc_dev( s, &r->state, sizeof(ulong) );
  if( s->tile[t].client != ( r->kind == FD_VERIFY_SVC_REQ_SIGS ) ) {
    /* a client posts signature records only, a verify tile never does */
    fprintf( stderr, "fd_verify_svc: tile %lu slot %lu: request kind %lu from a %s\n", t, slot, r->kind,
             s->tile[t].client ? "client" : "verify tile" );
    abort();
  }
  if( r->kind == FD_VERIFY_SVC_REQ_RANGE ) {
    if( r->link >= FD_VERIFY_SVC_LINK_MAX || !s->link[r->link].set || !r->rr_cnt || r->rr_idx >= r->rr_cnt ||
        r->seq_cnt > s->link[r->link].depth ||
        r->n != fd_verify_svc_range_cnt( r->seq0, r->seq_cnt, r->rr_cnt, r->rr_idx ) || r->n > g->slot_cap ) {
      fprintf( stderr, "fd_verify_svc: tile %lu slot %lu: bad range request (link %lu seq0 %lu cnt %lu rr %lu/%lu n %lu)\n",
               t, slot, r->link, r->seq0, r->seq_cnt, r->rr_idx, r->rr_cnt, r->n );
      abort();
    }
    d.src = (u64)s->link[r->link].d_mcache; d.aux0 = (u64)s->link[r->link].d_base;
    d.first = fd_verify_svc_range_first( r->seq0, r->rr_cnt, r->rr_idx ); d.stride = r->rr_cnt;
    d.line_mask = s->link[r->link].depth - 1ul; d.chunk0 = s->link[r->link].chunk0; d.wmark = s->link[r->link].wmark;
  } else if( r->kind == FD_VERIFY_SVC_REQ_FRAGS || r->kind == FD_VERIFY_SVC_REQ_SIGS ) {
    if( r->n > g->frag_cap ) {
      fprintf( stderr, "fd_verify_svc: tile %lu slot %lu: %lu frags over the frag area's %lu\n", t, slot, r->n, g->frag_cap );
      abort();
    }
    d.src  = (u64)svc_dev( s, fd_verify_svc_frag( g, t, slot ), r->n * FD_VERIFY_SVC_FRAG_STRIDE );
    d.aux0 = (u64)svc_dev( s, fd_verify_svc_frag_sz( g, t, slot ), 2ul * r->n );
    d.aux1 = (u64)svc_dev( s, fd_verify_svc_frag_kind( g, t, slot ), r->n );
  } else {
    fprintf( stderr, "fd_verify_svc: tile %lu slot %lu: request kind %lu\n", t, slot, r->kind );
    abort();
  }
}

/* a verify launch over ingested requests (their descriptors were made at ingest) */
static void
svc_launch_start( fd_verify_svc_t * s, svc_launch & L ) {
  fd_verify_svc_seg_t * g = s->seg;
  ulong n = 0;
  L.nreq = 0;
  while( s->pend_head != s->pend_tail && L.nreq < SVC_REQ_MAX ) {
    svc_pend const & p = s->pend[s->pend_head % s->pend_cap];
    if( n + p.n > s->batch_max ) break;
    L.h_desc[L.nreq] = s->sdesc[p.t * g->req_depth + p.slot];
    L.h_desc[L.nreq].base = n;
    L.h_desc[L.nreq].res  = (u64)svc_dev( s, fd_verify_svc_res( g, p.t, p.slot ), sizeof(fd_verify_svc_res_t) * p.n );
    L.req[L.nreq].t = p.t; L.req[L.nreq].slot = p.slot;
    L.nreq++; n += p.n;
    s->pend_frags -= p.n; s->pend_head++;
  }
  L.n = n; L.busy = 1; L.sig = 0;
  svc_device( s->dev );
  SV_CHECK( hipEventRecord( L.ev0, L.st ) );
  hipLaunchKernelGGL( k_svc_assemble, dim3( (unsigned)((n + 255ul) / 256ul) ), dim3( 256 ), 0, L.st, L.d_desc, (u32)L.nreq,
                      n, s->d_ing_sz, s->d_ing_kind, s->d_ing_tso, L.d_in_chunk, L.d_in_sz, L.d_in_kind, L.d_tso, L.d_seed,
                      L.d_stage_chunk );
  SV_CHECK( hipGetLastError() );
  fd_txn_hip_batch_core( L.ctx, L.st, n, s->d_ing, L.d_in_chunk, L.d_in_sz, L.d_in_kind, s->d_stage, L.d_stage_chunk,
                         L.d_seed, L.d_tsz, L.d_tag, L.d_bid, L.d_first, L.d_cnt, L.d_misc, L.d_rsig, L.d_rpub,
                         L.d_rmoff, L.d_rmsz, L.rcap, L.d_rcode, L.d_tcode, L.d_fdesc );
  hipLaunchKernelGGL( k_svc_results, dim3( (unsigned)((n + 255ul) / 256ul) ), dim3( 256 ), 0, L.st, L.d_desc, (u32)L.nreq, n,
                      L.d_tsz, L.d_tag, L.d_bid, L.d_cnt, L.d_tcode, L.d_fdesc, L.d_tso );
  SV_CHECK( hipGetLastError() );
  SV_CHECK( hipEventRecord( L.ev1, L.st ) );
  s->stat[0]++; s->stat[1] += n; s->stat[2] += L.nreq;
  if( n > s->stat[15] ) s->stat[15] = n;
}

/* a signature launch over ingested client requests: records -> the
   verify's inputs (k_svc_sigrec), fd_ed25519_verify per record on the
   launch's context, codes -> the slots' result arrays (k_svc_sigres) */
static void
svc_sig_launch_start( fd_verify_svc_t * s, svc_launch & L ) {
  fd_verify_svc_seg_t * g = s->seg;
  ulong n = 0;
  L.nreq = 0;
  while( s->spend_head != s->spend_tail && L.nreq < SVC_REQ_MAX ) {
    svc_pend const & p = s->spend[s->spend_head % s->pend_cap];
    if( n + p.n > s->batch_max ) break;
    L.h_desc[L.nreq] = s->sdesc[p.t * g->req_depth + p.slot];
    L.h_desc[L.nreq].base = n;
    L.h_desc[L.nreq].res  = (u64)svc_dev( s, fd_verify_svc_res( g, p.t, p.slot ), sizeof(fd_verify_svc_res_t) * p.n );
    L.req[L.nreq].t = p.t; L.req[L.nreq].slot = p.slot;
    L.nreq++; n += p.n;
    s->spend_head++;
  }
  L.n = n; L.busy = 1; L.sig = 1;
  svc_device( s->dev );
  SV_CHECK( hipEventRecord( L.ev0, L.st ) );
  ulong wgs = (n + 3ul) / 4ul;
  if( wgs > 2048ul ) wgs = 2048ul;
  hipLaunchKernelGGL( k_svc_sigrec, dim3( (unsigned)wgs ), dim3( 256 ), 0, L.st, L.d_desc, (u32)L.nreq, n,
                      (u8 const *)s->d_ing, (u16 const *)s->d_ing_sz, s->d_stage, L.d_rsig, L.d_rpub, L.d_rmoff, L.d_rmsz );
  SV_CHECK( hipGetLastError() );
  if( fd_ed25519_hip_verify_dev( L.ctx, n, L.d_rsig, L.d_rpub, s->d_stage, L.d_rmoff, L.d_rmsz, L.d_rcode, 0, L.st ) ) {
    fprintf( stderr, "fd_verify_svc: signature launch of %lu records failed\n", n );
    abort();
  }
  hipLaunchKernelGGL( k_svc_sigres, dim3( (unsigned)((n + 255ul) / 256ul) ), dim3( 256 ), 0, L.st, L.d_desc, (u32)L.nreq, n,
                      (u16 const *)s->d_ing_sz, (signed char const *)L.d_rcode );
  SV_CHECK( hipGetLastError() );
  SV_CHECK( hipEventRecord( L.ev1, L.st ) );
  s->stat[0]++; s->stat[1] += n; s->stat[2] += L.nreq;
}

/* the gather of the newly posted requests in I (their frags into the slots'
   HBM ingest frags), on the ingest stream */
static void
svc_ingest_start( fd_verify_svc_t * s, svc_ingest & I ) {
  svc_device( s->dev );
  hipStream_t const st = ( s->ing_nst == 2ul && ( s->ing_take & 1ul ) ) ? s->st_ing2 : s->st_ing;
  SV_CHECK( hipEventRecord( I.ev0, st ) );
  ulong wgs = s->gather_wave ? (I.n + 3ul) / 4ul : (I.n + 15ul) / 16ul;   /* frags per workgroup per trip: 4 / 16 */
  if( s->gather_wgs && wgs > s->gather_wgs ) wgs = s->gather_wgs;
  if( s->gather_wave ) {
    hipLaunchKernelGGL( k_svc_gather_wave, dim3( (unsigned)wgs ), dim3( 256 ), 0, st, I.d_desc,
                        (u32)I.nreq, I.n, s->d_ing, s->d_ing_sz, s->d_ing_kind, s->d_ing_tso, s->d_stage,
                        s->d_ing_ctr + (s->ing_take % SVC_ING_MAX) );
  } else
  hipLaunchKernelGGL( k_svc_gather, dim3( (unsigned)wgs ), dim3( 256 ), sizeof(svc_desc) * I.nreq, st, I.d_desc,
                      (u32)I.nreq, I.n, s->d_ing, s->d_ing_sz, s->d_ing_kind, s->d_ing_tso, s->d_stage,
                      s->d_ing_ctr + (s->ing_take % SVC_ING_MAX) );
  SV_CHECK( hipGetLastError() );
  SV_CHECK( hipEventRecord( I.ev1, st ) );
  I.busy = 1;
  s->stat[12]++;
}

static void
svc_flush_start( fd_verify_svc_t * s, ulong t, fd_verify_svc_flush_t const * f ) {
  fd_verify_svc_seg_t * g = s->seg;
  svc_tile & T = s->tile[t];
  if( f->slot >= g->req_depth || f->lo > f->hi || f->hi > g->slot_cap ) {
    fprintf( stderr, "fd_verify_svc: tile %lu: bad flush (slot %lu [%lu,%lu))\n", t, f->slot, f->lo, f->hi );
    abort();
  }
  ulong const m = f->hi - f->lo;
  fd_verify_svc_out_t const * out = fd_verify_svc_out( g, t, f->slot ) + f->lo;
  long const delta = (long)(T.chunk_base - T.h_out);              /* dcache offset of chunk c: 64 c + delta */
  if( m ) {
    /* the kernel checks every entry's chunks against the out dcache (the
       host does not walk the entries: the service thread drives every tile) */
    ulong wgs = (m + 3ul) / 4ul;
    if( s->flush_wgs && wgs > s->flush_wgs ) wgs = s->flush_wgs;
    hipLaunchKernelGGL( k_svc_compact, dim3( (unsigned)wgs ), dim3( 256 ), 0, T.st,
                        (fd_verify_svc_out_t const *)svc_dev( s, out, m * sizeof(fd_verify_svc_out_t) ), m,
                        (u8 const *)s->d_stage, svc_stage0( s, t, f->slot ), T.d_out, delta, T.out_sz, g->slot_cap,
                        T.d_err );
    SV_CHECK( hipGetLastError() );
    s->stat[6]++;
  }
  SV_CHECK( hipEventRecord( T.ev[T.flush_take % SVC_FLUSH_Q], T.st ) );
  s->stat[3]++; s->stat[4] += m;
}

/* the newly posted flushes of every tile (each tile's in order) into one
   k_svc_compact_batch launch; 1 if it started one */
static int
svc_flush_batch_start( fd_verify_svc_t * s, svc_fbatch & F ) {
  fd_verify_svc_seg_t * g = s->seg;
  F.nf = 0; F.n = 0;
  for( ulong t = 0; t < g->tile_cnt && F.nf < SVC_FB_FLUSH_MAX; t++ ) {
    svc_tile & T = s->tile[t];
    if( T.client ) continue;
    fd_verify_svc_tile_t * b = fd_verify_svc_tile( g, t );
    ulong const post = fd_verify_svc_ld( &b->flush_post );
    while( T.flush_take < post && F.nf < SVC_FB_FLUSH_MAX ) {
      fd_verify_svc_flush_t const * f = &b->flush[T.flush_take % FD_VERIFY_SVC_FLUSH_DEPTH];
      if( f->slot >= g->req_depth || f->lo > f->hi || f->hi > g->slot_cap ) {
        fprintf( stderr, "fd_verify_svc: tile %lu: bad flush (slot %lu [%lu,%lu))\n", t, f->slot, f->lo, f->hi );
        abort();
      }
      ulong const m = f->hi - f->lo;
      svc_fdesc & d = F.h_desc[F.nf];
      d.base = F.n;
      d.out = m ? (u64)svc_dev( s, fd_verify_svc_out( g, t, f->slot ) + f->lo, m * sizeof(fd_verify_svc_out_t) ) : 0ul;
      d.stage0 = svc_stage0( s, t, f->slot ); d.dcache = (u64)T.d_out; d.delta = (long)(T.chunk_base - T.h_out);
      d.out_sz = T.out_sz; d.err = (u64)T.d_err; d.rsv = 0;
      F.t[F.nf] = (u8)t;
      F.nf++; F.n += m;
      T.flush_take++;
      s->stat[3]++; s->stat[4] += m;
    }
  }
  if( !F.nf ) return 0;
  svc_device( s->dev );
  if( F.n ) {
    ulong wgs = (F.n + 3ul) / 4ul;
    if( s->flush_wgs && wgs > s->flush_wgs ) wgs = s->flush_wgs;
    hipLaunchKernelGGL( k_svc_compact_batch, dim3( (unsigned)wgs ), dim3( 256 ), 0, s->st_flush, F.d_desc, F.nf, F.n,
                        (u8 const *)s->d_stage, g->slot_cap );
    SV_CHECK( hipGetLastError() );
    s->stat[6]++;
  }
  SV_CHECK( hipEventRecord( F.ev, s->st_flush ) );
  F.busy = 1;
  return 1;
}

/* the ingest side of a poll: 1b. finished gathers, in order (their
   requests' frags are in HBM, the tiles may reuse the link space) into the
   handoff ring; 2. newly posted requests, in each tile's ring order, into
   one gather batch (a request waits while every batch is busy).  Runs on
   the ingest thread, or inside fd_verify_svc_poll without one; it alone
   touches the ING ring, the tiles' take counters, sdesc and stat[12..14] */
static int
svc_ingest_step( fd_verify_svc_t * s ) {
  fd_verify_svc_seg_t * g = s->seg;
  int did = 0;
  long const now0 = svc_now_ns();
  ulong tail = s->ih_tail;
  while( s->ing_fin < s->ing_take ) {
    svc_ingest & I = s->ING[s->ing_fin % SVC_ING_MAX];
    hipError_t e = hipEventQuery( I.ev1 );
    if( e == hipErrorNotReady ) break;
    SV_CHECK( e );
    float ms = 0.f;
    SV_CHECK( hipEventElapsedTime( &ms, I.ev0, I.ev1 ) );
    s->stat[13] += (ulong)((double)ms * 1e6);
    /* the gather's last workgroup has stored INGESTED into each slot (the
       tiles learn it from the GPU, not from this turn); here they go to the
       launch queues */
    for( ulong r = 0; r < I.nreq; r++ ) {
      svc_pend & p = s->ih[tail % s->ih_cap];
      p.t = I.req[r].t; p.slot = I.req[r].slot; p.n = I.h_desc[r].n; p.seen = now0;
      p.sig = I.h_desc[r].kind == FD_VERIFY_SVC_REQ_SIGS;
      tail++;
    }
    I.busy = 0; s->ing_fin++; did = 1;
  }
  __atomic_store_n( &s->ih_tail, tail, __ATOMIC_RELEASE );
  long const p1 = svc_now_ns();
  /* a range request holds its link until its gather has read it */
  if( s->ing_take - s->ing_fin < SVC_ING_MAX ) {
    svc_ingest & I = s->ING[s->ing_take % SVC_ING_MAX];
    I.nreq = 0; I.n = 0;
    for( ulong t = 0; t < g->tile_cnt && I.nreq < SVC_REQ_MAX; t++ ) {
      svc_tile & T = s->tile[t];
      while( I.nreq < SVC_REQ_MAX ) {
        ulong slot = T.take & (g->req_depth - 1ul);
        fd_verify_svc_req_t * q = fd_verify_svc_req( g, t, slot );
        if( fd_verify_svc_ld( &q->state ) != FD_VERIFY_SVC_POSTED ) break;
        if( q->id + g->req_depth == T.take ) break;          /* the slot's previous request, still on the GPU */
        if( q->id != T.take ) {
          fprintf( stderr, "fd_verify_svc: tile %lu posted request %lu in slot %lu, expected %lu\n", t, q->id, slot, T.take );
          abort();
        }
        T.take++; did = 1;
        if( !q->n ) {                                        /* nothing to verify: results at once */
          q->batch_frags = 0; fd_verify_svc_st( &q->state, FD_VERIFY_SVC_RESULTS );
          continue;
        }
        svc_desc & d = s->sdesc[t * g->req_depth + slot];
        svc_desc_of( s, t, slot, I.n, d );
        I.h_desc[I.nreq] = d;
        I.req[I.nreq].t = t; I.req[I.nreq].slot = slot;
        I.nreq++; I.n += q->n;
      }
    }
    if( I.nreq ) { svc_ingest_start( s, I ); s->ing_take++; }
  }
  s->stat[14] += (ulong)(svc_now_ns() - p1);
  return did;
}

static void *
svc_ingest_main( void * arg ) {
  fd_verify_svc_t * s = (fd_verify_svc_t *)arg;
  /* the thread's first HIP calls (the runtime's per-thread setup), an empty
     gather, an event and its query, and its first malloc (its arena) happen
     here, before fd_verify_svc_run returns and the GPU tile enters its
     sandbox: made after it, the setup's calls met the seccomp filter (one
     bench run of r06l ended in SIGSYS) */
  svc_device( s->dev );
  free( malloc( 4096 ) );
  hipLaunchKernelGGL( k_svc_gather, dim3( 1 ), dim3( 256 ), 0, s->st_ing, s->ING[0].d_desc, 0u, 0ul, s->d_ing, s->d_ing_sz,
                      s->d_ing_kind, s->d_ing_tso, s->d_stage, (u32 *)0 );
  SV_CHECK( hipGetLastError() );
  if( s->gather_wave ) {
    hipLaunchKernelGGL( k_svc_gather_wave, dim3( 1 ), dim3( 256 ), 0, s->st_ing, s->ING[0].d_desc, 0u, 0ul, s->d_ing,
                        s->d_ing_sz, s->d_ing_kind, s->d_ing_tso, s->d_stage, (u32 *)0 );
    SV_CHECK( hipGetLastError() );
  }
  SV_CHECK( hipEventRecord( s->ING[0].ev0, s->st_ing ) );
  SV_CHECK( hipEventRecord( s->ING[0].ev1, s->st_ing ) );
  SV_CHECK( hipStreamSynchronize( s->st_ing ) );
  if( s->st_ing2 ) {
    hipLaunchKernelGGL( k_svc_gather, dim3( 1 ), dim3( 256 ), 0, s->st_ing2, s->ING[1].d_desc, 0u, 0ul, s->d_ing, s->d_ing_sz,
                        s->d_ing_kind, s->d_ing_tso, s->d_stage, (u32 *)0 );
    SV_CHECK( hipGetLastError() );
    SV_CHECK( hipStreamSynchronize( s->st_ing2 ) );
  }
  SV_CHECK( hipEventQuery( s->ING[0].ev1 ) );
  float ms = 0.f;
  SV_CHECK( hipEventElapsedTime( &ms, s->ING[0].ev0, s->ING[0].ev1 ) );
  __atomic_store_n( &s->iready, 1, __ATOMIC_RELEASE );
  while( !__atomic_load_n( &s->istop, __ATOMIC_ACQUIRE ) )
    if( !svc_ingest_step( s ) ) __builtin_ia32_pause();
  __atomic_store_n( &s->iexited, 1, __ATOMIC_RELEASE );
  return 0;
}

extern "C" int fd_verify_svc_debug( fd_verify_svc_t const * s, char * buf, ulong sz );

extern "C" int
fd_verify_svc_poll( fd_verify_svc_t * s ) {
  fd_verify_svc_seg_t * g = s->seg;
  int did = 0;
  long const p0 = svc_now_ns();
  svc_device( s->dev );
  g->svc_heartbeat++;
  s->stat[11]++;
  if( !(s->stat[11] & 63ul) ) {
    ulong c[4] = { 0ul, 0ul, 0ul, 0ul };
    for( ulong t = 0; t < g->tile_cnt; t++ )
      for( ulong k = 0; k < g->req_depth; k++ ) {
        ulong st = fd_verify_svc_ld( &fd_verify_svc_req( g, t, k )->state );
        c[st == FD_VERIFY_SVC_POSTED ? 0 : st == FD_VERIFY_SVC_INGESTED ? 1 : st == FD_VERIFY_SVC_RESULTS ? 2 : 3]++;
      }
    ulong launched = 0;
    for( ulong k = 0; k < s->inflight; k++ ) if( s->L[k].busy ) launched += s->L[k].nreq;
    if( c[3] < g->tile_cnt * g->req_depth ) {                  /* only while some slot is in use */
      s->occ[0]++; s->occ[1] += c[0]; s->occ[2] += c[1] - launched; s->occ[3] += launched; s->occ[4] += c[2];
      s->occ[5] += c[3];
    }
  }
  if( s->io ) {
    svc_io_hctl const * hc = (svc_io_hctl const *)s->h_ctl;
    ulong const err = __atomic_load_n( &hc->err, __ATOMIC_ACQUIRE );
    if( err ) {
      static char const * const what[] = { "", "bad range request", "frag request over the frag area", "bad request kind",
                                           "request id out of ring order", "bad flush (slot / range)",
                                           "flush entry outside the slot's staging or the out dcache",
                                           "a job's descriptor is not the leader's" };
      fprintf( stderr, "fd_verify_svc: IO engine: %s (%lu, %lu, %lu)\n", err < 8ul ? what[err] : "?", hc->err_a,
               hc->err_b, hc->err_c );
      abort();
    }
    /* the engine never ends while the service runs: an end is a fault */
    if( !(s->stat[11] & 1023ul) ) {
      hipError_t e = hipEventQuery( s->io_ev );
      if( e != hipErrorNotReady ) {
        char b[ 1024 ];
        if( fd_verify_svc_debug( s, b, sizeof(b) ) > 0 ) { b[ sizeof(b)-2 ] = '\0'; fprintf( stderr, "fd_verify_svc: %s\n", b ); }
        fprintf( stderr, "fd_verify_svc: IO engine ended while running (%s)\n", hipGetErrorString( e ) );
        abort();
      }
    }
  }
  /* 1. finished verify launches: their slots' results are in the segment */
  ulong busy = 0;
  for( ulong k = 0; k < s->inflight; k++ ) {
    svc_launch & L = s->L[k];
    if( !L.busy ) continue;
    hipError_t e = hipEventQuery( L.ev1 );
    if( e == hipErrorNotReady ) {
      /* a launch that never ends (a stream sharing a hardware queue behind
         the IO engine would) ends the service loudly, not silently */
      if( p0 - s->launch_t0[k] > 20000000000L ) {
        fprintf( stderr, "fd_verify_svc: verify launch %lu (%lu frags) not done after 20 s\n", k, L.n );
        abort();
      }
      busy++; continue;
    }
    SV_CHECK( e );
    float ms = 0.f;
    SV_CHECK( hipEventElapsedTime( &ms, L.ev0, L.ev1 ) );
    s->stat[7] += (ulong)((double)ms * 1e6);
    for( ulong r = 0; r < L.nreq; r++ ) {
      fd_verify_svc_req_t * q = fd_verify_svc_req( g, L.req[r].t, L.req[r].slot );
      q->batch_frags = L.n;
      fd_verify_svc_st( &q->state, FD_VERIFY_SVC_RESULTS );
    }
    L.busy = 0; did = 1;
  }
  long const now0 = svc_now_ns();
  if( s->io ) {
    /* the IO engine ingests and flushes on the GPU: the requests it has
       ingested, in each tile's ring order, wait for a verify launch */
    for( ulong t = 0; t < g->tile_cnt; t++ ) {
      for( ;; ) {
        ulong const slot = s->pend_take[t] & (g->req_depth - 1ul);
        fd_verify_svc_req_t * q = fd_verify_svc_req( g, t, slot );
        if( fd_verify_svc_ld( &q->state ) != FD_VERIFY_SVC_INGESTED ) break;
        ulong const r = t * g->req_depth + slot;
        ulong const n = __atomic_load_n( &s->h_vd[2ul * r], __ATOMIC_ACQUIRE ), seed = s->h_vd[2ul * r + 1ul];
        s->pend_take[t]++; did = 1;
        if( !n ) { q->batch_frags = 0; fd_verify_svc_st( &q->state, FD_VERIFY_SVC_RESULTS ); continue; }
        svc_desc & d = s->sdesc[r];
        memset( &d, 0, sizeof(d) );
        d.n = n; d.seed = seed; d.stage0 = svc_stage0( s, t, slot ); d.ibase = r * g->slot_cap;
        svc_pend & p = s->pend[s->pend_tail % s->pend_cap];
        p.t = t; p.slot = slot; p.n = n; p.seen = now0; p.sig = 0ul;
        s->pend_tail++; s->pend_frags += n;
      }
    }
  }
  long const p1 = svc_now_ns();
  s->stat[10] += (ulong)(p1 - p0);
  /* 1b, 2: the ingest side, here when it has no thread of its own */
  if( !s->io && !s->ithread ) did |= svc_ingest_step( s );
  /* ingested requests join the launch queues (txn frags merge; signature
     requests ride their own launches) */
  {
    ulong const tail = __atomic_load_n( &s->ih_tail, __ATOMIC_ACQUIRE );
    for( ; s->ih_head < tail; s->ih_head++ ) {
      svc_pend const & h = s->ih[s->ih_head % s->ih_cap];
      if( h.sig ) { s->spend[s->spend_tail % s->pend_cap] = h; s->spend_tail++; }
      else        { s->pend[s->pend_tail % s->pend_cap] = h; s->pend_tail++; s->pend_frags += h.n; }
      did = 1;
    }
  }
  long const p2 = svc_now_ns();
  /* 3. flushes: retire in order, start the newly posted */
  while( s->flush_batch && s->fb_fin < s->fb_take ) {
    svc_fbatch & F = s->FB[s->fb_fin % SVC_FB_MAX];
    hipError_t e = hipEventQuery( F.ev );
    if( e == hipErrorNotReady ) break;
    SV_CHECK( e );
    for( u32 i = 0; i < F.nf; i++ ) {
      ulong const t = F.t[i];
      svc_tile & T = s->tile[t];
      if( *(volatile u32 *)T.h_err ) {
        fprintf( stderr, "fd_verify_svc: tile %lu: a flush entry's chunks lie outside the out dcache\n", t );
        abort();
      }
      T.flush_fin++;
      fd_verify_svc_st( &fd_verify_svc_tile( g, t )->flush_done, T.flush_fin );
    }
    F.busy = 0; s->fb_fin++; did = 1;
  }
  for( ulong t = 0; t < g->tile_cnt && !s->io && !s->flush_batch; t++ ) {
    svc_tile & T = s->tile[t];
    if( T.client ) continue;
    fd_verify_svc_tile_t * b = fd_verify_svc_tile( g, t );
    while( T.flush_fin < T.flush_take ) {
      hipError_t e = hipEventQuery( T.ev[T.flush_fin % SVC_FLUSH_Q] );
      if( e == hipErrorNotReady ) break;
      SV_CHECK( e );
      if( *(volatile u32 *)T.h_err ) {
        fprintf( stderr, "fd_verify_svc: tile %lu: a flush entry's chunks lie outside the out dcache\n", t );
        abort();
      }
      T.flush_fin++; did = 1;
      fd_verify_svc_st( &b->flush_done, T.flush_fin );
    }
  }

  for( ulong t = 0; t < g->tile_cnt && !s->io; t++ ) {
    svc_tile & T = s->tile[t];
    fd_verify_svc_tile_t * b = fd_verify_svc_tile( g, t );
    ulong post = fd_verify_svc_ld( &b->flush_post );
    if( T.client ) {
      if( post ) { fprintf( stderr, "fd_verify_svc: tile %lu is a client and posted a flush\n", t ); abort(); }
      continue;
    }
    if( s->flush_batch ) continue;
    while( T.flush_take < post && T.flush_take - T.flush_fin < SVC_FLUSH_Q ) {
      svc_flush_start( s, t, &b->flush[T.flush_take % FD_VERIFY_SVC_FLUSH_DEPTH] );
      T.flush_take++; did = 1;
    }
  }
  if( s->flush_batch && !s->io && s->fb_take - s->fb_fin < SVC_FB_MAX ) {
    if( svc_flush_batch_start( s, s->FB[s->fb_take % SVC_FB_MAX] ) ) { s->fb_take++; did = 1; }
  }
  long const now = svc_now_ns();
  s->stat[9] += (ulong)(now - p2);
  /* 4. a verify launch: when the ingested frags fill its merge target, or
     the oldest has waited merge_wait_ns, or (the GPU idle) merge_idle_ns --
     large launches while the GPU is busy (a 55 K-signature launch runs ~one
     wave per SIMD and costs 3x per signature), little added
     latency while it is not */
  /* 4a. signature requests (clients: a FEC set's root, a replay batch)
     launch as soon as a launch slot is free: they are few and wait on
     their caller, so no merge target */
  while( s->spend_head != s->spend_tail && busy < s->inflight ) {
    ulong k = 0;
    while( s->L[k].busy ) k++;
    long const l0 = svc_now_ns();
    s->launch_t0[k] = l0;
    svc_sig_launch_start( s, s->L[k] );
    s->stat[8] += (ulong)(svc_now_ns() - l0);
    busy++; did = 1;
  }
  while( s->pend_head != s->pend_tail && busy < s->inflight ) {
    long waited = now - s->pend[s->pend_head % s->pend_cap].seen;
    bool ready = s->pend_frags >= s->merge_min || waited >= s->merge_wait_ns || ( !busy && waited >= s->merge_idle_ns );
    if( !ready ) break;
    ulong k = 0;
    while( s->L[k].busy ) k++;
    long const l0 = svc_now_ns();
    s->launch_t0[k] = l0;
    svc_launch_start( s, s->L[k] );
    s->stat[8] += (ulong)(svc_now_ns() - l0);
    busy++; did = 1;
  }
  return did;
}

extern "C" void
fd_verify_svc_stats( fd_verify_svc_t const * s, ulong out[16] ) {
  for( int k = 0; k < 16; k++ ) out[k] = s->stat[k];
  if( s->io ) {                               /* the IO engine's counters (copied by its leader every 256 loops) */
    svc_io_hctl const * hc = (svc_io_hctl const *)s->h_ctl;
    out[12] = hc->st[IO_ST_REQS]; out[3] = hc->st[IO_ST_FLUSHES]; out[4] = hc->st[IO_ST_FLFRAGS]; out[6] = hc->st[IO_ST_JOBS];
  }
}

/* one line of the service's state, for a stalled run's log (svc_run.c
   SVC_DEBUG_S) */
extern "C" int
fd_verify_svc_debug( fd_verify_svc_t const * s, char * buf, ulong sz ) {
  fd_verify_svc_seg_t const * g = s->seg;
  int n = snprintf( buf, sz, "polls %lu launches %lu frags %lu pend %lu/%lu", s->stat[11], s->stat[0], s->stat[1],
                    s->pend_tail - s->pend_head, s->pend_frags );
  for( ulong k = 0; k < s->inflight && n > 0 && (ulong)n < sz; k++ )
    n += snprintf( buf + n, sz - (ulong)n, " L%lu:%d/%lu", k, s->L[k].busy, s->L[k].n );
  for( ulong t = 0; t < g->tile_cnt && t < 4ul && n > 0 && (ulong)n < sz; t++ ) {
    ulong st[4] = { 0, 0, 0, 0 };
    for( ulong k = 0; k < g->req_depth; k++ ) st[__atomic_load_n( &fd_verify_svc_req( (fd_verify_svc_seg_t *)g, t, k )->state, __ATOMIC_ACQUIRE ) & 3ul]++;
    n += snprintf( buf + n, sz - (ulong)n, " t%lu[take %lu free %lu posted %lu results %lu ingested %lu]", t, s->pend_take[t], st[0],
                   st[1], st[2], st[3] );
  }
  if( s->io && n > 0 && (ulong)n < sz ) {
    svc_io_hctl const * hc = (svc_io_hctl const *)s->h_ctl;
    n += snprintf( buf + n, sz - (ulong)n, " io[beat %lu reqs %lu frags %lu flushes %lu jobs %lu exited %lu tail %lu claim %lu "
                   "take %lu %lu ftake %lu ffin %lu err %lu taken %lu loaded %lu]", hc->beat, hc->st[0], hc->st[1], hc->st[2], hc->st[4], hc->st[5],
                   hc->dbg[0], hc->dbg[1], hc->dbg[2], hc->dbg[3], hc->dbg[6], hc->dbg[7], hc->err, hc->st[6], hc->st[7] );
  }
  return n;
}

extern "C" void
fd_verify_svc_occupancy( fd_verify_svc_t const * s, ulong out[6] ) {
  for( int k = 0; k < 6; k++ ) out[k] = s->occ[k];
}

/* Teardown waits for each stream's work with a deadline, stage by stage,
   so that a stuck shutdown says where it is stuck (a run's
   service did not finish its shutdown in 60 s and left no trace of where;
   hipDeviceSynchronize blocks without one).  A stage still running after
   2 s is named on stderr, after 30 s the process aborts naming it. */
static void
svc_drain( hipStream_t st, hipEvent_t ev, char const * what, ulong idx, fd_verify_svc_t const * s ) {
  int own = 0;
  /* each stage is named before its first HIP call: with CU-masked verify
     streams (FD_VERIFY_SVC_FREE_CUS) teardown hung with nothing said after
     "teardown" (profiles/r06/teardown) */
  if( getenv( "FD_VERIFY_SVC_TEARDOWN_LOG" ) ) fprintf( stderr, "fd_verify_svc: teardown: %s %lu\n", what, idx );
  if( !ev ) {
    SV_CHECK( hipEventCreateWithFlags( &ev, hipEventDisableTiming ) );
    if( getenv( "FD_VERIFY_SVC_TEARDOWN_LOG" ) ) fprintf( stderr, "fd_verify_svc: teardown: %s %lu: event created\n", what, idx );
    SV_CHECK( hipEventRecord( ev, st ) );
    if( getenv( "FD_VERIFY_SVC_TEARDOWN_LOG" ) ) fprintf( stderr, "fd_verify_svc: teardown: %s %lu: event recorded\n", what, idx );
    own = 1;
  }
  long const t0 = svc_now_ns();
  int warned = 0;
  for( ;; ) {
    hipError_t e = hipEventQuery( ev );
    if( e == hipSuccess ) break;
    if( e != hipErrorNotReady ) {
      fprintf( stderr, "fd_verify_svc: teardown: %s %lu: %s\n", what, idx, hipGetErrorString( e ) );
      abort();
    }
    long const dt = svc_now_ns() - t0;
    if( dt > 2000000000L && !warned ) {
      warned = 1;
      fprintf( stderr, "fd_verify_svc: teardown: %s %lu still running after 2 s\n", what, idx );
      if( s->io ) {
        svc_io_hctl const * hc = (svc_io_hctl const *)s->h_ctl;
        fprintf( stderr, "fd_verify_svc: teardown: IO engine: %lu waves of %lu left, leader beat %lu\n",
                 hc->st[IO_ST_EXITED], 4ul * s->io_wgs, hc->beat );
      }
    }
    if( dt > 30000000000L ) {
      fprintf( stderr, "fd_verify_svc: teardown: %s %lu not done after 30 s\n", what, idx );
      abort();
    }
    struct timespec ts = { 0, 100000L };
    nanosleep( &ts, 0 );
  }
  if( warned ) fprintf( stderr, "fd_verify_svc: teardown: %s %lu done after %.1f s\n", what, idx, 1e-9 * (double)(svc_now_ns() - t0) );
  if( own ) (void)hipEventDestroy( ev );
}

extern "C" void
fd_verify_svc_delete( fd_verify_svc_t * s ) {
  if( !s ) return;
  /* no HIP call before the ingest thread has stopped: a call that takes a
     runtime lock the thread holds inside a blocked HIP call would hang here
     with nothing said (profiles/r06/teardown: with CU-masked verify streams
     nothing came after "teardown" for 60 s) */
  if( getenv( "FD_VERIFY_SVC_TEARDOWN_LOG" ) ) fprintf( stderr, "fd_verify_svc: teardown: begin (ingest thread %d)\n", s->ithread );
  if( s->ithread ) {                          /* no new gathers from here on (the stream drains below) */
    __atomic_store_n( &s->istop, 1, __ATOMIC_RELEASE );
    /* a thread held inside a HIP call would hold pthread_join silently: the
       wait is staged as the streams' are (named after 2 s, abort after 30 s) */
    long const t0 = svc_now_ns();
    int warned = 0;
    while( !__atomic_load_n( &s->iexited, __ATOMIC_ACQUIRE ) ) {
      long const dt = svc_now_ns() - t0;
      if( dt > 2000000000L && !warned ) {
        warned = 1;
        fprintf( stderr, "fd_verify_svc: teardown: the ingest thread still in a HIP call after 2 s (gathers %lu started, "
                 "%lu retired)\n", s->ing_take, s->ing_fin );
      }
      if( dt > 30000000000L ) { fprintf( stderr, "fd_verify_svc: teardown: the ingest thread not done after 30 s\n" ); abort(); }
      struct timespec ts = { 0, 100000L };
      nanosleep( &ts, 0 );
    }
    (void)pthread_join( s->ith, 0 );
    s->ithread = 0;
  }
  svc_device( s->dev );                       /* the service thread's device (set by its polls already) */
  if( s->io && s->running ) {
    __atomic_store_n( &((svc_io_hctl *)s->h_ctl)->stop, 1ul, __ATOMIC_SEQ_CST );
    svc_drain( s->st_ing, s->io_ev, "the IO engine (k_svc_io)", 0ul, s );
  }
  for( ulong k = 0; k < s->inflight; k++ ) if( s->L[k].ctx ) svc_drain( s->L[k].st, 0, "verify launch stream", k, s );
  for( ulong t = 0; t < FD_VERIFY_SVC_TILE_MAX && !s->io && !s->flush_batch; t++ )
    if( s->tile[t].set && !s->tile[t].client ) svc_drain( s->tile[t].st, 0, "flush stream of tile", t, s );
  if( s->flush_batch ) svc_drain( s->st_flush, 0, "flush stream", 0ul, s );
  if( s->st_ing && !s->io ) svc_drain( s->st_ing, 0, "ingest stream", 0ul, s );
  if( s->st_ing2 ) svc_drain( s->st_ing2, 0, "ingest stream", 1ul, s );
  /* the null stream (the runtime's memsets) the same way, not
     hipDeviceSynchronize: with a CU-masked stream in the process
     (FD_VERIFY_SVC_FREE_CUS) hipDeviceSynchronize never returned although
     every stream above had drained -- the r05m and r06o shutdown hangs
     (profiles/r06/teardown) */
  svc_drain( 0, 0, "null stream", 0ul, s );
  for( ulong k = 0; k < SVC_LAUNCH_MAX; k++ ) launch_free( s->L[k] );
  for( ulong t = 0; t < FD_VERIFY_SVC_TILE_MAX; t++ ) {
    svc_tile & T = s->tile[t];
    if( !T.set ) continue;
    if( !s->io && !T.client && !s->flush_batch ) {
      (void)hipStreamDestroy( T.st );
      for( ulong k = 0; k < SVC_FLUSH_Q; k++ ) (void)hipEventDestroy( T.ev[k] );
    }
    if( T.h_err ) (void)hipHostFree( T.h_err );
  }
  if( s->io ) {
    (void)hipFree( s->d_io ); (void)hipHostFree( s->h_ctl ); (void)hipHostFree( s->h_vd ); (void)hipEventDestroy( s->io_ev );
  }
  (void)hipFree( s->d_stage );
  (void)hipFree( s->d_ing ); (void)hipFree( s->d_ing_sz ); (void)hipFree( s->d_ing_kind ); (void)hipFree( s->d_ing_tso );
  (void)hipFree( s->d_ing_ctr );
  for( ulong k = 0; k < SVC_ING_MAX; k++ ) {
    svc_ingest & I = s->ING[k];
    if( !I.h_desc ) continue;
    (void)hipHostFree( I.h_desc ); (void)hipEventDestroy( I.ev0 ); (void)hipEventDestroy( I.ev1 );
  }
  if( s->st_ing ) (void)hipStreamDestroy( s->st_ing );
  if( s->st_ing2 ) (void)hipStreamDestroy( s->st_ing2 );
  if( s->flush_batch ) {
    for( ulong k = 0; k < SVC_FB_MAX; k++ ) {
      if( !s->FB[k].h_desc ) continue;
      (void)hipHostFree( s->FB[k].h_desc ); (void)hipEventDestroy( s->FB[k].ev );
    }
    (void)hipStreamDestroy( s->st_flush );
  }
  free( s->sdesc );
  for( ulong k = 0; k < s->nreg; k++ ) (void)hipHostUnregister( s->reg[k].h );
  fd_verify_svc_st( &s->seg->svc_state, FD_VERIFY_SVC_SVC_STOPPED );
  free( s->pend ); free( s->spend ); free( s->ih );
  free( s );
}
