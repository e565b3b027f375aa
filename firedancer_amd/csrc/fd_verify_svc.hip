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
#define SVC_REQ_MAX       64u    /* requests per launch */
#define SVC_LAUNCH_MAX    8ul
#define SVC_GATHER_WGS    256ul  /* the gather's default grid: 1024 waves, enough to keep PCIe busy (64: 2x slower) */
#define SVC_FLUSH_WGS     256ul  /* the flush kernel's default grid */
#define SVC_FLUSH_Q       64ul   /* flushes in flight per tile */
#define SVC_REGION_MAX    64ul
#define SVC_ING_MAX       8ul    /* ingest batches in flight */

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
  u64 rsv[1];
};
static_assert( sizeof(svc_desc) == 128, "svc_desc layout" );

/**********************************************************************/
/* kernels                                                             */

__global__ __launch_bounds__(256)
void k_svc_gather( svc_desc const * __restrict__ desc, u32 nreq, ulong n, u8 * __restrict__ ing,
                   u16 * __restrict__ ing_sz, u8 * __restrict__ ing_kind, u32 * __restrict__ ing_tso,
                   u8 * __restrict__ stage ) {
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
      kind = ((u8 const *)d->aux1)[i];
      ok   = sz <= FD_VERIFY_SVC_FRAG_STRIDE;
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

/* a flush: out entry e's staging frag (its realized bytes, in whole 64-B
   chunks) straight into the tile's out dcache (registered host memory) at the
   entry's chunk; one wave per entry, 16-B stores, a frag's bytes contiguous */
__global__ __launch_bounds__(256)
void k_svc_compact( fd_verify_svc_out_t const * __restrict__ out, ulong m, u8 const * __restrict__ stage,
                    ulong stage0, u8 * __restrict__ dcache, long delta, ulong out_sz, u32 * __restrict__ err ) {
  u32 const lane = threadIdx.x & 63u;
  /* one wave per entry, grid-stride (a capped grid, flush_wgs, loops) */
  for( ulong e = (ulong)blockIdx.x * 4ul + (threadIdx.x >> 6); e < m; e += 4ul * gridDim.x ) {
    fd_verify_svc_out_t const o = out[e];
    if( o.flags & FD_VERIFY_SVC_OUT_HOSTWRITTEN ) continue;
    u32 const len = ((u32)o.sz + 63u) & ~63u;
    long const at = (long)(64ul * (ulong)o.chunk) + delta;
    /* the tile's chunk must lie inside its out dcache: a bad entry is
       reported (the service aborts at the flush's retirement), never written */
    if( at < 0 || at + (long)len > (long)out_sz ) { if( lane == 0u ) *(volatile u32 *)err = 1u; continue; }
    u8 const * src = stage + 64ul * (stage0 + FD_TXN_HIP_STAGE_CHUNKS * (ulong)o.idx);
    u8 *       dst = dcache + at;
    for( u32 p = 16u * lane; p < len; p += 1024u ) *(uint4 *)(dst + p) = *(uint4 const *)(src + p);
  }
}

/**********************************************************************/
/* service                                                             */

struct svc_launch {
  int                    busy;
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

struct svc_pend { ulong t, slot, n; long seen; };

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
  svc_ingest ING[SVC_ING_MAX];
  ulong    ing_take, ing_fin;  /* ingest batches started / retired (ring order) */
  svc_desc * sdesc;            /* per (tile, slot): the request's descriptor, made at ingest */
  svc_launch L[SVC_LAUNCH_MAX];
  svc_pend * pend; ulong pend_cap, pend_head, pend_tail, pend_frags;
  ulong    occ[6];             /* every 64th poll with a slot in use: samples, then the summed slot counts posted (not yet
                                  ingested), ingested and waiting for a launch, in a launch, results (the
                                  tile's ordered pass, flushes, publish), free */
  ulong    stat[16];           /* launches, frags, requests, flushes, flushed frags, flushed bytes, flush kernels, gpu ns;
                                  host ns starting launches, starting flushes, retiring, polls; ingests, ingest
                                  gpu ns, host ns starting ingests, the largest launch */
  long     merge_idle_ns;      /* a launch on an idle GPU once the oldest request has waited this long */
  int      running;
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
  if( !seg || inflight < 1ul || inflight > SVC_LAUNCH_MAX || batch_max < seg->slot_cap ) return 0;
  /* staging messages are addressed by 32-bit byte offsets (the verify's
     msg_off): the whole staging area stays below 4 GiB */
  ulong stage_sz = seg->tile_cnt * seg->req_depth * seg->slot_cap * FD_TXN_HIP_STAGE_CHUNKS * 64ul;
  if( stage_sz + 4096ul >= (1ul << 32) ) {
    fprintf( stderr, "fd_verify_svc: staging %lu B over 4 GiB (tiles x req_depth x slot_cap too large)\n", stage_sz );
    return 0;
  }
  /* ingest frags are addressed by 32-bit chunk indices (the parse's in_chunk) */
  ulong const ing_cnt = seg->tile_cnt * seg->req_depth * seg->slot_cap;
  if( SVC_INGEST_CHUNKS * ing_cnt >= (1ul << 32) ) {
    fprintf( stderr, "fd_verify_svc: %lu ingest frags over the 32-bit chunk index\n", ing_cnt );
    return 0;
  }
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
  SV_CHECK( hipStreamCreateWithFlags( &s->st_ing, hipStreamNonBlocking ) );
  for( ulong k = 0; k < SVC_ING_MAX; k++ ) {
    svc_ingest & I = s->ING[k];
    SV_CHECK( hipHostMalloc( &I.h_desc, sizeof(svc_desc) * SVC_REQ_MAX, hipHostMallocMapped ) );
    SV_CHECK( hipHostGetDevicePointer( (void **)&I.d_desc, I.h_desc, 0 ) );
    SV_CHECK( hipEventCreate( &I.ev0 ) ); SV_CHECK( hipEventCreate( &I.ev1 ) );
  }
  s->sdesc = (svc_desc *)calloc( seg->tile_cnt * seg->req_depth, sizeof(svc_desc) );
  for( ulong k = 0; k < inflight; k++ ) launch_alloc( s->L[k], device, batch_max );
  s->pend_cap = seg->tile_cnt * seg->req_depth;
  s->pend = (svc_pend *)calloc( s->pend_cap, sizeof(svc_pend) );
  SV_CHECK( hipDeviceSynchronize() );
  return s;
}

extern "C" int
fd_verify_svc_map( fd_verify_svc_t * s, void * host, ulong sz ) {
  if( !s || !host || !sz || s->nreg >= SVC_REGION_MAX ) return -1;
  ulong a = (ulong)host & ~4095ul, e = ((ulong)host + sz + 4095ul) & ~4095ul;
  SV_CHECK( hipSetDevice( s->dev ) );
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
  SV_CHECK( hipStreamCreateWithFlags( &T.st, hipStreamNonBlocking ) );
  for( ulong k = 0; k < SVC_FLUSH_Q; k++ ) SV_CHECK( hipEventCreateWithFlags( &T.ev[k], hipEventDisableTiming ) );
  T.set = 1;
  return 0;
}

extern "C" void
fd_verify_svc_set_merge( fd_verify_svc_t * s, ulong min_frags, ulong wait_ns, ulong idle_ns ) {
  s->merge_min = min_frags; s->merge_wait_ns = (long)wait_ns; s->merge_idle_ns = (long)idle_ns;
}

extern "C" int
fd_verify_svc_run( fd_verify_svc_t * s ) {
  for( ulong t = 0; t < s->seg->tile_cnt; t++ ) if( !s->tile[t].set ) return -1;
  svc_device( s->dev );
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
                      s->d_ing_kind, s->d_ing_tso, s->d_stage );
  SV_CHECK( hipGetLastError() );
  for( ulong t = 0; t < s->seg->tile_cnt; t++ ) {
    hipLaunchKernelGGL( k_svc_compact, dim3( 1 ), dim3( 256 ), 0, s->tile[t].st, (fd_verify_svc_out_t const *)0, 0ul,
                        (u8 const *)s->d_stage, 0ul, s->tile[t].d_out, 0L, 0ul, s->tile[t].d_err );
    SV_CHECK( hipGetLastError() );
  }
  SV_CHECK( hipDeviceSynchronize() );
  s->running = 1;
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
  } else if( r->kind == FD_VERIFY_SVC_REQ_FRAGS ) {
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
  L.n = n; L.busy = 1;
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

/* the gather of the newly posted requests in I (their frags into the slots'
   HBM ingest frags), on the ingest stream */
static void
svc_ingest_start( fd_verify_svc_t * s, svc_ingest & I ) {
  svc_device( s->dev );
  SV_CHECK( hipEventRecord( I.ev0, s->st_ing ) );
  ulong wgs = (I.n + 3ul) / 4ul;
  if( s->gather_wgs && wgs > s->gather_wgs ) wgs = s->gather_wgs;
  hipLaunchKernelGGL( k_svc_gather, dim3( (unsigned)wgs ), dim3( 256 ), 0, s->st_ing, I.d_desc,
                      (u32)I.nreq, I.n, s->d_ing, s->d_ing_sz, s->d_ing_kind, s->d_ing_tso, s->d_stage );
  SV_CHECK( hipGetLastError() );
  SV_CHECK( hipEventRecord( I.ev1, s->st_ing ) );
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
                        (u8 const *)s->d_stage, svc_stage0( s, t, f->slot ), T.d_out, delta, T.out_sz, T.d_err );
    SV_CHECK( hipGetLastError() );
    s->stat[6]++;
  }
  SV_CHECK( hipEventRecord( T.ev[T.flush_take % SVC_FLUSH_Q], T.st ) );
  s->stat[3]++; s->stat[4] += m;
}

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
  /* 1. finished verify launches: their slots' results are in the segment */
  ulong busy = 0;
  for( ulong k = 0; k < s->inflight; k++ ) {
    svc_launch & L = s->L[k];
    if( !L.busy ) continue;
    hipError_t e = hipEventQuery( L.ev1 );
    if( e == hipErrorNotReady ) { busy++; continue; }
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
  /* 1b. finished ingests, in order: their requests' frags are in HBM (the
     tiles may reuse the link space) and wait for a verify launch */
  long const now0 = svc_now_ns();
  while( s->ing_fin < s->ing_take ) {
    svc_ingest & I = s->ING[s->ing_fin % SVC_ING_MAX];
    hipError_t e = hipEventQuery( I.ev1 );
    if( e == hipErrorNotReady ) break;
    SV_CHECK( e );
    float ms = 0.f;
    SV_CHECK( hipEventElapsedTime( &ms, I.ev0, I.ev1 ) );
    s->stat[13] += (ulong)((double)ms * 1e6);
    for( ulong r = 0; r < I.nreq; r++ ) {
      fd_verify_svc_st( &fd_verify_svc_req( g, I.req[r].t, I.req[r].slot )->state, FD_VERIFY_SVC_INGESTED );
      svc_pend & p = s->pend[s->pend_tail % s->pend_cap];
      p.t = I.req[r].t; p.slot = I.req[r].slot; p.n = I.h_desc[r].n; p.seen = now0;
      s->pend_tail++; s->pend_frags += p.n;
    }
    I.busy = 0; s->ing_fin++; did = 1;
  }
  /* 2. flushes: retire in order, start the newly posted */
  for( ulong t = 0; t < g->tile_cnt; t++ ) {
    svc_tile & T = s->tile[t];
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
  long const p1 = svc_now_ns();
  s->stat[10] += (ulong)(p1 - p0);
  for( ulong t = 0; t < g->tile_cnt; t++ ) {
    svc_tile & T = s->tile[t];
    fd_verify_svc_tile_t * b = fd_verify_svc_tile( g, t );
    ulong post = fd_verify_svc_ld( &b->flush_post );
    while( T.flush_take < post && T.flush_take - T.flush_fin < SVC_FLUSH_Q ) {
      svc_flush_start( s, t, &b->flush[T.flush_take % FD_VERIFY_SVC_FLUSH_DEPTH] );
      T.flush_take++; did = 1;
    }
  }
  long const p2 = svc_now_ns();
  s->stat[9] += (ulong)(p2 - p1);
  /* 3. posted requests, in each tile's ring order, into one ingest batch
     (a request waits while every ingest slot is busy) */
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
  long const now = svc_now_ns();
  s->stat[14] += (ulong)(now - p2);
  /* 4. a verify launch: when the ingested frags fill its merge target, or
     the oldest has waited merge_wait_ns, or (the GPU idle) merge_idle_ns --
     large launches while the GPU is busy (a 55 K-signature launch runs ~one
     wave per SIMD and costs 3x per signature), little added
     latency while it is not */
  while( s->pend_head != s->pend_tail && busy < s->inflight ) {
    long waited = now - s->pend[s->pend_head % s->pend_cap].seen;
    bool ready = s->pend_frags >= s->merge_min || waited >= s->merge_wait_ns || ( !busy && waited >= s->merge_idle_ns );
    if( !ready ) break;
    ulong k = 0;
    while( s->L[k].busy ) k++;
    long const l0 = svc_now_ns();
    svc_launch_start( s, s->L[k] );
    s->stat[8] += (ulong)(svc_now_ns() - l0);
    busy++; did = 1;
  }
  return did;
}

extern "C" void
fd_verify_svc_stats( fd_verify_svc_t const * s, ulong out[16] ) {
  for( int k = 0; k < 16; k++ ) out[k] = s->stat[k];
}

extern "C" void
fd_verify_svc_occupancy( fd_verify_svc_t const * s, ulong out[6] ) {
  for( int k = 0; k < 6; k++ ) out[k] = s->occ[k];
}

extern "C" void
fd_verify_svc_delete( fd_verify_svc_t * s ) {
  if( !s ) return;
  (void)hipSetDevice( s->dev );
  (void)hipDeviceSynchronize();
  for( ulong k = 0; k < SVC_LAUNCH_MAX; k++ ) launch_free( s->L[k] );
  for( ulong t = 0; t < FD_VERIFY_SVC_TILE_MAX; t++ ) {
    svc_tile & T = s->tile[t];
    if( !T.set ) continue;
    (void)hipStreamDestroy( T.st );
    (void)hipHostFree( T.h_err );
    for( ulong k = 0; k < SVC_FLUSH_Q; k++ ) (void)hipEventDestroy( T.ev[k] );
  }
  (void)hipFree( s->d_stage );
  (void)hipFree( s->d_ing ); (void)hipFree( s->d_ing_sz ); (void)hipFree( s->d_ing_kind ); (void)hipFree( s->d_ing_tso );
  for( ulong k = 0; k < SVC_ING_MAX; k++ ) {
    svc_ingest & I = s->ING[k];
    if( !I.h_desc ) continue;
    (void)hipHostFree( I.h_desc ); (void)hipEventDestroy( I.ev0 ); (void)hipEventDestroy( I.ev1 );
  }
  if( s->st_ing ) (void)hipStreamDestroy( s->st_ing );
  free( s->sdesc );
  for( ulong k = 0; k < s->nreg; k++ ) (void)hipHostUnregister( s->reg[k].h );
  fd_verify_svc_st( &s->seg->svc_state, FD_VERIFY_SVC_SVC_STOPPED );
  free( s->pend );
  free( s );
}
