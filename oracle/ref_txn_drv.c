/* ref_txn_drv.c -- TEST/BASELINE INFRASTRUCTURE ONLY.

   Repo-owned driver linked (oracle/Makefile) against the reference's own
   objects, compiled from /root/reference/src: fd_txn_parse.c, util/fd_hash.c,
   the ed25519 verify path, and the util objects fd_log needs.  The verify
   decision itself is the reference's header-inline fd_txn_verify
   (src/disco/verify/fd_verify_tile.h:61-111) with its FD_TCACHE_QUERY /
   FD_TCACHE_INSERT macros (src/tango/tcache/fd_tcache.h:281-410), included
   here unchanged.  Only after_frag's bookkeeping around it
   (fd_verify_tile.c:101-161, a static function of the tile) is restated.

   Exports (ctypes, see tests/oracle_lib.py):
     fd_txn_parse_core, fd_hash                      (reference symbols)
     ref_verify_tile_run     sequential after_frag over a frag array
     ref_verify_tile_bench   T verify "tiles" on T pinned threads, frags
                             round-robined by seq (before_frag,
                             fd_verify_tile.c:38-58), timed
     ref_verify_tile_digest  one tile's round robin share: the published
                             sequence's payload digest and the outcome
                             counts (the service-mode bench's parity,
                             tools/svc_bench.py) */

#define _GNU_SOURCE
#include "disco/verify/fd_verify_tile.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define FRAG_PUBLISH      ( 0)
#define FRAG_PARSE_FAIL   (-3)
#define FRAG_BUNDLE_PEER  (-4)

typedef struct {
  fd_verify_ctx_t ctx;
  ulong           oldest;       /* the tcache's "oldest" (fd_tcache_oldest_laddr) */
  ulong *         tc_mem;       /* ring then map */
  fd_sha512_t *   sha_mem;
} ref_tile_t;

static ref_tile_t * tile_new( ulong seed, ulong depth, ulong map_cnt ) {
  ref_tile_t * t = (ref_tile_t *)calloc( 1, sizeof(ref_tile_t) );
  if( !map_cnt ) map_cnt = fd_tcache_map_cnt_default( depth );
  t->tc_mem = (ulong *)aligned_alloc( 128, 8UL*(depth + map_cnt) + 128 );
  t->ctx.hashmap_seed   = seed;
  t->ctx.tcache_depth   = depth;
  t->ctx.tcache_map_cnt = map_cnt;
  t->ctx.tcache_ring    = t->tc_mem;
  t->ctx.tcache_map     = t->tc_mem + depth;
  t->ctx.tcache_sync    = &t->oldest;
  *t->ctx.tcache_sync   = fd_tcache_reset( t->ctx.tcache_ring, depth, t->ctx.tcache_map, map_cnt );
  t->sha_mem = (fd_sha512_t *)aligned_alloc( FD_SHA512_ALIGN, sizeof(fd_sha512_t)*FD_TXN_ACTUAL_SIG_MAX );
  for( ulong i=0; i<FD_TXN_ACTUAL_SIG_MAX; i++ )
    t->ctx.sha[i] = fd_sha512_join( fd_sha512_new( t->sha_mem + i ) );
  return t;
}

static void tile_delete( ref_tile_t * t ) { free( t->tc_mem ); free( t->sha_mem ); free( t ); }

/* after_frag (fd_verify_tile.c:101-161) for one frag; the tile's out dcache
   is replaced by a caller buffer for the parsed fd_txn_t. */
static int after_frag( ref_tile_t * t, uchar const * payload, ushort payload_sz, ulong bundle_id,
                       uchar * txn_buf, ushort * txn_t_sz, ulong * tag ) {
  fd_verify_ctx_t * ctx = &t->ctx;
  fd_txn_t * txnt = (fd_txn_t *)txn_buf;
  ushort tsz = (ushort)fd_txn_parse( payload, payload_sz, txnt, NULL );
  if( txn_t_sz ) *txn_t_sz = tsz;
  *tag = 0;
  int is_bundle = !!bundle_id;
  if( is_bundle & (bundle_id!=ctx->bundle_id) ) { ctx->bundle_failed = 0; ctx->bundle_id = bundle_id; }
  if( is_bundle & (!!ctx->bundle_failed) ) { ctx->metrics.bundle_peer_fail_cnt++; return FRAG_BUNDLE_PEER; }
  if( !tsz ) { if( is_bundle ) ctx->bundle_failed = 1; ctx->metrics.parse_fail_cnt++; return FRAG_PARSE_FAIL; }
  ulong sig = 0;
  int res = fd_txn_verify( ctx, payload, payload_sz, txnt, !is_bundle, &sig );
  if( res!=FD_TXN_VERIFY_SUCCESS ) {
    if( is_bundle ) ctx->bundle_failed = 1;
    if( res==FD_TXN_VERIFY_DEDUP ) ctx->metrics.dedup_fail_cnt++; else ctx->metrics.verify_fail_cnt++;
    return res;
  }
  *tag = sig;
  return FRAG_PUBLISH;
}

/* Sequential run.  state: in/out {oldest, bundle_failed, bundle_id} so a test
   can feed one stream in several calls; tcache arrays are the caller's
   (reference layout).  metrics[4] += {parse, verify, dedup, bundle_peer}. */
void ref_verify_tile_run( ulong seed, ulong * ring, ulong depth, ulong * map, ulong map_cnt, ulong * state,
                          ulong n, uchar const * pool, uint const * off, ushort const * sz,
                          ulong const * bundle_id, signed char * result, ulong * tag, ushort * txn_t_sz,
                          ulong * metrics ) {
  ref_tile_t t[1]; memset( t, 0, sizeof(t) );
  fd_sha512_t shas[FD_TXN_ACTUAL_SIG_MAX] __attribute__((aligned(FD_SHA512_ALIGN)));
  for( ulong i=0; i<FD_TXN_ACTUAL_SIG_MAX; i++ ) t->ctx.sha[i] = fd_sha512_join( fd_sha512_new( shas + i ) );
  ulong oldest = state[0];
  t->ctx.hashmap_seed = seed;
  t->ctx.tcache_depth = depth; t->ctx.tcache_map_cnt = map_cnt;
  t->ctx.tcache_ring = ring; t->ctx.tcache_map = map; t->ctx.tcache_sync = &oldest;
  t->ctx.bundle_failed = (int)state[1]; t->ctx.bundle_id = state[2];
  uchar txn_buf[FD_TXN_MAX_SZ] __attribute__((aligned(8)));
  for( ulong j=0; j<n; j++ )
    result[j] = (signed char)after_frag( t, pool + off[j], sz[j], bundle_id ? bundle_id[j] : 0UL,
                                         txn_buf, txn_t_sz ? txn_t_sz + j : NULL, tag + j );
  state[0] = oldest; state[1] = (ulong)t->ctx.bundle_failed; state[2] = t->ctx.bundle_id;
  metrics[0] += t->ctx.metrics.parse_fail_cnt;  metrics[1] += t->ctx.metrics.verify_fail_cnt;
  metrics[2] += t->ctx.metrics.dedup_fail_cnt;  metrics[3] += t->ctx.metrics.bundle_peer_fail_cnt;
}

/* ---- multi-tile timing (CPU baseline for config C4) --------------------- */

typedef struct {
  ulong idx, cnt, n, repeat, depth, seed; int cpu;
  uchar const * pool; uint const * off; ushort const * sz;
  signed char * result; ulong sigs, published;
} bench_job_t;

static void * bench_worker( void * arg ) {
  bench_job_t * j = (bench_job_t *)arg;
  if( j->cpu >= 0 ) { cpu_set_t cs; CPU_ZERO( &cs ); CPU_SET( j->cpu, &cs ); sched_setaffinity( 0, sizeof(cs), &cs ); }
  ref_tile_t * t = tile_new( j->seed, j->depth, 0 );
  uchar txn_buf[FD_TXN_MAX_SZ] __attribute__((aligned(8)));
  for( ulong rep=0; rep<j->repeat; rep++ ) {
    /* a fresh hash seed per pass: repeated passes look like new traffic to
       the (still filling) tcache instead of one big duplicate burst */
    t->ctx.hashmap_seed = j->seed + rep;
    for( ulong s=j->idx; s<j->n; s+=j->cnt ) {           /* before_frag: seq % round_robin_cnt */
      ushort tsz; ulong tag;
      int r = after_frag( t, j->pool + j->off[s], j->sz[s], 0UL, txn_buf, &tsz, &tag );
      if( rep==j->repeat-1 ) j->result[s] = (signed char)r;
      if( tsz ) j->sigs += ((fd_txn_t *)txn_buf)->signature_cnt;
      j->published += r==FRAG_PUBLISH;
    }
  }
  tile_delete( t );
  return NULL;
}

static double now_s( void ) { struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts ); return (double)ts.tv_sec + 1e-9*(double)ts.tv_nsec; }

/* out[0]=seconds out[1]=frags processed out[2]=signatures of parsed frags
   out[3]=published.  Each thread is one verify tile with its own tcache of
   `depth` and sees every T-th frag. */
void ref_verify_tile_bench( int threads, int first_cpu, ulong repeat, ulong seed, ulong depth,
                            ulong n, uchar const * pool, uint const * off, ushort const * sz,
                            signed char * result, double * out ) {
  if( threads < 1 ) threads = 1;
  if( threads > 256 ) threads = 256;
  pthread_t th[256]; bench_job_t jb[256];
  double t0 = now_s();
  for( int i=0;i<threads;i++ ) {
    jb[i] = (bench_job_t){ .idx=(ulong)i, .cnt=(ulong)threads, .n=n, .repeat=repeat ? repeat : 1, .depth=depth,
                           .seed=seed, .cpu = first_cpu>=0 ? first_cpu+i : -1, .pool=pool, .off=off, .sz=sz,
                           .result=result };
    pthread_create( &th[i], NULL, bench_worker, &jb[i] );
  }
  ulong sigs = 0, pub = 0;
  for( int i=0;i<threads;i++ ) { pthread_join( th[i], NULL ); sigs += jb[i].sigs; pub += jb[i].published; }
  out[0] = now_s() - t0; out[1] = (double)(n*(repeat ? repeat : 1)); out[2] = (double)sigs; out[3] = (double)pub;
}

/* ---- a tile's published sequence, for the service-mode stage's parity ----

   Tile t of T over one quic_verify link (seq = frag index): the frags
   j % T == t in order through after_frag.  fd_txn_verify's signature check
   is a pure function of the frag, so it runs first over the share on
   `threads` threads (the reference's fd_txn_parse and
   fd_ed25519_verify_batch_single_msg, the AVX-512 build); the order-dependent
   rest -- bundle state, tcache query, verdict, tcache insert
   (fd_verify_tile.h:61-111 with FD_TCACHE_QUERY / FD_TCACHE_INSERT) -- then
   runs in arrival order.  digest chains fd_hash( digest, payload,
   payload_sz ) over the published frags from 0x5eedd16e57, as
   integration/svc_tile_run.c's consumer does.  out: digest, published,
   parse, verify, dedup, bundle_peer, signatures of parsed frags. */

typedef struct {
  ulong t, tiles, n, lo, hi; uchar const * pool; uint const * off; ushort const * sz;
  signed char * code; ushort * tsz; uchar * nsig;
} digest_job_t;

static void * digest_worker( void * arg ) {
  digest_job_t * j = (digest_job_t *)arg;
  fd_sha512_t shas[FD_TXN_ACTUAL_SIG_MAX] __attribute__((aligned(FD_SHA512_ALIGN)));
  fd_sha512_t * sp[FD_TXN_ACTUAL_SIG_MAX];
  for( ulong i=0; i<FD_TXN_ACTUAL_SIG_MAX; i++ ) sp[i] = fd_sha512_join( fd_sha512_new( shas + i ) );
  uchar txn_buf[FD_TXN_MAX_SZ] __attribute__((aligned(8)));
  for( ulong k=j->lo; k<j->hi; k++ ) {
    ulong s = j->t + k*j->tiles;
    uchar const * pay = j->pool + j->off[s];
    fd_txn_t * txn = (fd_txn_t *)txn_buf;
    ushort tsz = (ushort)fd_txn_parse( pay, j->sz[s], txn, NULL );
    j->tsz[k] = tsz; j->code[k] = 0; j->nsig[k] = 0;
    if( !tsz ) continue;
    j->nsig[k] = txn->signature_cnt;
    j->code[k] = (signed char)fd_ed25519_verify_batch_single_msg( pay + txn->message_off, (ulong)j->sz[s] - txn->message_off,
                                                                  pay + txn->signature_off, pay + txn->acct_addr_off, sp,
                                                                  txn->signature_cnt );
  }
  return NULL;
}

void ref_verify_tile_digest( ulong tiles, ulong t, ulong seed, ulong depth, ulong n, uchar const * pool,
                             uint const * off, ushort const * sz, ulong const * bundle_id, int threads, ulong * out ) {
  ulong m = t<n ? ( n - 1UL - t )/tiles + 1UL : 0UL;
  signed char * code = (signed char *)malloc( m + 1UL );
  ushort *      tsz  = (ushort *)malloc( 2UL*m + 2UL );
  uchar *       nsig = (uchar *)malloc( m + 1UL );
  if( threads < 1 ) threads = 1;
  if( threads > 256 ) threads = 256;
  pthread_t th[256]; digest_job_t jb[256];
  for( int i=0; i<threads; i++ ) {
    jb[i] = (digest_job_t){ .t=t, .tiles=tiles, .n=n, .lo=m*(ulong)i/(ulong)threads, .hi=m*(ulong)(i+1)/(ulong)threads,
                            .pool=pool, .off=off, .sz=sz, .code=code, .tsz=tsz, .nsig=nsig };
    pthread_create( &th[i], NULL, digest_worker, &jb[i] );
  }
  for( int i=0; i<threads; i++ ) pthread_join( th[i], NULL );
  ref_tile_t * rt = tile_new( seed, depth, 0 );
  fd_verify_ctx_t * ctx = &rt->ctx;
  ulong digest = 0x5eedd16e57UL, pub = 0UL, sigs = 0UL;
  for( ulong k=0; k<m; k++ ) {
    ulong s = t + k*tiles;
    uchar const * pay = pool + off[s];
    ulong bid = bundle_id ? bundle_id[s] : 0UL;
    int is_bundle = !!bid;
    if( is_bundle & (bid!=ctx->bundle_id) ) { ctx->bundle_failed = 0; ctx->bundle_id = bid; }
    if( is_bundle & (!!ctx->bundle_failed) ) { ctx->metrics.bundle_peer_fail_cnt++; continue; }
    if( !tsz[k] ) { if( is_bundle ) ctx->bundle_failed = 1; ctx->metrics.parse_fail_cnt++; continue; }
    sigs += nsig[k];
    uchar txn_buf[FD_TXN_MAX_SZ] __attribute__((aligned(8)));
    fd_txn_t * txn = (fd_txn_t *)txn_buf;
    fd_txn_parse( pay, sz[s], txn, NULL );
    ulong tag = fd_hash( ctx->hashmap_seed, pay + txn->signature_off, 64UL );
    int res = FD_TXN_VERIFY_SUCCESS, ha_dup = 0;
    if( !is_bundle ) {
      FD_FN_UNUSED ulong map_idx = 0;
      FD_TCACHE_QUERY( ha_dup, map_idx, ctx->tcache_map, ctx->tcache_map_cnt, tag );
      if( ha_dup ) res = FD_TXN_VERIFY_DEDUP;
    }
    if( res==FD_TXN_VERIFY_SUCCESS && code[k]!=FD_ED25519_SUCCESS ) res = FD_TXN_VERIFY_FAILED;
    if( res==FD_TXN_VERIFY_SUCCESS && !is_bundle ) {
      FD_TCACHE_INSERT( ha_dup, *ctx->tcache_sync, ctx->tcache_ring, ctx->tcache_depth, ctx->tcache_map, ctx->tcache_map_cnt, tag );
      if( ha_dup ) res = FD_TXN_VERIFY_DEDUP;
    }
    if( res!=FD_TXN_VERIFY_SUCCESS ) {
      if( is_bundle ) ctx->bundle_failed = 1;
      if( res==FD_TXN_VERIFY_DEDUP ) ctx->metrics.dedup_fail_cnt++; else ctx->metrics.verify_fail_cnt++;
      continue;
    }
    digest = fd_hash( digest, pay, sz[s] );
    pub++;
  }
  out[0] = digest; out[1] = pub; out[2] = ctx->metrics.parse_fail_cnt; out[3] = ctx->metrics.verify_fail_cnt;
  out[4] = ctx->metrics.dedup_fail_cnt; out[5] = ctx->metrics.bundle_peer_fail_cnt; out[6] = sigs;
  tile_delete( rt ); free( code ); free( tsz ); free( nsig );
}
