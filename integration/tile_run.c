/* tile_run.c -- the reference's verify tile with integration/fd_verify_tile_hip.patch
   applied, run and timed in the reference's own run loop.

   Not test infrastructure: this is the north star's operating point, the
   unchanged tile (src/disco/verify/fd_verify_tile.c + the patch) handing its
   frags to the engine.  Built by integration/Makefile from the reference's
   sources where they lie (no copies) against firedancer_amd/libfd_ed25519_hip.so;
   driven by tools/tile_bench.py.

   The topology is the reference's quic -> verify fan-out
   (src/app/fdctl/topology.c:90,173): ONE quic_verify link that every verify
   tile polls, each tile taking seq % tile_cnt == kind_id (before_frag,
   fd_verify_tile.c:37-58), each with its own verify_dedup out link.

     tile_run produce <shm> <stream.bin> <tile_cnt> <in_depth>
         The quic side: creates <shm> (a file in /dev/shm), lays every frag
         of the stream into the quic_verify dcache as fd_txn_m_t frags (the
         copy the quic tile would have made), prints READY, waits for the
         tiles, then publishes the frags' mcache lines in seq order, never
         more than in_depth - 64 (less the frags a GPU-copy tile holds
         unread, RING x 2 x BATCH_MAX) ahead of the slowest tile's fseq (the
         reference link is unreliable and would drop frags past its depth; a
         throughput bench must not), and prints one JSON line once every
         tile is done.
     tile_run tile <shm> <tile_idx>      (TILE_RUN_WALK=1: walk mode, below)
         Verify tile tile_idx: the mock topology around the shared in link
         (tile_drv.c's shape, src/disco/verify/test_verify_tile.c:45-85),
         privileged_init (HIP context, GPU tile_idx % device count),
         unprivileged_init, then stem_run1 (src/disco/stem/fd_stem.c) with
         the patched callbacks until its share of the stream is published
         or dropped and nothing is left on the GPU.

   Range mode (environment TILE_RUN_RANGE=1 on the producer and the tiles):
   the tiles' quic_verify in link is FD_TOPOB_UNPOLLED (as
   integration/fd_verify_topo_hip.patch makes it in the reference's
   topologies), so the stem polls no in link and the patched tile reads the
   link by published seq ranges from after_credit, the GPU reading the
   mcache lines (fd_verify_hip_tile_submit_range).  Such a tile moves its
   fseq only once the GPU has read a range, so the producer needs no margin
   for frags a tile holds unread.

   Prelay (environment TILE_RUN_PRELAY=1 on the producer): the dcache holds
   the whole stream (in_depth >= the frag count) and every frag is laid into
   it before READY, so the timed loop only publishes mcache lines: the rate
   is the verify stage's, not one producer core's copy (~15-20 M frags/s of
   C4 frags on the GPU box).

   Links (environment TILE_RUN_LINKS=L on the producer, 1..4): L quic_verify
   links, as with L quic tiles (topology.c:90,173: every verify tile reads
   every quic_verify link); frag j of the stream goes to link j % L as that
   link's seq j / L.  Each tile takes seq % T of every link.

   Walk mode (environment TILE_RUN_WALK=1 on the tiles, one link): each tile's round
   robin count is set past every seq, so before_frag filters every frag and
   the tile only walks the link (mcache poll, before_frag, fseq updates)
   until its in-link fseq reaches the stream's end: the rate at which ONE
   consumer can walk the shared quic_verify link, which bounds every verify
   tile of the fan-out (each walks all frags of the link).

   Stream file: "FDT1" u64 n, u64 seed, u64 tcache_depth, per frag u64
   bundle_id, u16 payload_sz, payload bytes (oracle/tile_drv.c's format). */

#define FD_TILE_TEST
static int drv_should_shutdown( void * ctx );
#define STEM_CALLBACK_SHOULD_SHUTDOWN( ctx ) drv_should_shutdown( ctx )
#include TILE_SRC
static int     drv_walk;            /* TILE_RUN_WALK: filter every frag, shut down at the link's end */
static int     drv_range;           /* TILE_RUN_RANGE: the in link unpolled, read by range */
static ulong * drv_in_fseq;
static ulong   drv_n;
#include "../topo/fd_topob.h"
#include "../metrics/fd_metrics.h"
#include "../../tango/fseq/fd_fseq.h"
#include "../../tango/tempo/fd_tempo.h"
#include "../quic/fd_tpu.h"
#include <errno.h>
#include <pthread.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#if !FD_HAS_HIP
#error "tile_run drives the patched tile (FD_HAS_HIP)"
#endif

#if defined(fd_boot)                         /* integration/Makefile renames fd_boot / fd_halt (tile_drv.c) */
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

#define RUN_MAGIC     (0xfd7111e5a11ce5ULL)
#define RUN_TILE_MAX  (16UL)
#define RUN_LINK_MAX  (4UL)
/* verify_dedup depth: deep enough that the out chunk ring never holds back a
   throughput run (the tile's frags on the GPU hold chunks: verify_hip_room);
   TILE_RUN_OUT_DEPTH sets it (the reference's default is 16384,
   tiles.verify.receive_buffer_size) */
static ulong run_out_depth( void ) {
  char const * v = getenv( "TILE_RUN_OUT_DEPTH" );
  return v ? fd_ulong_pow2_up( strtoul( v, NULL, 0 ) ) : (1UL<<20);
}
#define RUN_OUT_DEPTH run_out_depth()

typedef struct {
  volatile long t_ready, t_end;
  volatile ulong done, frags, sigs, pub, parse, verify, dedup, bundle, overrun;
  volatile ulong batches;
  volatile double gpu_ms, host_ms;           /* sums over the tile's batches (fd_verify_hip_tile_hist sums) */
  volatile ulong regime[ 8 ];                /* the stem's REGIME_DURATION_NANOS ticks (fd_stem.c:406-712) */
  volatile ulong cons_digest, cons_cnt, cons_bad;   /* TILE_RUN_CONS: the out link's consumer */
} run_res_t;

typedef struct {
  ulong magic;
  ulong n, tile_cnt, seed, tcache_depth, in_depth, link_cnt;
  ulong mcache_off[ RUN_LINK_MAX ], dcache_off[ RUN_LINK_MAX ];
  ulong fseq_off[ RUN_LINK_MAX ];            /* link l, tile t's fseq at fseq_off[l] + t*fseq_stride */
  ulong fseq_stride, dcache_data_sz, map_sz;
  volatile ulong ready, start;
  volatile long  t0;
  run_res_t res[ RUN_TILE_MAX ];
} run_hdr_t;

static void * drv_map( char const * path, ulong sz, int create ) {
  int fd = open( path, create ? (O_RDWR|O_CREAT|O_EXCL) : O_RDWR, 0600 );
  if( fd<0 ) FD_LOG_ERR(( "open(%s) failed (%i-%s)", path, errno, fd_io_strerror( errno ) ));
  if( create && ftruncate( fd, (off_t)sz ) ) FD_LOG_ERR(( "ftruncate failed" ));
  if( !create ) {
    run_hdr_t h;
    if( pread( fd, &h, sizeof(h), 0 )!=(long)sizeof(h) || h.magic!=RUN_MAGIC ) FD_LOG_ERR(( "%s: not a tile_run segment", path ));
    sz = h.map_sz;
  }
  void * p = mmap( NULL, sz, PROT_READ|PROT_WRITE, MAP_SHARED, fd, 0 );
  if( p==MAP_FAILED ) FD_LOG_ERR(( "mmap failed (%i-%s)", errno, fd_io_strerror( errno ) ));
  close( fd );
  return p;
}

static uchar * read_all( char const * path, ulong * sz ) {
  FILE * f = fopen( path, "rb" ); FD_TEST( f );
  fseek( f, 0, SEEK_END ); long n = ftell( f ); fseek( f, 0, SEEK_SET );
  uchar * b = malloc( (ulong)n ); FD_TEST( b );
  FD_TEST( fread( b, 1, (ulong)n, f )==(ulong)n );
  fclose( f );
  *sz = (ulong)n;
  return b;
}

/* ---- produce ------------------------------------------------------------ */

static int
produce( char const * path, char const * stream, ulong tile_cnt, ulong in_depth ) {
  FD_TEST( tile_cnt>=1UL && tile_cnt<=RUN_TILE_MAX && fd_ulong_is_pow2( in_depth ) );
  ulong in_sz; uchar * in = read_all( stream, &in_sz );
  FD_TEST( in_sz>=28UL && !memcmp( in, "FDT1", 4 ) );
  ulong n, seed, depth;
  memcpy( &n, in+4, 8 ); memcpy( &seed, in+12, 8 ); memcpy( &depth, in+20, 8 );

  /* the stream's frags, in order (offsets into the file image) */
  ushort * fsz = malloc( n*sizeof(ushort) ); ulong * poff = malloc( n*sizeof(ulong) );
  FD_TEST( fsz && poff );
  ulong off = 28UL;
  for( ulong j=0UL; j<n; j++ ) {
    ushort psz; memcpy( &psz, in+off+8, 2 );
    poff[ j ] = off; off += 10UL + psz;
    FD_TEST( off<=in_sz && psz<=FD_TPU_MTU );
    fsz[ j ] = (ushort)( sizeof(fd_txn_m_t) + psz );
  }
  /* the quic_verify dcache: a ring of in_depth frags, as the quic tile's
     (the producer writes each frag into it just before publishing it, so a
     tile's during_frag copies recently written bytes, as it would behind a
     quic tile) */
  char const * le = getenv( "TILE_RUN_LINKS" );
  ulong const L = le ? strtoul( le, NULL, 0 ) : 1UL;
  if( FD_UNLIKELY( L<1UL || L>RUN_LINK_MAX ) ) FD_LOG_ERR(( "TILE_RUN_LINKS %lu not in [1,%lu]", L, RUN_LINK_MAX ));
  int const prelay = !!getenv( "TILE_RUN_PRELAY" );
  if( FD_UNLIKELY( prelay && in_depth<(n+L-1UL)/L ) ) FD_LOG_ERR(( "prelay: in_depth %lu < %lu frags", in_depth, n ));
  ulong data_sz = fd_dcache_req_data_sz( FD_TPU_RAW_MTU, in_depth, 1UL, 1 );
  if( prelay ) {                                             /* every frag at its own place: no wrap */
    ulong most = 0UL;
    for( ulong l=0UL; l<L; l++ ) {
      ulong sz_l = 2UL*FD_TPU_RAW_MTU + 4096UL;
      for( ulong j=l; j<n; j+=L ) sz_l += fd_ulong_align_up( fsz[ j ], 2UL*FD_CHUNK_SZ );
      most = fd_ulong_max( most, sz_l );
    }
    data_sz = fd_ulong_align_up( most, 4096UL );
  }
  ulong fs_strd = fd_ulong_align_up( fd_fseq_footprint(), 128UL );
  ulong mc_off[ RUN_LINK_MAX ], fs_off[ RUN_LINK_MAX ], dc_off[ RUN_LINK_MAX ];
  ulong at = sizeof(run_hdr_t);
  for( ulong l=0UL; l<L; l++ ) {
    /* page-aligned: a range tile maps each link's mcache and dcache for the GPU */
    mc_off[ l ] = fd_ulong_align_up( at, 4096UL );
    fs_off[ l ] = fd_ulong_align_up( mc_off[ l ] + fd_mcache_footprint( in_depth, 0UL ), 4096UL );
    dc_off[ l ] = fd_ulong_align_up( fs_off[ l ] + tile_cnt*fs_strd, 4096UL );
    at          = dc_off[ l ] + fd_dcache_footprint( data_sz, 0UL );
  }
  ulong map_sz  = fd_ulong_align_up( at, 4096UL );

  uchar * base = drv_map( path, map_sz, 1 );
  run_hdr_t * hdr = (run_hdr_t *)base;
  memset( hdr, 0, sizeof(run_hdr_t) );
  fd_frag_meta_t * mcache[ RUN_LINK_MAX ];
  ulong chunk0[ RUN_LINK_MAX ], wmark[ RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    mcache[ l ] = fd_mcache_join( fd_mcache_new( base + mc_off[ l ], in_depth, 0UL, 0UL ) );
    for( ulong t=0UL; t<tile_cnt; t++ ) FD_TEST( fd_fseq_join( fd_fseq_new( base + fs_off[ l ] + t*fs_strd, 0UL ) ) );
    uchar * dcache = fd_dcache_join( fd_dcache_new( base + dc_off[ l ], data_sz, 0UL ) );
    FD_TEST( mcache[ l ] && dcache );
    chunk0[ l ] = fd_dcache_compact_chunk0( base, dcache );
    wmark [ l ] = fd_dcache_compact_wmark ( base, dcache, FD_TPU_RAW_MTU );
    hdr->mcache_off[ l ] = mc_off[ l ]; hdr->dcache_off[ l ] = dc_off[ l ]; hdr->fseq_off[ l ] = fs_off[ l ];
  }
  hdr->n = n; hdr->tile_cnt = tile_cnt; hdr->seed = seed; hdr->tcache_depth = depth; hdr->in_depth = in_depth;
  hdr->link_cnt = L; hdr->fseq_stride = fs_strd; hdr->dcache_data_sz = data_sz; hdr->map_sz = map_sz;
  ulong * pchunk = NULL;
  if( prelay ) {
    pchunk = malloc( n*sizeof(ulong) ); FD_TEST( pchunk );
    for( ulong l=0UL; l<L; l++ ) {
      ulong c = chunk0[ l ];
      for( ulong j=l; j<n; j+=L ) {
        fd_txn_m_t * m = (fd_txn_m_t *)fd_chunk_to_laddr( base, c );
        memset( m, 0, sizeof(fd_txn_m_t) );
        memcpy( &m->block_engine.bundle_id, in+poff[ j ], 8 );
        m->payload_sz = (ushort)( fsz[ j ] - sizeof(fd_txn_m_t) );
        memcpy( fd_txn_m_payload( m ), in+poff[ j ]+10UL, m->payload_sz );
        pchunk[ j ] = c;
        ulong nc = fd_dcache_compact_next( c, fsz[ j ], chunk0[ l ], wmark[ l ] );
        if( FD_UNLIKELY( nc<c && j+L<n ) ) FD_LOG_ERR(( "prelay: dcache wrapped at frag %lu", j ));
        c = nc;
      }
    }
  }
  FD_COMPILER_MFENCE();
  hdr->magic = RUN_MAGIC;
  FD_COMPILER_MFENCE();
  printf( "READY\n" ); fflush( stdout );

  for( long tw=fd_log_wallclock(); hdr->ready<tile_cnt; FD_SPIN_PAUSE() )
    if( fd_log_wallclock()-tw > 120L*1000000000L ) FD_LOG_ERR(( "tiles not ready after 120 s (%lu of %lu)", hdr->ready, tile_cnt ));

  ulong const * fseq[ RUN_LINK_MAX ][ RUN_TILE_MAX ];
  for( ulong l=0UL; l<L; l++ )
    for( ulong t=0UL; t<tile_cnt; t++ ) fseq[ l ][ t ] = fd_fseq_join( base + fs_off[ l ] + t*fs_strd );
  long t0 = fd_log_wallclock();
  hdr->t0 = t0;
  FD_COMPILER_MFENCE();
  hdr->start = 1UL;
  ulong ctl = fd_frag_meta_ctl( 0UL, 1, 1, 0 );
  /* a tile with the GPU-side during_frag holds up to RING x 2 x BATCH_MAX frags
     between the stem consuming them (its fseq) and the GPU reading them:
     the producer stays that much (times the tile count: each tile takes
     every T-th seq) further behind, so nothing is overrun */
  ulong const hold = ( FD_VERIFY_HIP_GPU_COPY && !getenv( "TILE_RUN_NO_MARGIN" )    /* the env: overrun tests */
                       && !getenv( "TILE_RUN_RANGE" ) )                           /* range tiles hold none */
                     ? FD_VERIFY_HIP_RING*2UL*FD_VERIFY_HIP_BATCH_MAX*tile_cnt : 0UL;  /* seq % T: held frags
                                                                                          span T x the seqs */
  if( FD_UNLIKELY( in_depth<hold+128UL ) ) FD_LOG_ERR(( "in_depth %lu too small for the GPU copy's %lu held frags", in_depth, hold ));
  ulong lim[ RUN_LINK_MAX ], chunk[ RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    lim  [ l ] = getenv( "TILE_RUN_NO_FLOW" ) ? ULONG_MAX : 0UL;   /* the env: the reference's unreliable link, no
                                                                     flow control at all (overrun tests) */
    chunk[ l ] = chunk0[ l ];
  }
  for( ulong j=0UL; j<n; j++ ) {
    ulong l = j % L, seq = j / L;                              /* frag j: link j % L, its seq j / L */
    while( seq>=lim[ l ] ) {                                   /* flow control against the slowest tile */
      ulong m = ULONG_MAX;
      for( ulong t=0UL; t<tile_cnt; t++ ) m = fd_ulong_min( m, fd_fseq_query( fseq[ l ][ t ] ) );
      lim[ l ] = m + in_depth - 64UL - hold;
      if( seq>=lim[ l ] ) FD_SPIN_PAUSE();
      if( fd_log_wallclock()-t0 > 600L*1000000000L ) FD_LOG_ERR(( "tiles stalled at link %lu seq %lu", l, seq ));
    }
    if( prelay ) chunk[ l ] = pchunk[ j ];
    else {
      fd_txn_m_t * m = (fd_txn_m_t *)fd_chunk_to_laddr( base, chunk[ l ] );
      memset( m, 0, sizeof(fd_txn_m_t) );
      memcpy( &m->block_engine.bundle_id, in+poff[ j ], 8 );
      m->payload_sz = (ushort)( fsz[ j ] - sizeof(fd_txn_m_t) );
      memcpy( fd_txn_m_payload( m ), in+poff[ j ]+10UL, m->payload_sz );
    }
    ulong ts = (ulong)fd_frag_meta_ts_comp( fd_tickcount() );
    fd_mcache_publish( mcache[ l ], in_depth, seq, 0UL, chunk[ l ], fsz[ j ], ctl, ts, ts );
    if( !prelay ) chunk[ l ] = fd_dcache_compact_next( chunk[ l ], fsz[ j ], chunk0[ l ], wmark[ l ] );
  }
  long t_pub = fd_log_wallclock();
  ulong done = 0UL;
  while( done<tile_cnt ) {
    done = 0UL;
    for( ulong t=0UL; t<tile_cnt; t++ ) done += hdr->res[ t ].done;
    if( fd_log_wallclock()-t0 > 900L*1000000000L ) FD_LOG_ERR(( "tiles not done after 900 s" ));
    FD_SPIN_PAUSE();
  }
  long t_end = t0; ulong sigs = 0UL, frags = 0UL, pub = 0UL, batches = 0UL, reg[ 8 ] = { 0UL };
  ulong parse = 0UL, verify = 0UL, dedup = 0UL, bundle = 0UL, overrun = 0UL; double gpu_ms = 0.0, host_ms = 0.0;
  printf( "{\"tiles\": [" );
  for( ulong t=0UL; t<tile_cnt; t++ ) {
    run_res_t * r = &hdr->res[ t ];
    t_end = fd_long_max( t_end, r->t_end );
    sigs += r->sigs; frags += r->frags; pub += r->pub; batches += r->batches;
    parse += r->parse; verify += r->verify; dedup += r->dedup; bundle += r->bundle; overrun += r->overrun;
    gpu_ms += r->gpu_ms; host_ms += r->host_ms;
    for( ulong k=0UL; k<8UL; k++ ) reg[ k ] += r->regime[ k ];
    printf( "%s{\"frags\": %lu, \"sigs\": %lu, \"published\": %lu, \"batches\": %lu, \"s\": %.6f, "
            "\"gpu_ms_per_batch\": %.4f, \"host_ms_per_batch\": %.4f, \"parse_fail\": %lu, \"verify_fail\": %lu, "
            "\"dedup\": %lu, \"bundle_peer_fail\": %lu, \"cons_digest\": \"%016lx\", \"consumed\": %lu, "
            "\"cons_bad\": %lu}", t ? ", " : "", r->frags, r->sigs, r->pub,
            r->batches, (double)( r->t_end - t0 )*1e-9, r->batches ? r->gpu_ms/(double)r->batches : 0.0,
            r->batches ? r->host_ms/(double)r->batches : 0.0, r->parse, r->verify, r->dedup, r->bundle,
            r->cons_digest, r->cons_cnt, r->cons_bad );
  }
  double s = (double)( t_end - t0 )*1e-9;
  double rt = (double)( reg[0]+reg[1]+reg[2]+reg[3]+reg[4]+reg[5]+reg[6]+reg[7] ) + 1e-9;
  printf( "], " );
  /* fd_stem.c's regimes: {housekeeping, prefrag (before/after_credit), postfrag (the frag callbacks)}
     x {caught up, processing, backpressured} */
  printf( "\"regime\": {\"caught_up\": %.4f, \"processing\": %.4f, \"backpressure\": %.4f, "
          "\"hk_caught_up\": %.4f, \"hk_processing\": %.4f, \"pre_caught_up\": %.4f, \"pre_processing\": %.4f, "
          "\"post_caught_up\": %.4f, \"post_processing\": %.4f}, ",
          (double)( reg[0]+reg[3]+reg[6] )/rt, (double)( reg[1]+reg[4]+reg[7] )/rt, (double)( reg[2]+reg[5] )/rt,
          (double)reg[0]/rt, (double)reg[1]/rt, (double)reg[3]/rt, (double)reg[4]/rt, (double)reg[6]/rt,
          (double)reg[7]/rt );
  printf( "\"frags\": %lu, \"sigs\": %lu, \"published\": %lu, \"parse_fail\": %lu, \"verify_fail\": %lu, "
          "\"dedup\": %lu, \"bundle_peer_fail\": %lu, \"seconds\": %.6f, \"publish_s\": %.6f, "
          "\"verifies_per_s\": %.1f, \"frags_per_s\": %.1f, \"batches\": %lu, \"gpu_ms_per_batch\": %.4f, "
          "\"host_ms_per_batch\": %.4f, \"batch_max\": %lu, \"batch_cap\": %lu, \"inflight\": %lu, "
          "\"flush_ns\": %ld, \"in_depth\": %lu, \"tile_cnt\": %lu, \"overrun\": %lu, \"gpu_copy\": %d, "
          "\"range\": %d, \"range_batch_max\": %lu, \"links\": %lu}\n",
          frags, sigs, pub, parse, verify, dedup, bundle, s, (double)( t_pub - t0 )*1e-9, (double)sigs/s,
          (double)frags/s, batches, batches ? gpu_ms/(double)batches : 0.0, batches ? host_ms/(double)batches : 0.0,
          FD_VERIFY_HIP_BATCH_MAX, FD_VERIFY_HIP_BATCH_CAP, FD_VERIFY_HIP_INFLIGHT, (long)FD_VERIFY_HIP_FLUSH_NS,
          in_depth, tile_cnt, overrun, (int)FD_VERIFY_HIP_GPU_COPY, !!getenv( "TILE_RUN_RANGE" ),
          FD_VERIFY_HIP_RANGE_BATCH_MAX, L );
  fflush( stdout );
  munmap( base, map_sz );
  unlink( path );
  free( in ); free( fsz ); free( poff ); free( pchunk );
  return 0;
}

/* ---- tile --------------------------------------------------------------- */

static uchar * drv_arena;
static ulong   drv_arena_sz, drv_arena_used;

static void *
drv_malloc( ulong align, ulong sz ) {
  ulong off = fd_ulong_align_up( drv_arena_used, align );
  FD_TEST( off+sz<=drv_arena_sz );
  drv_arena_used = off + sz;
  return drv_arena + off;
}

static fd_verify_ctx_t * drv_ctx;
static ulong             drv_share;           /* frags of the stream this tile takes */
static long              drv_deadline;

/* TILE_RUN_CONS: a reliable consumer of the tile's verify_dedup link (as
   the dedup tile), on a thread of the tile process.  It stalls
   TILE_RUN_CONS_STALL_MS first, then reads every frag in seq order, checks
   the line still holds the seq after reading (an overwritten frag counts in
   cons_bad), chains the payloads into a digest (tests/svc_io.py digest_of:
   fd_hash from 0x5eedd16e57) and returns credits through its fseq. */
typedef struct {
  fd_frag_meta_t const * mcache;
  ulong                  depth;
  void const *           mem;                 /* the out dcache's chunk base */
  ulong *                fseq;
  long                   stall_ns;
  volatile ulong         target;              /* ULONG_MAX until the tile is done: then its published count */
  ulong                  digest, cnt, bad;
} drv_cons_t;

static void *
drv_cons( void * _c ) {
  drv_cons_t * c = (drv_cons_t *)_c;
  for( long t = fd_log_wallclock(); fd_log_wallclock()-t < c->stall_ns; ) FD_SPIN_PAUSE();
  ulong seq = 0UL, digest = 0x5eedd16e57UL;
  while( seq<c->target ) {
    fd_frag_meta_t const * line = c->mcache + fd_mcache_line_idx( seq, c->depth );
    ulong found = fd_frag_meta_seq_query( line );
    long  diff  = fd_seq_diff( found, seq );
    if( diff<0L ) { fd_fseq_update( c->fseq, seq ); FD_SPIN_PAUSE(); continue; }
    if( FD_UNLIKELY( diff>0L ) ) { c->bad++; seq = found; continue; }   /* lapped: cannot happen to a reliable consumer */
    FD_COMPILER_MFENCE();
    ulong chunk = (ulong)line->chunk;
    FD_COMPILER_MFENCE();
    fd_txn_m_t const * m = (fd_txn_m_t const *)fd_chunk_to_laddr_const( c->mem, chunk );
    ulong d = fd_hash( digest, fd_txn_m_payload_const( m ), m->payload_sz );
    FD_COMPILER_MFENCE();
    if( FD_UNLIKELY( fd_frag_meta_seq_query( line )!=seq ) ) c->bad++;
    digest = d;
    seq++;
    if( !( seq & 63UL ) ) fd_fseq_update( c->fseq, seq );
  }
  fd_fseq_update( c->fseq, seq );
  c->digest = digest; c->cnt = seq;
  return NULL;
}

static int
drv_should_shutdown( void * _ctx ) {
  static ulong calls;                                           /* every stem iteration: look every 64th */
  if( FD_LIKELY( (++calls) & 63UL ) ) return 0;
  fd_verify_ctx_t * ctx = (fd_verify_ctx_t *)_ctx;
  if( drv_walk ) {
    if( FD_UNLIKELY( fd_log_wallclock()>drv_deadline ) ) FD_LOG_ERR(( "walk: not at the end after the deadline" ));
    return fd_fseq_query( drv_in_fseq )>=drv_n;
  }
  ulong m[ 6 ];
  fd_verify_hip_tile_metrics( ctx->hip_tile, m );
  ulong seen = m[0] + m[1] + m[2] + m[3] + m[4]             /* parse, verify, dedup, bundle failures, published */
             + ctx->hip_overrun_cnt;                        /* and frags dropped as overrun after the GPU's read */
  if( FD_UNLIKELY( fd_log_wallclock()>drv_deadline ) ) FD_LOG_ERR(( "tile: %lu of %lu frags after the deadline", seen, drv_share ));
  return seen>=drv_share && FD_VERIFY_HIP_IDLE( ctx );
}

static int
tile( char const * path, ulong t ) {
  uchar * base = drv_map( path, 0UL, 0 );
  run_hdr_t * hdr = (run_hdr_t *)base;
  FD_TEST( t<hdr->tile_cnt );
  ulong in_depth = hdr->in_depth;

  fd_topo_t * topo = fd_topob_new( aligned_alloc( alignof(fd_topo_t), fd_ulong_align_up( sizeof(fd_topo_t), alignof(fd_topo_t) ) ),
                                   "verify-run" );
  fd_topo_wksp_t * qw = fd_topob_wksp( topo, "quic_verify" );   /* the shared segment */
  fd_topo_wksp_t * tw = fd_topob_wksp( topo, "verify" );        /* this tile's own memory */
  fd_topo_tile_t * tile = fd_topob_tile( topo, "verify", "verify", "verify", 0UL, 0, 0 );
  tile->verify.tcache_depth = hdr->tcache_depth;
  ulong out_data = fd_dcache_req_data_sz( FD_TPU_PARSED_MTU, RUN_OUT_DEPTH, FD_VERIFY_HIP_STEM_BURST, 1 );
  drv_arena_sz = 4096UL + scratch_footprint( tile ) + scratch_align() + fd_mcache_footprint( RUN_OUT_DEPTH, 0UL ) +
                 fd_dcache_footprint( out_data, 0UL ) + fd_mcache_align() + fd_dcache_align() + 4096UL;
  drv_arena = aligned_alloc( 4096UL, fd_ulong_align_up( drv_arena_sz, 4096UL ) );
  FD_TEST( drv_arena );
  memset( drv_arena, 0, drv_arena_sz );
  drv_arena_used = 4096UL;
  qw->wksp = (fd_wksp_t *)base;
  tw->wksp = (fd_wksp_t *)drv_arena;
  void * scratch = drv_malloc( scratch_align(), scratch_footprint( tile ) );
  topo->objs[ tile->tile_obj_id ].offset = (ulong)scratch - (ulong)drv_arena;

  ulong const L = hdr->link_cnt;
  fd_topo_link_t * quic[ RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    quic[ l ] = fd_topob_link( topo, "quic_verify", "quic_verify", in_depth, FD_TPU_REASM_MTU, 1UL );
    quic[ l ]->mcache = fd_mcache_join( base + hdr->mcache_off[ l ] );
    quic[ l ]->dcache = fd_dcache_join( base + hdr->dcache_off[ l ] );
    FD_TEST( quic[ l ]->mcache && quic[ l ]->dcache );
    quic[ l ]->mtu = FD_TPU_REASM_MTU;
  }
  fd_topo_link_t * out = fd_topob_link( topo, "verify_dedup", "verify", RUN_OUT_DEPTH, FD_TPU_PARSED_MTU,
                                        FD_VERIFY_HIP_STEM_BURST );
  out->mcache = fd_mcache_join( fd_mcache_new( drv_malloc( fd_mcache_align(), fd_mcache_footprint( RUN_OUT_DEPTH, 0UL ) ),
                                               RUN_OUT_DEPTH, 0UL, 0UL ) );
  out->dcache = fd_dcache_join( fd_dcache_new( drv_malloc( fd_dcache_align(), fd_dcache_footprint( out_data, 0UL ) ),
                                               out_data, 0UL ) );
  FD_TEST( out->mcache && out->dcache );
  drv_range = !!getenv( "TILE_RUN_RANGE" );
  ulong * in_fseq[ RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    fd_topob_tile_in( topo, "verify", 0UL, "verify", "quic_verify", l, FD_TOPOB_UNRELIABLE,
                      drv_range ? FD_TOPOB_UNPOLLED : FD_TOPOB_POLLED );
    in_fseq[ l ] = fd_fseq_join( base + hdr->fseq_off[ l ] + t*hdr->fseq_stride );
    tile->in_link_fseq[ l ] = in_fseq[ l ];                     /* fd_topo_fill_tile's: the range tile moves it */
  }
  fd_topob_tile_out( topo, "verify", 0UL, "verify_dedup", 0UL );
  tile->kind_id = t;                                            /* GPU t % devices; round robin index */
  out->mtu = FD_TPU_PARSED_MTU;

  privileged_init( topo, tile );
  fd_verify_ctx_t * ctx = (fd_verify_ctx_t *)scratch;
  if( getenv( "TILE_RUN_CU_SPLIT" ) ) {                         /* A/B: tile t on CUs [t, t+1) x cus/T */
    uint cus = (uint)strtoul( getenv( "TILE_RUN_CU_SPLIT" ), NULL, 0 ), mask[ 16 ] = { 0U };
    uint lo = (uint)( t*cus/hdr->tile_cnt ), hi = (uint)( (t+1UL)*cus/hdr->tile_cnt );
    FD_TEST( cus>0U && cus<=512U );
    for( uint c=lo; c<hi; c++ ) mask[ c>>5 ] |= 1U<<( c&31U );
    if( FD_UNLIKELY( fd_verify_hip_tile_set_cu_mask( ctx->hip_tile, mask, (cus+31U)/32U ) ) )
      FD_LOG_ERR(( "fd_verify_hip_tile_set_cu_mask failed" ));
  }
  ctx->hashmap_seed = hdr->seed + t;                            /* fixed per tile: runs are reproducible */
  unprivileged_init( topo, tile );
  ctx->round_robin_cnt = hdr->tile_cnt; ctx->round_robin_idx = t;
  drv_walk = !!getenv( "TILE_RUN_WALK" );
  if( drv_walk ) ctx->round_robin_cnt = ULONG_MAX;              /* seq % cnt == seq: only seq t would pass, t < tile_cnt */
  drv_ctx   = ctx;
  drv_share = 0UL;                                              /* seq % T of every link */
  for( ulong l=0UL; l<L; l++ ) {
    ulong nl = ( hdr->n + L - 1UL - l )/L;                      /* frags on link l */
    drv_share += nl/hdr->tile_cnt + ( t<nl%hdr->tile_cnt ? 1UL : 0UL );
  }

  /* the stem's run loop state (fd_stem.c:207-394): metrics, scratch, the
     in link's fseq in the shared segment (the producer's flow control), a
     consumer of the out link that returns every credit (STEM_SHUTDOWN_SEQ) */
  ulong * metrics = aligned_alloc( FD_METRICS_ALIGN, fd_ulong_align_up( FD_METRICS_FOOTPRINT( L, 1UL ), FD_METRICS_ALIGN ) );
  fd_metrics_register( fd_metrics_new( metrics, L, 1UL ) );
  void * stem_scratch = aligned_alloc( FD_STEM_SCRATCH_ALIGN,
                                       fd_ulong_align_up( stem_scratch_footprint( L, 1UL, 1UL ), FD_STEM_SCRATCH_ALIGN ) );
  if( FD_UNLIKELY( drv_walk && L!=1UL ) ) FD_LOG_ERR(( "walk mode takes one link" ));
  drv_in_fseq = in_fseq[ 0 ]; drv_n = hdr->n;
  uchar cons_mem[ 256 ] __attribute__((aligned(128)));
  FD_TEST( fd_fseq_footprint()<=sizeof(cons_mem) );
  int const with_cons = !!getenv( "TILE_RUN_CONS" );
  ulong * cons_fseq = fd_fseq_join( fd_fseq_new( cons_mem, with_cons ? 0UL : STEM_SHUTDOWN_SEQ ) );
  static drv_cons_t cons;
  pthread_t cons_thread;
  if( with_cons ) {
    char const * st = getenv( "TILE_RUN_CONS_STALL_MS" );
    cons = (drv_cons_t){ .mcache = out->mcache, .depth = fd_mcache_depth( out->mcache ), .mem = ctx->out_mem,
                         .fseq = cons_fseq, .stall_ns = st ? 1000000L*strtol( st, NULL, 0 ) : 0L, .target = ULONG_MAX };
  }
  fd_rng_t rng_mem[ 1 ];
  fd_rng_t * rng = fd_rng_join( fd_rng_new( rng_mem, (uint)(hdr->seed + t), 0UL ) );
  fd_frag_meta_t const * in_mcache[ RUN_LINK_MAX ];
  ulong *                in_fseqs [ RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) { in_mcache[ l ] = quic[ l ]->mcache; in_fseqs[ l ] = in_fseq[ l ]; }
  fd_frag_meta_t *       out_mcache[ 1 ] = { out->mcache };
  ulong                  cons_out[ 1 ] = { 0UL };
  ulong *                cons_fseqs[ 1 ] = { cons_fseq };
  (void)fd_tempo_tick_per_ns( NULL );                           /* calibrate before the clock starts */

  hdr->res[ t ].t_ready = fd_log_wallclock();
  __atomic_fetch_add( &hdr->ready, 1UL, __ATOMIC_SEQ_CST );
  while( !hdr->start ) FD_SPIN_PAUSE();
  if( with_cons ) FD_TEST( !pthread_create( &cons_thread, NULL, drv_cons, &cons ) );
  drv_deadline = fd_log_wallclock() + 600L*1000000000L;
  stem_run1( drv_range ? 0UL : L, in_mcache, in_fseqs, 1UL, out_mcache, 1UL, cons_out, cons_fseqs, FD_VERIFY_HIP_STEM_BURST, 0L, rng,
             stem_scratch, ctx );
  long t_end = fd_log_wallclock();

  ulong m[ 6 ];
  fd_verify_hip_tile_metrics( ctx->hip_tile, m );
  ulong cnt[ 16 ], sum_gpu = 0UL, sum_host = 0UL, nb = 0UL;
  fd_verify_hip_tile_hist( ctx->hip_tile, 0, cnt, NULL, &sum_gpu );
  for( ulong k=0UL; k<16UL; k++ ) nb += cnt[ k ];
  fd_verify_hip_tile_hist( ctx->hip_tile, 1, NULL, NULL, &sum_host );
  run_res_t * r = &hdr->res[ t ];
  r->t_end = t_end; r->frags = m[0] + m[1] + m[2] + m[3] + m[4]; r->sigs = m[5]; r->pub = m[4];
  r->parse = m[0]; r->verify = m[1]; r->dedup = m[2]; r->bundle = m[3]; r->overrun = ctx->hip_overrun_cnt;
  r->batches = nb; r->gpu_ms = (double)sum_gpu*1e-6; r->host_ms = (double)sum_host*1e-6;
  for( ulong k=0UL; k<8UL; k++ ) r->regime[ k ] = fd_metrics_tl[ MIDX( COUNTER, TILE, REGIME_DURATION_NANOS ) + k ];
  if( with_cons ) {
    cons.target = m[4];
    FD_TEST( !pthread_join( cons_thread, NULL ) );
    r->cons_digest = cons.digest; r->cons_cnt = cons.cnt; r->cons_bad = cons.bad;
  }
  FD_COMPILER_MFENCE();
  r->done = 1UL;
  return 0;
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  if( argc>=6 && !strcmp( argv[1], "produce" ) )
    return produce( argv[2], argv[3], strtoul( argv[4], NULL, 0 ), strtoul( argv[5], NULL, 0 ) );
  if( argc>=4 && !strcmp( argv[1], "tile" ) )
    return tile( argv[2], strtoul( argv[3], NULL, 0 ) );
  fprintf( stderr, "usage: %s produce <shm> <stream.bin> <tile_cnt> <in_depth> | tile <shm> <tile_idx>\n", argv[0] );
  return 2;
}
