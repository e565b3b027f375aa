/* tile_drv.c -- TEST INFRASTRUCTURE ONLY (repo-owned).

   Drives a verify tile compiled from TILE_SRC -- the reference's own
   src/disco/verify/fd_verify_tile.c, or that file with
   integration/fd_verify_tile_hip.patch applied (FD_HAS_HIP) -- through the
   reference's mock topology (the fd_topob / malloc-backed mcache+dcache
   set-up of src/disco/verify/test_verify_tile.c:45-85, with an explicit
   verify_dedup out link), one frag at a time in stem_run's callback order
   (src/disco/stem/fd_stem.c:506-712): after_credit (the patched tile), then
   before_frag, during_frag, after_frag.  After the last frag it keeps
   calling after_credit until the tile has published everything it holds.

   usage: tile_drv <in.bin> <out.bin>
   in.bin : "FDT1" u64 n, u64 seed, u64 tcache_depth,
            per frag: u64 bundle_id, u16 payload_sz, payload bytes
   out.bin: "FDO1" u64 pub_cnt, then per published frag: u64 sig, u64 sz,
            u64 tsorig, sz bytes (the frag's dcache bytes: fd_txn_m_t header,
            payload and fd_txn_t); then the metrics (5 x u64: parse, verify,
            dedup, bundle_peer, gossiped_votes), the tcache oldest, ring
            and map (u64 each).
   Frags arrive on the quic_verify link with tsorig = frag index, so the
   published tsorig names the input frag. */

#define FD_TILE_TEST
#include TILE_SRC
#include "../topo/fd_topob.h"
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#if FD_HAS_HIP
#include <signal.h>
#include <ucontext.h>
#include <sys/prctl.h>

/* TILE_DRV_SECCOMP=1: the frag loop runs under the patched tile's seccomp
   filter (verify_hip_seccomp), installed as fd_sandbox does
   (util/sandbox/fd_sandbox.c:544-551), with the output file's fd in the
   logfile slot.  tile_drv_hip is built with FD_VERIFY_HIP_SECCOMP_FAIL =
   SECCOMP_RET_TRAP so that a syscall outside the policy is reported here
   (number, then the call fails with ENOSYS) instead of killing the test. */
static volatile int drv_trap_nr[ 16 ];
static volatile int drv_trap_cnt;
static void
drv_sigsys( int sig, siginfo_t * si, void * uc ) {
  (void)sig;
  if( drv_trap_cnt<16 ) drv_trap_nr[ drv_trap_cnt ] = si->si_syscall;
  drv_trap_cnt++;
  char msg[ 48 ] = "tile_drv: seccomp trap on syscall ";      /* at once: a trap may end in an abort */
  int  len = 34, nr = si->si_syscall;
  char dig[ 12 ]; int nd = 0;
  do { dig[ nd++ ] = (char)('0' + nr % 10); nr /= 10; } while( nr && nd<11 );
  while( nd ) msg[ len++ ] = dig[ --nd ];
  msg[ len++ ] = '\n';
  (void)!write( 2, msg, (ulong)len );
  ((ucontext_t *)uc)->uc_mcontext.gregs[ REG_RAX ] = -ENOSYS;
}
#endif

/* fd_boot / fd_halt bring up the shmem and tile layers, which this driver
   does not link: oracle/Makefile renames them (-Dfd_boot=...) to these */
#if defined(fd_boot)
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

/* the out link's burst: the patched tile's (fd_verify_tile.h, FD_HAS_HIP:
   the reference's 1, its publishes stay within the stem's credits) */
#if FD_HAS_HIP
#define DRV_OUT_BURST FD_VERIFY_HIP_STEM_BURST
#else
#define DRV_OUT_BURST 1UL
#endif

/* One arena stands in for the workspace: the tile addresses frags as
   64-byte chunks relative to its workspace base, and an mcache line holds
   the chunk in 32 bits, so every link and the tile scratch are carved from
   one block whose base is the workspace pointer. */
static uchar * drv_arena;
static ulong   drv_arena_sz, drv_arena_used;

static void *
drv_malloc( ulong align, ulong sz ) {
  ulong off = fd_ulong_align_up( drv_arena_used, align );
  FD_TEST( off+sz<=drv_arena_sz );
  drv_arena_used = off + sz;
  return drv_arena + off;
}

static fd_topo_link_t *
drv_link( fd_topo_t * topo, char const * name, ulong depth, ulong mtu, ulong burst ) {
  fd_topo_link_t * link = fd_topob_link( topo, name, "wksp", depth, mtu, burst );
  ulong data_sz = fd_dcache_req_data_sz( mtu, depth, burst, 1 );
  link->mcache = fd_mcache_join( fd_mcache_new( drv_malloc( fd_mcache_align(), fd_mcache_footprint( depth, 0UL ) ),
                                                depth, 0UL, 0UL ) );
  link->dcache = fd_dcache_join( fd_dcache_new( drv_malloc( fd_dcache_align(), fd_dcache_footprint( data_sz, 0UL ) ),
                                                data_sz, 0UL ) );
  return link;
}

static ulong
drv_link_footprint( ulong depth, ulong mtu, ulong burst ) {
  return fd_mcache_footprint( depth, 0UL ) + fd_dcache_footprint( fd_dcache_req_data_sz( mtu, depth, burst, 1 ), 0UL ) +
         fd_mcache_align() + fd_dcache_align();
}

static uchar *
read_all( char const * path, ulong * sz ) {
  FILE * f = fopen( path, "rb" ); FD_TEST( f );
  fseek( f, 0, SEEK_END ); long n = ftell( f ); fseek( f, 0, SEEK_SET );
  uchar * b = malloc( (ulong)n ); FD_TEST( b );
  FD_TEST( fread( b, 1, (ulong)n, f )==(ulong)n );
  fclose( f );
  *sz = (ulong)n;
  return b;
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  if( argc<3 ) FD_LOG_ERR(( "usage: %s in.bin out.bin", argv[0] ));
  ulong in_sz; uchar * in = read_all( argv[1], &in_sz );
  FD_TEST( in_sz>=28 && !memcmp( in, "FDT1", 4 ) );
  ulong n, seed, depth;
  memcpy( &n, in+4, 8 ); memcpy( &seed, in+12, 8 ); memcpy( &depth, in+20, 8 );

  /* mock topology: one verify tile, the quic in link, the dedup out link,
     every frag fits in the links without wrapping */
  ulong link_depth = fd_ulong_pow2_up( n+16UL );
  fd_topo_t * topo = fd_topob_new( aligned_alloc( alignof(fd_topo_t), fd_ulong_align_up( sizeof(fd_topo_t), alignof(fd_topo_t) ) ),
                                   "verify-drv" );
  fd_topo_wksp_t * wksp = fd_topob_wksp( topo, "wksp" );
  fd_topo_tile_t * tile = fd_topob_tile( topo, "verify", "wksp", "wksp", 0UL, 0, 0 );
  tile->verify.tcache_depth = depth;
  drv_arena_sz = 4096UL + scratch_footprint( tile ) + scratch_align() + fd_fseq_footprint() + fd_fseq_align() +
                 drv_link_footprint( link_depth, FD_TPU_RAW_MTU, 1UL ) +
                 drv_link_footprint( link_depth, FD_TPU_PARSED_MTU, DRV_OUT_BURST );
  drv_arena = aligned_alloc( 4096UL, fd_ulong_align_up( drv_arena_sz, 4096UL ) );
  FD_TEST( drv_arena );
  memset( drv_arena, 0, drv_arena_sz );
  drv_arena_used = 4096UL;                                  /* obj offset 0 means "none" (fd_topo.c:20) */
  wksp->wksp = (fd_wksp_t *)drv_arena;
  void * scratch = drv_malloc( scratch_align(), scratch_footprint( tile ) );
  topo->objs[ tile->tile_obj_id ].offset = (ulong)scratch - (ulong)drv_arena;
  fd_topo_link_t * quic = drv_link( topo, "quic_verify", link_depth, FD_TPU_RAW_MTU, 1UL );
  fd_topo_link_t * out  = drv_link( topo, "verify_dedup", link_depth, FD_TPU_PARSED_MTU, DRV_OUT_BURST );
  /* TILE_DRV_RANGE (patched tile, FD_HAS_HIP): the quic link unpolled, as
     integration/fd_verify_topo_hip.patch makes it -- the driver only
     publishes the frags and the tile reads them by range from after_credit */
  int const range = !!getenv( "TILE_DRV_RANGE" );
  fd_topob_tile_in ( topo, "verify", 0UL, "wksp", "quic_verify", 0UL, 0, !range );
  fd_topob_tile_out( topo, "verify", 0UL, "verify_dedup", 0UL );
  quic->mtu = FD_TPU_RAW_MTU; out->mtu = FD_TPU_PARSED_MTU;
  ulong * in_fseq = fd_fseq_join( fd_fseq_new( drv_malloc( fd_fseq_align(), fd_fseq_footprint() ), 0UL ) );
  FD_TEST( in_fseq );
  tile->in_link_fseq[ 0 ] = in_fseq;

  privileged_init( topo, tile );
  fd_verify_ctx_t * ctx = (fd_verify_ctx_t *)scratch;
  ctx->hashmap_seed = seed;                                 /* the fixture's seed, not fd_rng_secure's */
  unprivileged_init( topo, tile );
  ctx->round_robin_cnt = 1UL; ctx->round_robin_idx = 0UL;

  /* stem context for the one out link (fd_stem.c:506-516), credits never short */
  fd_frag_meta_t * out_mcache[1] = { out->mcache };
  ulong out_depth[1] = { link_depth }, out_seq[1] = { 0UL }, cr_avail[1] = { ULONG_MAX/2 }, min_cr_avail = ULONG_MAX/2;
  fd_stem_context_t stem = { .mcaches = out_mcache, .depths = out_depth, .seqs = out_seq,
                             .cr_avail = cr_avail, .min_cr_avail = &min_cr_avail, .cr_decrement_amount = 1UL };

  /* output assembled in memory and written with one write() at the end:
     under the sandbox only write() to this fd is allowed */
  int out_fd = open( argv[2], O_WRONLY|O_CREAT|O_TRUNC, 0644 );
  FD_TEST( out_fd>=0 );
  ulong   obuf_sz = 64UL + n*(24UL+FD_TPU_PARSED_MTU) + 8UL*(1UL+ctx->tcache_depth+ctx->tcache_map_cnt);
  uchar * obuf    = malloc( obuf_sz );
  FD_TEST( obuf );
  int sandboxed = 0;
#if FD_HAS_HIP
  if( getenv( "TILE_DRV_SECCOMP" ) ) {
    struct sigaction sa; memset( &sa, 0, sizeof(sa) );
    sa.sa_sigaction = drv_sigsys; sa.sa_flags = SA_SIGINFO;
    FD_TEST( !sigaction( SIGSYS, &sa, NULL ) );
    struct sock_filter filter[ 128 ];
    ulong cnt = verify_hip_seccomp( 128UL, filter, (uint)out_fd, ctx->hip_fd, ctx->hip_fd_cnt );
    struct sock_fprog prog = { .len = (ushort)cnt, .filter = filter };
    FD_TEST( !prctl( PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0 ) );
    FD_TEST( !syscall( SYS_seccomp, SECCOMP_SET_MODE_FILTER, 0, &prog ) );
    sandboxed = 1;
  }
#endif
  (void)sandboxed;

  ulong const in_chunk0 = fd_dcache_compact_chunk0( drv_arena, quic->dcache );   /* = ctx->in[0] when polled */
  ulong const in_wmark  = fd_dcache_compact_wmark ( drv_arena, quic->dcache, quic->mtu );
  ulong   in_chunk = in_chunk0;
  ulong   off = 28UL;
  for( ulong j=0UL; j<n; j++ ) {
#if FD_HAS_HIP
    /* as the stem: after_credit until it lets the next frag in (fd_stem.c:545-550) */
    for( long t0 = fd_log_wallclock();; ) {
      int poll_in = 1, busy = 0;
      after_credit( ctx, &stem, &poll_in, &busy );
      if( poll_in ) break;
      if( FD_UNLIKELY( fd_log_wallclock()-t0 > 30L*1000L*1000L*1000L ) ) FD_LOG_ERR(( "frag %lu: after_credit never let it in", j ));
    }
#endif
    ulong bid; ushort psz;
    memcpy( &bid, in+off, 8 ); memcpy( &psz, in+off+8, 2 ); off += 10UL;
    FD_TEST( off+psz<=in_sz );
    uchar * frag = fd_chunk_to_laddr( drv_arena, in_chunk );
    fd_txn_m_t * m = (fd_txn_m_t *)frag;
    memset( m, 0, sizeof(fd_txn_m_t) );
    m->payload_sz = psz; m->block_engine.bundle_id = bid;
    memcpy( fd_txn_m_payload( m ), in+off, psz ); off += psz;
    ulong sz = sizeof(fd_txn_m_t) + psz;
    fd_mcache_publish( quic->mcache, link_depth, j, 0UL, in_chunk, sz, 0UL, j, j );
    if( !range && !before_frag( ctx, 0UL, j, 0UL ) ) {
      during_frag( ctx, 0UL, j, 0UL, in_chunk, sz, 0UL );
      after_frag( ctx, 0UL, j, 0UL, sz, j, j, &stem );
    }
    in_chunk = fd_dcache_compact_next( in_chunk, sz, in_chunk0, in_wmark );
  }
#if FD_HAS_HIP
  /* drain: the tile flushes a partial batch after its timeout and
     publishes completed batches from after_credit */
  /* range mode: idle is not enough, the tile must also have read the link
     to its end (it reads ranges only from after_credit) */
#define DRV_DONE( ctx ) ( FD_VERIFY_HIP_IDLE( ctx ) && ( !range || (ctx)->hip_rlink[ 0 ].seq>=n ) )
  for( long t0 = fd_log_wallclock(); fd_log_wallclock()-t0 < 30L*1000L*1000L*1000L; ) {
    int poll_in = 1, busy = 0;
    after_credit( ctx, &stem, &poll_in, &busy );
    if( DRV_DONE( ctx ) ) break;
  }
  FD_TEST( DRV_DONE( ctx ) );
#undef DRV_DONE
#endif

  ulong pub = out_seq[0];
  ulong o = 0UL;
#define PUT( p, k ) do { FD_TEST( o+(k)<=obuf_sz ); memcpy( obuf+o, (p), (k) ); o += (k); } while(0)
  PUT( "FDO1", 4 ); PUT( &pub, 8 );
  for( ulong s=0UL; s<pub; s++ ) {
    fd_frag_meta_t const * meta = out->mcache + fd_mcache_line_idx( s, link_depth );
    FD_TEST( meta->seq==s );
    ulong sig = meta->sig, sz = meta->sz, tsorig = meta->tsorig;
    PUT( &sig, 8 ); PUT( &sz, 8 ); PUT( &tsorig, 8 );
    PUT( fd_chunk_to_laddr( ctx->out_mem, meta->chunk ), sz );
  }
#if FD_HAS_HIP
  verify_hip_metrics_pull( ctx );
#endif
  ulong met[5] = { ctx->metrics.parse_fail_cnt, ctx->metrics.verify_fail_cnt, ctx->metrics.dedup_fail_cnt,
                   ctx->metrics.bundle_peer_fail_cnt, ctx->metrics.gossiped_votes_cnt };
  PUT( met, 40 );
  PUT( ctx->tcache_sync, 8 );
  PUT( ctx->tcache_ring, 8UL*ctx->tcache_depth );
  PUT( ctx->tcache_map,  8UL*ctx->tcache_map_cnt );
#undef PUT
  FD_TEST( write( out_fd, obuf, o )==(long)o );
  FD_LOG_NOTICE(( "published %lu of %lu frags", pub, n ));
#if FD_HAS_HIP
  if( sandboxed ) {
    FD_LOG_NOTICE(( "seccomp traps: %d", drv_trap_cnt ));
    for( int k=0; k<drv_trap_cnt && k<16; k++ ) FD_LOG_NOTICE(( "seccomp trap: syscall %d", drv_trap_nr[ k ] ));
    /* a sandboxed tile never returns; leave without the runtime's exit
       handlers (their munmap/mbind/close are outside the policy) */
    syscall( SYS_exit_group, drv_trap_cnt ? 1 : 0 );
  }
#endif
  free( obuf ); free( drv_arena ); free( topo ); free( in );
  fd_halt();
  return 0;
}
