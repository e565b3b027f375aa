/* svc_tile_run.c -- the reference's verify stage in service mode, run and
   timed in the reference's own run loop: quic_verify producer -> verify
   tiles (src/disco/verify/fd_verify_tile.c + integration/fd_verify_tile_svc.patch,
   FD_HAS_HIP_SVC, no HIP in the process) -> verify_dedup consumers, with the
   GPU tile (integration/svc_run.c) serving the tiles through the segment
   of include/fd_verify_svc.h.  Built by integration/Makefile from the
   reference's sources where they lie; driven by tools/svc_bench.py.

   The topology is the reference's quic -> verify -> dedup fan-out
   (src/app/fdctl/topology.c:90,173,181): quic_verify links that every
   verify tile reads (range mode: unpolled, as integration/fd_verify_topo_hip.patch
   makes them), each tile taking seq % tile_cnt == kind_id (before_frag), each
   with its own verify_dedup link of the reference's sizing (depth
   SVC_RUN_OUT_DEPTH, default 16384 = tiles.verify.receive_buffer_size's
   default, burst 1) read by a reliable consumer.

     svc_tile_run produce <shm> <stream.bin> <tile_cnt> <in_depth>
         Creates <shm> (integration/svc_run.h), prints READY, waits for the
         GPU tile, the tiles and the consumers, then publishes the stream's
         frags on the quic_verify links and prints one JSON line once every
         tile and consumer is done.  Environment:
           SVC_RUN_LINKS=L      quic_verify links (frag j: link j % L, seq j / L)
           SVC_RUN_PRELAY=1     the dcache holds the whole stream, laid in
                                before the clock starts (the stage's rate,
                                not one producer core's copy); the mcache
                                keeps in_depth lines, so a producer that
                                laps a tile still overruns it
           SVC_RUN_RATE=R       offered rate, frags/s, with NO flow control
                                (the reference's unreliable link,
                                topology.c:173): frags the tiles do not read
                                in time are overrun (counted, not fatal);
                                default 0: flow control against the slowest
                                tile's fseq, nothing dropped
           SVC_RUN_OUT_DEPTH    verify_dedup depth (default 16384)
           SVC_RUN_LIE=k        every k-th frag's mcache sz is 8 bytes short
                                of its header's payload_sz (no reference
                                producer does this, fd_tpu_reasm.c:278):
                                after_frag parses stale out-dcache bytes,
                                which the tile redoes on its core
                                (FD_VERIFY_SVC_RES_HOST)
           SVC_RUN_POLLED=1     the quic_verify links polled by the stem (frag
                                requests through the frag area); =m (m > 1):
                                a bit mask, link l polled if bit l is set,
                                the others read by range (both kinds of in
                                link on one tile)
           SVC_RUN_REQ_DEPTH, SVC_RUN_SLOT_CAP, SVC_RUN_FRAG_CAP   the segment
     svc_tile_run tile <shm> <t>
         Verify tile t: the mock topology around the shared links (the shape
         of src/disco/verify/test_verify_tile.c:45-85), privileged_init
         (records its thread count and device fds), unprivileged_init, then
         stem_run1 with the patched callbacks until its share is verified,
         dropped or overrun and every published frag is out.
     svc_tile_run consume <shm> <t>
         The dedup side of tile t's verify_dedup link: a reliable consumer
         (its fseq is the tile's credit) that reads every published frag,
         checks its size, digests its payload in order (fd_hash chain: the
         same digest the reference tile's run gives, oracle/ref_txn_drv.c)
         and histograms tspub - tsorig and consume time - tsorig.
         SVC_RUN_CONS_STALL_MS=m: it sleeps m ms before reading anything.
     svc_tile_run host <shm> <clients> <req_depth> <slot_cap> <frag_cap>
         A run of client tiles only (see host() below).
   produce with SVC_RUN_CLIENTS=k adds k client tiles to the segment after
   the verify tiles (a replay or shred tile beside them,
   integration/svc_client.h) and ends the run only once each has set
   clients_done.

   Stream file: "FDT1" u64 n, u64 seed, u64 tcache_depth, per frag u64
   bundle_id, u16 payload_sz, payload bytes (oracle/tile_drv.c's format). */

#define FD_TILE_TEST
static int drv_should_shutdown( void * ctx );
#define STEM_CALLBACK_SHOULD_SHUTDOWN( ctx ) drv_should_shutdown( ctx )
#include TILE_SRC
#include "../topo/fd_topob.h"
#include "../metrics/fd_metrics.h"
#include "../../tango/fseq/fd_fseq.h"
#include "../../tango/tempo/fd_tempo.h"
#include "../../util/pod/fd_pod_format.h"
#include "../quic/fd_tpu.h"
#include "../../util/sandbox/fd_sandbox.h"
#include "svc_run.h"
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#if !FD_HAS_HIP_SVC
#error "svc_tile_run drives the service-mode tile (FD_HAS_HIP_SVC)"
#endif

#if defined(fd_boot)                         /* integration/Makefile renames fd_boot / fd_halt (tile_drv.c) */
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

static ulong env_ulong( char const * k, ulong def ) { char const * v = getenv( k ); return v ? strtoul( v, NULL, 0 ) : def; }

static void *
drv_map( char const * path, ulong sz, int create ) {
  int fd = open( path, create ? (O_RDWR|O_CREAT|O_EXCL) : O_RDWR, 0600 );
  if( fd<0 ) FD_LOG_ERR(( "open(%s) failed (%i-%s)", path, errno, fd_io_strerror( errno ) ));
  if( create && ftruncate( fd, (off_t)sz ) ) FD_LOG_ERR(( "ftruncate failed" ));
  if( !create ) {
    svc_run_hdr_t h;
    if( pread( fd, &h, sizeof(h), 0 )!=(long)sizeof(h) || h.magic!=SVC_RUN_MAGIC ) FD_LOG_ERR(( "%s: not a svc_run segment", path ));
    sz = h.map_sz;
  }
  void * p = mmap( NULL, sz, PROT_READ|PROT_WRITE, MAP_SHARED, fd, 0 );
  if( p==MAP_FAILED ) FD_LOG_ERR(( "mmap failed (%i-%s)", errno, fd_io_strerror( errno ) ));
  close( fd );
  return p;
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

static ulong
lat_bucket( double ns ) {                     /* bucket k: [2^(k/4), 2^((k+1)/4)) ns */
  if( ns<1.0 ) return 0UL;
  ulong k = (ulong)( 4.0*log2( ns ) );
  return k<SVC_RUN_LAT_B ? k : SVC_RUN_LAT_B-1UL;
}

/* ---- produce ------------------------------------------------------------ */

static void
print_lat( char const * name, ulong const * h ) {
  ulong tot = 0UL;
  for( ulong k=0UL; k<SVC_RUN_LAT_B; k++ ) tot += h[ k ];
  double q[ 3 ] = { 0.5, 0.99, 0.999 }, v[ 3 ] = { 0.0, 0.0, 0.0 };
  for( int i=0; i<3; i++ ) {
    ulong want = (ulong)( q[ i ]*(double)tot ), acc = 0UL;
    for( ulong k=0UL; k<SVC_RUN_LAT_B; k++ ) {
      acc += h[ k ];
      if( acc>want || k==SVC_RUN_LAT_B-1UL ) { v[ i ] = pow( 2.0, ((double)k + 1.0)/4.0 )*1e-3; break; }   /* bucket's upper edge, us */
    }
  }
  printf( "\"%s\": {\"p50_us\": %.1f, \"p99_us\": %.1f, \"p999_us\": %.1f, \"n\": %lu}", name, v[0], v[1], v[2], tot );
}

static int
produce( char const * path, char const * stream, ulong tile_cnt, ulong in_depth ) {
  FD_TEST( tile_cnt>=1UL && tile_cnt<=SVC_RUN_TILE_MAX && fd_ulong_is_pow2( in_depth ) );
  ulong in_sz; uchar * in = read_all( stream, &in_sz );
  FD_TEST( in_sz>=28UL && !memcmp( in, "FDT1", 4 ) );
  ulong n, seed, depth;
  memcpy( &n, in+4, 8 ); memcpy( &seed, in+12, 8 ); memcpy( &depth, in+20, 8 );
  ushort * fsz = malloc( n*sizeof(ushort) ); ulong * poff = malloc( n*sizeof(ulong) );
  FD_TEST( fsz && poff );
  ulong off = 28UL;
  for( ulong j=0UL; j<n; j++ ) {
    ushort psz; memcpy( &psz, in+off+8, 2 );
    poff[ j ] = off; off += 10UL + psz;
    FD_TEST( off<=in_sz && psz<=FD_TPU_MTU );
    fsz[ j ] = (ushort)( sizeof(fd_txn_m_t) + psz );
  }
  ulong const L         = env_ulong( "SVC_RUN_LINKS", 1UL );
  int   const prelay    = !!getenv( "SVC_RUN_PRELAY" );
  ulong const rate      = env_ulong( "SVC_RUN_RATE", 0UL );
  ulong const lie       = env_ulong( "SVC_RUN_LIE", 0UL );
  ulong const out_depth = env_ulong( "SVC_RUN_OUT_DEPTH", 16384UL );
  ulong const req_depth = env_ulong( "SVC_RUN_REQ_DEPTH", 16UL );
  ulong const slot_cap  = env_ulong( "SVC_RUN_SLOT_CAP", 32768UL );
  /* a polled link's frag area: 4096 frags per request, at most the slot's capacity (a frag area over
     slot_cap is no segment: the shallow-link shape's 2048-frag slots made every polled run fail) */
  ulong const frag_cap  = env_ulong( "SVC_RUN_FRAG_CAP", getenv( "SVC_RUN_POLLED" ) ? fd_ulong_min( 4096UL, slot_cap ) : 0UL );
  if( FD_UNLIKELY( L<1UL || L>SVC_RUN_LINK_MAX ) ) FD_LOG_ERR(( "SVC_RUN_LINKS %lu not in [1,%lu]", L, SVC_RUN_LINK_MAX ));
  if( FD_UNLIKELY( !fd_ulong_is_pow2( out_depth ) ) ) FD_LOG_ERR(( "SVC_RUN_OUT_DEPTH %lu not a power of 2", out_depth ));
  /* clients (integration/svc_client.h: a replay or shred tile beside the verify tiles): frag areas for their records */
  ulong const clients   = env_ulong( "SVC_RUN_CLIENTS", 0UL );
  ulong const frag_capc = clients ? fd_ulong_max( frag_cap, fd_ulong_min( 256UL, slot_cap ) ) : frag_cap;
  ulong svc_sz = fd_verify_svc_footprint( tile_cnt+clients, req_depth, slot_cap, frag_capc );
  if( FD_UNLIKELY( !svc_sz ) ) FD_LOG_ERR(( "bad service segment parameters (%lu tiles, %lu clients, %lu slots x %lu frags, frag area %lu)",
                                          tile_cnt, clients, req_depth, slot_cap, frag_capc ));

  ulong data_sz = fd_dcache_req_data_sz( FD_TPU_RAW_MTU, in_depth, 1UL, 1 );
  if( prelay ) {
    ulong most = 0UL;
    for( ulong l=0UL; l<L; l++ ) {
      ulong sz_l = 2UL*FD_TPU_RAW_MTU + 4096UL;
      for( ulong j=l; j<n; j+=L ) sz_l += fd_ulong_align_up( fsz[ j ], 2UL*FD_CHUNK_SZ );
      most = fd_ulong_max( most, sz_l );
    }
    data_sz = fd_ulong_max( data_sz, fd_ulong_align_up( most, 4096UL ) );
  }
  ulong out_data = fd_dcache_req_data_sz( FD_TPU_PARSED_MTU, out_depth, 1UL, 1 );
  ulong fs_strd  = fd_ulong_align_up( fd_fseq_footprint(), 128UL );
  ulong at = fd_ulong_align_up( sizeof(svc_run_hdr_t), 4096UL );
  ulong mc_off[ SVC_RUN_LINK_MAX ], fs_off[ SVC_RUN_LINK_MAX ], dc_off[ SVC_RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    mc_off[ l ] = at;
    fs_off[ l ] = fd_ulong_align_up( mc_off[ l ] + fd_mcache_footprint( in_depth, 0UL ), 4096UL );
    dc_off[ l ] = fd_ulong_align_up( fs_off[ l ] + tile_cnt*fs_strd, 4096UL );
    at          = fd_ulong_align_up( dc_off[ l ] + fd_dcache_footprint( data_sz, 0UL ), 4096UL );
  }
  ulong omc_off[ SVC_RUN_TILE_MAX ], odc_off[ SVC_RUN_TILE_MAX ], cfs_off[ SVC_RUN_TILE_MAX ];
  for( ulong t=0UL; t<tile_cnt; t++ ) {
    omc_off[ t ] = at;
    odc_off[ t ] = fd_ulong_align_up( omc_off[ t ] + fd_mcache_footprint( out_depth, 0UL ), 4096UL );
    cfs_off[ t ] = fd_ulong_align_up( odc_off[ t ] + fd_dcache_footprint( out_data, 0UL ), 4096UL );
    at           = fd_ulong_align_up( cfs_off[ t ] + fs_strd, 4096UL );
  }
  ulong svc_off = at;
  ulong map_sz  = fd_ulong_align_up( svc_off + svc_sz, 4096UL );

  uchar * base = drv_map( path, map_sz, 1 );
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;
  memset( hdr, 0, sizeof(svc_run_hdr_t) );
  fd_frag_meta_t * mcache[ SVC_RUN_LINK_MAX ];
  ulong chunk0[ SVC_RUN_LINK_MAX ], wmark[ SVC_RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    mcache[ l ] = fd_mcache_join( fd_mcache_new( base + mc_off[ l ], in_depth, 0UL, 0UL ) );
    for( ulong t=0UL; t<tile_cnt; t++ ) FD_TEST( fd_fseq_join( fd_fseq_new( base + fs_off[ l ] + t*fs_strd, 0UL ) ) );
    uchar * dcache = fd_dcache_join( fd_dcache_new( base + dc_off[ l ], data_sz, 0UL ) );
    FD_TEST( mcache[ l ] && dcache );
    chunk0[ l ] = fd_dcache_compact_chunk0( base, dcache );
    wmark [ l ] = fd_dcache_compact_wmark ( base, dcache, FD_TPU_RAW_MTU );
    hdr->mcache_off[ l ] = mc_off[ l ]; hdr->dcache_off[ l ] = dc_off[ l ]; hdr->fseq_off[ l ] = fs_off[ l ];
  }
  for( ulong t=0UL; t<tile_cnt; t++ ) {
    FD_TEST( fd_mcache_join( fd_mcache_new( base + omc_off[ t ], out_depth, 0UL, 0UL ) ) );
    FD_TEST( fd_dcache_join( fd_dcache_new( base + odc_off[ t ], out_data, 0UL ) ) );
    FD_TEST( fd_fseq_join( fd_fseq_new( base + cfs_off[ t ], 0UL ) ) );
    hdr->out_mcache_off[ t ] = omc_off[ t ]; hdr->out_dcache_off[ t ] = odc_off[ t ]; hdr->cons_fseq_off[ t ] = cfs_off[ t ];
  }
  FD_TEST( fd_verify_svc_new( base + svc_off, tile_cnt+clients, req_depth, slot_cap, frag_capc ) );
  hdr->client_cnt = clients;
  hdr->n = n; hdr->tile_cnt = tile_cnt; hdr->seed = seed; hdr->tcache_depth = depth; hdr->in_depth = in_depth;
  hdr->link_cnt = L; hdr->out_depth = out_depth; hdr->fseq_stride = fs_strd; hdr->dcache_data_sz = data_sz;
  hdr->out_data_sz = out_data; hdr->svc_off = svc_off; hdr->svc_sz = svc_sz; hdr->req_depth = req_depth;
  hdr->slot_cap = slot_cap; hdr->frag_cap = frag_capc; hdr->map_sz = map_sz;
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
  hdr->magic = SVC_RUN_MAGIC;
  FD_COMPILER_MFENCE();
  printf( "READY\n" ); fflush( stdout );

  for( long tw=fd_log_wallclock(); hdr->svc_ready<1UL || hdr->tiles_ready<tile_cnt || hdr->cons_ready<tile_cnt; FD_SPIN_PAUSE() )
    if( fd_log_wallclock()-tw > 180L*1000000000L )
      FD_LOG_ERR(( "not ready after 180 s (service %lu, tiles %lu, consumers %lu of %lu)", hdr->svc_ready,
                   hdr->tiles_ready, hdr->cons_ready, tile_cnt ));

  ulong const * fseq[ SVC_RUN_LINK_MAX ][ SVC_RUN_TILE_MAX ];
  for( ulong l=0UL; l<L; l++ )
    for( ulong t=0UL; t<tile_cnt; t++ ) fseq[ l ][ t ] = fd_fseq_join( base + fs_off[ l ] + t*fs_strd );
  double tick_per_ns = fd_tempo_tick_per_ns( NULL );
  long t0 = fd_log_wallclock();
  hdr->t0 = t0;
  FD_COMPILER_MFENCE();
  hdr->start = 1UL;
  ulong ctl = fd_frag_meta_ctl( 0UL, 1, 1, 0 );
  ulong lim[ SVC_RUN_LINK_MAX ], chunk[ SVC_RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) { lim[ l ] = rate ? ULONG_MAX : 0UL; chunk[ l ] = chunk0[ l ]; }
  double const ticks_per_frag = rate ? tick_per_ns*1e9/(double)rate : 0.0;
  long   const tick0 = fd_tickcount();
  for( ulong j=0UL; j<n; j++ ) {
    ulong l = j % L, seq = j / L;
    while( seq>=lim[ l ] ) {                                   /* flow control against the slowest tile */
      ulong m = ULONG_MAX;
      for( ulong t=0UL; t<tile_cnt; t++ ) m = fd_ulong_min( m, fd_fseq_query( fseq[ l ][ t ] ) );
      lim[ l ] = m + in_depth - 64UL;
      if( seq>=lim[ l ] ) FD_SPIN_PAUSE();
      if( fd_log_wallclock()-t0 > 600L*1000000000L ) FD_LOG_ERR(( "tiles stalled at link %lu seq %lu", l, seq ));
    }
    if( rate ) while( (double)( fd_tickcount()-tick0 )<(double)j*ticks_per_frag ) FD_SPIN_PAUSE();   /* paced */
    if( prelay ) chunk[ l ] = pchunk[ j ];
    else {
      fd_txn_m_t * m = (fd_txn_m_t *)fd_chunk_to_laddr( base, chunk[ l ] );
      memset( m, 0, sizeof(fd_txn_m_t) );
      memcpy( &m->block_engine.bundle_id, in+poff[ j ], 8 );
      m->payload_sz = (ushort)( fsz[ j ] - sizeof(fd_txn_m_t) );
      memcpy( fd_txn_m_payload( m ), in+poff[ j ]+10UL, m->payload_sz );
    }
    ulong ts = (ulong)fd_frag_meta_ts_comp( fd_tickcount() );
    ulong psz_lie = lie && j%lie==lie-1UL && fsz[ j ]>=sizeof(fd_txn_m_t)+8UL ? 8UL : 0UL;
    fd_mcache_publish( mcache[ l ], in_depth, seq, 0UL, chunk[ l ], fsz[ j ]-psz_lie, ctl, ts, ts );
    if( !prelay ) chunk[ l ] = fd_dcache_compact_next( chunk[ l ], fsz[ j ], chunk0[ l ], wmark[ l ] );
  }
  long t_pub = fd_log_wallclock();
  hdr->t_pub = t_pub;
  for( ;; ) {
    ulong done = 0UL;
    for( ulong t=0UL; t<tile_cnt; t++ ) done += hdr->tile[ t ].done + hdr->cons[ t ].done;
    if( done==2UL*tile_cnt && hdr->clients_done>=clients ) break;
    if( fd_log_wallclock()-t0 > 900L*1000000000L ) FD_LOG_ERR(( "tiles / consumers / clients not done after 900 s" ));
    FD_SPIN_PAUSE();
  }
  /* the GPU tile's threads while it still runs: each one's seccomp mode
     (2: filtered) and no_new_privs, from /proc (its sandbox, svc_run.c) */
  ulong svc_threads = 0UL, svc_filtered = 0UL, svc_nnp = 0UL;
  if( hdr->svc_pid ) {
    char dpath[ 64 ];
    snprintf( dpath, sizeof(dpath), "/proc/%lu/task", hdr->svc_pid );
    DIR * d = opendir( dpath );
    for( struct dirent * e; d && (e = readdir( d )); ) {
      if( e->d_name[0]=='.' ) continue;
      char spath[ 384 ], line[ 256 ];
      snprintf( spath, sizeof(spath), "%s/%s/status", dpath, e->d_name );
      FILE * f = fopen( spath, "r" );
      if( !f ) continue;
      svc_threads++;
      while( fgets( line, sizeof(line), f ) ) {
        if( !strncmp( line, "Seccomp:", 8 ) && strtoul( line+8, NULL, 10 )==2UL ) svc_filtered++;
        if( !strncmp( line, "NoNewPrivs:", 11 ) && strtoul( line+11, NULL, 10 )==1UL ) svc_nnp++;
      }
      fclose( f );
    }
    if( d ) closedir( d );
  }
  hdr->shutdown = 1UL;
  for( long tw=fd_log_wallclock(); !hdr->svc_done; FD_SPIN_PAUSE() )
    if( fd_log_wallclock()-tw > 60L*1000000000L ) FD_LOG_ERR(( "service not done 60 s after shutdown" ));

  long t_end = t0;
  ulong sigs = 0UL, frags = 0UL, pub = 0UL, parse = 0UL, verify = 0UL, dedup = 0UL, bundle = 0UL, ovr = 0UL, lapped = 0UL;
  ulong host = 0UL, reg[ 8 ] = { 0UL }, lat[ SVC_RUN_LAT_B ] = { 0UL }, latq[ SVC_RUN_LAT_B ] = { 0UL };
  ulong cons_frags = 0UL, cons_bad = 0UL, metrics_ok = 1UL, threads_max = 0UL, dev_fds = 0UL;
  long  t_last = t0;
  printf( "{\"tiles\": [" );
  for( ulong t=0UL; t<tile_cnt; t++ ) {
    svc_run_tile_res_t * r = &hdr->tile[ t ];
    svc_run_cons_res_t * c = &hdr->cons[ t ];
    t_end = fd_long_max( t_end, r->t_end ); t_last = fd_long_max( t_last, c->t_last );
    sigs += r->sigs; frags += r->frags; pub += r->pub; parse += r->parse; verify += r->verify; dedup += r->dedup;
    bundle += r->bundle; ovr += r->overrun; lapped += r->lapped; host += r->host;
    cons_frags += c->frags; cons_bad += c->bad; metrics_ok &= r->metrics_ok;
    threads_max = fd_ulong_max( threads_max, r->threads ); dev_fds += r->dev_fds;
    for( ulong k=0UL; k<8UL; k++ ) reg[ k ] += r->regime[ k ];
    for( ulong k=0UL; k<SVC_RUN_LAT_B; k++ ) { lat[ k ] += c->lat[ k ]; latq[ k ] += c->lat_q[ k ]; }
    printf( "%s{\"frags\": %lu, \"sigs\": %lu, \"published\": %lu, \"parse_fail\": %lu, \"verify_fail\": %lu, "
            "\"dedup\": %lu, \"bundle_peer_fail\": %lu, \"overrun\": %lu, \"lapped\": %lu, \"s\": %.6f, "
            "\"consumed\": %lu, \"digest\": \"%016lx\", \"threads\": %lu, \"dev_fds\": %lu, \"metrics_ok\": %lu, \"sandboxed\": %lu, "
            "\"link\": {\"consumed\": %lu, \"filtered\": %lu, \"overrun_polling\": %lu, \"overrun_polling_frags\": %lu, "
            "\"overrun_reading\": %lu, \"overrun_reading_frags\": %lu}, "
            "\"busy_s\": {\"publish\": %.4f, \"pass\": %.4f, \"flush\": %.4f, \"post\": %.4f}, \"early_credits\": %lu, "
            "\"gpu_metrics\": {\"signatures\": %lu, \"host_redone\": %lu, \"ingest_n\": %lu, \"ingest_mean_us\": %.1f, "
            "\"batch_n\": %lu, \"batch_mean_us\": %.1f, \"ingest_p50_us\": %.1f, \"ingest_p99_us\": %.1f, "
            "\"ingest_max_us\": %.1f}}",
            t ? ", " : "", r->frags, r->sigs, r->pub, r->parse, r->verify, r->dedup, r->bundle, r->overrun, r->lapped,
            (double)( r->t_end - t0 )*1e-9, c->frags, c->digest, r->threads, r->dev_fds, r->metrics_ok, r->sandboxed,
            r->link_consumed, r->link_filtered, r->link_ovr_poll, r->link_ovr_poll_frags, r->link_ovr_read,
            r->link_ovr_read_frags, r->sec_pub, r->sec_pass, r->sec_flush, r->sec_post, r->early,
            r->m_sigs, r->m_host, r->m_ing_n, r->m_ing_n ? 1e-3*(double)r->m_ing_sum/(double)r->m_ing_n : 0.0,
            r->m_batch_n, r->m_batch_n ? 1e-3*(double)r->m_batch_sum/(double)r->m_batch_n : 0.0,
            1e-3*(double)r->ing_p50, 1e-3*(double)r->ing_p99, 1e-3*(double)r->ing_max );
  }
  double s  = (double)( t_end - t0 )*1e-9;
  double rt = (double)( reg[0]+reg[1]+reg[2]+reg[3]+reg[4]+reg[5]+reg[6]+reg[7] ) + 1e-9;
  printf( "], \"regime\": {\"caught_up\": %.4f, \"processing\": %.4f, \"backpressure\": %.4f}, ",
          (double)( reg[0]+reg[3]+reg[6] )/rt, (double)( reg[1]+reg[4]+reg[7] )/rt, (double)( reg[2]+reg[5] )/rt );
  print_lat( "latency", lat ); printf( ", " );
  print_lat( "latency_to_consumer", latq ); printf( ", " );
  double occ_n = (double)hdr->svc_occ[0] + 1e-9;
  printf( "\"svc\": {\"launches\": %lu, \"frags\": %lu, \"requests\": %lu, \"flushes\": %lu, \"flushed_frags\": %lu, "
          "\"spans\": %lu, \"gpu_s\": %.6f, \"host_launch_s\": %.6f, \"host_flush_s\": %.6f, "
          "\"host_poll_s\": %.6f, \"polls\": %lu, \"ingests\": %lu, \"ingest_gpu_s\": %.6f, \"host_ingest_s\": %.6f, "
          "\"launch_max\": %lu, \"slots\": {\"posted\": %.3f, \"waiting\": %.3f, \"launched\": %.3f, \"results\": %.3f, "
          "\"free\": %.3f}}, ",
          hdr->svc_stats[0], hdr->svc_stats[1], hdr->svc_stats[2], hdr->svc_stats[3], hdr->svc_stats[4],
          hdr->svc_stats[6], (double)hdr->svc_stats[7]*1e-9, (double)hdr->svc_stats[8]*1e-9,
          (double)hdr->svc_stats[9]*1e-9, (double)hdr->svc_stats[10]*1e-9, hdr->svc_stats[11], hdr->svc_stats[12],
          (double)hdr->svc_stats[13]*1e-9, (double)hdr->svc_stats[14]*1e-9, hdr->svc_stats[15],
          (double)hdr->svc_occ[1]/occ_n, (double)hdr->svc_occ[2]/occ_n, (double)hdr->svc_occ[3]/occ_n,
          (double)hdr->svc_occ[4]/occ_n, (double)hdr->svc_occ[5]/occ_n );
  printf( "\"svc_sandbox\": {\"sandboxed\": %lu, \"threads\": %lu, \"seccomp_threads\": %lu, \"nnp_threads\": %lu, "
          "\"traps\": %lu, \"trap_nr\": [", hdr->svc_sandboxed, svc_threads, svc_filtered, svc_nnp, hdr->svc_traps );
  for( ulong k=0UL; k<fd_ulong_min( hdr->svc_traps, 16UL ); k++ ) printf( "%s%lu", k ? ", " : "", hdr->svc_trap_nr[ k ] );
  printf( "]}, " );
  printf( "\"frags\": %lu, \"sigs\": %lu, \"published\": %lu, \"parse_fail\": %lu, \"verify_fail\": %lu, "
          "\"dedup\": %lu, \"bundle_peer_fail\": %lu, \"overrun\": %lu, \"lapped\": %lu, \"host_redone\": %lu, "
          "\"consumed\": %lu, \"consumer_bad\": %lu, \"digest_on\": %d, \"metrics_ok\": %lu, \"tile_threads_max\": %lu, \"tile_dev_fds\": %lu, "
          "\"seconds\": %.6f, \"publish_s\": %.6f, \"consumer_s\": %.6f, \"verifies_per_s\": %.1f, \"frags_per_s\": %.1f, "
          "\"offered_rate\": %lu, \"in_depth\": %lu, \"out_depth\": %lu, \"tile_cnt\": %lu, \"links\": %lu, \"prelay\": %d, "
          "\"polled\": %d, \"req_depth\": %lu, \"slot_cap\": %lu, \"range_max\": %lu, \"stream_frags\": %lu, \"unseen\": %lu}\n",
          frags, sigs, pub, parse, verify, dedup, bundle, ovr, lapped, host, cons_frags, cons_bad, !!getenv( "SVC_RUN_DIGEST" ), metrics_ok, threads_max,
          dev_fds, s, (double)( t_pub - t0 )*1e-9, (double)( t_last - t0 )*1e-9, (double)sigs/s, (double)frags/s, rate,
          in_depth, out_depth, tile_cnt, L, prelay, !!getenv( "SVC_RUN_POLLED" ), req_depth, slot_cap,
          (ulong)FD_VERIFY_SVC_RANGE_MAX, n,
          /* unseen: published frags no tile counted, processed or overrun -- a polled link's overruns
             are the stem's own (its link metrics), so a polled run's losses show here */
          n>frags+ovr+lapped ? n-frags-ovr-lapped : 0UL );
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

static ulong           drv_share;           /* seqs of the stream this tile takes */
/* the polled links: the stem's fseq for each (its consumed seq, written at
   housekeeping) and the seq one past the link's last frag.  A polled
   link's overruns are the stem's own (its link-in metrics count every
   lapped frag, whichever tile's share it held), so a lapped tile cannot
   count its share to the end: it is done once the stem has passed every
   polled link's last seq (each frag processed, filtered or skipped) */
static ulong           drv_polled_cnt;
static ulong *         drv_polled_fseq[ SVC_RUN_LINK_MAX ];
static ulong           drv_polled_end [ SVC_RUN_LINK_MAX ];
static svc_run_hdr_t * drv_hdr;
static long            drv_deadline;
static svc_run_tile_res_t * drv_res;

/* frags of this tile's share accounted for: an after_frag outcome, or
   dropped by the stem's overrun checks (lapped while polling, overwritten
   before the GPU's read) */
static ulong
drv_seen( fd_verify_ctx_t * ctx ) {
  ulong seen = ctx->metrics.parse_fail_cnt + ctx->metrics.verify_fail_cnt + ctx->metrics.dedup_fail_cnt +
               ctx->metrics.bundle_peer_fail_cnt + ctx->svc_pub_cnt;
  for( ulong k=0UL; k<ctx->svc_rlink_cnt; k++ )
    seen += ctx->svc_rlink[ k ].overrun_polling_frag_cnt + ctx->svc_rlink[ k ].overrun_reading_frag_cnt;
  return seen;
}

static int
drv_should_shutdown( void * _ctx ) {
  static ulong calls;                                           /* every stem iteration: look every 64th */
  if( FD_LIKELY( (++calls) & 63UL ) ) return 0;
  fd_verify_ctx_t * ctx = (fd_verify_ctx_t *)_ctx;
  ulong seen = drv_seen( ctx );
  if( FD_UNLIKELY( fd_log_wallclock()>drv_deadline ) ) FD_LOG_ERR(( "tile: %lu of %lu frags after the deadline", seen, drv_share ));
  int drained = drv_polled_cnt && drv_hdr->t_pub;             /* the producer is done publishing */
  for( ulong k=0UL; drained && k<drv_polled_cnt; k++ ) drained = fd_fseq_query( drv_polled_fseq[ k ] )>=drv_polled_end[ k ];
  return ( seen>=drv_share || drained ) && FD_VERIFY_SVC_IDLE( ctx );
}

/* threads of this process and its open device fds (the GPU test's check
   that a tile can enter fd_sandbox: unshare( CLONE_NEWUSER ) needs one
   thread, fd_sandbox.c:640-655) */
static void
drv_process_census( ulong * threads, ulong * dev_fds ) {
  *threads = 0UL; *dev_fds = 0UL;
  DIR * d = opendir( "/proc/self/task" );
  if( d ) { struct dirent * e; while( (e = readdir( d )) ) *threads += e->d_name[0]!='.'; closedir( d ); }
  d = opendir( "/proc/self/fd" );
  if( d ) {
    struct dirent * e; char p[ 320 ], tgt[ 256 ];
    while( (e = readdir( d )) ) {
      if( e->d_name[0]=='.' ) continue;
      snprintf( p, sizeof(p), "/proc/self/fd/%s", e->d_name );
      long k = readlink( p, tgt, sizeof(tgt)-1UL );
      if( k<=0L ) continue;
      tgt[ k ] = 0;
      if( !strncmp( tgt, "/dev/kfd", 8 ) || !strncmp( tgt, "/dev/dri", 8 ) ) (*dev_fds)++;
    }
    closedir( d );
  }
}

static int
tile( char const * path, ulong t ) {
  uchar * base = drv_map( path, 0UL, 0 );
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;
  FD_TEST( t<hdr->tile_cnt );
  ulong in_depth = hdr->in_depth;
  ulong const pmask = env_ulong( "SVC_RUN_POLLED", 0UL );
  ulong const polled_mask = pmask==1UL ? ~0UL : pmask;          /* 1: every link; m > 1: the links of mask m */

  fd_topo_t * topo = fd_topob_new( aligned_alloc( alignof(fd_topo_t), fd_ulong_align_up( sizeof(fd_topo_t), alignof(fd_topo_t) ) ),
                                   "verify-svc-run" );
  fd_topo_wksp_t * sw = fd_topob_wksp( topo, "stage" );         /* the shared file: every link and the segment */
  fd_topo_wksp_t * tw = fd_topob_wksp( topo, "verify" );        /* this tile's own memory */
  fd_topo_tile_t * tile = fd_topob_tile( topo, "verify", "verify", "verify", 0UL, 0, 0 );
  tile->verify.tcache_depth = hdr->tcache_depth;
  drv_arena_sz = 4096UL + scratch_footprint( tile ) + scratch_align() + 4096UL;
  drv_arena = aligned_alloc( 4096UL, fd_ulong_align_up( drv_arena_sz, 4096UL ) );
  FD_TEST( drv_arena );
  memset( drv_arena, 0, drv_arena_sz );
  drv_arena_used = 4096UL;
  sw->wksp = (fd_wksp_t *)base;
  tw->wksp = (fd_wksp_t *)drv_arena;
  void * scratch = drv_malloc( scratch_align(), scratch_footprint( tile ) );
  topo->objs[ tile->tile_obj_id ].offset = (ulong)scratch - (ulong)drv_arena;

  ulong const L = hdr->link_cnt;
  fd_topo_link_t * quic[ SVC_RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    quic[ l ] = fd_topob_link( topo, "quic_verify", "stage", in_depth, FD_TPU_REASM_MTU, 1UL );
    quic[ l ]->mcache = fd_mcache_join( base + hdr->mcache_off[ l ] );
    quic[ l ]->dcache = fd_dcache_join( base + hdr->dcache_off[ l ] );
    FD_TEST( quic[ l ]->mcache && quic[ l ]->dcache );
    quic[ l ]->mtu = FD_TPU_REASM_MTU;
  }
  fd_topo_link_t * out = fd_topob_link( topo, "verify_dedup", "stage", hdr->out_depth, FD_TPU_PARSED_MTU, 1UL );
  out->mcache = fd_mcache_join( base + hdr->out_mcache_off[ t ] );
  out->dcache = fd_dcache_join( base + hdr->out_dcache_off[ t ] );
  FD_TEST( out->mcache && out->dcache );
  out->mtu = FD_TPU_PARSED_MTU;
  ulong * in_fseq[ SVC_RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ ) {
    fd_topob_tile_in( topo, "verify", 0UL, "verify", "quic_verify", l, FD_TOPOB_UNRELIABLE,
                      ( polled_mask>>l )&1UL ? FD_TOPOB_POLLED : FD_TOPOB_UNPOLLED );
    in_fseq[ l ] = fd_fseq_join( base + hdr->fseq_off[ l ] + t*hdr->fseq_stride );
    tile->in_link_fseq[ l ] = in_fseq[ l ];
  }
  fd_topob_tile_out( topo, "verify", 0UL, "verify_dedup", 0UL );
  tile->kind_id = t;
  /* the verify service object (fd_verify_svc.h): one GPU */
  fd_topo_obj_t * svc = fd_topob_obj( topo, "verify_svc", "stage" );
  svc->offset = hdr->svc_off;
  FD_TEST( fd_pod_insert_ulong( topo->props, "verify_svc.gpu_cnt", 1UL ) );
  FD_TEST( fd_pod_insertf_ulong( topo->props, svc->id, "verify_svc.%lu", 0UL ) );

  /* everything the run loop uses, allocated before the sandbox (which
     leaves no address space to map) */
  ulong * metrics = aligned_alloc( FD_METRICS_ALIGN, fd_ulong_align_up( FD_METRICS_FOOTPRINT( L, 1UL ), FD_METRICS_ALIGN ) );
  fd_metrics_register( fd_metrics_new( metrics, L, 1UL ) );
  ulong polled_cnt = 0UL;
  fd_frag_meta_t const * in_mcache[ SVC_RUN_LINK_MAX ];
  ulong *                in_fseqs [ SVC_RUN_LINK_MAX ];
  for( ulong l=0UL; l<L; l++ )                                  /* the stem's ins: the polled links, in link order */
    if( ( polled_mask>>l )&1UL ) {
      in_mcache[ polled_cnt ] = quic[ l ]->mcache; in_fseqs[ polled_cnt ] = in_fseq[ l ];
      drv_polled_fseq[ polled_cnt ] = in_fseq[ l ];
      drv_polled_end [ polled_cnt ] = ( hdr->n + L - 1UL - l )/L;   /* frags j = l mod L: seqs 0 .. end-1 */
      polled_cnt++;
    }
  drv_polled_cnt = polled_cnt; drv_hdr = hdr;
  void * stem_scratch = aligned_alloc( FD_STEM_SCRATCH_ALIGN,
                                       fd_ulong_align_up( stem_scratch_footprint( polled_cnt, 1UL, 1UL ), FD_STEM_SCRATCH_ALIGN ) );
  fd_rng_t rng_mem[ 1 ];
  fd_rng_t * rng = fd_rng_join( fd_rng_new( rng_mem, (uint)(hdr->seed + t), 0UL ) );
  fd_frag_meta_t *       out_mcache[ 1 ] = { out->mcache };
  ulong                  cons_out[ 1 ] = { 0UL };
  ulong *                cons_fseqs[ 1 ] = { fd_fseq_join( base + hdr->cons_fseq_off[ t ] ) };
  (void)fd_tempo_tick_per_ns( NULL );                           /* calibrate before the clock starts */

  privileged_init( topo, tile );
  drv_res = &hdr->tile[ t ];
  { ulong th, fds; drv_process_census( &th, &fds ); drv_res->threads = th; drv_res->dev_fds = fds; }
  fd_verify_ctx_t * ctx = (fd_verify_ctx_t *)scratch;
  ctx->hashmap_seed = hdr->seed + t;                            /* fixed per tile: runs are reproducible */

  /* SVC_RUN_SANDBOX=1: the reference's sandbox, entered where
     fd_topo_run_tile enters it (src/disco/topo/fd_topo_run.c:86-135: after
     privileged_init, with the tile's own populate_allowed_fds and
     populate_allowed_seccomp -- the reference's policy, write and fsync
     only): a user namespace, pivot_root, landlock, rlimits, no
     capabilities, seccomp.  The process keeps only stderr (fdctl's boot
     closes the rest; here the driver does).  The loop's exit is not in the
     policy: the tile dies of SIGSYS after reporting, as a reference tile
     never returns. */
  drv_res->sandboxed = 0UL;
  if( getenv( "SVC_RUN_SANDBOX" ) ) {
    int   fds[ 256 ];
    ulong fd_cnt = populate_allowed_fds( topo, tile, 256UL, fds );
    struct sock_filter filter[ 256 ];
    ulong filter_cnt = populate_allowed_seccomp( topo, tile, 256UL, filter );
    for( int f=0; f<1024; f++ ) {
      int keep = 0;
      for( ulong k=0UL; k<fd_cnt; k++ ) keep |= fds[ k ]==f;
      if( !keep ) close( f );
    }
    fd_sandbox_enter( (uint)getuid(), (uint)getgid(), 0, 0, 0, 1, 0, 0UL, 0UL, 0UL, fd_cnt, fds, filter_cnt, filter );
    drv_res->sandboxed = 1UL;
  }

  unprivileged_init( topo, tile );
  ctx->round_robin_cnt = hdr->tile_cnt; ctx->round_robin_idx = t;
  drv_share = 0UL;                                              /* seq % T of every link */
  for( ulong l=0UL; l<L; l++ ) {
    ulong nl = ( hdr->n + L - 1UL - l )/L;
    drv_share += nl/hdr->tile_cnt + ( t<nl%hdr->tile_cnt ? 1UL : 0UL );
  }

  __atomic_fetch_add( &hdr->tiles_ready, 1UL, __ATOMIC_SEQ_CST );
  while( !hdr->start ) FD_SPIN_PAUSE();
  drv_deadline = fd_log_wallclock() + 600L*1000000000L;
  stem_run1( polled_cnt, in_mcache, in_fseqs, 1UL, out_mcache, 1UL, cons_out, cons_fseqs, 1UL, 0L, rng,
             stem_scratch, ctx );
  long t_end = fd_log_wallclock();

  svc_run_tile_res_t * r = drv_res;
  ulong lp = 0UL, lpf = 0UL, lr = 0UL, lrf = 0UL, lc = 0UL, lfl = 0UL;
  for( ulong k=0UL; k<ctx->svc_rlink_cnt; k++ ) {
    fd_verify_svc_rlink_t const * rl = &ctx->svc_rlink[ k ];
    lp += rl->overrun_polling_cnt; lpf += rl->overrun_polling_frag_cnt; lr += rl->overrun_reading_cnt;
    lrf += rl->overrun_reading_frag_cnt; lc += rl->consumed_cnt; lfl += rl->filtered_cnt;
  }
  r->t_end = t_end;
  r->pub    = ctx->svc_pub_cnt;
  r->parse  = ctx->metrics.parse_fail_cnt; r->verify = ctx->metrics.verify_fail_cnt; r->dedup = ctx->metrics.dedup_fail_cnt;
  r->bundle = ctx->metrics.bundle_peer_fail_cnt;
  r->frags  = r->pub + r->parse + r->verify + r->dedup + r->bundle;
  r->sigs   = ctx->svc_sig_cnt; r->overrun = lrf; r->lapped = lpf; r->host = ctx->svc_host_cnt; r->early = ctx->svc_early_cnt;
  r->link_consumed = lc; r->link_filtered = lfl; r->link_ovr_poll = lp; r->link_ovr_poll_frags = lpf;
  r->link_ovr_read = lr; r->link_ovr_read_frags = lrf;
  /* the link-in metric slots after the polled ones hold the range links' counts (metrics_write) */
  metrics_write( ctx );
  ulong ok = 1UL;
  for( ulong k=0UL; k<ctx->svc_rlink_cnt; k++ ) {
    fd_verify_svc_rlink_t const * rl = &ctx->svc_rlink[ k ];
    volatile ulong const * m = fd_metrics_link_in( fd_metrics_base_tl, ctx->svc_polled_cnt + k );
    ok &= m[ FD_METRICS_COUNTER_LINK_CONSUMED_COUNT_OFF ]==rl->consumed_cnt &&
          m[ FD_METRICS_COUNTER_LINK_FILTERED_COUNT_OFF ]==rl->filtered_cnt &&
          m[ FD_METRICS_COUNTER_LINK_OVERRUN_POLLING_FRAG_COUNT_OFF ]==rl->overrun_polling_frag_cnt &&
          m[ FD_METRICS_COUNTER_LINK_OVERRUN_READING_FRAG_COUNT_OFF ]==rl->overrun_reading_frag_cnt;
  }
  /* the GPU service's metrics (fd_verify_metrics_hip.patch), as metrics_write left them */
  r->m_sigs = fd_metrics_tl[ MIDX( COUNTER, VERIFY, GPU_SIGNATURES ) ];
  r->m_host = fd_metrics_tl[ MIDX( COUNTER, VERIFY, GPU_HOST_REDONE ) ];
  ulong in_ = 0UL, bn = 0UL;
  for( ulong k=0UL; k<FD_HISTF_BUCKET_CNT; k++ ) {
    in_ += fd_metrics_tl[ MIDX( HISTOGRAM, VERIFY, GPU_INGEST_LATENCY_NANOS ) + k ];
    bn  += fd_metrics_tl[ MIDX( HISTOGRAM, VERIFY, GPU_BATCH_LATENCY_NANOS  ) + k ];
  }
  r->m_ing_n = in_; r->m_batch_n = bn;
  r->ing_p50 = fd_histf_percentile( ctx->svc_ing_hist, 50, 0UL );
  r->ing_p99 = fd_histf_percentile( ctx->svc_ing_hist, 99, 0UL );
  r->ing_max = 0UL;
  for( ulong k=0UL; k<fd_histf_bucket_cnt( ctx->svc_ing_hist ); k++ )
    if( fd_histf_cnt( ctx->svc_ing_hist, k ) ) r->ing_max = fd_histf_right( ctx->svc_ing_hist, k );
  r->m_ing_sum   = FD_MHIST_SUM( VERIFY, GPU_INGEST_LATENCY_NANOS );
  r->m_batch_sum = FD_MHIST_SUM( VERIFY, GPU_BATCH_LATENCY_NANOS );
  ok &= r->m_sigs==ctx->svc_sig_cnt && r->m_host==ctx->svc_host_cnt;
  r->metrics_ok = ok;
  double tpn = fd_tempo_tick_per_ns( NULL );
  r->sec_pub  = (double)ctx->svc_ticks[ 0 ]/tpn*1e-9; r->sec_pass = (double)ctx->svc_ticks[ 1 ]/tpn*1e-9;
  r->sec_flush = (double)ctx->svc_ticks[ 2 ]/tpn*1e-9; r->sec_post = (double)ctx->svc_ticks[ 3 ]/tpn*1e-9;
  for( ulong k=0UL; k<8UL; k++ ) r->regime[ k ] = fd_metrics_tl[ MIDX( COUNTER, TILE, REGIME_DURATION_NANOS ) + k ];
  FD_COMPILER_MFENCE();
  r->done = 1UL;
  return 0;
}

/* ---- consume ------------------------------------------------------------- */

static int
consume( char const * path, ulong t ) {
  uchar * base = drv_map( path, 0UL, 0 );
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;
  FD_TEST( t<hdr->tile_cnt );
  fd_frag_meta_t const * mcache = fd_mcache_join( base + hdr->out_mcache_off[ t ] );
  ulong *                fseq   = fd_fseq_join( base + hdr->cons_fseq_off[ t ] );
  ulong                  depth  = hdr->out_depth;
  FD_TEST( mcache && fseq );
  double tick_per_ns = fd_tempo_tick_per_ns( NULL );
  ulong stall_ms = env_ulong( "SVC_RUN_CONS_STALL_MS", 0UL );
  /* SVC_RUN_DIGEST=1: read every frag's bytes (size checks, the payload
     digest); otherwise only the mcache lines (the credits and the latency):
     a consumer that reads ~700 B per frag is ~100-200 ns a frag, as the
     reference's dedup tile's copy is, and would bound a bench of the
     verify stage at its own rate */
  int const digest_on = !!getenv( "SVC_RUN_DIGEST" );
  svc_run_cons_res_t * c = &hdr->cons[ t ];
  __atomic_fetch_add( &hdr->cons_ready, 1UL, __ATOMIC_SEQ_CST );
  while( !hdr->start ) FD_SPIN_PAUSE();
  if( stall_ms ) usleep( (uint)( stall_ms*1000UL ) );
  ulong seq = 0UL, digest = 0x5eedd16e57UL, bytes = 0UL, bad = 0UL, ovr = 0UL;
  ulong lat[ SVC_RUN_LAT_B ] = { 0UL }, latq[ SVC_RUN_LAT_B ] = { 0UL };
  long  deadline = fd_log_wallclock() + 900L*1000000000L;
  long  t_last = fd_log_wallclock();
  for( ulong it=0UL;; it++ ) {
    fd_frag_meta_t const * line = mcache + fd_mcache_line_idx( seq, depth );
    ulong found = fd_frag_meta_seq_query( line );
    long  diff  = fd_seq_diff( found, seq );
    if( diff<0L ) {                                             /* caught up */
      if( hdr->tile[ t ].done && seq>=hdr->tile[ t ].pub ) break;
      if( !( it & 1023UL ) && fd_log_wallclock()>deadline ) FD_LOG_ERR(( "consumer %lu stuck at seq %lu", t, seq ));
      FD_SPIN_PAUSE();
      continue;
    }
    if( FD_UNLIKELY( diff>0L ) ) { ovr += (ulong)diff; seq = found; continue; }   /* a reliable consumer never sees this */
    FD_COMPILER_MFENCE();
    ulong chunk = line->chunk, sz = line->sz, tsorig = line->tsorig, tspub = line->tspub;
    ulong d2 = digest, b2 = 0UL;
    if( digest_on ) {
      uchar const * frag = (uchar const *)fd_chunk_to_laddr_const( base, chunk );
      fd_txn_m_t const * m = (fd_txn_m_t const *)frag;
      ulong psz = m->payload_sz, tsz = m->txn_t_sz;
      ulong want = fd_ulong_align_up( sizeof(fd_txn_m_t) + psz, fd_txn_align() ) + tsz;
      d2 = fd_hash( digest, fd_txn_m_payload_const( m ), psz );
      b2 = ( want!=sz || !tsz || psz>FD_TPU_MTU );
    }
    FD_COMPILER_MFENCE();
    if( FD_UNLIKELY( fd_frag_meta_seq_query( line )!=seq ) ) { ovr++; continue; }
    bad    += b2;
    digest  = d2;
    bytes  += sz;
    long now = fd_tickcount();
    long to  = fd_frag_meta_ts_decomp( tsorig, now ), tp = fd_frag_meta_ts_decomp( tspub, now );
    lat [ lat_bucket( (double)( tp - to )/tick_per_ns ) ]++;
    latq[ lat_bucket( (double)( now - to )/tick_per_ns ) ]++;
    seq++;
    if( !( seq & 63UL ) ) fd_fseq_update( fseq, seq );
    t_last = fd_log_wallclock();
  }
  fd_fseq_update( fseq, seq );
  c->frags = seq; c->bytes = bytes; c->digest = digest; c->overrun = ovr; c->bad = bad; c->t_last = t_last;
  for( ulong k=0UL; k<SVC_RUN_LAT_B; k++ ) { c->lat[ k ] = lat[ k ]; c->lat_q[ k ] = latq[ k ]; }
  FD_COMPILER_MFENCE();
  c->done = 1UL;
  return 0;
}

/* svc_tile_run host <shm> <clients> <req_depth> <slot_cap> <frag_cap>: a
   run of clients only (no link, no verify tile): creates <shm> with a
   segment of <clients> client tiles, prints READY, waits for the GPU tile
   (svc_run or oracle/svc_mock on the same file) and for every client
   process (integration/svc_client.h: each sets clients_done when done),
   then shuts the service down and prints the service's counters */
static int
host( char const * path, ulong clients, ulong req_depth, ulong slot_cap, ulong frag_cap ) {
  FD_TEST( clients>=1UL && clients<=FD_VERIFY_SVC_TILE_MAX );
  ulong svc_sz = fd_verify_svc_footprint( clients, req_depth, slot_cap, frag_cap );
  if( FD_UNLIKELY( !svc_sz ) ) FD_LOG_ERR(( "bad segment parameters (%lu clients, %lu slots x %lu, frag area %lu)",
                                          clients, req_depth, slot_cap, frag_cap ));
  ulong svc_off = fd_ulong_align_up( sizeof(svc_run_hdr_t), 4096UL );
  ulong map_sz  = fd_ulong_align_up( svc_off + svc_sz, 4096UL );
  uchar * base = drv_map( path, map_sz, 1 );
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;
  memset( hdr, 0, sizeof(svc_run_hdr_t) );
  FD_TEST( fd_verify_svc_new( base + svc_off, clients, req_depth, slot_cap, frag_cap ) );
  hdr->tile_cnt = 0UL; hdr->client_cnt = clients; hdr->link_cnt = 0UL;
  hdr->svc_off = svc_off; hdr->svc_sz = svc_sz; hdr->req_depth = req_depth; hdr->slot_cap = slot_cap;
  hdr->frag_cap = frag_cap; hdr->map_sz = map_sz;
  FD_COMPILER_MFENCE();
  hdr->magic = SVC_RUN_MAGIC;
  FD_COMPILER_MFENCE();
  printf( "READY\n" ); fflush( stdout );
  long t0 = fd_log_wallclock();
  while( hdr->svc_ready<1UL ) {
    if( fd_log_wallclock()-t0 > 180L*1000000000L ) FD_LOG_ERR(( "GPU tile not ready after 180 s" ));
    FD_SPIN_PAUSE();
  }
  hdr->start = 1UL;
  while( hdr->clients_done<clients ) {
    if( fd_log_wallclock()-t0 > 900L*1000000000L ) FD_LOG_ERR(( "clients not done after 900 s (%lu of %lu)", hdr->clients_done, clients ));
    FD_SPIN_PAUSE();
  }
  long t1 = fd_log_wallclock();
  hdr->shutdown = 1UL;
  while( !hdr->svc_done ) {
    if( fd_log_wallclock()-t1 > 120L*1000000000L ) FD_LOG_ERR(( "GPU tile not done 120 s after shutdown" ));
    FD_SPIN_PAUSE();
  }
  printf( "{\"clients\": %lu, \"seconds\": %.6f, \"svc\": {\"launches\": %lu, \"records\": %lu, \"requests\": %lu, "
          "\"gpu_ns\": %lu, \"largest_launch\": %lu}, \"svc_sandboxed\": %lu, \"svc_traps\": %lu}\n", clients,
          (double)( t1-t0 )*1e-9, hdr->svc_stats[ 0 ], hdr->svc_stats[ 1 ], hdr->svc_stats[ 2 ], hdr->svc_stats[ 7 ],
          hdr->svc_stats[ 15 ], hdr->svc_sandboxed, hdr->svc_traps );
  return 0;
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  if( argc>=6 && !strcmp( argv[1], "produce" ) )
    return produce( argv[2], argv[3], strtoul( argv[4], NULL, 0 ), strtoul( argv[5], NULL, 0 ) );
  if( argc>=4 && !strcmp( argv[1], "tile" ) )    return tile( argv[2], strtoul( argv[3], NULL, 0 ) );
  if( argc>=4 && !strcmp( argv[1], "consume" ) ) return consume( argv[2], strtoul( argv[3], NULL, 0 ) );
  if( argc>=7 && !strcmp( argv[1], "host" ) )
    return host( argv[2], strtoul( argv[3], NULL, 0 ), strtoul( argv[4], NULL, 0 ), strtoul( argv[5], NULL, 0 ),
                 strtoul( argv[6], NULL, 0 ) );
  fprintf( stderr, "usage: %s produce <shm> <stream.bin> <tile_cnt> <in_depth> | tile <shm> <t> | consume <shm> <t> | "
                   "host <shm> <clients> <req_depth> <slot_cap> <frag_cap>\n", argv[0] );
  return 2;
}
