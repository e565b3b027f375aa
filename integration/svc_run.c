/* svc_run.c -- the GPU tile of the service-mode verify stage run
   (integration/svc_tile_run.c, integration/svc_run.h): one process that
   owns the HIP context and serves every verify tile of the run through the
   segment of include/fd_verify_svc.h.

     svc_run <shm> <gpu>

   Maps the run's shared file, registers it for the GPU once (every link's
   mcache and dcache, the tiles' verify_dedup dcaches and the segment lie
   in it), names the quic_verify links (service link l = link kind_id l)
   and the tiles' out dcaches (the segment's client tiles, after them, get
   fd_verify_svc_set_client), then polls until the producer sets shutdown.
   Environment: SVC_BATCH_MAX (frags per merged launch, default 262144),
   SVC_INFLIGHT (launches at once, default 2), SVC_MERGE_MIN (frags that
   start a launch at once, default batch_max / 2), SVC_MERGE_WAIT_NS
   (default 2000000), SVC_MERGE_IDLE_NS (the wait with no launch in flight,
   default 20000), SVC_HW_QUEUES (GPU_MAX_HW_QUEUES for this process,
   default 8, set over the environment's), SVC_SANDBOX (kill, the default:
   after the service is running the process enters
   fd_hip_tile_sandbox_process -- fd allow-list, rlimits, no capabilities,
   no new privileges, a seccomp filter over every thread with
   SECCOMP_RET_KILL_PROCESS; trap: the same filter with SECCOMP_RET_TRAP, a
   refused call is recorded and fails with ENOSYS; 0: none),
   SVC_SANDBOX_PROBE=1 (a refused call right after entering: the process
   must die of SIGSYS).

   The integration's GPU tile (integration/fd_verify_gpu_tile.c) does the
   same from the topology's objects. */

#include "../../tango/mcache/fd_mcache.h"
#include "../../tango/dcache/fd_dcache.h"
#include "../quic/fd_tpu.h"
#include "fd_verify_svc.h"
#include "fd_hip_tile_sandbox.h"
#include "svc_run.h"
#include <errno.h>
#include <dlfcn.h>
#include <signal.h>
#include <ucontext.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#if defined(fd_boot)
void fd_boot( int * pargc, char *** pargv ) { (void)pargc; (void)pargv; }
void fd_halt( void ) {}
#endif

static ulong env_ulong( char const * k, ulong def ) { char const * v = getenv( k ); return v ? strtoul( v, NULL, 0 ) : def; }

/* SVC_SANDBOX=trap: a refused call is recorded (its number, once) and
   returns -ENOSYS to the caller, so one run lists every call the filter is
   missing */
static svc_run_hdr_t * svc_hdr;
static int             hdr_sandboxed;

/* SIGTERM (the driver's timeout): leave the poll loop and tear the service
   down -- the IO engine stopped and drained -- rather than die with a
   kernel running on the GPU */
static volatile int svc_term;
static void svc_sigterm( int sig ) { (void)sig; svc_term = 1; }
static void
svc_sigsys( int sig, siginfo_t * si, void * uc_ ) {
  (void)sig;
  ucontext_t * uc = (ucontext_t *)uc_;
  uc->uc_mcontext.gregs[ REG_RAX ] = -ENOSYS;
  ulong nr = (ulong)si->si_syscall;
  static ulong traps;
  ulong k = traps++;
  if( svc_hdr ) {                                               /* NULL once the segment is unmapped */
    __atomic_fetch_add( &svc_hdr->svc_traps, 1UL, __ATOMIC_RELAXED );
    if( k<16UL ) svc_hdr->svc_trap_nr[ k ] = nr;
  }
  /* a path argument, when the call has one (openat, newfstatat: rsi; open, stat, access: rdi) */
  char const * path = nr==257UL || nr==262UL ? (char const *)uc->uc_mcontext.gregs[ REG_RSI ] :
                      nr==2UL || nr==4UL || nr==21UL ? (char const *)uc->uc_mcontext.gregs[ REG_RDI ] : NULL;
  char m[ 192 ]; int n = snprintf( m, sizeof(m), "svc_run: seccomp trap, syscall %lu, thread %ld%s%.100s\n", nr,
                                   (long)syscall( SYS_gettid ), path ? ", path " : "", path ? path : "" );
  if( n>0 ) (void)!write( 2, m, (ulong)n );
  /* where from: the faulting pc and the words on the stack that fall in a
     loaded object's code, named by dladdr (no unwinder: its first use in a
     thread makes calls the filter refuses, and a refused call inside this
     handler -- SIGSYS blocked -- kills the process) */
  if( k<4UL ) {
    ulong const * sp = (ulong const *)uc->uc_mcontext.gregs[ REG_RSP ];
    ulong pcs[ 9 ]; ulong np = 0UL;
    pcs[ np++ ] = (ulong)uc->uc_mcontext.gregs[ REG_RIP ];
    for( ulong w=0UL; w<256UL && np<9UL; w++ ) {
      Dl_info di;
      if( sp[ w ]>4096UL && dladdr( (void *)sp[ w ], &di ) && di.dli_fname && di.dli_sname ) pcs[ np++ ] = sp[ w ];
    }
    for( ulong i=0UL; i<np; i++ ) {
      Dl_info di; memset( &di, 0, sizeof(di) );
      (void)dladdr( (void *)pcs[ i ], &di );
      n = snprintf( m, sizeof(m), "  %s %s+0x%lx\n", di.dli_fname ? strrchr( di.dli_fname, '/' ) ? strrchr( di.dli_fname, '/' )+1 : di.dli_fname : "?",
                    di.dli_sname ? di.dli_sname : "?", di.dli_saddr ? pcs[ i ]-(ulong)di.dli_saddr : 0UL );
      if( n>0 ) (void)!write( 2, m, fd_ulong_min( (ulong)n, sizeof(m)-1UL ) );
    }
  }
}

int
main( int argc, char ** argv ) {
  fd_boot( &argc, &argv );
  if( argc<3 ) { fprintf( stderr, "usage: %s <shm> <gpu>\n", argv[0] ); return 2; }
  int fd = open( argv[1], O_RDWR );
  if( fd<0 ) FD_LOG_ERR(( "open(%s) failed (%i-%s)", argv[1], errno, fd_io_strerror( errno ) ));
  svc_run_hdr_t h;
  if( pread( fd, &h, sizeof(h), 0 )!=(long)sizeof(h) || h.magic!=SVC_RUN_MAGIC ) FD_LOG_ERR(( "%s: not a svc_run segment", argv[1] ));
  uchar * base = mmap( NULL, h.map_sz, PROT_READ|PROT_WRITE, MAP_SHARED, fd, 0 );
  if( base==MAP_FAILED ) FD_LOG_ERR(( "mmap failed (%i-%s)", errno, fd_io_strerror( errno ) ));
  close( fd );
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;

  /* hardware queues for this process's streams: the ingest and flush
     streams must not wait behind a verify launch in a shared queue
     (DESIGN.md section 10).  SVC_HW_QUEUES (default 8: the launch, ingest
     and tile streams of up to 5 tiles, while leaving the device's queue
     slots to other processes) replaces the environment's
     GPU_MAX_HW_QUEUES: the GPU boxes export HIP's default of 4 for every
     process (profiles/r05af/host.txt) */
  {
    ulong hwq = env_ulong( "SVC_HW_QUEUES", 8UL );
    if( hwq<1UL || hwq>32UL ) FD_LOG_ERR(( "SVC_HW_QUEUES %lu not in [1,32]", hwq ));
    char q[ 24 ]; snprintf( q, sizeof(q), "%lu", hwq ); setenv( "GPU_MAX_HW_QUEUES", q, 1 );
  }
  ulong batch_max = env_ulong( "SVC_BATCH_MAX", 262144UL );
  ulong inflight  = env_ulong( "SVC_INFLIGHT", 2UL );
  fd_verify_svc_t * svc = fd_verify_svc_boot( base + hdr->svc_off, (int)strtol( argv[2], NULL, 0 ), batch_max, inflight );
  if( !svc ) FD_LOG_ERR(( "fd_verify_svc_boot failed (batch_max %lu, inflight %lu)", batch_max, inflight ));
  fd_verify_svc_set_merge( svc, env_ulong( "SVC_MERGE_MIN", batch_max/2UL ), env_ulong( "SVC_MERGE_WAIT_NS", 2000000UL ),
                           env_ulong( "SVC_MERGE_IDLE_NS", 20000UL ) );
  if( fd_verify_svc_map( svc, base, hdr->map_sz ) ) FD_LOG_ERR(( "registering %lu B for the GPU failed", hdr->map_sz ));
  for( ulong l=0UL; l<hdr->link_cnt; l++ ) {
    fd_frag_meta_t const * mcache = fd_mcache_join( base + hdr->mcache_off[ l ] );
    uchar const *          dcache = fd_dcache_join( base + hdr->dcache_off[ l ] );
    if( !mcache || !dcache ) FD_LOG_ERR(( "link %lu: join failed", l ));
    /* during_frag's range, from the link's mtu as the tile sees it (svc_tile_run.c: FD_TPU_REASM_MTU) */
    if( fd_verify_svc_set_link( svc, l, mcache, fd_mcache_depth( mcache ), base, fd_dcache_compact_chunk0( base, dcache ),
                                fd_dcache_compact_wmark( base, dcache, FD_TPU_REASM_MTU ) ) )
      FD_LOG_ERR(( "fd_verify_svc_set_link %lu failed", l ));
  }
  for( ulong t=0UL; t<hdr->tile_cnt; t++ ) {
    uchar * dcache = fd_dcache_join( base + hdr->out_dcache_off[ t ] );
    if( !dcache || fd_verify_svc_set_tile( svc, t, dcache, fd_dcache_data_sz( dcache ), base ) )
      FD_LOG_ERR(( "fd_verify_svc_set_tile %lu failed", t ));
  }
  for( ulong c=0UL; c<hdr->client_cnt; c++ )
    if( fd_verify_svc_set_client( svc, hdr->tile_cnt+c ) ) FD_LOG_ERR(( "fd_verify_svc_set_client %lu failed", hdr->tile_cnt+c ));
  if( fd_verify_svc_run( svc ) ) FD_LOG_ERR(( "fd_verify_svc_run failed" ));

  {                                                             /* before the sandbox: rt_sigaction is not in its filter */
    struct sigaction sa;
    memset( &sa, 0, sizeof(sa) );
    sa.sa_handler = svc_sigterm;
    if( sigaction( SIGTERM, &sa, NULL ) ) FD_LOG_ERR(( "sigaction(SIGTERM) failed" ));
  }
  /* the GPU tile's sandbox: everything HIP needs is set up, so from here on
     the process opens nothing, starts no thread and makes only the calls of
     fd_hip_tile_seccomp_process (include/fd_hip_tile_sandbox.h) */
  hdr->svc_pid = (ulong)getpid();
  char const * sb = getenv( "SVC_SANDBOX" );
  if( !sb || strcmp( sb, "0" ) ) {
    int trap = sb && !strcmp( sb, "trap" );
    svc_hdr = hdr;
    if( trap ) {
      struct sigaction sa;
      memset( &sa, 0, sizeof(sa) );
      sa.sa_sigaction = svc_sigsys; sa.sa_flags = SA_SIGINFO;
      if( sigaction( SIGSYS, &sa, NULL ) ) FD_LOG_ERR(( "sigaction(SIGSYS) failed" ));
    }
    close( 0 ); close( 1 );                                     /* the driver's stdin and stdout (/dev/null) */
    int dev[ FD_HIP_TILE_FD_MAX ];
    long nd = fd_hip_tile_device_fds( dev, FD_HIP_TILE_FD_MAX );
    if( nd<0L ) FD_LOG_ERR(( "the HIP device fds could not be listed" ));
    char why[ 160 ];
    if( fd_hip_tile_sandbox_process( -1, dev, (ulong)nd, 1, trap ? SECCOMP_RET_TRAP : SECCOMP_RET_KILL_PROCESS, why, sizeof(why) ) )
      FD_LOG_ERR(( "sandbox: %s", why ));
    hdr->svc_sandboxed = 1UL; hdr_sandboxed = 1;
    if( getenv( "SVC_SANDBOX_PROBE" ) ) (void)syscall( SYS_getppid );   /* refused: the process dies here */
  }
  FD_COMPILER_MFENCE();
  hdr->svc_ready = 1UL;
  long deadline = fd_log_wallclock() + 1200L*1000000000L;
  /* SVC_DEBUG_S=s: the service's state on stderr every s seconds (a stalled
     run's log names where it stalled) */
  long dbg_ns = (long)env_ulong( "SVC_DEBUG_S", 0UL )*1000000000L, dbg_next = fd_log_wallclock() + dbg_ns;
  for( ulong it=0UL; !hdr->shutdown && !svc_term; it++ ) {
    if( !fd_verify_svc_poll( svc ) ) FD_SPIN_PAUSE();
    if( !( it & 0xffffUL ) ) {
      long now = fd_log_wallclock();
      if( now>deadline ) { fprintf( stderr, "svc_run: no shutdown after 1200 s\n" ); break; }
      if( dbg_ns && now>dbg_next ) {
        char b[ 1024 ]; int n = fd_verify_svc_debug( svc, b, sizeof(b) );
        if( n>0 ) { b[ sizeof(b)-2 ] = '\0'; fprintf( stderr, "svc_run: %s\n", b ); }
        dbg_next = now + dbg_ns;
      }
    }
  }
  if( svc_term || !hdr->shutdown ) {
    char b[ 1024 ]; int n = fd_verify_svc_debug( svc, b, sizeof(b) );
    if( n>0 ) { b[ sizeof(b)-2 ] = '\0'; fprintf( stderr, "svc_run: stopped before shutdown: %s\n", b ); }
  }
  (void)!write( 2, "svc_run: teardown\n", 18UL );
  ulong st[ 16 ];
  fd_verify_svc_stats( svc, st );
  for( ulong k=0UL; k<16UL; k++ ) hdr->svc_stats[ k ] = st[ k ];
  ulong occ[ 6 ];
  fd_verify_svc_occupancy( svc, occ );
  for( ulong k=0UL; k<6UL; k++ ) hdr->svc_occ[ k ] = occ[ k ];
  fd_verify_svc_delete( svc );
  (void)!write( 2, "svc_run: deleted\n", 17UL );
  FD_COMPILER_MFENCE();
  hdr->svc_done = 1UL;
  svc_hdr = NULL;
  munmap( base, h.map_sz );
  /* a sandboxed process leaves with exit_group: the HIP runtime's exit-time
     destructors close descriptors and free what the kernel frees anyway,
     calls the filter refuses (the GPU's work was drained by
     fd_verify_svc_delete above) */
  if( hdr_sandboxed ) { fflush( stderr ); _exit( 0 ); }
  return 0;
}
