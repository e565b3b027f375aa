/* svc_probe.c -- the verify service's IO engine step by step, with no tile
   process: one segment in this process's memory, the service on GPU 0, and
   requests posted by hand (fd_verify_svc.h's tile-side calls).  Each step
   prints one line with the service's state (fd_verify_svc_debug) and fails
   loudly with a deadline, so a run names the step an engine change broke:

     idle       the engine runs 0.5 s with nothing posted
     empty      a frag request with no frags: INGESTED by the engine, RESULTS
     frags      a frag request of 64 frags in the frag area: ingested, verified
                (zero bytes: every frag fails its parse), RESULTS; the tile
                side frees the slots
     flush      a flush of host-written entries (nothing to copy): flush_done
     delete     teardown (the engine stopped and drained)

   svc_probe [frags]          (default 64)
   Built by integration/Makefile (svc-probe), run by tests/test_gpu_svc_io.py. */

#define _GNU_SOURCE
#include "fd_verify_svc.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

static long now_ns( void ) { struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t ); return t.tv_sec*1000000000L + t.tv_nsec; }

static fd_verify_svc_t * svc;
static char const * volatile step_now = "boot";

/* a step that blocks inside a HIP call: say which, every 5 s */
static void
on_alarm( int sig ) {
  (void)sig;
  char b[ 1024 ];
  int  n = svc ? fd_verify_svc_debug( svc, b, sizeof(b) ) : 0;
  printf( "%s: STILL RUNNING | %s\n", step_now, n>0 ? b : "" );
  fflush( stdout );
  alarm( 5 );
}

static void
say( char const * step, char const * what ) {
  char b[ 1024 ];
  int  n = fd_verify_svc_debug( svc, b, sizeof(b) );
  printf( "%s: %s | %s\n", step, what, n>0 ? b : "" );
  fflush( stdout );
}

/* poll until *p reaches want (or the deadline) */
static int
wait_state( char const * step, ulong * p, ulong want, long ms ) {
  long end = now_ns() + ms*1000000L;
  while( fd_verify_svc_ld( p )!=want ) {
    fd_verify_svc_poll( svc );
    if( now_ns()>end ) { say( step, "TIMEOUT" ); return -1; }
  }
  return 0;
}

int
main( int argc, char ** argv ) {
  ulong nfr = argc>1 ? strtoul( argv[1], NULL, 0 ) : 64UL;
  ulong T = 1UL, D = 8UL, cap = 1024UL, fcap = 256UL;
  if( nfr>fcap ) nfr = fcap;
  ulong fp = fd_verify_svc_footprint( T, D, cap, fcap );
  void * mem = aligned_alloc( 4096UL, fp );
  ulong out_sz = 1UL<<22;
  uchar * out = aligned_alloc( 4096UL, out_sz );
  if( !mem || !out ) { printf( "alloc failed\n" ); return 1; }
  memset( mem, 0, fp ); memset( out, 0, out_sz );
  signal( SIGALRM, on_alarm );
  alarm( 5 );
  fd_verify_svc_seg_t * seg = fd_verify_svc_new( mem, T, D, cap, fcap );
  svc = fd_verify_svc_boot( seg, 0, 65536UL, 2UL );
  if( !svc ) { printf( "boot failed\n" ); return 1; }
  if( fd_verify_svc_map( svc, mem, fp ) || fd_verify_svc_map( svc, out, out_sz ) ) { printf( "map failed\n" ); return 1; }
  if( fd_verify_svc_set_tile( svc, 0UL, out, out_sz, out ) ) { printf( "set_tile failed\n" ); return 1; }
  step_now = "run";
  if( fd_verify_svc_run( svc ) ) { printf( "run failed\n" ); return 1; }
  say( "run", "ok" );

  step_now = "idle";
  long end = now_ns() + 500000000L;
  while( now_ns()<end ) fd_verify_svc_poll( svc );
  say( "idle", "ok" );

  step_now = "empty";
  /* request 0: no frags */
  fd_verify_svc_req_t * r0 = fd_verify_svc_req( seg, 0UL, 0UL );
  if( fd_verify_svc_post_frags( seg, 0UL, 0UL, 0UL, 1UL, 0L ) ) { printf( "post 0 refused\n" ); return 1; }
  if( wait_state( "empty", &r0->state, FD_VERIFY_SVC_RESULTS, 2000L ) ) return 1;
  say( "empty", "ok" );
  fd_verify_svc_st( &r0->state, FD_VERIFY_SVC_FREE );

  step_now = "frags";
  /* request 1: nfr frags of zero bytes (80-byte fd_txn_m_t header, payload_sz 0) */
  uchar *  fa  = fd_verify_svc_frag( seg, 0UL, 1UL );
  ushort * fsz = fd_verify_svc_frag_sz( seg, 0UL, 1UL );
  uchar *  fk  = fd_verify_svc_frag_kind( seg, 0UL, 1UL );
  for( ulong j=0UL; j<nfr; j++ ) { memset( fa + j*FD_VERIFY_SVC_FRAG_STRIDE, 0, 128UL ); fsz[ j ] = 96; fk[ j ] = 0; }
  fd_verify_svc_req_t * r1 = fd_verify_svc_req( seg, 0UL, 1UL );
  if( fd_verify_svc_post_frags( seg, 0UL, 1UL, nfr, 1UL, 0L ) ) { printf( "post 1 refused\n" ); return 1; }
  long t0 = now_ns();
  while( !fd_verify_svc_state_ingested( fd_verify_svc_ld( &r1->state ) ) ) {
    fd_verify_svc_poll( svc );
    if( now_ns()-t0>2000000000L ) { say( "frags", "TIMEOUT before INGESTED" ); return 1; }
  }
  long t1 = now_ns();
  if( wait_state( "frags", &r1->state, FD_VERIFY_SVC_RESULTS, 5000L ) ) return 1;
  long t2 = now_ns();
  fd_verify_svc_res_t const * res = fd_verify_svc_res( seg, 0UL, 1UL );
  ulong parse_fail = 0UL;
  for( ulong j=0UL; j<nfr; j++ ) parse_fail += !res[ j ].txn_t_sz && !(res[ j ].flags & FD_VERIFY_SVC_RES_BAD);
  char m[ 160 ];
  snprintf( m, sizeof(m), "ok: %lu frags, %lu parse failures, ingested in %.1f us, results %.1f us later, batch %lu",
            nfr, parse_fail, 1e-3*(double)(t1-t0), 1e-3*(double)(t2-t1), r1->batch_frags );
  say( "frags", m );
  if( parse_fail!=nfr ) { printf( "frags: expected every frag to fail its parse\n" ); return 1; }

  step_now = "flush";
  /* flush 0: two host-written entries of slot 1 (nothing for the GPU to copy) */
  fd_verify_svc_out_t * o = fd_verify_svc_out( seg, 0UL, 1UL );
  for( ulong j=0UL; j<2UL; j++ ) { o[ j ].idx = (uint)j; o[ j ].chunk = 0U; o[ j ].sz = 64; o[ j ].flags = FD_VERIFY_SVC_OUT_HOSTWRITTEN; }
  fd_verify_svc_tile_t * tb = fd_verify_svc_tile( seg, 0UL );
  if( fd_verify_svc_post_flush( seg, 0UL, 1UL, 0UL, 2UL ) ) { printf( "flush refused\n" ); return 1; }
  if( wait_state( "flush", &tb->flush_done, 1UL, 2000L ) ) return 1;
  say( "flush", "ok" );
  fd_verify_svc_st( &r1->state, FD_VERIFY_SVC_FREE );

  /* latency: 32 more frag requests one at a time, post -> INGESTED */
  step_now = "latency";
  double lat[ 32 ]; ulong nl = 0UL;
  for( ulong k=2UL; k<34UL; k++ ) {
    ulong slot = k & ( D-1UL );
    fd_verify_svc_req_t * rq = fd_verify_svc_req( seg, 0UL, slot );
    uchar * fb = fd_verify_svc_frag( seg, 0UL, slot );
    ushort * fs = fd_verify_svc_frag_sz( seg, 0UL, slot );
    uchar * fkk = fd_verify_svc_frag_kind( seg, 0UL, slot );
    for( ulong j=0UL; j<nfr; j++ ) { memset( fb + j*FD_VERIFY_SVC_FRAG_STRIDE, 0, 128UL ); fs[ j ] = 96; fkk[ j ] = 0; }
    if( fd_verify_svc_post_frags( seg, 0UL, k, nfr, 1UL, 0L ) ) { printf( "post %lu refused\n", k ); return 1; }
    long a = now_ns();
    while( !fd_verify_svc_state_ingested( fd_verify_svc_ld( &rq->state ) ) ) {
      fd_verify_svc_poll( svc );
      if( now_ns()-a>2000000000L ) { say( "latency", "TIMEOUT before INGESTED" ); return 1; }
    }
    lat[ nl++ ] = 1e-3*(double)( now_ns()-a );
    if( wait_state( "latency", &rq->state, FD_VERIFY_SVC_RESULTS, 5000L ) ) return 1;
    fd_verify_svc_st( &rq->state, FD_VERIFY_SVC_FREE );
  }
  for( ulong i=1UL; i<nl; i++ ) for( ulong j=i; j>0UL && lat[ j-1UL ]>lat[ j ]; j-- ) { double x = lat[ j ]; lat[ j ] = lat[ j-1UL ]; lat[ j-1UL ] = x; }
  snprintf( m, sizeof(m), "post -> INGESTED over %lu requests of %lu frags: min %.1f, median %.1f, max %.1f us", nl, nfr,
            lat[ 0 ], lat[ nl/2UL ], lat[ nl-1UL ] );
  say( "latency", m );

  step_now = "delete";
  fd_verify_svc_delete( svc );
  svc = NULL;
  printf( "delete: ok\nPROBE OK\n" );
  return 0;
}
