/* svc_client.h -- a client process of the service-mode run's GPU tile
   (integration/svc_run.h, svc_tile_run.c produce / host): the harnesses of
   the shred tile's resolver (integration/fec_run.c) and of the replay
   scheduler (integration/sched_run.c) built with FD_HAS_HIP_SVC join the
   run's segment as one of its client tiles and verify through
   fd_verify_svc_client_t (include/fd_verify_svc.h): no HIP in the process.

     SVC_CLIENT_SHM=<shm>   the run's file
     SVC_CLIENT_IDX=<c>     which client (default 0): segment tile
                            tile_cnt + c

   svc_client_attach maps the file, waits for the GPU tile (svc_ready) and
   the run's start, and returns the segment and tile; svc_client_done
   counts the client done (the run's host or producer then shuts the
   service down). */
#ifndef HEADER_svc_client_h
#define HEADER_svc_client_h

#include "fd_verify_svc.h"
#include "svc_run.h"
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

static svc_run_hdr_t * svc_client_hdr;

static fd_verify_svc_seg_t *
svc_client_attach( ulong * t ) {
  char const * path = getenv( "SVC_CLIENT_SHM" );
  if( !path ) { fprintf( stderr, "svc_client: SVC_CLIENT_SHM not set\n" ); exit( 2 ); }
  char const * ie = getenv( "SVC_CLIENT_IDX" );
  ulong c = ie ? strtoul( ie, NULL, 0 ) : 0UL;
  int fd = -1;
  svc_run_hdr_t h;
  long t0 = fd_log_wallclock();
  for( ;; ) {                                                    /* the host may still be creating the file */
    fd = open( path, O_RDWR );
    if( fd>=0 && pread( fd, &h, sizeof(h), 0 )==(long)sizeof(h) && h.magic==SVC_RUN_MAGIC ) break;
    if( fd>=0 ) close( fd );
    if( fd_log_wallclock()-t0 > 180L*1000000000L ) { fprintf( stderr, "svc_client: %s not a run file after 180 s\n", path ); exit( 2 ); }
    usleep( 10000 );
  }
  uchar * base = mmap( NULL, h.map_sz, PROT_READ|PROT_WRITE, MAP_SHARED, fd, 0 );
  close( fd );
  if( base==MAP_FAILED ) { fprintf( stderr, "svc_client: mmap failed\n" ); exit( 2 ); }
  svc_run_hdr_t * hdr = (svc_run_hdr_t *)base;
  if( c>=hdr->client_cnt ) { fprintf( stderr, "svc_client: client %lu of %lu\n", c, hdr->client_cnt ); exit( 2 ); }
  fd_verify_svc_seg_t * seg = fd_verify_svc_join( base + hdr->svc_off );
  if( !seg ) { fprintf( stderr, "svc_client: no segment\n" ); exit( 2 ); }
  __atomic_fetch_add( &hdr->clients_ready, 1UL, __ATOMIC_ACQ_REL );
  while( !hdr->svc_ready || !hdr->start ) {
    if( fd_log_wallclock()-t0 > 300L*1000000000L ) { fprintf( stderr, "svc_client: the run did not start in 300 s\n" ); exit( 2 ); }
    FD_SPIN_PAUSE();
  }
  svc_client_hdr = hdr;
  *t = hdr->tile_cnt + c;
  return seg;
}

static void
svc_client_done( void ) {
  if( svc_client_hdr ) __atomic_fetch_add( &svc_client_hdr->clients_done, 1UL, __ATOMIC_ACQ_REL );
}

/* threads and /dev/kfd|/dev/dri fds of this process (the client keeps the
   reference's process model: 1 and 0) */
static void
svc_client_census( ulong * threads, ulong * dev_fds ) {
  char p[ 64 ], l[ 256 ];
  *threads = 0UL; *dev_fds = 0UL;
  FILE * f = fopen( "/proc/self/status", "r" );
  while( f && fgets( l, sizeof(l), f ) ) if( !strncmp( l, "Threads:", 8 ) ) *threads = strtoul( l+8, NULL, 10 );
  if( f ) fclose( f );
  for( int k=0; k<1024; k++ ) {
    snprintf( p, sizeof(p), "/proc/self/fd/%d", k );
    ssize_t n = readlink( p, l, sizeof(l)-1UL );
    if( n<=0 ) continue;
    l[ n ] = '\0';
    if( !strncmp( l, "/dev/kfd", 8 ) || !strncmp( l, "/dev/dri", 8 ) ) (*dev_fds)++;
  }
}

#endif /* HEADER_svc_client_h */
