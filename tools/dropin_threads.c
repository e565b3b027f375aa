/* dropin_threads.c -- concurrent callers of the drop-in API, in C.

   T host threads each call fd_ed25519_verify_batch_single_msg (K signatures
   over one message: the shape of fd_executor_txn_verify's per-transaction
   call, src/flamenco/runtime/fd_executor.c:1608-1617) in a loop for S
   seconds, the way replay's exec tiles call the reference
   (fd_ed25519.h:89-94: re-entrant, no shared state).  Every call's result is
   checked against the expected code.  Prints one JSON line: calls, aggregate
   signatures/s, per-call latency percentiles, launches (the drop-in's
   combining counters).  No Python in the measured loop (ctypes callers hold
   the GIL between calls).

   Input file (written by tests/test_gpu_dropin_concurrent.py):
     u32 T, u32 K, u32 msg_sz, u32 expect_code (as int32)
     then per thread t: msg[msg_sz] sigs[K*64] pubs[K*32]

   usage: dropin_threads <input> <seconds> [threads to use (<= T)] */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned char uchar;
typedef unsigned long ulong;

int fd_ed25519_verify_batch_single_msg( uchar const msg[], ulong const msg_sz, uchar const signatures[ 64 ],
                                        uchar const pubkeys[ 32 ], void * shas[ 1 ], uchar const batch_sz );
int fd_ed25519_hip_dropin_init( int device );
void fd_ed25519_hip_dropin_stats( ulong out[ 2 ] );

#define LAT_CAP (1u << 20)

typedef struct {
  uchar const * msg; uchar const * sigs; uchar const * pubs;
  uint32_t k, msg_sz; int32_t expect;
  double deadline;
  float * lat; ulong ncall, nbad;
} worker_t;

static double now( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void * run( void * arg ) {
  worker_t * w = (worker_t *)arg;
  while( now() < w->deadline ) {
    double t0 = now();
    int r = fd_ed25519_verify_batch_single_msg( w->msg, w->msg_sz, w->sigs, w->pubs, NULL, (uchar)w->k );
    double t1 = now();
    if( w->ncall < LAT_CAP ) w->lat[ w->ncall ] = (float)((t1 - t0) * 1e6);
    w->ncall++;
    if( r != w->expect ) w->nbad++;
  }
  return NULL;
}

static int cmpf( void const * a, void const * b ) {
  float x = *(float const *)a, y = *(float const *)b;
  return (x > y) - (x < y);
}

int main( int argc, char ** argv ) {
  if( argc < 3 ) { fprintf( stderr, "usage: %s input seconds [threads]\n", argv[0] ); return 2; }
  FILE * f = fopen( argv[1], "rb" );
  if( !f ) { perror( "open" ); return 2; }
  uint32_t hdr[4];
  if( fread( hdr, 4, 4, f ) != 4 ) { fprintf( stderr, "short header\n" ); return 2; }
  uint32_t T = hdr[0], K = hdr[1], msz = hdr[2];
  int32_t expect = (int32_t)hdr[3];
  if( !T || !K || K > 16 ) { fprintf( stderr, "bad header\n" ); return 2; }
  ulong per = (ulong)msz + 96ul * K;
  uchar * data = (uchar *)malloc( per * T );
  if( fread( data, 1, per * T, f ) != per * T ) { fprintf( stderr, "short data\n" ); return 2; }
  fclose( f );
  double secs = atof( argv[2] );
  uint32_t use = argc > 3 ? (uint32_t)atoi( argv[3] ) : T;
  if( !use || use > T ) use = T;

  if( fd_ed25519_hip_dropin_init( 0 ) ) { fprintf( stderr, "dropin_init failed\n" ); return 1; }
  worker_t * w = (worker_t *)calloc( use, sizeof(worker_t) );
  for( uint32_t t=0; t<use; t++ ) {
    uchar const * p = data + per * t;
    w[t].msg = p; w[t].sigs = p + msz; w[t].pubs = p + msz + 64ul * K;
    w[t].k = K; w[t].msg_sz = msz; w[t].expect = expect;
    w[t].lat = (float *)malloc( sizeof(float) * LAT_CAP );
  }
  /* warm: one call per thread's inputs, serially (first-call setup, tables) */
  for( uint32_t t=0; t<use; t++ ) {
    int r = fd_ed25519_verify_batch_single_msg( w[t].msg, msz, w[t].sigs, w[t].pubs, NULL, (uchar)K );
    if( r != expect ) { fprintf( stderr, "warm call %u: %d != %d\n", t, r, expect ); return 1; }
  }
  ulong s0[2]; fd_ed25519_hip_dropin_stats( s0 );
  pthread_t * th = (pthread_t *)calloc( use, sizeof(pthread_t) );
  double t0 = now();
  for( uint32_t t=0; t<use; t++ ) { w[t].deadline = t0 + secs; pthread_create( &th[t], NULL, run, &w[t] ); }
  for( uint32_t t=0; t<use; t++ ) pthread_join( th[t], NULL );
  double dt = now() - t0;
  ulong s1[2]; fd_ed25519_hip_dropin_stats( s1 );

  ulong calls = 0, bad = 0, nl = 0;
  for( uint32_t t=0; t<use; t++ ) { calls += w[t].ncall; bad += w[t].nbad; nl += w[t].ncall < LAT_CAP ? w[t].ncall : LAT_CAP; }
  float * all = (float *)malloc( sizeof(float) * (nl ? nl : 1) );
  ulong o = 0;
  for( uint32_t t=0; t<use; t++ ) {
    ulong m = w[t].ncall < LAT_CAP ? w[t].ncall : LAT_CAP;
    memcpy( all + o, w[t].lat, m * sizeof(float) ); o += m;
  }
  qsort( all, nl, sizeof(float), cmpf );
#define PCT( q ) (nl ? all[ (ulong)((double)(nl - 1) * (q)) ] : 0.f)
  ulong launches = s1[0] - s0[0], lcalls = s1[1] - s0[1];
  printf( "{\"threads\": %u, \"sigs_per_call\": %u, \"msg_sz\": %u, \"seconds\": %.3f, \"calls\": %lu, "
          "\"bad\": %lu, \"sigs_per_s\": %.1f, \"calls_per_s\": %.1f, \"p50_us\": %.1f, \"p90_us\": %.1f, "
          "\"p99_us\": %.1f, \"max_us\": %.1f, \"launches\": %lu, \"calls_per_launch\": %.2f}\n",
          use, K, msz, dt, calls, bad, (double)calls * K / dt, (double)calls / dt, PCT( 0.50 ), PCT( 0.90 ),
          PCT( 0.99 ), nl ? all[nl - 1] : 0.f, launches, launches ? (double)lcalls / (double)launches : 0.0 );
  return bad ? 1 : 0;
}
