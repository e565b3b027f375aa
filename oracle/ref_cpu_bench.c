/* ref_cpu_bench.c -- TEST/BASELINE INFRASTRUCTURE ONLY.

   Repo-owned driver linked against the reference's own verify objects
   (oracle/Makefile builds them from /root/reference sources into _ref/).
   It times fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:135) or
   fd_ed25519_verify_batch_single_msg (:232) over a record file written by
   bench.py / tests, on T host threads (one contiguous slice per thread,
   each pinned to its own core), and writes the per-record codes so callers
   can compare bitmaps.

   usage: ref_cpu_bench <in.bin> <threads> <codes_out.bin|-> [first_cpu] [repeat]
          (each thread verifies its slice `repeat` times; codes from the last pass)
   input  : "FDV1" u64 n, u64 pool_sz, u64 nbatch,
            sigs[64n] pubs[32n] msg_off[u32 n] msg_sz[u32 n] pool[pool_sz]
            batch_first[u32 nbatch] batch_cnt[u8 nbatch]   (nbatch==0: single verifies)
   output : JSON line {"verifies":..,"seconds":..,"threads":..,"rate":..}
            codes: one int8 per record (single) or per batch (batch mode). */

#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned char uchar;
typedef unsigned long ulong;

typedef struct { _Alignas(128) uchar mem[256]; } sha_t;   /* fd_sha512_t footprint 256, align 128 (fd_sha512.h:56-77) */

extern int fd_ed25519_verify( uchar const msg[], ulong msg_sz, uchar const sig[64],
                              uchar const public_key[32], void * sha );
extern int fd_ed25519_verify_batch_single_msg( uchar const msg[], ulong const msg_sz,
                                               uchar const signatures[64], uchar const pubkeys[32],
                                               void * shas[1], uchar const batch_sz );
extern void * fd_sha512_init( void * sha );

static uint64_t n, pool_sz, nbatch;
static uchar *sigs, *pubs, *pool, *bcnt;
static uint32_t *moff, *msz, *bfirst;
static int8_t * codes;
static int repeat = 1;

typedef struct { uint64_t lo, hi; int cpu; } job_t;

static void * worker( void * arg ) {
  job_t * j = (job_t *)arg;
  if( j->cpu >= 0 ) {
    cpu_set_t cs; CPU_ZERO( &cs ); CPU_SET( j->cpu, &cs );
    sched_setaffinity( 0, sizeof(cs), &cs );
  }
  static __thread sha_t shas[16];
  void * shp[16];
  for( int i=0;i<16;i++ ) { fd_sha512_init( &shas[i] ); shp[i] = &shas[i]; }
  for( int rep=0; rep<repeat; rep++ ) {
  if( !nbatch ) {
    for( uint64_t i=j->lo; i<j->hi; i++ )
      codes[i] = (int8_t)fd_ed25519_verify( pool + moff[i], msz[i], sigs + 64*i, pubs + 32*i, shp[0] );
  } else {
    for( uint64_t b=j->lo; b<j->hi; b++ ) {
      uint32_t f = bfirst[b];
      codes[b] = (int8_t)fd_ed25519_verify_batch_single_msg( pool + moff[f], msz[f], sigs + 64*(uint64_t)f,
                                                            pubs + 32*(uint64_t)f, shp, bcnt[b] );
    }
  }
  }
  return NULL;
}

static double now( void ) { struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t ); return (double)t.tv_sec + 1e-9*(double)t.tv_nsec; }

int main( int argc, char ** argv ) {
  if( argc < 4 ) { fprintf( stderr, "usage: %s in.bin threads codes_out|- [first_cpu]\n", argv[0] ); return 2; }
  FILE * f = fopen( argv[1], "rb" ); if( !f ) { perror( "open" ); return 1; }
  char magic[4];
  if( fread( magic, 1, 4, f )!=4 || memcmp( magic, "FDV1", 4 ) ) { fprintf( stderr, "bad magic\n" ); return 1; }
  if( fread( &n, 8, 1, f )!=1 || fread( &pool_sz, 8, 1, f )!=1 || fread( &nbatch, 8, 1, f )!=1 ) return 1;
  sigs = malloc( 64*n ); pubs = malloc( 32*n ); moff = malloc( 4*n ); msz = malloc( 4*n ); pool = malloc( pool_sz+1 );
  if( fread( sigs, 64, n, f )!=n || fread( pubs, 32, n, f )!=n || fread( moff, 4, n, f )!=n ||
      fread( msz, 4, n, f )!=n || fread( pool, 1, pool_sz, f )!=pool_sz ) { fprintf( stderr, "short read\n" ); return 1; }
  if( nbatch ) {
    bfirst = malloc( 4*nbatch ); bcnt = malloc( nbatch );
    if( fread( bfirst, 4, nbatch, f )!=nbatch || fread( bcnt, 1, nbatch, f )!=nbatch ) { fprintf( stderr, "short read\n" ); return 1; }
  }
  fclose( f );
  int T = atoi( argv[2] ); if( T<1 ) T = 1;
  int first_cpu = argc>4 ? atoi( argv[4] ) : -1;
  repeat = argc>5 ? atoi( argv[5] ) : 1; if( repeat<1 ) repeat = 1;
  uint64_t units = nbatch ? nbatch : n;
  codes = calloc( units, 1 );
  pthread_t th[1024]; job_t jb[1024]; if( T>1024 ) T = 1024;
  double t0 = now();
  for( int t=0;t<T;t++ ) {
    jb[t].lo = units*(uint64_t)t/(uint64_t)T; jb[t].hi = units*(uint64_t)(t+1)/(uint64_t)T;
    jb[t].cpu = first_cpu>=0 ? first_cpu + t : -1;
    pthread_create( &th[t], NULL, worker, &jb[t] );
  }
  for( int t=0;t<T;t++ ) pthread_join( th[t], NULL );
  double dt = now() - t0;
  uint64_t sigcnt = n*(uint64_t)repeat;   /* signatures verified (batch mode: all sigs of all batches) */
  if( strcmp( argv[3], "-" ) ) { FILE * o = fopen( argv[3], "wb" ); fwrite( codes, 1, units, o ); fclose( o ); }
  printf( "{\"verifies\": %lu, \"calls\": %lu, \"seconds\": %.6f, \"threads\": %d, \"repeat\": %d, \"rate\": %.1f}\n",
          (ulong)sigcnt, (ulong)units*(ulong)repeat, dt, T, repeat, (double)sigcnt/dt );
  return 0;
}
