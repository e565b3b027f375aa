// Host-side cost of the HIP calls the verify service makes per ingest and
// per flush (hipLaunchKernelGGL, hipEventRecord with and without timing,
// hipEventQuery), alone and beside a long kernel on another stream, and
// from two threads at once.  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/hip_host_costs tools/hip_host_costs.hip -lpthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <algorithm>

#define CK( x ) do { hipError_t e_ = (x); if( e_ != hipSuccess ) { fprintf( stderr, "%s: %s\n", #x, hipGetErrorString( e_ ) ); exit( 1 ); } } while( 0 )

__global__ void k_small( unsigned * p, unsigned n ) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if( i < n ) p[ i ] += 1u;
}

/* a kernel that keeps every CU busy for about `iters` loop trips */
__global__ void k_long( unsigned * p, unsigned iters ) {
  unsigned x = threadIdx.x;
  for( unsigned k = 0; k < iters; k++ ) x = x * 1664525u + 1013904223u;
  if( x == 0x12345678u ) p[ 0 ] = x;
}

static double now_us( void ) {
  return std::chrono::duration<double, std::micro>( std::chrono::steady_clock::now().time_since_epoch() ).count();
}

struct res { double p50, p99, mean; };
static res stats( std::vector<double> & v ) {
  std::sort( v.begin(), v.end() );
  double s = 0; for( double x : v ) s += x;
  return { v[ v.size() / 2 ], v[ (v.size() * 99) / 100 ], s / (double)v.size() };
}

/* mode: 0 launch only, 1 launch + timing event, 2 launch + no-timing event,
   3 launch + 2 timing events (the service's ingest), 4 event query of a done event */
static res run( hipStream_t st, unsigned * d, int mode, int n ) {
  hipEvent_t et0, et1, en;
  CK( hipEventCreate( &et0 ) ); CK( hipEventCreate( &et1 ) );
  CK( hipEventCreateWithFlags( &en, hipEventDisableTiming ) );
  std::vector<double> v;
  for( int i = 0; i < n + 50; i++ ) {
    double t0 = now_us();
    if( mode == 4 ) {
      (void)hipEventQuery( en );
    } else {
      if( mode == 3 ) CK( hipEventRecord( et0, st ) );
      hipLaunchKernelGGL( k_small, dim3( 4 ), dim3( 256 ), 0, st, d, 1024u );
      if( mode == 1 || mode == 3 ) CK( hipEventRecord( et1, st ) );
      if( mode == 2 ) CK( hipEventRecord( en, st ) );
    }
    double t1 = now_us();
    if( i >= 50 ) v.push_back( t1 - t0 );
    if( mode != 4 && (i & 15) == 15 ) CK( hipStreamSynchronize( st ) );
    if( mode == 4 && i == 0 ) { CK( hipEventRecord( en, st ) ); CK( hipStreamSynchronize( st ) ); }
  }
  CK( hipStreamSynchronize( st ) );
  CK( hipEventDestroy( et0 ) ); CK( hipEventDestroy( et1 ) ); CK( hipEventDestroy( en ) );
  return stats( v );
}

int main( int argc, char ** argv ) {
  int n = argc > 1 ? atoi( argv[ 1 ] ) : 2000;
  CK( hipSetDevice( 0 ) );
  unsigned * d; CK( hipMalloc( &d, 1 << 20 ) ); CK( hipMemset( d, 0, 1 << 20 ) );
  hipStream_t a, b, c;
  CK( hipStreamCreateWithFlags( &a, hipStreamNonBlocking ) );
  CK( hipStreamCreateWithFlags( &b, hipStreamNonBlocking ) );
  CK( hipStreamCreateWithFlags( &c, hipStreamNonBlocking ) );
  hipLaunchKernelGGL( k_small, dim3( 4 ), dim3( 256 ), 0, a, d, 1024u );
  hipLaunchKernelGGL( k_long, dim3( 1 ), dim3( 64 ), 0, b, d, 10u );
  CK( hipDeviceSynchronize() );
  char const * name[] = { "launch", "launch_ev_timing", "launch_ev_notiming", "launch_2ev_timing", "query_done" };
  printf( "{" );
  for( int m = 0; m < 5; m++ ) {
    res r = run( a, d, m, n );
    printf( "\"%s\": {\"p50_us\": %.2f, \"p99_us\": %.2f, \"mean_us\": %.2f}, ", name[ m ], r.p50, r.p99, r.mean );
  }
  /* beside a chip-filling kernel on another stream */
  for( int m = 0; m < 4; m++ ) {
    hipLaunchKernelGGL( k_long, dim3( 4096 ), dim3( 256 ), 0, b, d, 2000000u );
    res r = run( a, d, m, n / 4 );
    CK( hipDeviceSynchronize() );
    printf( "\"busy_%s\": {\"p50_us\": %.2f, \"p99_us\": %.2f, \"mean_us\": %.2f}, ", name[ m ], r.p50, r.p99, r.mean );
  }
  /* two threads, each launching + one no-timing event on its own stream */
  {
    res r0, r1;
    std::thread t0( [ & ] { r0 = run( a, d, 2, n ); } );
    std::thread t1( [ & ] { r1 = run( c, d + 65536, 2, n ); } );
    t0.join(); t1.join();
    printf( "\"two_threads\": [{\"p50_us\": %.2f, \"p99_us\": %.2f, \"mean_us\": %.2f}, {\"p50_us\": %.2f, \"p99_us\": %.2f, "
            "\"mean_us\": %.2f}], ", r0.p50, r0.p99, r0.mean, r1.p50, r1.p99, r1.mean );
  }
  /* end-to-end latency of one small launch observed through a host-mapped flag */
  printf( "\"n\": %d}\n", n );
  return 0;
}
