// pcie_probe.hip -- host-link rates the verify tile's range mode depends on.
//
// Range mode moves every frag over PCIe twice from kernels (k_txnm_batch reads
// the in-link dcache in pinned host memory, k_out_flush writes the out dcache),
// DESIGN.md section 9.  This measures, on one GPU, 1 GiB each way:
//   kread    a kernel reading pinned host memory, 16 B per lane, coalesced
//   kwrite   a kernel writing pinned host memory, 16 B per lane, coalesced
//   kboth    both kernels at once on two streams (the tile's two legs)
//   sdma_h2d / sdma_d2h   hipMemcpyAsync (the copy engines)
// Prints one JSON line (GB/s, 1e9 bytes).  Diagnostic only: not on any
// product path.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/pcie_probe tools/pcie_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK( x ) do { hipError_t e_ = (x); if( e_ != hipSuccess ) { \
  fprintf( stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString( e_ ) ); exit( 1 ); } } while( 0 )

__global__ void kread( uint4 const * __restrict__ h, uint4 * __restrict__ d, size_t n ) {
  for( size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x ) d[i] = h[i];
}
__global__ void kwrite( uint4 const * __restrict__ d, uint4 * __restrict__ h, size_t n ) {
  for( size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x ) h[i] = d[i];
}

int main() {
  size_t const sz = (size_t)1 << 30, n = sz / 16;
  uint4 *h_in, *h_out, *d_a, *d_b;
  CK( hipHostMalloc( (void **)&h_in, sz, 0 ) ); CK( hipHostMalloc( (void **)&h_out, sz, 0 ) );
  CK( hipMalloc( (void **)&d_a, sz ) ); CK( hipMalloc( (void **)&d_b, sz ) );
  for( size_t i = 0; i < sz / 8; i++ ) ((unsigned long *)h_in)[i] = i * 0x9e3779b97f4a7c15ul;
  CK( hipMemset( d_a, 1, sz ) ); CK( hipMemset( d_b, 2, sz ) );
  hipStream_t s0, s1;
  CK( hipStreamCreateWithFlags( &s0, hipStreamNonBlocking ) ); CK( hipStreamCreateWithFlags( &s1, hipStreamNonBlocking ) );
  hipEvent_t e0, e1, f0, f1;
  CK( hipEventCreate( &e0 ) ); CK( hipEventCreate( &e1 ) ); CK( hipEventCreate( &f0 ) ); CK( hipEventCreate( &f1 ) );
  dim3 grid( 256 * 32 ), blk( 256 );
  auto gbs = []( size_t b, float ms ) { return (double)b / ( (double)ms * 1e6 ); };
  float ms;
  double r[5] = { 0 };
  for( int rep = 0; rep < 3; rep++ ) {       /* best of three */
    CK( hipEventRecord( e0, s0 ) ); hipLaunchKernelGGL( kread, grid, blk, 0, s0, h_in, d_a, n ); CK( hipEventRecord( e1, s0 ) );
    CK( hipEventSynchronize( e1 ) ); CK( hipEventElapsedTime( &ms, e0, e1 ) ); if( gbs( sz, ms ) > r[0] ) r[0] = gbs( sz, ms );
    CK( hipEventRecord( e0, s0 ) ); hipLaunchKernelGGL( kwrite, grid, blk, 0, s0, d_b, h_out, n ); CK( hipEventRecord( e1, s0 ) );
    CK( hipEventSynchronize( e1 ) ); CK( hipEventElapsedTime( &ms, e0, e1 ) ); if( gbs( sz, ms ) > r[1] ) r[1] = gbs( sz, ms );
    CK( hipDeviceSynchronize() );
    CK( hipEventRecord( e0, s0 ) ); CK( hipStreamWaitEvent( s1, e0, 0 ) );
    hipLaunchKernelGGL( kread, grid, blk, 0, s0, h_in, d_a, n );
    hipLaunchKernelGGL( kwrite, grid, blk, 0, s1, d_b, h_out, n );
    CK( hipEventRecord( f0, s1 ) ); CK( hipStreamWaitEvent( s0, f0, 0 ) ); CK( hipEventRecord( e1, s0 ) );
    CK( hipEventSynchronize( e1 ) ); CK( hipEventElapsedTime( &ms, e0, e1 ) ); if( gbs( 2 * sz, ms ) > r[2] ) r[2] = gbs( 2 * sz, ms );
    CK( hipEventRecord( e0, s0 ) ); CK( hipMemcpyAsync( d_a, h_in, sz, hipMemcpyHostToDevice, s0 ) ); CK( hipEventRecord( e1, s0 ) );
    CK( hipEventSynchronize( e1 ) ); CK( hipEventElapsedTime( &ms, e0, e1 ) ); if( gbs( sz, ms ) > r[3] ) r[3] = gbs( sz, ms );
    CK( hipEventRecord( e0, s0 ) ); CK( hipMemcpyAsync( h_out, d_b, sz, hipMemcpyDeviceToHost, s0 ) ); CK( hipEventRecord( e1, s0 ) );
    CK( hipEventSynchronize( e1 ) ); CK( hipEventElapsedTime( &ms, e0, e1 ) ); if( gbs( sz, ms ) > r[4] ) r[4] = gbs( sz, ms );
  }
  printf( "{\"bytes_each_way\": %zu, \"kread_GBps\": %.1f, \"kwrite_GBps\": %.1f, \"kboth_GBps_total\": %.1f, "
          "\"sdma_h2d_GBps\": %.1f, \"sdma_d2h_GBps\": %.1f}\n", sz, r[0], r[1], r[2], r[3], r[4] );
  CK( hipHostFree( h_in ) ); CK( hipHostFree( h_out ) ); CK( hipFree( d_a ) ); CK( hipFree( d_b ) );
  return 0;
}
