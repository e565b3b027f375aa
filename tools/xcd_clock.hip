// tools/xcd_clock.hip -- diagnostic: the shader clock a lone single-workgroup
// launch runs at, per launch.  Each launch runs one wave whose lane 0 does a
// dependent chain of v_mad_u64_u32 (~0.3 ms), timed by s_memtime (shader
// cycles) and s_memrealtime (100 MHz constant clock); it also records
// HW_REG_XCC_ID and HW_REG_HW_ID.  Launches are issued one at a time with a
// host sync in between, as the drop-in's single calls are.
// Output: one line per launch: launch xcc hw_id cycles ticks clock_GHz us
// Mode "chase" (argv[3]): the lane instead follows a dependent pointer chain
// through a 64 MB buffer in HBM (one cache line per step), so the time per
// step is the load latency from wherever the launch was placed.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k_probe( uint64_t * out, uint32_t iters, uint64_t seed ) {
  if( threadIdx.x != 0 ) return;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t x = seed | 1;
  for( uint32_t i = 0; i < iters; i++ ) x = (uint64_t)(uint32_t)x * (uint32_t)(x >> 32) + x;
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0; out[1] = r1 - r0; out[2] = x;
  out[3] = (uint32_t)__builtin_amdgcn_s_getreg( (3 << 11) | (0 << 6) | 20 );      // XCC_ID
  out[4] = (uint32_t)__builtin_amdgcn_s_getreg( (31 << 11) | (0 << 6) | 4 );      // HW_ID
}

__global__ void k_chase( uint64_t * out, uint32_t const * __restrict__ buf, uint32_t steps ) {
  if( threadIdx.x != 0 ) return;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t j = 0;
  for( uint32_t i = 0; i < steps; i++ ) j = __builtin_nontemporal_load( buf + j );
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0; out[1] = r1 - r0; out[2] = j;
  out[3] = (uint32_t)__builtin_amdgcn_s_getreg( (3 << 11) | (0 << 6) | 20 );
  out[4] = (uint32_t)__builtin_amdgcn_s_getreg( (31 << 11) | (0 << 6) | 4 );
}

int main( int argc, char ** argv ) {
  int n = argc > 1 ? atoi( argv[1] ) : 64;
  uint32_t iters = argc > 2 ? (uint32_t)atoi( argv[2] ) : 200000u;
  int chase = argc > 3 && argv[3][0] == 'c';
  uint64_t * d, h[5];
  if( hipMalloc( &d, sizeof(h) ) != hipSuccess ) return 1;
  uint32_t * buf = 0;
  if( chase ) {                                   /* a random cycle over 64 MB, one 128-B line per node */
    const uint32_t lines = (64u << 20) / 128u, stride = 32u;
    uint32_t * h_buf = (uint32_t *)calloc( (size_t)lines * stride, 4 );
    uint32_t * perm = (uint32_t *)malloc( (size_t)lines * 4 );
    for( uint32_t i = 0; i < lines; i++ ) perm[i] = i;
    uint64_t x = 88172645463325252ull;
    for( uint32_t i = lines - 1; i > 0; i-- ) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; uint32_t r = (uint32_t)(x % (i + 1)); uint32_t t = perm[i]; perm[i] = perm[r]; perm[r] = t; }
    for( uint32_t i = 0; i < lines; i++ ) h_buf[(size_t)perm[i] * stride] = perm[(i + 1) % lines] * stride;
    if( hipMalloc( &buf, (size_t)lines * stride * 4 ) != hipSuccess ) return 1;
    if( hipMemcpy( buf, h_buf, (size_t)lines * stride * 4, hipMemcpyHostToDevice ) != hipSuccess ) return 1;
    free( h_buf ); free( perm );
  }
  for( int k = 0; k < n; k++ ) {
    if( chase ) hipLaunchKernelGGL( k_chase, dim3( 1 ), dim3( 64 ), 0, 0, d, buf, iters );
    else        hipLaunchKernelGGL( k_probe, dim3( 1 ), dim3( 64 ), 0, 0, d, iters, (uint64_t)k );
    if( hipMemcpy( h, d, sizeof(h), hipMemcpyDeviceToHost ) != hipSuccess ) return 1;
    double us = (double)h[1] / 100.0;                                          // 100 MHz realtime counter
    printf( "%d %llu 0x%08llx %llu %llu %.3f %.1f\n", k, (unsigned long long)h[3], (unsigned long long)h[4],
            (unsigned long long)h[0], (unsigned long long)h[1], (double)h[0] / (us * 1e3), us );
  }
  (void)hipFree( d );
  if( buf ) (void)hipFree( buf );
  return 0;
}
