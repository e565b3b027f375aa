// tools/xcd_clock.hip -- diagnostic: the shader clock a lone single-workgroup
// launch runs at, per launch.  Each launch runs one wave whose lane 0 does a
// dependent chain of v_mad_u64_u32 (~0.3 ms), timed by s_memtime (shader
// cycles) and s_memrealtime (100 MHz constant clock); it also records
// HW_REG_XCC_ID and HW_REG_HW_ID.  Launches are issued one at a time with a
// host sync in between, as the drop-in's single calls are.
// Output: one line per launch: launch xcc hw_id cycles ticks clock_GHz us
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

int main( int argc, char ** argv ) {
  int n = argc > 1 ? atoi( argv[1] ) : 64;
  uint32_t iters = argc > 2 ? (uint32_t)atoi( argv[2] ) : 200000u;
  uint64_t * d, h[5];
  if( hipMalloc( &d, sizeof(h) ) != hipSuccess ) return 1;
  for( int k = 0; k < n; k++ ) {
    hipLaunchKernelGGL( k_probe, dim3( 1 ), dim3( 64 ), 0, 0, d, iters, (uint64_t)k );
    if( hipMemcpy( h, d, sizeof(h), hipMemcpyDeviceToHost ) != hipSuccess ) return 1;
    double us = (double)h[1] / 100.0;                                          // 100 MHz realtime counter
    printf( "%d %llu 0x%08llx %llu %llu %.3f %.1f\n", k, (unsigned long long)h[3], (unsigned long long)h[4],
            (unsigned long long)h[0], (unsigned long long)h[1], (double)h[0] / (us * 1e3), us );
  }
  hipFree( d );
  return 0;
}
