/* Batched SHA-512 on gfx950: include/fd_sha512_hip.h.

   The GPU counterpart of the reference's multi-message SHA-512
   (src/ballet/sha512/fd_sha512.h:232-419, fd_sha512_batch_avx512.c: 8
   messages per AVX-512 call).  Here a launch hashes any number of messages,
   one per lane, with the wave-cooperative LDS-staged block loader that
   k_verify_prep uses for SHA-512(R||A||M) (fd_ed25519_dev.h
   sha512_prefixed_coop, empty prefix).  The hash is VALU-bound (about 5 000
   32-bit operations per 128-byte block against 128 bytes of HBM traffic), so
   the kernel is sized for occupancy: 256-thread workgroups, 9 KB of LDS per
   wave. */

#include "../../include/fd_sha512_hip.h"
#include "fd_ed25519_dev.h"

#include <hip/hip_runtime.h>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SHA_CHECK( x ) do {                                                           \
    hipError_t e_ = (x);                                                               \
    if( e_ != hipSuccess ) {                                                           \
      fprintf( stderr, "fd_sha512_hip: %s failed at %s:%d: %s\n", #x, __FILE__,      \
               __LINE__, hipGetErrorString( e_ ) );                                    \
      abort();                                                                         \
    }                                                                                  \
  } while( 0 )

#define SHA_WAVE_WORDS (64*36)      /* sha512_prefixed_coop: 64 windows of 144 B per wave */

__global__ __launch_bounds__(256)
void k_sha512_batch( ulong n, uchar const * __restrict__ pool, uint const * __restrict__ off,
                     uint const * __restrict__ sz, uchar * __restrict__ hash ) {
  __shared__ __attribute__((aligned(16))) u32 lds_msg_all[4*SHA_WAVE_WORDS];
  __shared__ u64 lds_meta_all[4*64];
  ulong wave0 = (ulong)blockIdx.x * 256ul + (threadIdx.x & ~63u);
  if( wave0 >= n ) return;                          /* wave-uniform: the hash below needs all 64 lanes */
  u32 lane = threadIdx.x & 63u;
  ulong i = wave0 + lane;
  bool live = i < n;
  u32 x[16];
  sha512_prefixed_coop<0u>( x, nullptr, nullptr, pool + (live ? off[i] : 0u), live ? sz[i] : 0u,
                            lds_msg_all + SHA_WAVE_WORDS*(threadIdx.x >> 6), lds_meta_all + 64*(threadIdx.x >> 6),
                            lane );
  if( !live ) return;
  uint4 * o = (uint4 *)(hash + 64ul*i);
  #pragma unroll
  for( int q=0; q<4; q++ ) o[q] = make_uint4( x[4*q], x[4*q+1], x[4*q+2], x[4*q+3] );
}

/* the drop-in's process-wide context (fd_ed25519_hip.hip) */
extern "C" fd_ed25519_hip_ctx_t * fd_ed25519_hip_private_default_ctx( void );

struct __attribute__((aligned(FD_SHA512_HIP_BATCH_ALIGN))) fd_sha512_hip_batch {
  fd_ed25519_hip_ctx_t * ctx;
  ulong                  cnt;
  void const *           data[ FD_SHA512_HIP_BATCH_MAX ];
  ulong                  sz  [ FD_SHA512_HIP_BATCH_MAX ];
  void *                 hash[ FD_SHA512_HIP_BATCH_MAX ];
};

/* pinned, device-mapped staging shared by every host batch (flushes are
   serialised on its lock): off[MAX] sz[MAX] hash[64*MAX] then the messages,
   each 16-byte aligned, and 16 zero bytes */
#define STG_OFF  0ul
#define STG_SZ   (4ul*FD_SHA512_HIP_BATCH_MAX)
#define STG_HASH (8ul*FD_SHA512_HIP_BATCH_MAX)
#define STG_DATA (72ul*FD_SHA512_HIP_BATCH_MAX)

static std::mutex g_stg_lock;
static uchar *    g_stg;
static ulong      g_stg_cap;

static void
batch_flush( fd_sha512_hip_batch_t * b ) {
  ulong n = b->cnt;
  b->cnt = 0ul;
  if( !n ) return;
  fd_ed25519_hip_ctx_t * ctx = b->ctx ? b->ctx : fd_ed25519_hip_private_default_ctx();
  std::lock_guard<std::mutex> lk( g_stg_lock );
  ulong j0 = 0ul;
  while( j0 < n ) {
    /* as many records as keep every offset below 2^32 */
    ulong tot = 0ul, j1 = j0;
    while( j1 < n ) {
      ulong a = (b->sz[j1] + 15ul) & ~15ul;
      if( j1 > j0 && tot + a + 16ul > (ulong)UINT32_MAX ) break;
      tot += a; j1++;
    }
    ulong need = STG_DATA + tot + 16ul;
    if( need > g_stg_cap ) {
      if( g_stg ) fd_ed25519_hip_host_free( g_stg );
      g_stg_cap = need < (1ul << 22) ? (1ul << 22) : need + need/4;
      g_stg = (uchar *)fd_ed25519_hip_host_alloc( g_stg_cap );
    }
    uint * off = (uint *)(g_stg + STG_OFF), * sz = (uint *)(g_stg + STG_SZ);
    ulong o = 0ul;
    for( ulong j=j0; j<j1; j++ ) {
      off[j-j0] = (uint)o; sz[j-j0] = (uint)b->sz[j];
      if( b->sz[j] ) memcpy( g_stg + STG_DATA + o, b->data[j], b->sz[j] );
      o += (b->sz[j] + 15ul) & ~15ul;
    }
    memset( g_stg + STG_DATA + o, 0, 16ul );
    fd_sha512_hip_batch_dev( ctx, j1 - j0, g_stg + STG_DATA, off, sz, g_stg + STG_HASH, NULL );
    SHA_CHECK( hipStreamSynchronize( (hipStream_t)fd_ed25519_hip_ctx_stream( ctx ) ) );
    for( ulong j=j0; j<j1; j++ ) memcpy( b->hash[j], g_stg + STG_HASH + 64ul*(j-j0), 64ul );
    j0 = j1;
  }
}

extern "C" {

int
fd_sha512_hip_batch_dev( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_pool, uint const * d_off,
                         uint const * d_sz, uchar * d_hash, void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)fd_ed25519_hip_ctx_stream( ctx );
  SHA_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( ctx ) ) );
  if( !n ) return 0;
  ulong const per_launch = 256ul << 23;                        /* 2^23 workgroups per launch */
  for( ulong i0=0ul; i0<n; i0+=per_launch ) {
    ulong m = n - i0 < per_launch ? n - i0 : per_launch;
    hipLaunchKernelGGL( k_sha512_batch, dim3( (unsigned)((m + 255ul)/256ul) ), dim3( 256 ), 0, s, m, d_pool,
                        d_off + i0, d_sz + i0, d_hash + 64ul*i0 );
    SHA_CHECK( hipGetLastError() );
  }
  return 0;
}

ulong fd_sha512_hip_batch_align    ( void ) { return FD_SHA512_HIP_BATCH_ALIGN; }
ulong fd_sha512_hip_batch_footprint( void ) { return sizeof(fd_sha512_hip_batch_t); }

fd_sha512_hip_batch_t *
fd_sha512_hip_batch_init( void * mem, fd_ed25519_hip_ctx_t * ctx ) {
  fd_sha512_hip_batch_t * b = (fd_sha512_hip_batch_t *)mem;
  b->ctx = ctx;
  b->cnt = 0ul;
  return b;
}

fd_sha512_hip_batch_t *
fd_sha512_hip_batch_add( fd_sha512_hip_batch_t * b, void const * data, ulong sz, void * hash ) {
  if( sz > FD_SHA512_HIP_MSG_MAX ) {
    fprintf( stderr, "fd_sha512_hip_batch_add: sz %lu exceeds FD_SHA512_HIP_MSG_MAX (%lu)\n", sz,
             (ulong)FD_SHA512_HIP_MSG_MAX );
    abort();
  }
  ulong c = b->cnt;
  b->data[c] = data; b->sz[c] = sz; b->hash[c] = hash;
  b->cnt = c + 1ul;
  if( b->cnt == FD_SHA512_HIP_BATCH_MAX ) batch_flush( b );
  return b;
}

void *
fd_sha512_hip_batch_fini( fd_sha512_hip_batch_t * b ) {
  batch_flush( b );
  return (void *)b;
}

void *
fd_sha512_hip_batch_abort( fd_sha512_hip_batch_t * b ) {
  b->cnt = 0ul;
  return (void *)b;
}

} /* extern "C" */
