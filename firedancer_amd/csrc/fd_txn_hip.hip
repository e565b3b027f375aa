/* fd_txn_hip.hip -- verify-tile layer of the gfx950 engine: GPU txn parse,
   sig0 tags, txn -> signature-record expansion, and the ordered host pass
   (tcache dedup + bundle state).  C ABI: include/fd_verify_hip.h.

   Per batch of frags (one lane per frag, 256-thread workgroups):

     k_txn_parse   fd_txn_parse_core (fd_txn_parse.c:7-254) on the payload,
                   fd_txn_t out, tag = fd_hash(seed, sig0, 64), and the
                   signature span to verify
     k_txn_expand  slot allocation (one atomic per wave, ballot prefix sums)
                   and 16-B-aligned signature records for the verify
                   pipeline; first/cnt per txn for the reduce
     fd_ed25519_hip_verify_dev_count + fd_ed25519_hip_group_reduce_dev
                   (the record count never leaves the device)
     D2H           txn_t_sz (2 B), code (1 B), tag (8 B) per frag

   The ordered host pass restates after_frag (fd_verify_tile.c:101-161)
   around fd_txn_verify (fd_verify_tile.h:61-111) with the tcache of
   fd_tcache.h:237-410, prefetching map slots a few frags ahead.

   The replay caller (include/fd_replay_hip.h) reuses the expansion and the
   reduce on caller-parsed transactions: k_desc_spans turns fd_txn_t fields
   into the same spans, k_exec_codes maps the per-txn code to the runtime's. */

#include "../../include/fd_verify_hip.h"
#include "../../include/fd_replay_hip.h"
#include "fd_hip_order.h"
#include "fd_txn_hip_int.h"

#include <hip/hip_runtime.h>
#include <chrono>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TX_CHECK( x ) do {                                                            \
    hipError_t e_ = (x);                                                               \
    if( e_ != hipSuccess ) {                                                           \
      fprintf( stderr, "fd_verify_hip: %s failed at %s:%d: %s\n", #x, __FILE__,      \
               __LINE__, hipGetErrorString( e_ ) );                                    \
      abort();                                                                         \
    }                                                                                  \
  } while( 0 )

typedef uint8_t  u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

#define DEVI __device__ __forceinline__
#define HD   __host__ __device__ __forceinline__

#define SIG_VERIFY_MAX 16u   /* fd_ed25519_user.c:238: batch_sz > 16 -> ERR_SIG */

/**********************************************************************/
/* fd_hash (util/fd_hash.c:6-72), shared by host and device            */

#define XH_P1 11400714785074694791ULL
#define XH_P2 14029467366897019727ULL
#define XH_P3  1609587929392839161ULL
#define XH_P4  9650029242287828579ULL
#define XH_P5  2870177450012600261ULL

HD u64 xh_rotl( u64 x, int r ) { return (x << r) | (x >> (64 - r)); }
HD u64 xh_round( u64 acc, u64 w ) { return xh_rotl( acc + w*XH_P2, 31 ) * XH_P1; }
HD u64 xh_avalanche( u64 h ) {
  h ^= h >> 33; h *= XH_P2; h ^= h >> 29; h *= XH_P3; h ^= h >> 32;
  return h;
}

/* the 64-byte case the verify tile hashes (sig0): two 32-byte stripes, no tail */
HD u64 xh_hash64( u64 seed, u64 const w[8] ) {
  u64 a = seed + XH_P1 + XH_P2, b = seed + XH_P2, c = seed, d = seed - XH_P1;
  a = xh_round( a, w[0] ); b = xh_round( b, w[1] ); c = xh_round( c, w[2] ); d = xh_round( d, w[3] );
  a = xh_round( a, w[4] ); b = xh_round( b, w[5] ); c = xh_round( c, w[6] ); d = xh_round( d, w[7] );
  u64 h = xh_rotl( a, 1 ) + xh_rotl( b, 7 ) + xh_rotl( c, 12 ) + xh_rotl( d, 18 );
  h ^= xh_round( 0, a ); h = h*XH_P1 + XH_P4;
  h ^= xh_round( 0, b ); h = h*XH_P1 + XH_P4;
  h ^= xh_round( 0, c ); h = h*XH_P1 + XH_P4;
  h ^= xh_round( 0, d ); h = h*XH_P1 + XH_P4;
  h += 64u;
  return xh_avalanche( h );
}

extern "C" ulong fd_verify_hip_hash( ulong seed, void const * buf, ulong sz ) {
  u8 const * p = (u8 const *)buf, * end = p + sz;
  u64 h;
  if( sz < 32 ) h = seed + XH_P5;
  else {
    u64 a = seed + XH_P1 + XH_P2, b = seed + XH_P2, c = seed, d = seed - XH_P1, w[4];
    do {
      memcpy( w, p, 32 );
      a = xh_round( a, w[0] ); b = xh_round( b, w[1] ); c = xh_round( c, w[2] ); d = xh_round( d, w[3] );
      p += 32;
    } while( end - p >= 32 );
    h = xh_rotl( a, 1 ) + xh_rotl( b, 7 ) + xh_rotl( c, 12 ) + xh_rotl( d, 18 );
    h ^= xh_round( 0, a ); h = h*XH_P1 + XH_P4;
    h ^= xh_round( 0, b ); h = h*XH_P1 + XH_P4;
    h ^= xh_round( 0, c ); h = h*XH_P1 + XH_P4;
    h ^= xh_round( 0, d ); h = h*XH_P1 + XH_P4;
  }
  h += sz;
  for( ; end - p >= 8; p += 8 ) { u64 w; memcpy( &w, p, 8 ); h ^= xh_round( 0, w ); h = xh_rotl( h, 27 )*XH_P1 + XH_P4; }
  if( end - p >= 4 ) { u32 w; memcpy( &w, p, 4 ); h ^= (u64)w*XH_P1; h = xh_rotl( h, 23 )*XH_P2 + XH_P3; p += 4; }
  for( ; p < end; p++ ) { h ^= (u64)p[0]*XH_P5; h = xh_rotl( h, 11 )*XH_P1; }
  return xh_avalanche( h );
}

/**********************************************************************/
/* GPU parse                                                           */

/* Unaligned 32-bit load from global memory: two aligned dwords and a funnel
   shift.  Only used inside a payload at offsets with >= 4 valid bytes after
   the loaded word's last byte (signatures and pubkeys are followed by more
   payload), so the second dword never leaves the payload. */
DEVI u32 ld_u32u( u8 const * p ) {
  uintptr_t a = (uintptr_t)p;
  u32 const * q = (u32 const *)(a & ~(uintptr_t)3);
  u32 sh = (u32)(a & 3u) * 8u;
  u32 lo = q[0];
  if( !sh ) return lo;
  return __builtin_amdgcn_alignbit( q[1], lo, sh );
}

/* The per-frag verify span produced by the parse. */
struct txn_span {
  u32 sig_at, acct_at, msg_at, msg_sz;
  u32 nsig;          /* signatures to verify: sig_cnt if parsed and <= 16, else 0 */
  u32 tsz;           /* fd_txn_t footprint or 0 */
};

/* fd_cu16_dec_sz + fd_cu16_dec_fixed (fd_compact_u16.h:38-92) */
template<class P>
DEVI bool cu16_rd( P const & p, u32 sz, u32 & i, u32 & v ) {
  u32 left = sz - i;
  u32 b0 = left >= 1 ? p[i] : 0u;
  if( left >= 1 && !(b0 & 0x80u) ) { v = b0; i += 1; return true; }
  u32 b1 = left >= 2 ? p[i+1] : 0u;
  if( left >= 2 && !(b1 & 0x80u) ) {
    if( !b1 ) return false;
    v = (b0 & 0x7fu) | (b1 << 7); i += 2; return true;
  }
  u32 b2 = left >= 3 ? p[i+2] : 0u;
  if( left >= 3 && !(b2 & 0xfcu) ) {
    if( !b2 ) return false;
    v = (b0 & 0x7fu) | ((b1 & 0x7fu) << 7) | (b2 << 14); i += 3; return true;
  }
  return false;
}

DEVI void put8 ( u8 * o, u32 off, u32 v ) { if( o ) o[off] = (u8)v; }
DEVI void put16( u8 * o, u32 off, u32 v ) { if( o ) *(u16 *)(o + off) = (u16)v; }   /* off even, o 2-aligned */

/* fd_txn_parse_core(payload, sz, out, NULL, NULL, FD_TXN_INSTR_MAX): returns
   the footprint or 0.  Check order follows fd_txn_parse.c line by line;
   `need(n)` is CHECK_LEFT.  P: a byte pointer, or any type with a byte
   operator[] (k_txnm_batch's out-frag view). */
template<class P>
DEVI u32 txn_parse( P const & p, u32 sz, u8 * out, txn_span & sp ) {
  u32 i = 0;
#define NEED( n ) do { if( (u32)(n) > sz - i ) return 0u; } while( 0 )
  if( sz > (u32)FD_TXN_HIP_MTU ) return 0u;                                 /* :82 */
  NEED( 1 ); u32 sig_cnt = p[i]; i++;
  if( sig_cnt < 1u || sig_cnt > 127u ) return 0u;                           /* :91 */
  NEED( 64u*sig_cnt ); u32 sig_off = i; i += 64u*sig_cnt;
  u32 msg_off = i;
  NEED( 1 ); u32 b0 = p[i]; i++;
  u32 version;
  if( b0 & 0x80u ) {                                                        /* :98-104 */
    version = b0 & 0x7fu;
    if( version != 0u ) return 0u;
    NEED( 1 ); if( p[i] != sig_cnt ) return 0u; i++;
  } else {
    version = 0xffu;
    if( b0 != sig_cnt ) return 0u;
  }
  NEED( 1 ); u32 ro_signed = p[i]; i++;
  if( ro_signed >= sig_cnt ) return 0u;                                     /* :111 */
  NEED( 1 ); u32 ro_unsigned = p[i]; i++;
  u32 acct_cnt;
  if( !cu16_rd( p, sz, i, acct_cnt ) ) return 0u;
  if( sig_cnt > acct_cnt || acct_cnt > 128u ) return 0u;                    /* :117 */
  if( sig_cnt + ro_unsigned > acct_cnt ) return 0u;                         /* :118 */
  NEED( 32u*acct_cnt ); u32 acct_off = i; i += 32u*acct_cnt;
  NEED( 32 ); u32 bh_off = i; i += 32u;
  u32 instr_cnt;
  if( !cu16_rd( p, sz, i, instr_cnt ) ) return 0u;
  if( instr_cnt > 64u ) return 0u;                                          /* :129 */
  NEED( 3u*instr_cnt );
  if( !( acct_cnt > (instr_cnt ? 1u : 0u) ) ) return 0u;                    /* :134 */
  put8( out, 0, version ); put8( out, 1, sig_cnt ); put16( out, 2, sig_off ); put16( out, 4, msg_off );
  put8( out, 6, ro_signed ); put8( out, 7, ro_unsigned ); put16( out, 8, acct_cnt ); put16( out, 10, acct_off );
  put16( out, 12, bh_off ); put16( out, 18, instr_cnt );
  u32 max_acct = 0;
  for( u32 j = 0; j < instr_cnt; j++ ) {                                    /* :153-184 */
    NEED( 3 ); u32 prog = p[i]; i++;
    u32 ia_cnt, data_sz;
    if( !cu16_rd( p, sz, i, ia_cnt ) ) return 0u;
    NEED( ia_cnt ); u32 ia_off = i;
    for( u32 k = 0; k < ia_cnt; k++ ) { u32 x = p[ia_off + k]; max_acct = x > max_acct ? x : max_acct; }
    i += ia_cnt;
    if( !cu16_rd( p, sz, i, data_sz ) ) return 0u;
    NEED( data_sz ); u32 data_off = i; i += data_sz;
    if( !( prog > 0u && prog < acct_cnt ) ) return 0u;                      /* :171 */
    u32 o = 20u + 10u*j;
    put8( out, o, prog ); put8( out, o+1, 0 ); put16( out, o+2, ia_cnt ); put16( out, o+4, data_sz );
    put16( out, o+6, ia_off ); put16( out, o+8, data_off );
  }
  u32 lut_cnt = 0, adtl_w = 0, adtl = 0;
  if( version == 0u ) {                                                     /* :193-226 */
    if( !cu16_rd( p, sz, i, lut_cnt ) ) return 0u;
    if( lut_cnt > 127u ) return 0u;
    NEED( 34u*lut_cnt );
    for( u32 j = 0; j < lut_cnt; j++ ) {
      NEED( 32 ); u32 a_off = i; i += 32u;
      u32 w, ro;
      if( !cu16_rd( p, sz, i, w ) ) return 0u;
      NEED( w ); u32 w_off = i; i += w;
      if( !cu16_rd( p, sz, i, ro ) ) return 0u;
      NEED( ro ); u32 ro_off = i; i += ro;
      if( w > 128u - acct_cnt || ro > 128u - acct_cnt || w + ro < 1u ) return 0u;
      u32 o = 20u + 10u*instr_cnt + 8u*j;
      put16( out, o, a_off ); put8( out, o+2, w ); put8( out, o+3, ro ); put16( out, o+4, w_off ); put16( out, o+6, ro_off );
      adtl_w += w; adtl += w + ro;
    }
  }
  if( i != sz ) return 0u;                                                  /* :229 */
  if( acct_cnt + adtl > 128u ) return 0u;                                   /* :231 */
  if( !( max_acct < acct_cnt + adtl ) ) return 0u;                          /* :234 */
#undef NEED
  put8( out, 14, lut_cnt ); put8( out, 15, adtl_w ); put8( out, 16, adtl ); put8( out, 17, 0 );
  sp.sig_at = sig_off; sp.acct_at = acct_off; sp.msg_at = msg_off; sp.msg_sz = sz - msg_off;
  sp.nsig = sig_cnt <= SIG_VERIFY_MAX ? sig_cnt : 0u;
  return 20u + 10u*instr_cnt + 8u*lut_cnt;
}

/* packed per-frag results for the host pass (k_tile_results, below) */
struct __attribute__((packed)) tile_res { u64 tag; u64 bid; u16 tsz; signed char tcode; u8 kind; u32 pad; };
static_assert( sizeof(tile_res) == 24, "tile_res layout" );
#define TILE_RES_HDR 32ul   /* u32 record count, u32 flag, u64 pad, u64 ingest bytes read, written */
#define TILE_RES_BAD 0x40u  /* or'd into tile_res.kind: the frag itself is corrupt (known per frag with out staging) */

/* per-frag SoA scratch written by k_txn_parse */
struct parse_out {
  u16 * tsz;      /* fd_txn_t footprint, 0 = parse failure */
  u8  * nsig;     /* signatures to verify */
  u32 * sig_at;   /* absolute pool offsets */
  u32 * acct_at;
  u32 * msg_at;
  u32 * msg_sz;
  u64 * tag;
};

/* tout (fd_txn_m_t frag mode): fd_txn_t of frag j at pool + tout[j] (the
   fd_txn_m_txn_t address, fd_txn_m.h:101-104) instead of txn_out + 852*j,
   and txn_t_sz written into the frag header (pool + off[j] - 80 + 10) as
   after_frag does (fd_verify_tile.c:120) */
__global__ __launch_bounds__(256)
void k_txn_parse( ulong n, u8 const * __restrict__ pool, u32 const * __restrict__ off,
                  u16 const * __restrict__ sz, u8 * __restrict__ txn_out, u64 seed, parse_out po,
                  u32 const * __restrict__ tout ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  u32 base = off[j];
  u8 const * p = pool + base;
  u8 * out = tout ? (u8 *)pool + tout[j] : txn_out ? txn_out + (ulong)FD_TXN_HIP_MAX_SZ * j : (u8 *)0;
  txn_span sp = { 0u, 0u, 0u, 0u, 0u, 0u };
  u32 tsz = txn_parse( p, sz[j], out, sp );
  if( tout ) *(u16 *)((u8 *)pool + base - FD_VERIFY_HIP_TXNM_SZ + FD_VERIFY_HIP_TXNM_TXN_T_SZ_OFF) = (u16)tsz;
  if( !po.tsz ) { return; }
  po.tsz[j] = (u16)tsz;
  if( !po.nsig ) return;
  u64 tag = 0;
  if( tsz ) {
    u64 w[8];
    u8 const * s = p + sp.sig_at;
    #pragma unroll
    for( int q = 0; q < 8; q++ ) w[q] = (u64)ld_u32u( s + 8*q ) | ((u64)ld_u32u( s + 8*q + 4 ) << 32);
    tag = xh_hash64( seed, w );
  }
  po.nsig[j]    = (u8)(tsz ? sp.nsig : 0u);
  po.sig_at[j]  = base + sp.sig_at;
  po.acct_at[j] = base + sp.acct_at;
  po.msg_at[j]  = base + sp.msg_at;
  po.msg_sz[j]  = sp.msg_sz;
  po.tag[j]     = tag;
}

/* NW little-endian words from an unaligned byte address: NW (+1 when
   unaligned) aligned dword loads and one funnel shift per word; never reads
   past the dword holding the last byte */
template<int NW>
DEVI void ld_words_u( u32 w[NW], u8 const * p ) {
  uintptr_t a = (uintptr_t)p;
  u32 const * q = (u32 const *)(a & ~(uintptr_t)3);
  u32 sh = (u32)(a & 3u) * 8u;
  u32 d[NW+1];
  #pragma unroll
  for( int i=0; i<NW; i++ ) d[i] = q[i];
  d[NW] = sh ? q[NW] : 0u;
  #pragma unroll
  for( int i=0; i<NW; i++ ) w[i] = __builtin_amdgcn_alignbit( d[i+1], d[i], sh );
}

/* Slot allocation + record expansion.  Each wave computes exclusive prefix
   sums of its lanes' nsig (< 32, five ballots + mbcnt) and takes one
   atomicAdd on the record counter.  Records of a wave are contiguous and in
   frag order; waves land in any order (first[] says where).  The wave then
   copies its records cooperatively, one record per lane per round (the frag
   of record t found by binary search over the wave's prefix sums in LDS):
   ceil(records/64) rounds instead of the largest per-frag count, and the
   record writes coalesce. */
__global__ __launch_bounds__(256)
void k_txn_expand( ulong n, u8 const * __restrict__ pool, u8 const * __restrict__ nsig_a,
                   u32 const * __restrict__ sig_at, u32 const * __restrict__ acct_at,
                   u32 const * __restrict__ msg_at, u32 const * __restrict__ msg_sz,
                   u32 * __restrict__ counter, u32 * __restrict__ first, u8 * __restrict__ cnt,
                   u8 * __restrict__ rsig, u8 * __restrict__ rpub, u32 * __restrict__ rmoff,
                   u32 * __restrict__ rmsz, ulong cap ) {
  __shared__ u32 l_excl[256], l_c[256], l_sig[256], l_acct[256], l_mo[256], l_ms[256];
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  u32 c = j < n ? nsig_a[j] : 0u;
  u32 excl = 0, tot = 0;
  #pragma unroll
  for( int b = 0; b < 5; b++ ) {
    unsigned long long m = __ballot( (c >> b) & 1u );
    u32 below = __builtin_amdgcn_mbcnt_hi( (u32)(m >> 32), __builtin_amdgcn_mbcnt_lo( (u32)m, 0u ) );
    excl += below << b;
    tot  += (u32)__popcll( m ) << b;
  }
  u32 base = 0;
  if( (threadIdx.x & 63u) == 0u && tot ) base = atomicAdd( counter, tot );
  base = __shfl( base, 0 );
  u32 lc = c;
  if( j < n ) {
    u32 f = base + excl;
    first[j] = f; cnt[j] = (u8)c;
    if( (ulong)f + c > cap ) { cnt[j] = 0; lc = 0; }      /* host sizes cap; never taken */
    l_sig[threadIdx.x] = sig_at[j]; l_acct[threadIdx.x] = acct_at[j];
    l_mo[threadIdx.x] = msg_at[j];  l_ms[threadIdx.x] = msg_sz[j];
  }
  l_excl[threadIdx.x] = excl; l_c[threadIdx.x] = lc;
  __syncthreads();
  u32 w0 = threadIdx.x & ~63u;
  for( u32 t = threadIdx.x & 63u; t < tot; t += 64u ) {
    u32 lo = 0, hi = 63;                                  /* last lane with excl <= t */
    #pragma unroll
    for( int s = 0; s < 6; s++ ) {
      u32 mid = (lo + hi + 1u) >> 1;
      bool le = l_excl[w0 + mid] <= t;
      lo = le ? mid : lo; hi = le ? hi : mid - 1u;
    }
    u32 L = w0 + lo, k = t - l_excl[L];
    if( k >= l_c[L] ) continue;                           /* capped frag */
    u32 r = base + t;
    u32 w[16];
    ld_words_u<16>( w, pool + l_sig[L] + 64u*k );
    uint4 * ds = (uint4 *)(rsig + 64ul*r);
    #pragma unroll
    for( int q = 0; q < 4; q++ ) ds[q] = make_uint4( w[4*q], w[4*q+1], w[4*q+2], w[4*q+3] );
    ld_words_u<8>( w, pool + l_acct[L] + 32u*k );
    uint4 * dp = (uint4 *)(rpub + 32ul*r);
    #pragma unroll
    for( int q = 0; q < 2; q++ ) dp[q] = make_uint4( w[4*q], w[4*q+1], w[4*q+2], w[4*q+3] );
    rmoff[r] = l_mo[L]; rmsz[r] = l_ms[L];
  }
}

/* fd_txn_m_t frag ingest: during_frag (fd_verify_tile.c:64-99) for a batch.
   One wave per frag (frags strided over the grid's waves), 64 B-aligned
   dcache chunks in and out (fd_chunk_to_laddr: mem + 64*chunk):
     QUIC / BUNDLE / SEND  copy the sz-byte frag in -> out (16 B per lane per
                           round, coalesced); sz > FD_TPU_RAW_MTU or a
                           header payload_sz > FD_TPU_MTU is a corrupt frag
     GOSSIP                fd_gossip_update_message_t vote -> fd_txn_m_t:
                           payload_sz = vote.txn_sz, bundle_id = 0,
                           source_ipv4 = vote.socket.addr, source_tpu =
                           GOSSIP, payload = vote.txn; sz > 2048 (or a
                           txn_sz past the 1232-B vote buffer) is corrupt
   A QUIC / BUNDLE / SEND frag whose in chunk is its out chunk is left in
   place (a host tile whose during_frag already copied the frag into its out
   dcache, integration/fd_verify_tile_hip.patch).
   Per frag it emits the payload span for k_txn_parse, the fd_txn_m_txn_t
   offset and the header's bundle_id for the ordered host pass.  A corrupt
   frag sets bit 0 of *flag (the reference's FD_LOG_ERR: the host aborts in
   complete()) and is parsed as an empty payload. */
DEVI void copy_bytes( u8 * __restrict__ d, u8 const * __restrict__ s, u32 nb, u32 lane ) {   /* d, s 16-B aligned */
  u32 full = nb >> 4;
  for( u32 q = lane; q < full; q += 64u ) ((uint4 *)d)[q] = ((uint4 const *)s)[q];
  u32 t = full << 4;
  if( lane < nb - t ) d[t + lane] = s[t + lane];                 /* < 16 tail bytes, one per lane */
}

__global__ __launch_bounds__(256)
void k_txnm_ingest( ulong n, u8 const * in, u32 const * __restrict__ in_chunk,
                    u16 const * __restrict__ in_sz, u8 const * __restrict__ in_kind, u8 * out,
                    u32 const * __restrict__ out_chunk, u32 * __restrict__ pay_off, u16 * __restrict__ pay_sz,
                    u32 * __restrict__ tout, u64 * __restrict__ bid, u32 * __restrict__ flag ) {
  u32 lane = threadIdx.x & 63u;
  ulong w = ((ulong)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((ulong)gridDim.x * blockDim.x) >> 6;
  for( ulong j = w; j < n; j += nw ) {
    u32 ob = 64u * out_chunk[j];
    u8 * dst = out + ob;
    u32 sz = in_sz[j], kind = in_kind[j], psz = 0u, bad = 0u;
    u8 const * src = (kind & FD_VERIFY_HIP_IN_HOSTCOPY) ? dst : in + 64ul * in_chunk[j];   /* host did during_frag */
    u64 b = 0ul;
    if( kind == FD_VERIFY_HIP_IN_GOSSIP ) {
      u64 tsz = *(u64 const *)(src + FD_VERIFY_HIP_GOSSIP_VOTE_TXN_SZ_OFF);
      bad = sz > 2048u || tsz > FD_TXN_HIP_MTU;
      psz = bad ? 0u : (u32)tsz;
      copy_bytes( dst + FD_VERIFY_HIP_TXNM_SZ, src + FD_VERIFY_HIP_GOSSIP_VOTE_TXN_OFF, psz, lane );
      if( lane == 0u ) {
        *(u16 *)(dst + FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF) = (u16)psz;
        *(u64 *)(dst + FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF) = 0ul;
        *(u32 *)(dst + FD_VERIFY_HIP_TXNM_SRC_IPV4_OFF) = *(u32 const *)(src + FD_VERIFY_HIP_GOSSIP_VOTE_ADDR_OFF);
        dst[FD_VERIFY_HIP_TXNM_SRC_TPU_OFF] = (u8)FD_VERIFY_HIP_TPU_SOURCE_GOSSIP;
      }
    } else {
      bad = sz > FD_VERIFY_HIP_TPU_RAW_MTU;
      if( src != dst ) copy_bytes( dst, src, bad ? 0u : sz, lane );   /* in place: the tile copied it already */
      psz = bad ? 0u : *(u16 const *)(src + FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF);
      b   = bad ? 0ul : *(u64 const *)(src + FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF);
      if( psz > FD_TXN_HIP_MTU ) { bad = 1u; psz = 0u; }
    }
    if( lane == 0u ) {
      u32 po = ob + FD_VERIFY_HIP_TXNM_SZ;
      pay_off[j] = po; pay_sz[j] = (u16)psz;
      tout[j] = (po + psz + (FD_VERIFY_HIP_TXN_ALIGN - 1u)) & ~(FD_VERIFY_HIP_TXN_ALIGN - 1u);
      bid[j] = b;
      if( bad ) atomicOr( flag, 1u );
    }
  }
}

/**********************************************************************/
/* k_txnm_batch: ingest + parse + record expansion in one pass          */

/* One 64-thread workgroup per group of F fd_txn_m_t frags; the frags go
   through LDS once:

   1. stage   every 16-B piece of the group's frags (the header and the
              bytes during_frag copies; for a gossip vote its txn) is loaded
              once, pieces dealt to lanes over the group's piece prefix sums
              so that all 64 lanes load and the loads coalesce; each piece is
              stored to LDS at its prefix position (packed: a frag takes its
              own size, ~30 pieces in a txn stream, not the 82 of the MTU)
              and, where during_frag copies it, to the out dcache
              (fd_verify_tile.c:64-99)
   2. parse   lane f parses frag f's payload from LDS (fd_txn_parse_core,
              fd_txn_parse.c:7-254, restated as txn_parse above but reading
              4 bytes per LDS access), writes the fd_txn_t at fd_txn_m_txn_t
              and txn_t_sz into the out header (after_frag, :118-120), and
              hashes sig0 for the tcache tag (fd_txn_verify, fd_verify_tile.h:76)
   3. expand  the group's signatures get one contiguous record range (one
              atomic per group), and the wave copies each record's signature
              and public key out of LDS as 16-B pieces (coalesced stores);
              per-record message spans; the block-count histogram prep's
              order is built from (fd_hip_order.h)

   Against k_txnm_ingest + k_txn_parse + k_txn_expand (+ k_msg_hist) this
   reads each frag from HBM once instead of three times, and the parse's
   dependent byte loads hit LDS instead of HBM.  The kernel is bound by the
   bytes it keeps in flight, so the LDS per group is a budget of
   FB_PIECES_PER_FRAG pieces per frag (10 KB for 16 frags: 16 workgroups per
   CU) rather than an MTU-sized slot per frag (21 KB: 7 workgroups per CU,
   profiles/r04b trace: the staging phase was 58% of a workgroup's life).

   The global path: after_frag parses the OUT frag, so where during_frag's
   copy did not reach (a header whose payload_sz exceeds the frag, a frag
   shorter than its header) it reads the out dcache's stale bytes.  A group
   with such a frag, or whose pieces overflow the budget, parses, hashes and
   expands through frag_view (in-frag bytes below the copy's end, out-frag
   bytes past it, loaded from global memory) instead of LDS: the same bytes
   the reference's parse sees.  A corrupt frag sets *flag (the host aborts
   in complete()) and parses as an empty payload, as in k_txnm_ingest. */

/* FD_TXNM_TRACE builds (diagnostic variants only, firedancer_amd/build.py
   <variant> FD_TXNM_TRACE=1): lane 0 of every k_txnm_batch workgroup
   records s_memtime at each phase boundary; fd_verify_hip_txnm_trace()
   copies them out. */
#ifndef FD_TXNM_TRACE
#define FD_TXNM_TRACE 0
#endif
#if FD_TXNM_TRACE
#define TXTR_SLOTS 8
#define TXTR_MAX   (1ul << 17)
__device__ u64 g_txnm_trace[ TXTR_MAX * TXTR_SLOTS ];
#define TXTR( k ) do { if( threadIdx.x == 0u && blockIdx.x < TXTR_MAX ) \
    g_txnm_trace[ (ulong)blockIdx.x * TXTR_SLOTS + (k) ] = __builtin_amdgcn_s_memtime(); } while( 0 )
extern "C" int fd_verify_hip_txnm_trace( void * out, ulong n_wg ) {
  if( n_wg > TXTR_MAX ) n_wg = TXTR_MAX;
  return (int)hipMemcpyFromSymbol( out, HIP_SYMBOL( g_txnm_trace ), n_wg * TXTR_SLOTS * sizeof(u64), 0,
                                   hipMemcpyDeviceToHost );
}
#else
#define TXTR( k ) do {} while( 0 )
#endif

/* FD_TXNM_ABLATE (diagnostic variants only; results are wrong): bit 0 no
   fd_txn_t stores, bit 1 no out-frag copy stores, bit 2 no parse, bit 3 no
   record stores */
#ifndef FD_TXNM_ABLATE
#define FD_TXNM_ABLATE 0
#endif

#define FB_PIECES_PER_FRAG 40u   /* LDS budget: 640 B per frag on average (a normal stream's mean is ~30 pieces) */
#define FB_LB        8    /* pieces in flight per lane */

/* 4 bytes at LDS byte offset i (two aligned dword reads and a funnel shift;
   reads up to 7 bytes past i) */
DEVI u32 lds_ld4( u8 const * l, u32 i ) {
  u32 const * q = (u32 const *)(l + (i & ~3u));
  return __builtin_amdgcn_alignbit( q[1], q[0], (i & 3u) * 8u );
}

/* fd_cu16_dec (fd_compact_u16.h:38-92) on the 4 bytes w = p[i..i+3], left =
   sz - i bytes remaining: same accept/reject as cu16_rd */
DEVI bool cu16_w( u32 w, u32 left, u32 & len, u32 & v ) {
  u32 b0 = w & 0xffu, b1 = (w >> 8) & 0xffu, b2 = (w >> 16) & 0xffu;
  if( left >= 1u && !(b0 & 0x80u) ) { v = b0; len = 1u; return true; }
  if( left >= 2u && !(b1 & 0x80u) ) {
    if( !b1 ) return false;
    v = (b0 & 0x7fu) | (b1 << 7); len = 2u; return true;
  }
  if( left >= 3u && !(b2 & 0xfcu) ) {
    if( !b2 ) return false;
    v = (b0 & 0x7fu) | ((b1 & 0x7fu) << 7) | (b2 << 14); len = 3u; return true;
  }
  return false;
}

/* txn_parse (above) over a payload in LDS: identical checks, order and
   output; out (global, 2-aligned) receives the fd_txn_t */
DEVI u32 txn_parse_lds( u8 const * p, u32 sz, u8 * out, txn_span & sp ) {
  u32 i = 0, len, w;
#define NEED( n ) do { if( (u32)(n) > sz - i ) return 0u; } while( 0 )
  if( sz > (u32)FD_TXN_HIP_MTU ) return 0u;                                 /* :82 */
  NEED( 1 ); u32 sig_cnt = p[0]; i = 1u;
  if( sig_cnt < 1u || sig_cnt > 127u ) return 0u;                           /* :91 */
  NEED( 64u*sig_cnt ); u32 sig_off = i; i += 64u*sig_cnt;
  u32 msg_off = i;
  u32 h0 = lds_ld4( p, i ), h1 = lds_ld4( p, i + 4u );                       /* message header, one LDS round */
  NEED( 1 ); u32 b0 = h0 & 0xffu; i++;
  u32 version, hb = 1u;                                                     /* hb: header bytes consumed from h */
  if( b0 & 0x80u ) {                                                        /* :98-104 */
    version = b0 & 0x7fu;
    if( version != 0u ) return 0u;
    NEED( 1 ); if( ((h0 >> 8) & 0xffu) != sig_cnt ) return 0u; i++; hb = 2u;
  } else {
    version = 0xffu;
    if( b0 != sig_cnt ) return 0u;
  }
  u32 h = __builtin_amdgcn_alignbit( h1, h0, hb * 8u );                     /* bytes msg_off+hb .. +hb+3 */
  NEED( 1 ); u32 ro_signed = h & 0xffu; i++;
  if( ro_signed >= sig_cnt ) return 0u;                                     /* :111 */
  NEED( 1 ); u32 ro_unsigned = (h >> 8) & 0xffu; i++;
  u32 acct_cnt;
  w = hb == 1u ? __builtin_amdgcn_alignbit( h1, h0, 24u ) : h1;            /* the varint's (up to) 3 bytes */
  if( !cu16_w( w, sz - i, len, acct_cnt ) ) return 0u;
  i += len;
  if( sig_cnt > acct_cnt || acct_cnt > 128u ) return 0u;                    /* :117 */
  if( sig_cnt + ro_unsigned > acct_cnt ) return 0u;                         /* :118 */
  NEED( 32u*acct_cnt ); u32 acct_off = i; i += 32u*acct_cnt;
  NEED( 32 ); u32 bh_off = i; i += 32u;
  u32 instr_cnt;
  if( !cu16_w( lds_ld4( p, i ), sz - i, len, instr_cnt ) ) return 0u;
  i += len;
  if( instr_cnt > 64u ) return 0u;                                          /* :129 */
  NEED( 3u*instr_cnt );
  if( !( acct_cnt > (instr_cnt ? 1u : 0u) ) ) return 0u;                    /* :134 */
  put8( out, 0, version ); put8( out, 1, sig_cnt ); put16( out, 2, sig_off ); put16( out, 4, msg_off );
  put8( out, 6, ro_signed ); put8( out, 7, ro_unsigned ); put16( out, 8, acct_cnt ); put16( out, 10, acct_off );
  put16( out, 12, bh_off ); put16( out, 18, instr_cnt );
  u32 max_acct = 0;
  for( u32 j = 0; j < instr_cnt; j++ ) {                                    /* :153-184 */
    NEED( 3 );
    w = lds_ld4( p, i );
    u32 prog = w & 0xffu; i++;
    u32 ia_cnt, data_sz;
    if( !cu16_w( w >> 8, sz - i, len, ia_cnt ) ) return 0u;
    i += len;
    NEED( ia_cnt ); u32 ia_off = i;
    i += ia_cnt;
    u32 wd = lds_ld4( p, i );                                               /* data_sz varint: before the max loop */
    for( u32 k = 0; k < ia_cnt; k += 4u ) {                                 /* max account index, 4 bytes a read */
      u32 x = lds_ld4( p, ia_off + k ), left = ia_cnt - k;
      if( left < 4u ) x &= (1u << (8u*left)) - 1u;
      u32 m = max( max( x & 0xffu, (x >> 8) & 0xffu ), max( (x >> 16) & 0xffu, x >> 24 ) );
      max_acct = m > max_acct ? m : max_acct;
    }
    if( !cu16_w( wd, sz - i, len, data_sz ) ) return 0u;
    i += len;
    NEED( data_sz ); u32 data_off = i; i += data_sz;
    if( !( prog > 0u && prog < acct_cnt ) ) return 0u;                      /* :171 */
    u32 o = 20u + 10u*j;
    put8( out, o, prog ); put8( out, o+1, 0 ); put16( out, o+2, ia_cnt ); put16( out, o+4, data_sz );
    put16( out, o+6, ia_off ); put16( out, o+8, data_off );
  }
  u32 lut_cnt = 0, adtl_w = 0, adtl = 0;
  if( version == 0u ) {                                                     /* :193-226 */
    if( !cu16_w( lds_ld4( p, i ), sz - i, len, lut_cnt ) ) return 0u;
    i += len;
    if( lut_cnt > 127u ) return 0u;
    NEED( 34u*lut_cnt );
    for( u32 j = 0; j < lut_cnt; j++ ) {
      NEED( 32 ); u32 a_off = i; i += 32u;
      u32 wl, ro;
      if( !cu16_w( lds_ld4( p, i ), sz - i, len, wl ) ) return 0u;
      i += len;
      NEED( wl ); u32 w_off = i; i += wl;
      if( !cu16_w( lds_ld4( p, i ), sz - i, len, ro ) ) return 0u;
      i += len;
      NEED( ro ); u32 ro_off = i; i += ro;
      if( wl > 128u - acct_cnt || ro > 128u - acct_cnt || wl + ro < 1u ) return 0u;
      u32 o = 20u + 10u*instr_cnt + 8u*j;
      put16( out, o, a_off ); put8( out, o+2, wl ); put8( out, o+3, ro ); put16( out, o+4, w_off ); put16( out, o+6, ro_off );
      adtl_w += wl; adtl += wl + ro;
    }
  }
  if( i != sz ) return 0u;                                                  /* :229 */
  if( acct_cnt + adtl > 128u ) return 0u;                                   /* :231 */
  if( !( max_acct < acct_cnt + adtl ) ) return 0u;                          /* :234 */
#undef NEED
  put8( out, 14, lut_cnt ); put8( out, 15, adtl_w ); put8( out, 16, adtl ); put8( out, 17, 0 );
  sp.sig_at = sig_off; sp.acct_at = acct_off; sp.msg_at = msg_off; sp.msg_sz = sz - msg_off;
  sp.nsig = sig_cnt <= SIG_VERIFY_MAX ? sig_cnt : 0u;
  return 20u + 10u*instr_cnt + 8u*lut_cnt;
}

/* 16 bytes at LDS byte offset a, any alignment */
DEVI uint4 lds_ld16u( u8 const * l, u32 a ) {
  u32 const * q = (u32 const *)(l + (a & ~3u));
  u32 sh = (a & 3u) * 8u;
  u32 d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
  return make_uint4( __builtin_amdgcn_alignbit( d1, d0, sh ), __builtin_amdgcn_alignbit( d2, d1, sh ),
                     __builtin_amdgcn_alignbit( d3, d2, sh ), __builtin_amdgcn_alignbit( d4, d3, sh ) );
}

/* the first nb (< 16) bytes of v to d (16-B aligned): whole dwords, then bytes */
DEVI void store_head( u8 * d, uint4 v, u32 nb ) {
  u32 w[4] = { v.x, v.y, v.z, v.w };
  u32 nd = nb >> 2;
  #pragma unroll
  for( u32 k = 0; k < 3; k++ ) if( k < nd ) ((u32 *)d)[k] = w[k];
  u32 t = nb & 3u, x = w[nd & 3u];
  u8 * e = d + 4u*nd;
  if( t > 0u ) e[0] = (u8)x;
  if( t > 1u ) e[1] = (u8)(x >> 8);
  if( t > 2u ) e[2] = (u8)(x >> 16);
}

/* which of the group's F frags item q belongs to: the last f with
   start_f <= q, where lane f holds start_f (ascending over the lanes, start_0
   = 0; lanes past the group's frags hold the total, past every item).  A
   binary search over __shfl reads: call with every lane of the wave active. */
template<int F>
DEVI u32 group_of( u32 start, u32 q ) {
  u32 f = 0u;
  #pragma unroll
  for( u32 step = (u32)F / 2u; step; step >>= 1 ) {
    u32 c = f + step;
    f = (u32)__shfl( (int)start, (int)c ) <= q ? c : f;
  }
  return f;
}

/* a tile slot's misc block (memset per batch): a header line ([0] total
   record count, written by the verify's k_seg_reduce; [1] corrupt-frag
   flag), then one fd_hip_order.h segment per record segment: its counter
   line (count, and the u64 ingest byte counter at SEG_BYTES_W) and its
   block-count histogram line */
#define SEG_BYTES_W        2u
#define FB_SEGS           64u      /* record segments of a batch at most (fd_hip_order.h: ~1000 claims per counter) */
#define SLOT_MISC_WORDS   (32u + FD_HIP_SEG_MAX*FD_HIP_SEG_STRIDE)
#define SLOT_MISC_BYTES   (4ul*SLOT_MISC_WORDS)
#define SLOT_SEG_SLACK    (16ul*(FB_SEGS + 1ul))   /* frags of rounding per batch: records sized 12 x (n + slack) */

/* The out frag as after_frag reads it, byte by byte: during_frag's copy
   [lo, cend) comes from the in frag, everything else is the out dcache's
   (k_txnm_batch's global path) */
struct frag_view {
  u8 const * src; u8 const * dst; u32 cend;
  DEVI u32 operator[]( u32 x ) const { return x < cend ? src[x] : dst[x]; }
};
struct pay_view {                                          /* the payload: frag offset 80 + i */
  frag_view f;
  DEVI u32 operator[]( u32 i ) const { return f[FD_VERIFY_HIP_TXNM_SZ + i]; }
};

/* Out staging (hout != 0, fd_verify_hip_tile_set_staging): out / out_chunk
   are a staging area in HBM and hout / hout_chunk the caller's out dcache
   (pinned host memory).  The kernel then works on HBM only -- the copy, the
   fd_txn_t and the signature records' messages (which the verify reads)
   land in the staging frag -- and k_out_flush copies to the out dcache
   exactly the bytes the reference writes there (fdesc[j]: the copy's end,
   payload_sz, txn_t_sz, gossip, corrupt).  Bytes after_frag reads but
   during_frag did not copy (a frag shorter than its header or its
   payload_sz: the out dcache's own bytes) are read from the out dcache, and
   a host-copied frag (FD_VERIFY_HIP_IN_HOSTCOPY) is read from it too. */
template<int F>
__global__ __launch_bounds__(64)
void k_txnm_batch( ulong n, u8 const * in, u32 const * __restrict__ in_chunk, u16 const * __restrict__ in_sz,
                   u8 const * __restrict__ in_kind, u8 * out, u32 const * __restrict__ out_chunk, u64 seed,
                   u16 * __restrict__ tsz_o, u64 * __restrict__ tag_o, u64 * __restrict__ bid_o,
                   u32 * __restrict__ first_o, u8 * __restrict__ cnt_o, u32 * __restrict__ misc,
                   u8 * __restrict__ rsig, u8 * __restrict__ rpub, u32 * __restrict__ rmoff,
                   u32 * __restrict__ rmsz, u32 n_seg, ulong seg_cap, u8 const * hout,
                   u32 const * __restrict__ hout_chunk, u64 * __restrict__ fdesc,
                   u64 const * __restrict__ seedv ) {
  constexpr u32 BUDGET = FB_PIECES_PER_FRAG * (u32)F;                        /* staged pieces per group */
  __shared__ __attribute__((aligned(16))) u8 lds[16u * BUDGET + 32u];       /* + over-read of the last piece */
  /* this group's record segment (fd_hip_order.h): claims, histogram and
     byte counts go to its own lines, ~nwg/n_seg groups per counter */
  u32 const sx = blockIdx.x % n_seg;
  u32 * const flag = misc + 1, * const seg = misc + 32u + sx * FD_HIP_SEG_STRIDE;
  u32 const lane = threadIdx.x;
  ulong const j0 = (ulong)blockIdx.x * (ulong)F;
  if( j0 >= n ) return;
  u32 const nf = n - j0 < (ulong)F ? (u32)(n - j0) : (u32)F;
  TXTR( 0 );

  /* per-frag metadata on lanes [0, nf) */
  bool const fl = lane < nf;
  ulong const j = j0 + lane;
  u32 ic = 0u, oc = 0u, sz = 0u, kind = 0u, hoc = 0u;
  if( fl ) { oc = out_chunk[j]; sz = in_sz[j]; kind = in_kind[j]; }
  if( fl && !(kind & FD_VERIFY_HIP_IN_HOSTCOPY) ) ic = in_chunk[j];
  if( fl && hout ) hoc = hout_chunk[j];
  u8 *       dst = out + 64ul * oc;
  u8 const * hdst = hout ? hout + 64ul * hoc : (u8 const *)dst;              /* the out dcache's frag */
  u8 const * src = (kind & FD_VERIFY_HIP_IN_HOSTCOPY) ? hdst : in + 64ul * ic;  /* host did during_frag */
  u32 const src_lo = (u32)(u64)src, src_hi = (u32)((u64)src >> 32);
  bool const gossip = fl && kind == FD_VERIFY_HIP_IN_GOSSIP;
  u32 tsz_g = 0u;
  if( __ballot( gossip ) && gossip ) {
    u64 t = *(u64 const *)(src + FD_VERIFY_HIP_GOSSIP_VOTE_TXN_SZ_OFF);
    tsz_g = t > (u64)FD_TXN_HIP_MTU ? 0xffffffffu : (u32)t;
  }
  /* staged byte range [lo, hi) of the in frag (whole pieces); the bytes
     during_frag copies to the same offsets of the out frag: [lo, cend) */
  u32 bad = 0u, lo = 0u, hi = 0u, cend = 0u;
  if( fl ) {
    if( gossip ) {
      bad = sz > 2048u || tsz_g == 0xffffffffu;
      u32 psz = bad ? 0u : tsz_g;
      lo = FD_VERIFY_HIP_GOSSIP_VOTE_TXN_OFF; hi = lo + psz; cend = hi;     /* vote.txn -> the payload */
    } else {
      bad = sz > FD_VERIFY_HIP_TPU_RAW_MTU;
      if( !bad ) {
        hi = sz > FD_VERIFY_HIP_TXNM_SZ ? sz : FD_VERIFY_HIP_TXNM_SZ;       /* with the whole header */
        cend = src == (u8 const *)dst ? 0u : sz;                            /* in place: copied by the host tile */
      }
    }
  }
  u32 const np = (((hi + 15u) & ~15u) - lo) >> 4;                           /* pieces, <= 82 */

  /* piece prefix sums over the group (np < 128: seven ballots): frag f's
     pieces are the group's pieces [excl_f, excl_f + np_f), staged at LDS
     byte 16 excl_f (packed: a frag takes its own size, not the MTU) */
  u32 excl = 0u, tot = 0u;
  #pragma unroll
  for( int b = 0; b < 7; b++ ) {
    unsigned long long m = __ballot( (np >> b) & 1u );
    excl += __builtin_amdgcn_mbcnt_hi( (u32)(m >> 32), __builtin_amdgcn_mbcnt_lo( (u32)m, 0u ) ) << b;
    tot  += (u32)__popcll( m ) << b;
  }
  bool const packed = tot <= BUDGET;                                        /* wave-uniform */
  TXTR( 1 );

  /* 1. stage: piece q of the group -> lane q % 64; to LDS (if the group
     fits) and, where during_frag copies it, to the out frag */
  for( u32 q0 = 0u; q0 < tot; q0 += 64u * FB_LB ) {
    uint4 v[FB_LB];
    u32 ce[FB_LB];
    u8 * da[FB_LB];
    #pragma unroll
    for( int r = 0; r < FB_LB; r++ ) {
      u32 q = q0 + 64u * (u32)r + lane;
      u32 f = group_of<F>( excl, q < tot ? q : 0u );
      u32 fsl = __shfl( src_lo, (int)f ), fsh = __shfl( src_hi, (int)f ), foc = __shfl( oc, (int)f );
      u32 flo = __shfl( lo, (int)f ), fce = __shfl( cend, (int)f ), fex = __shfl( excl, (int)f );
      u32 b = flo + 16u * (q - fex);                                         /* byte offset in the frag */
      da[r] = out + 64ul * foc + b;
      ce[r] = q < tot ? (fce > b ? fce - b : 0u) : 0u;                       /* bytes of this piece to copy */
      if( q < tot ) v[r] = *(uint4 const *)((u8 const *)(((u64)fsh << 32) | (u64)fsl) + b);
    }
    #pragma unroll
    for( int r = 0; r < FB_LB; r++ ) {
      u32 q = q0 + 64u * (u32)r + lane;
      if( packed && q < tot ) *(uint4 *)(lds + 16u * q) = v[r];
      if( FD_TXNM_ABLATE & 2 ) continue;
      if( ce[r] >= 16u )     *(uint4 *)da[r] = v[r];
      else if( ce[r] )       store_head( da[r], v[r], ce[r] );
    }
  }
  __syncthreads();
  TXTR( 2 );

  /* 2. header and parse (lanes [0, nf)).  after_frag reads the OUT frag:
     where during_frag's copy did not reach (a frag shorter than its header,
     a payload_sz past the frag) those are the out dcache's own bytes.  A
     group with such a frag, or one whose pieces overflow the LDS budget,
     parses through frag_view from global memory instead of LDS. */
  frag_view const fv = { src, hdst, cend };
  u32 const hb = 16u * excl;                                                /* the frag's first staged byte in LDS */
  u32 psz = 0u, tsz = 0u, nsig = 0u, side = 0u;
  u64 bid = 0ul, tag = 0ul;
  txn_span sp = { 0u, 0u, 0u, 0u, 0u, 0u };
  if( fl ) {
    if( gossip ) {
      psz = bad ? 0u : tsz_g;
    } else if( !bad ) {
      bool short_hdr = src != (u8 const *)dst && sz < FD_VERIFY_HIP_TXNM_SZ;
      if( packed && !short_hdr ) {
        psz = *(u16 const *)(lds + hb + FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF);
        bid = *(u64 const *)(lds + hb + FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF);
      } else {
        psz = fv[FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF] | (fv[FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF + 1u] << 8);
        #pragma unroll
        for( u32 k = 0; k < 8u; k++ ) bid |= (u64)fv[FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF + k] << (8u*k);
      }
      if( psz > FD_TXN_HIP_MTU ) { bad = 1u; psz = 0u; }
      u32 have = src == (u8 const *)dst ? ((hi + 15u) & ~15u) : sz;         /* bytes of the out frag staged */
      side = short_hdr || FD_VERIFY_HIP_TXNM_SZ + psz > have;               /* parse reads bytes not staged */
      /* out staging: the payload bytes past the copy are the out dcache's
         (stale) bytes, and the verify hashes the message from the staging
         frag -- bring them over (a frag shorter than its payload_sz only) */
      if( hout && !bad )
        for( u32 x = cend; x < FD_VERIFY_HIP_TXNM_SZ + psz; x++ ) dst[x] = hdst[x];
    }
    if( bad ) atomicOr( flag, 1u );
  }
  bool const glob = !packed || __ballot( side );
  /* the copy's stores precede the parse's where they can meet: a lying
     payload_sz can place the fd_txn_t over copied bytes, and the reference
     writes it after the copy (no frag of a normal stream: its fd_txn_t
     starts at or past the copied end) */
  u32 const po = FD_VERIFY_HIP_TXNM_SZ + psz;
  u32 const to = (po + (FD_VERIFY_HIP_TXN_ALIGN - 1u)) & ~(FD_VERIFY_HIP_TXN_ALIGN - 1u);
  if( __ballot( fl && to < cend ) ) __builtin_amdgcn_s_waitcnt( 0 );
  TXTR( 3 );
  u32 const pb = hb + FD_VERIFY_HIP_TXNM_SZ - lo;                           /* payload byte 0 in LDS */
  pay_view const pv = { fv };
  if( fl ) {
    if( gossip ) {                                                          /* fd_verify_tile.c:90-95 */
      *(u16 *)(dst + FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF) = (u16)psz;
      *(u64 *)(dst + FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF) = 0ul;
      *(u32 *)(dst + FD_VERIFY_HIP_TXNM_SRC_IPV4_OFF) = *(u32 const *)(src + FD_VERIFY_HIP_GOSSIP_VOTE_ADDR_OFF);
      dst[FD_VERIFY_HIP_TXNM_SRC_TPU_OFF] = (u8)FD_VERIFY_HIP_TPU_SOURCE_GOSSIP;
    }
    u8 * tout = (FD_TXNM_ABLATE & 1) ? (u8 *)0 : dst + to;
    u32 psz_p = (FD_TXNM_ABLATE & 4) ? 0u : psz;
    tsz = glob ? txn_parse( pv, psz_p, tout, sp ) : txn_parse_lds( lds + pb, psz_p, tout, sp );
    *(u16 *)(dst + FD_VERIFY_HIP_TXNM_TXN_T_SZ_OFF) = (u16)tsz;
    nsig = tsz ? sp.nsig : 0u;
    if( fdesc ) fdesc[j] = (u64)cend | ((u64)psz << 12) | ((u64)tsz << 23) | ((u64)gossip << 33) | ((u64)bad << 34);
  }
  TXTR( 4 );

  /* 3. expand: records of the group contiguous, in frag order; the range
     is claimed before the tag hash so that the atomic's round trip overlaps
     it */
  u32 rex = 0u, rtot = 0u;
  #pragma unroll
  for( int b = 0; b < 5; b++ ) {                                            /* nsig <= 16 */
    unsigned long long m = __ballot( (nsig >> b) & 1u );
    rex  += __builtin_amdgcn_mbcnt_hi( (u32)(m >> 32), __builtin_amdgcn_mbcnt_lo( (u32)m, 0u ) ) << b;
    rtot += (u32)__popcll( m ) << b;
  }
  u32 base = 0u;
  if( lane == 0u && rtot ) base = atomicAdd( seg + FD_HIP_SEG_CNT_W, rtot );
  if( fl && tsz ) {
    u64 w[8];
    if( glob ) {
      #pragma unroll
      for( int q = 0; q < 8; q++ ) {
        u64 x = 0ul;
        #pragma unroll
        for( u32 k = 0; k < 8u; k++ ) x |= (u64)pv[sp.sig_at + 8u*q + k] << (8u*k);
        w[q] = x;
      }
    } else {
      #pragma unroll
      for( int q = 0; q < 8; q++ )
        w[q] = (u64)lds_ld4( lds, pb + sp.sig_at + 8u*q ) | ((u64)lds_ld4( lds, pb + sp.sig_at + 8u*q + 4u ) << 32);
    }
    tag = xh_hash64( seedv ? seedv[j] : seed, w );                         /* seedv: the service's per-frag seeds */
  }
  base = (u32)__builtin_amdgcn_readfirstlane( (int)base );
  TXTR( 5 );
  u32 lc = nsig;
  if( fl ) {
    if( (ulong)base + rex + nsig > seg_cap ) lc = 0u;                       /* sized 12 per frag: never taken */
    tsz_o[j] = (u16)tsz; tag_o[j] = tag; bid_o[j] = bid;
    first_o[j] = (u32)((ulong)sx * seg_cap + base + rex); cnt_o[j] = (u8)lc;
  }
  base = (u32)((ulong)sx * seg_cap + base);                                 /* the group's first record index */
  u32 const msz = sp.msg_sz, mat = sp.msg_at, aat = sp.acct_at, sat = sp.sig_at;
  /* sig (4 pieces) and pubkey (2 pieces) of each record.  Trip counts are
     wave-uniform: every lane takes part in the __shfl (ds_bpermute) reads
     of the frag lanes' values, whatever its own piece. */
  for( u32 q0 = 0u; q0 < 6u * rtot; q0 += 64u ) {
    u32 q = q0 + lane;
    u32 t = (q * 0xaaabu) >> 18, p = q - 6u * t;                            /* q / 6 (q < 2^17) */
    u32 f = group_of<F>( rex, t );
    u32 k = t - __shfl( rex, (int)f ), flc = __shfl( lc, (int)f );
    u32 fs = __shfl( sat, (int)f ), fa = __shfl( aat, (int)f ), fpb = __shfl( pb, (int)f );
    u32 at = p < 4u ? fs + 64u*k + 16u*p : fa + 32u*k + 16u*(p - 4u);       /* payload offset of the piece */
    bool live = q < 6u * rtot && k < flc;                                   /* k >= flc: a capped frag */
    uint4 v;
    if( glob ) {
      u32 fsl = __shfl( src_lo, (int)f ), fsh = __shfl( src_hi, (int)f ), fce = __shfl( cend, (int)f );
      u32 fhl = __shfl( (u32)(u64)hdst, (int)f ), fhh = __shfl( (u32)((u64)hdst >> 32), (int)f );
      pay_view const fp = { { (u8 const *)(((u64)fsh << 32) | (u64)fsl), (u8 const *)(((u64)fhh << 32) | (u64)fhl),
                              fce } };
      u32 w[4] = { 0u, 0u, 0u, 0u };
      if( live )
        for( u32 x = 0; x < 16u; x++ ) w[x >> 2] |= fp[at + x] << (8u*(x & 3u));
      v = make_uint4( w[0], w[1], w[2], w[3] );
    } else {
      v = live ? lds_ld16u( lds, fpb + at ) : make_uint4( 0u, 0u, 0u, 0u );
    }
    if( live && !(FD_TXNM_ABLATE & 8) ) {
      ulong r = (ulong)base + t;
      if( p < 4u ) *(uint4 *)(rsig + 64ul*r + 16u*p) = v;
      else         *(uint4 *)(rpub + 32ul*r + 16u*(p - 4u)) = v;
    }
  }
  for( u32 t0 = 0u; t0 < rtot; t0 += 64u ) {
    u32 t = t0 + lane;
    u32 f = group_of<F>( rex, t );
    u32 k = t - __shfl( rex, (int)f ), flc = __shfl( lc, (int)f );
    u32 fo = __shfl( oc, (int)f ), fm = __shfl( mat, (int)f ), fz = __shfl( msz, (int)f );
    if( t < rtot && k < flc ) {
      ulong r = (ulong)base + t;
      rmoff[r] = 64u * fo + FD_VERIFY_HIP_TXNM_SZ + fm; rmsz[r] = fz;
    }
  }
  TXTR( 6 );
  /* block-count histogram: one atomic per distinct key in the group, on the
     segment's histogram line */
  u32 key = fd_hip_msg_key( msz );
  bool has = fl && lc;
  u32 * hc = seg + FD_HIP_SEG_HIST_W;
  for( unsigned long long pend = __ballot( has ); pend; ) {
    u32 k0 = (u32)__builtin_amdgcn_readlane( (int)key, (int)__builtin_ctzll( pend ) );
    bool mine = has && key == k0;
    unsigned long long mm = __ballot( mine );
    u32 c = 0u;
    #pragma unroll
    for( int b = 0; b < 5; b++ ) c += (u32)__popcll( __ballot( mine && ((lc >> b) & 1u) ) ) << b;
    if( lane == 0u ) atomicAdd( hc + k0, c );
    pend &= ~mm;
  }
  /* ingest byte accounting (fd_verify_hip_tile_ingest_stats): in-frag bytes
     during_frag reads (low word) and writes (high word), one 64-bit atomic
     per group on its segment's counter line */
  u32 rd = fl && !bad ? (gossip ? psz : sz) : 0u, wr = cend > lo ? cend - lo : 0u;
  u64 acc = 0ul;
  #pragma unroll
  for( int g = 0; g < F; g++ )
    acc += (u64)(u32)__builtin_amdgcn_readlane( (int)rd, g ) | ((u64)(u32)__builtin_amdgcn_readlane( (int)wr, g ) << 32);
  if( lane == 0u ) atomicAdd( (unsigned long long *)(seg + SEG_BYTES_W), (unsigned long long)acc );
  TXTR( 7 );
}

/* Out staging's last step: frag j's staging bytes to the out dcache, only
   those the reference writes there (fd_verify_tile.c:64-99 and :118-120):
   during_frag's copy [0, cend) -- for a gossip vote the header fields and
   the payload [80, 80 + payload_sz) -- txn_t_sz, and the fd_txn_t at
   fd_txn_m_txn_t; every other byte of the out chunk keeps its value.  One
   wave per frag, a 16-byte piece per lane: whole pieces as one store
   (coalesced across the wave), the edge pieces by dword and byte. */
DEVI u32 piece_mask( u32 p0, u32 a, u32 b ) {               /* bytes of [p0, p0+16) in [a, b), as a 16-bit mask */
  u32 lo = a > p0 ? a - p0 : 0u, hi = b < p0 + 16u ? (b > p0 ? b - p0 : 0u) : 16u;
  return hi > lo ? ((0xffffu >> (16u - (hi - lo))) << lo) & 0xffffu : 0u;
}

__global__ __launch_bounds__(256)
void k_out_flush( ulong n, u8 const * __restrict__ stage, u32 const * __restrict__ stage_chunk, u8 * hout,
                  u32 const * __restrict__ hout_chunk, u64 const * __restrict__ fdesc ) {
  ulong const j = (ulong)blockIdx.x * 4ul + (threadIdx.x >> 6);
  u32 const lane = threadIdx.x & 63u;
  if( j >= n ) return;
  u64 const d = fdesc[j];
  u32 const cend = (u32)(d & 0xfffu), psz = (u32)((d >> 12) & 0x7ffu), tsz = (u32)((d >> 23) & 0x3ffu);
  bool const gossip = (d >> 33) & 1u, bad = (d >> 34) & 1u;
  if( bad ) return;                                          /* the tile aborts on it (or skips it as overrun) */
  u32 const to = (FD_VERIFY_HIP_TXNM_SZ + psz + (FD_VERIFY_HIP_TXN_ALIGN - 1u)) & ~(FD_VERIFY_HIP_TXN_ALIGN - 1u);
  u32 const end = max( max( cend, 12u ), tsz ? to + tsz : 0u );
  u8 const * s = stage + 64ul * stage_chunk[j];
  u8 *       h = hout  + 64ul * hout_chunk[j];
  for( u32 p0 = 16u * lane; p0 < end; p0 += 1024u ) {
    u32 m = piece_mask( p0, FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF + 2u, FD_VERIFY_HIP_TXNM_TXN_T_SZ_OFF + 2u );  /* txn_t_sz */
    if( gossip ) {
      m |= piece_mask( p0, FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF, FD_VERIFY_HIP_TXNM_SRC_TPU_OFF + 1u );   /* psz .. source_tpu */
      m |= piece_mask( p0, FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF, FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF + 8u );
      m |= piece_mask( p0, FD_VERIFY_HIP_TXNM_SZ, cend );
    } else {
      m |= piece_mask( p0, 0u, cend );
    }
    if( tsz ) m |= piece_mask( p0, to, to + tsz );
    if( !m ) continue;
    uint4 const v = *(uint4 const *)(s + p0);
    if( m == 0xffffu ) { *(uint4 *)(h + p0) = v; continue; }
    u32 const w[4] = { v.x, v.y, v.z, v.w };
    #pragma unroll
    for( u32 k = 0; k < 4u; k++ ) {
      u32 mk = (m >> (4u*k)) & 0xfu;
      if( mk == 0xfu ) { *(u32 *)(h + p0 + 4u*k) = w[k]; continue; }
      #pragma unroll
      for( u32 b = 0; b < 4u; b++ ) if( (mk >> b) & 1u ) h[p0 + 4u*k + b] = (u8)(w[k] >> (8u*b));
    }
  }
}

extern "C" int
fd_txn_hip_parse_dev( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_pool, uint const * d_txn_off,
                      ushort const * d_txn_sz, uchar * d_txn_out, ushort * d_txn_t_sz, void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)fd_ed25519_hip_ctx_stream( ctx );
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( ctx ) ) );
  if( !n ) return 0;
  parse_out po = { d_txn_t_sz, 0, 0, 0, 0, 0, 0 };
  hipLaunchKernelGGL( k_txn_parse, dim3( (unsigned)((n + 255)/256) ), dim3( 256 ), 0, s,
                      n, d_pool, d_txn_off, d_txn_sz, d_txn_out, (u64)0, po, (u32 const *)0 );
  TX_CHECK( hipGetLastError() );
  return 0;
}

/**********************************************************************/
/* tcache (fd_tcache.h:115-410) on the reference memory layout          */

static inline ulong tc_probe( ulong const * map, ulong map_cnt, ulong tag, int & found ) {
  ulong m = map_cnt - 1, i = tag & m;
  for( ;; ) {
    ulong t = map[i];
    if( t == tag ) { found = 1; return i; }
    if( !t )       { found = 0; return i; }
    i = (i + 1) & m;
  }
}

static inline void tc_remove( ulong * map, ulong map_cnt, ulong tag ) {
  if( !tag ) return;
  int f; ulong hole = tc_probe( map, map_cnt, tag, f );
  if( !f ) return;
  ulong m = map_cnt - 1;
  for( ;; ) {
    map[hole] = 0;
    ulong s = hole;
    for( ;; ) {
      s = (s + 1) & m;
      ulong t = map[s];
      if( !t ) return;
      ulong home = t & m;
      bool chained = hole <= s ? (home > hole && home <= s) : (home > hole || home <= s);
      if( !chained ) { map[hole] = t; hole = s; break; }
    }
  }
}

extern "C" ulong fd_verify_hip_tcache_map_cnt_default( ulong depth ) {
  if( !depth || depth == ~0ul ) return 0;
  int lg = 63 - __builtin_clzl( depth + 1 ) + 2;     /* FD_TCACHE_SPARSE_DEFAULT */
  return lg > 63 ? 0 : 1ul << lg;
}

extern "C" ulong fd_verify_hip_tcache_reset( ulong * ring, ulong depth, ulong * map, ulong map_cnt ) {
  memset( ring, 0, depth*sizeof(ulong) ); memset( map, 0, map_cnt*sizeof(ulong) );
  return 0;
}

extern "C" int fd_verify_hip_tcache_query( ulong const * map, ulong map_cnt, ulong tag ) {
  int f; tc_probe( map, map_cnt, tag, f ); return f;
}

extern "C" int fd_verify_hip_tcache_insert( ulong * oldest, ulong * ring, ulong depth, ulong * map,
                                            ulong map_cnt, ulong tag ) {
  int f; ulong slot = tc_probe( map, map_cnt, tag, f );
  if( f ) return 1;
  map[slot] = tag;
  ulong o = *oldest, ev = ring[o];
  ring[o] = tag;
  *oldest = o + 1 >= depth ? 0 : o + 1;
  tc_remove( map, map_cnt, ev );
  return 0;
}

/**********************************************************************/
/* verify tile engine                                                  */

struct tile_slot {
  ulong         n, nsig;
  /* per frag, device */
  u16 *         d_tsz; u8 * d_nsig; u32 * d_sig_at; u32 * d_acct_at; u32 * d_msg_at; u32 * d_msg_sz;
  u64 *         d_tag; u32 * d_first; u8 * d_cnt; signed char * d_tcode; u32 * d_counter;
  /* per signature record, device (grown on demand) */
  ulong         rcap;
  u8 *          d_rsig; u8 * d_rpub; u32 * d_rmoff; u32 * d_rmsz; signed char * d_rcode;
  /* per frag results, packed (k_tile_results): device and pinned host */
  u8 *          d_res; u8 * h_res;
  /* fd_txn_m_t frag mode (submit_frags): payload spans, fd_txn_t offsets,
     header bundle ids, in kinds and the corrupt-frag flag */
  u32 *         d_pay_off; u16 * d_pay_sz; u32 * d_tout; u64 * d_bid; u32 * d_flag;
  u32 *         d_misc;     /* counter, flag, record segments (SLOT_MISC_*) */
  /* mcache range mode (submit_range): the frag list k_range_gather builds
     from the in link's mcache lines, and each frag's tsorig (device, host) */
  u32 *         d_rin; u16 * d_rsz; u8 * d_rkind; u32 * d_tso; u32 * h_tso;
  int           range;
  /* out staging (set_staging): staging frags (STAGE_CHUNKS 64-B chunks
     each, frag j at chunk STAGE_CHUNKS*j) and k_out_flush's descriptors */
  u8 *          d_stage; u32 * d_stage_chunk; u64 * d_fdesc;
  fd_ed25519_hip_ctx_t * ctx;   /* the verify context (stream and scratch) the slot's batches run on */
  int           own_ctx;    /* created by set_inflight: batches of different slots run concurrently */
  u32           n_seg;      /* the last batch's record segments (0: not k_txnm_batch) */
  hipEvent_t    ev_ing0, ev_ing1;   /* around the ingest kernel (ingest timing) */
  int           ing_timed;
  int           frags;
  hipEvent_t    ev_start, ev_done;
  /* out staging: k_out_flush runs on a stream of its own beside the verify
     (it needs only k_txnm_batch's staging frags), joined before ev_done */
  hipStream_t   st_flush; hipEvent_t ev_fork, ev_join;
  int           busy;
};

/* batch latency histograms in fd_histf's shape (src/util/hist/fd_histf.h:
   16 buckets, [0,min) and [max,inf) at the ends, integer edges growing
   geometrically between, no bucket empty) */
#define HIST_B FD_VERIFY_HIP_HIST_BUCKET_CNT
struct lat_hist { ulong counts[HIST_B]; ulong edge[HIST_B]; ulong sum; };

/* the edges fd_histf_new computes (fd_histf.h:88-118): each interior edge
   spreads the remaining ratio max/edge over the buckets left, rounded and
   kept above the previous edge */
extern "C" int fd_verify_hip_hist_edges( ulong min_v, ulong max_v, ulong edge[ HIST_B ] ) {
  if( max_v <= min_v ) return -1;
  if( min_v < 1ul ) min_v = 1ul;
  if( max_v < min_v + HIST_B - 2ul ) max_v = min_v + HIST_B - 2ul;
  edge[0] = 0ul; edge[1] = min_v;
  for( ulong i = 2; i < HIST_B - 1ul; i++ ) {
    double prev = (double)edge[i-1];
    ulong e = (ulong)(0.5 + prev * pow( (double)max_v / prev, 1.0 / (double)(HIST_B - i) ));
    edge[i] = e > edge[i-1] ? e : edge[i-1] + 1ul;
  }
  edge[HIST_B-1] = max_v;
  return 0;
}

static void hist_sample( lat_hist & h, ulong v ) {
  h.sum += v;
  ulong b = HIST_B - 1ul;
  while( v < h.edge[b] ) b--;                     /* edge[0] == 0 stops it */
  h.counts[b]++;
}

struct fd_verify_hip_tile {
  fd_ed25519_hip_ctx_t * ctx;
  ulong      max_txn, seed;
  /* tcache: the tile's own, or the caller's (join_tcache) */
  ulong *    own_mem;
  ulong      own_oldest;
  ulong *    oldest; ulong * ring; ulong depth; ulong * map; ulong map_cnt;
  /* bundle state (fd_verify_ctx_t bundle_failed / bundle_id) */
  int        bundle_failed; ulong bundle_id;
  ulong      m_parse, m_verify, m_dedup, m_bundle, m_pub, m_sigs, m_gossip;
  tile_slot  slot[FD_VERIFY_HIP_INFLIGHT_MAX];
  ulong      nslot;          /* batches in flight at most: the slot ring (fd_verify_hip_tile_set_inflight; 2) */
  ulong      nalloc;         /* slots allocated */
  ulong      submitted, completed;
  int        ingest_split;   /* FD_VERIFY_HIP_INGEST=split: the three-kernel frag ingest (A/B runs) */
  int        fb;             /* k_txnm_batch frags per workgroup (FD_VERIFY_HIP_FB: 8 or 16) */
  int        ingest_timing;  /* fd_verify_hip_tile_set_ingest_timing */
  int        staging;        /* fd_verify_hip_tile_set_staging */
  double     last_ingest[4]; /* fd_verify_hip_tile_ingest_stats */
  double     last_gpu_ms, last_host_ms, last_sigs;
  lat_hist   hist[2];        /* batch latency: GPU, host pass (ns) */
};

static void slot_alloc( tile_slot & s, ulong n ) {
  memset( &s, 0, sizeof(s) );
  TX_CHECK( hipMalloc( &s.d_tsz, 2*n ) );     TX_CHECK( hipMalloc( &s.d_nsig, n ) );
  TX_CHECK( hipMalloc( &s.d_sig_at, 4*n ) );  TX_CHECK( hipMalloc( &s.d_acct_at, 4*n ) );
  TX_CHECK( hipMalloc( &s.d_msg_at, 4*n ) );  TX_CHECK( hipMalloc( &s.d_msg_sz, 4*n ) );
  TX_CHECK( hipMalloc( &s.d_tag, 8*n ) );     TX_CHECK( hipMalloc( &s.d_first, 4*n ) );
  TX_CHECK( hipMalloc( &s.d_cnt, n ) );       TX_CHECK( hipMalloc( &s.d_tcode, n ) );
  TX_CHECK( hipMalloc( &s.d_misc, SLOT_MISC_BYTES ) );
  TX_CHECK( hipMemset( s.d_misc, 0, SLOT_MISC_BYTES ) );
  s.d_counter = s.d_misc; s.d_flag = s.d_misc + 1;
  TX_CHECK( hipMalloc( &s.d_res, TILE_RES_HDR + 24*n ) );  TX_CHECK( hipHostMalloc( &s.h_res, TILE_RES_HDR + 24*n, 0 ) );
  TX_CHECK( hipMalloc( &s.d_pay_off, 4*n ) );     TX_CHECK( hipMalloc( &s.d_pay_sz, 2*n ) );
  TX_CHECK( hipMalloc( &s.d_tout, 4*n ) );        TX_CHECK( hipMalloc( &s.d_bid, 8*n ) );
  TX_CHECK( hipMalloc( &s.d_rin, 4*n ) );         TX_CHECK( hipMalloc( &s.d_rsz, 2*n ) );
  TX_CHECK( hipMalloc( &s.d_rkind, n ) );         TX_CHECK( hipMalloc( &s.d_tso, 4*n ) );
  TX_CHECK( hipHostMalloc( &s.h_tso, 4*n, 0 ) );
  TX_CHECK( hipEventCreate( &s.ev_start ) ); TX_CHECK( hipEventCreate( &s.ev_done ) );
  TX_CHECK( hipEventCreate( &s.ev_ing0 ) ); TX_CHECK( hipEventCreate( &s.ev_ing1 ) );
  TX_CHECK( hipStreamCreateWithFlags( &s.st_flush, hipStreamNonBlocking ) );
  TX_CHECK( hipEventCreateWithFlags( &s.ev_fork, hipEventDisableTiming ) );
  TX_CHECK( hipEventCreateWithFlags( &s.ev_join, hipEventDisableTiming ) );
}

static void slot_free_records( tile_slot & s ) {
  (void)hipFree( s.d_rsig ); (void)hipFree( s.d_rpub ); (void)hipFree( s.d_rmoff );
  (void)hipFree( s.d_rmsz ); (void)hipFree( s.d_rcode );
  s.d_rsig = s.d_rpub = 0; s.d_rmoff = s.d_rmsz = 0; s.d_rcode = 0; s.rcap = 0;
}

static void slot_records( tile_slot & s, ulong need ) {   /* (re)size the per-signature record buffers */
  slot_free_records( s );
  TX_CHECK( hipMalloc( &s.d_rsig, 64*need ) ); TX_CHECK( hipMalloc( &s.d_rpub, 32*need ) );
  TX_CHECK( hipMalloc( &s.d_rmoff, 4*need ) ); TX_CHECK( hipMalloc( &s.d_rmsz, 4*need ) );
  TX_CHECK( hipMalloc( &s.d_rcode, need ) );
  s.rcap = need;
}

#define STAGE_CHUNKS 34ul   /* FD_TPU_PARSED_MTU (2168 B) in 64-B chunks */

static void slot_stage_alloc( tile_slot & s, ulong n ) {
  if( s.d_stage ) return;
  TX_CHECK( hipMalloc( &s.d_stage, 64ul*STAGE_CHUNKS*n ) );
  TX_CHECK( hipMalloc( &s.d_stage_chunk, 4ul*n ) );
  TX_CHECK( hipMalloc( &s.d_fdesc, 8ul*n ) );
  u32 * h = (u32 *)malloc( 4ul*n );
  for( ulong j = 0; j < n; j++ ) h[j] = (u32)(STAGE_CHUNKS*j);
  TX_CHECK( hipMemcpy( s.d_stage_chunk, h, 4ul*n, hipMemcpyHostToDevice ) );
  free( h );
}

static void slot_free( tile_slot & s ) {
  (void)hipFree( s.d_stage ); (void)hipFree( s.d_stage_chunk ); (void)hipFree( s.d_fdesc );
  (void)hipFree( s.d_tsz ); (void)hipFree( s.d_nsig ); (void)hipFree( s.d_sig_at ); (void)hipFree( s.d_acct_at );
  (void)hipFree( s.d_msg_at ); (void)hipFree( s.d_msg_sz ); (void)hipFree( s.d_tag ); (void)hipFree( s.d_first );
  (void)hipFree( s.d_cnt ); (void)hipFree( s.d_tcode ); (void)hipFree( s.d_misc );
  (void)hipFree( s.d_res ); (void)hipHostFree( s.h_res );
  (void)hipFree( s.d_pay_off ); (void)hipFree( s.d_pay_sz ); (void)hipFree( s.d_tout ); (void)hipFree( s.d_bid );
  (void)hipFree( s.d_rin ); (void)hipFree( s.d_rsz ); (void)hipFree( s.d_rkind ); (void)hipFree( s.d_tso );
  (void)hipHostFree( s.h_tso );
  (void)hipEventDestroy( s.ev_start ); (void)hipEventDestroy( s.ev_done );
  (void)hipEventDestroy( s.ev_ing0 ); (void)hipEventDestroy( s.ev_ing1 );
  (void)hipStreamSynchronize( s.st_flush ); (void)hipStreamDestroy( s.st_flush );
  (void)hipEventDestroy( s.ev_fork ); (void)hipEventDestroy( s.ev_join );
  slot_free_records( s );
}

__global__ __launch_bounds__(256)
void k_tile_results( ulong n, u16 const * __restrict__ tsz, signed char const * __restrict__ tcode,
                     u64 const * __restrict__ tag, u64 const * __restrict__ bid, u8 const * __restrict__ kind,
                     u32 const * __restrict__ counter, u32 const * __restrict__ flag, u32 n_seg,
                     u8 const * __restrict__ out, u32 const * __restrict__ out_chunk, u64 const * __restrict__ fdesc,
                     u8 * __restrict__ res );

/* a slot's record buffers at their bound and the results kernel loaded (a
   tile is created in privileged_init: its sandboxed steady state allocates
   nothing and loads no code) */
static void slot_warm( tile_slot & s, ulong max_txn, hipStream_t st ) {
  slot_records( s, 12ul*(max_txn + SLOT_SEG_SLACK) );
  hipLaunchKernelGGL( k_tile_results, dim3( 1 ), dim3( 64 ), 0, st, 0ul, s.d_tsz, s.d_tcode, s.d_tag,
                      (u64 const *)0, (u8 const *)0, s.d_counter, (u32 const *)0, 0u, (u8 const *)0,
                      (u32 const *)0, (u64 const *)0, s.d_res );
  TX_CHECK( hipGetLastError() );
}

extern "C" fd_verify_hip_tile_t *
fd_verify_hip_tile_new( fd_ed25519_hip_ctx_t * ctx, ulong max_txn, ulong seed, ulong depth, ulong map_cnt ) {
  if( !ctx || !max_txn || !depth ) return 0;
  if( !map_cnt ) map_cnt = fd_verify_hip_tcache_map_cnt_default( depth );
  if( !map_cnt || (map_cnt & (map_cnt - 1)) || map_cnt < depth + 2 ) return 0;
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( ctx ) ) );
  fd_ed25519_hip_ctx_reserve( ctx, 12ul*(max_txn + SLOT_SEG_SLACK) );   /* one verify launch pair per batch */
  fd_verify_hip_tile_t * t = (fd_verify_hip_tile_t *)calloc( 1, sizeof(fd_verify_hip_tile_t) );
  t->ctx = ctx; t->max_txn = max_txn; t->seed = seed;
  {
    char const * e = getenv( "FD_VERIFY_HIP_INGEST" );
    t->ingest_split = e && !strcmp( e, "split" );
    char const * f = getenv( "FD_VERIFY_HIP_FB" );
    t->fb = f && atoi( f ) == 8 ? 8 : 16;
  }
  t->own_mem = (ulong *)malloc( sizeof(ulong)*(depth + map_cnt) );
  t->oldest = &t->own_oldest; t->ring = t->own_mem; t->depth = depth; t->map = t->own_mem + depth; t->map_cnt = map_cnt;
  t->own_oldest = fd_verify_hip_tcache_reset( t->ring, depth, t->map, map_cnt );
  t->nslot = t->nalloc = 2ul;
  slot_alloc( t->slot[0], max_txn ); slot_alloc( t->slot[1], max_txn );
  t->slot[0].ctx = t->slot[1].ctx = ctx;                  /* one stream: the two batches run back to back */
  fd_verify_hip_tile_hist_init( t, 10000ul, 1000000000ul );   /* 10 us .. 1 s */
  /* Everything the batch path would otherwise do lazily, done now: record
     buffers at their bound (12 signatures per frag) and this module's code
     object loaded (the runtime loads a translation unit's kernels at their
     first launch: file opens and NUMA queries).  A tile creates this in
     privileged_init, so its sandboxed steady state needs neither
     (integration/fd_verify_tile_hip.patch, verify_hip_seccomp). */
  hipStream_t st = (hipStream_t)fd_ed25519_hip_ctx_stream( ctx );
  for( int k = 0; k < 2; k++ ) slot_warm( t->slot[k], max_txn, st );
  TX_CHECK( hipStreamSynchronize( st ) );
  {
    /* one empty-payload frag through the whole batch path (ingest, parse,
       expansion, verify launches, reduce, results, completion), then the
       counters reset: the first real batch finds nothing left to set up */
    u8 * d = 0;
    TX_CHECK( hipMalloc( &d, 512 ) );
    TX_CHECK( hipMemset( d, 0, 512 ) );
    u32 * d_chunk = (u32 *)(d + 256); u16 * d_sz = (u16 *)(d + 260); u8 * d_kind = d + 262;
    u16 const hsz = (u16)FD_VERIFY_HIP_TXNM_SZ;
    TX_CHECK( hipMemcpy( d_sz, &hsz, 2, hipMemcpyHostToDevice ) );
    signed char r = 0;
    if( fd_verify_hip_tile_submit_frags( t, 1, d, d_chunk, d_sz, d_kind, d + 128, d_chunk ) ||
        fd_verify_hip_tile_complete( t, NULL, &r, NULL, NULL ) || r != FD_VERIFY_HIP_FRAG_PARSE_FAIL ) {
      fprintf( stderr, "fd_verify_hip: tile warm-up batch failed (%d)\n", (int)r );
      abort();
    }
    TX_CHECK( hipFree( d ) );
    t->m_parse = t->m_verify = t->m_dedup = t->m_bundle = t->m_pub = t->m_sigs = t->m_gossip = 0;
    t->bundle_failed = 0; t->bundle_id = 0;
    fd_verify_hip_tile_hist_init( t, 10000ul, 1000000000ul );
  }
  return t;
}

extern "C" int fd_verify_hip_tile_hist_init( fd_verify_hip_tile_t * t, ulong min_ns, ulong max_ns ) {
  ulong edge[HIST_B];
  if( fd_verify_hip_hist_edges( min_ns, max_ns, edge ) ) return -1;
  for( int w = 0; w < 2; w++ ) {
    memset( &t->hist[w], 0, sizeof(lat_hist) );
    memcpy( t->hist[w].edge, edge, sizeof(edge) );
  }
  return 0;
}

extern "C" int fd_verify_hip_tile_hist( fd_verify_hip_tile_t const * t, int which, ulong counts[ HIST_B ],
                                        ulong left_edge_ns[ HIST_B ], ulong * sum_ns ) {
  if( which < 0 || which > 1 ) return -1;
  lat_hist const & h = t->hist[which];
  if( counts )       memcpy( counts, h.counts, sizeof(h.counts) );
  if( left_edge_ns ) memcpy( left_edge_ns, h.edge, sizeof(h.edge) );
  if( sum_ns )       *sum_ns = h.sum;
  return 0;
}

extern "C" void
fd_verify_hip_tile_join_tcache( fd_verify_hip_tile_t * t, ulong * sync, ulong * ring, ulong depth, ulong * map,
                                ulong map_cnt ) {
  t->oldest = sync; t->ring = ring; t->depth = depth; t->map = map; t->map_cnt = map_cnt;
}

extern "C" void fd_verify_hip_tile_tcache_reset( fd_verify_hip_tile_t * t ) {
  *t->oldest = fd_verify_hip_tcache_reset( t->ring, t->depth, t->map, t->map_cnt );
}

extern "C" void fd_verify_hip_tile_set_seed( fd_verify_hip_tile_t * t, ulong seed ) { t->seed = seed; }

extern "C" void fd_verify_hip_tile_delete( fd_verify_hip_tile_t * t ) {
  if( !t ) return;
  (void)hipSetDevice( fd_ed25519_hip_ctx_device( t->ctx ) );
  (void)hipStreamSynchronize( (hipStream_t)fd_ed25519_hip_ctx_stream( t->ctx ) );
  for( ulong k = 0; k < t->nalloc; k++ ) {
    if( t->slot[k].own_ctx ) (void)hipStreamSynchronize( (hipStream_t)fd_ed25519_hip_ctx_stream( t->slot[k].ctx ) );
    slot_free( t->slot[k] );
    if( t->slot[k].own_ctx ) fd_ed25519_hip_ctx_delete( t->slot[k].ctx );
  }
  free( t->own_mem ); free( t );
}

/* Per-frag results to the host as one packed array and one D2H copy per
   batch (instead of one hipMemcpyAsync per field array, each a blit kernel
   on the tile's stream): k_tile_results packs txn_t_sz, per-txn code, tag
   and, in frag mode, the header bundle id and in kind into 24-byte records
   behind a 16-byte header (record count, corrupt-frag flag).  Writing the
   fields into mapped host memory from the kernel instead measured slower
   (C4 99.7 / 75.1 vs 102-104M verifies/s: small PCIe writes from a kernel
   that holds CU slots). */

__global__ __launch_bounds__(256)
void k_tile_results( ulong n, u16 const * __restrict__ tsz, signed char const * __restrict__ tcode,
                     u64 const * __restrict__ tag, u64 const * __restrict__ bid, u8 const * __restrict__ kind,
                     u32 const * __restrict__ counter, u32 const * __restrict__ flag, u32 n_seg,
                     u8 const * __restrict__ out, u32 const * __restrict__ out_chunk, u64 const * __restrict__ fdesc,
                     u8 * __restrict__ res ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j == 0ul ) {
    ((u32 *)res)[0] = *counter; ((u32 *)res)[1] = flag ? *flag : 0u;
    u64 rd = 0ul, wr = 0ul;
    for( u32 x = 0; x < n_seg; x++ ) {                       /* k_txnm_batch: flag = misc + 1, segments after */
      u64 b = *(u64 const *)(flag - 1 + 32u + x*FD_HIP_SEG_STRIDE + SEG_BYTES_W);
      rd += b & 0xffffffffull; wr += b >> 32;
    }
    ((u64 *)res)[2] = rd; ((u64 *)res)[3] = wr;
  }
  if( j >= n ) return;
  tile_res r;
  r.tag = tag[j]; r.bid = bid ? bid[j] : 0ul; r.tsz = tsz[j]; r.tcode = tcode[j]; r.kind = kind ? kind[j] : 0u;
  if( fdesc && ((fdesc[j] >> 34) & 1u) ) r.kind |= (u8)TILE_RES_BAD;   /* this frag is corrupt (out staging) */
  /* frag mode: the out header's payload_sz (after the GPU's own during_frag),
     for the caller's fd_txn_m_realized_footprint */
  r.pad = fdesc ? (u32)((fdesc[j] >> 12) & 0x7ffu)
        : out   ? (u32)*(u16 const *)(out + 64ul*out_chunk[j] + FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF) : 0u;
  *(tile_res *)(res + TILE_RES_HDR + 24ul*j) = r;
}

/* the part of a batch both submit forms share: record capacity, expansion,
   verify, per-txn reduce and the D2H of the per-frag results; the payloads
   are pool[ off[j], +sz[j] ) after k_txn_parse has filled the slot */
static void
submit_verify( fd_verify_hip_tile_t * t, tile_slot & s, hipStream_t st, ulong n, uchar const * d_pool ) {
  dim3 grid( (unsigned)((n + 255)/256) ), blk( 256 );
  /* record capacity: a parsed frag carries at most 12 signatures (96 B of
     sig + pubkey each within FD_TXN_MTU, fd_txn.h:68); grow to that bound
     once instead of reading the count back twice */
  ulong need = 12ul * n;
  if( s.rcap < need ) {                                    /* n <= max_txn: sized at tile_new */
    TX_CHECK( hipStreamSynchronize( st ) );
    slot_records( s, need );
  }
  TX_CHECK( hipMemsetAsync( s.d_counter, 0, 4, st ) );
  hipLaunchKernelGGL( k_txn_expand, grid, blk, 0, st, n, d_pool, s.d_nsig, s.d_sig_at, s.d_acct_at, s.d_msg_at,
                      s.d_msg_sz, s.d_counter, s.d_first, s.d_cnt, s.d_rsig, s.d_rpub, s.d_rmoff, s.d_rmsz, s.rcap );
  TX_CHECK( hipGetLastError() );
  /* the record count stays on the device: no host round trip between the
     expansion and the verify, so submit never waits on the GPU */
  fd_ed25519_hip_verify_dev_count( s.ctx, need, s.d_counter, s.d_rsig, s.d_rpub, d_pool, s.d_rmoff, s.d_rmsz,
                                   s.d_rcode, NULL, st );
  fd_ed25519_hip_group_reduce_dev( s.ctx, n, s.d_first, s.d_cnt, s.d_rcode, s.d_tcode, st );
}

static void
submit_results( tile_slot & s, hipStream_t st, ulong n, uchar const * d_in_kind, uchar const * d_out = 0,
                uint const * d_out_chunk = 0, u64 const * fdesc = 0 ) {
  hipLaunchKernelGGL( k_tile_results, dim3( (unsigned)((n + 255)/256) ), dim3( 256 ), 0, st, n, s.d_tsz, s.d_tcode,
                      s.d_tag, s.frags ? s.d_bid : (u64 const *)0, (u8 const *)d_in_kind, s.d_counter,
                      s.frags ? s.d_flag : (u32 const *)0, s.n_seg, (u8 const *)d_out, (u32 const *)d_out_chunk,
                      fdesc, s.d_res );
  TX_CHECK( hipGetLastError() );
  TX_CHECK( hipMemcpyAsync( s.h_res, s.d_res, TILE_RES_HDR + 24ul*n, hipMemcpyDeviceToHost, st ) );
}

static tile_slot *
submit_begin( fd_verify_hip_tile_t * t, ulong n, hipStream_t & st, int & rc ) {
  rc = 0;
  if( n > t->max_txn ) { rc = -1; return 0; }
  tile_slot & s = t->slot[t->submitted % t->nslot];
  if( s.busy ) { rc = -2; return 0; }                        /* two batches outstanding */
  st = (hipStream_t)fd_ed25519_hip_ctx_stream( s.ctx );
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( s.ctx ) ) );
  s.n = n; s.nsig = 0; s.busy = 1; s.frags = 0; s.range = 0; s.ing_timed = 0; s.n_seg = 0; t->submitted++;
  TX_CHECK( hipEventRecord( s.ev_start, st ) );
  return &s;
}

extern "C" int
fd_verify_hip_tile_submit( fd_verify_hip_tile_t * t, ulong n, uchar const * d_pool, uint const * d_txn_off,
                           ushort const * d_txn_sz, uchar * d_txn_out ) {
  hipStream_t st; int rc;
  tile_slot * sp = submit_begin( t, n, st, rc );
  if( !sp ) return rc;
  tile_slot & s = *sp;
  if( !n ) { TX_CHECK( hipEventRecord( s.ev_done, st ) ); return 0; }
  dim3 grid( (unsigned)((n + 255)/256) ), blk( 256 );
  parse_out po = { s.d_tsz, s.d_nsig, s.d_sig_at, s.d_acct_at, s.d_msg_at, s.d_msg_sz, s.d_tag };
  hipLaunchKernelGGL( k_txn_parse, grid, blk, 0, st, n, d_pool, d_txn_off, d_txn_sz, d_txn_out, (u64)t->seed, po,
                      (u32 const *)0 );
  TX_CHECK( hipGetLastError() );
  submit_verify( t, s, st, n, d_pool );
  submit_results( s, st, n, (uchar const *)0 );
  TX_CHECK( hipEventRecord( s.ev_done, st ) );
  return 0;
}

/* a frag batch after submit_begin, n > 0: ingest (copy, parse, records),
   verify, per-txn reduce and the results D2H on the slot's stream */
static void
submit_frags_body( fd_verify_hip_tile_t * t, tile_slot & s, hipStream_t st, ulong n, uchar const * d_in,
                   uint const * d_in_chunk, ushort const * d_in_sz, uchar const * d_in_kind, uchar * d_out,
                   uint const * d_out_chunk, int misc_zeroed = 0 ) {
  dim3 grid( (unsigned)((n + 255)/256) ), blk( 256 );
  if( t->ingest_split ) {
    /* the three-kernel form (ingest copy, one-lane parse, expansion, then
       k_msg_hist in the verify): kept for A/B runs, FD_VERIFY_HIP_INGEST=split */
    TX_CHECK( hipMemsetAsync( s.d_flag, 0, 4, st ) );
    /* one wave per frag: up to 4 frags per 256-thread workgroup, grid capped */
    ulong wgs = (n + 3ul) / 4ul; if( wgs > 8192ul ) wgs = 8192ul;
    hipLaunchKernelGGL( k_txnm_ingest, dim3( (unsigned)wgs ), blk, 0, st, n, d_in, d_in_chunk, d_in_sz, d_in_kind,
                        d_out, d_out_chunk, s.d_pay_off, s.d_pay_sz, s.d_tout, s.d_bid, s.d_flag );
    TX_CHECK( hipGetLastError() );
    parse_out po = { s.d_tsz, s.d_nsig, s.d_sig_at, s.d_acct_at, s.d_msg_at, s.d_msg_sz, s.d_tag };
    hipLaunchKernelGGL( k_txn_parse, grid, blk, 0, st, n, (u8 const *)d_out, s.d_pay_off, s.d_pay_sz, (u8 *)0,
                        (u64)t->seed, po, s.d_tout );
    TX_CHECK( hipGetLastError() );
    submit_verify( t, s, st, n, d_out );
  } else {
    /* k_txnm_batch: ingest, parse and record expansion in one pass, the
       records in n_seg segments of seg_cap (fd_hip_order.h) */
    ulong F = t->fb == 8 ? 8ul : 16ul, nwg = (n + F - 1ul) / F;
    u32 n_seg = nwg < FB_SEGS ? (u32)nwg : FB_SEGS;
    ulong seg_cap = 12ul * F * ((nwg + n_seg - 1ul) / n_seg);
    ulong need = (ulong)n_seg * seg_cap;                     /* <= 12 x (n + SLOT_SEG_SLACK): sized at tile_new */
    if( s.rcap < need ) { TX_CHECK( hipStreamSynchronize( st ) ); slot_records( s, need ); }
    s.n_seg = n_seg;
    if( !misc_zeroed )                                       /* submit_range: k_range_gather zeroed it */
      TX_CHECK( hipMemsetAsync( s.d_misc, 0, 4ul*(32ul + (ulong)n_seg*FD_HIP_SEG_STRIDE), st ) );
    s.ing_timed = t->ingest_timing;
    if( s.ing_timed ) TX_CHECK( hipEventRecord( s.ev_ing0, st ) );
    /* out staging: the batch works on HBM staging frags, then k_out_flush
       writes the out dcache (pinned host memory) with coalesced stores */
    bool const stg = t->staging;
    uchar *        k_out   = stg ? s.d_stage : d_out;
    uint const *   k_chunk = stg ? s.d_stage_chunk : d_out_chunk;
    u8 const *     h_out   = stg ? (u8 const *)d_out : (u8 const *)0;
    u32 const *    h_chunk = stg ? (u32 const *)d_out_chunk : (u32 const *)0;
    u64 *          fdesc   = stg ? s.d_fdesc : (u64 *)0;
    if( F == 8ul )
      hipLaunchKernelGGL( k_txnm_batch<8>, dim3( (unsigned)nwg ), dim3( 64 ), 0, st, n, d_in,
                          d_in_chunk, d_in_sz, d_in_kind, k_out, k_chunk, (u64)t->seed, s.d_tsz, s.d_tag, s.d_bid,
                          s.d_first, s.d_cnt, s.d_misc, s.d_rsig, s.d_rpub, s.d_rmoff, s.d_rmsz, n_seg, seg_cap,
                          h_out, h_chunk, fdesc, (u64 const *)0 );
    else
      hipLaunchKernelGGL( k_txnm_batch<16>, dim3( (unsigned)nwg ), dim3( 64 ), 0, st, n, d_in,
                          d_in_chunk, d_in_sz, d_in_kind, k_out, k_chunk, (u64)t->seed, s.d_tsz, s.d_tag, s.d_bid,
                          s.d_first, s.d_cnt, s.d_misc, s.d_rsig, s.d_rpub, s.d_rmoff, s.d_rmsz, n_seg, seg_cap,
                          h_out, h_chunk, fdesc, (u64 const *)0 );
    TX_CHECK( hipGetLastError() );
    if( s.ing_timed ) TX_CHECK( hipEventRecord( s.ev_ing1, st ) );
    if( stg ) {                                              /* off the verify's critical path */
      TX_CHECK( hipEventRecord( s.ev_fork, st ) );
      TX_CHECK( hipStreamWaitEvent( s.st_flush, s.ev_fork, 0 ) );
      hipLaunchKernelGGL( k_out_flush, dim3( (unsigned)((n + 3ul)/4ul) ), dim3( 256 ), 0, s.st_flush, n,
                          (u8 const *)k_out, (u32 const *)k_chunk, (u8 *)d_out, (u32 const *)d_out_chunk,
                          (u64 const *)fdesc );
      TX_CHECK( hipGetLastError() );
      TX_CHECK( hipEventRecord( s.ev_join, s.st_flush ) );
    }
    fd_hip_segs_t segs = { s.d_misc + 32u, n_seg, seg_cap, s.d_counter };
    if( fd_ed25519_hip_verify_segs( s.ctx, segs, s.d_rsig, s.d_rpub, k_out, s.d_rmoff, s.d_rmsz, s.d_rcode, st ) ) {
      fprintf( stderr, "fd_verify_hip: segmented verify refused (%u x %lu records)\n", n_seg, seg_cap );
      abort();
    }
    fd_ed25519_hip_group_reduce_dev( s.ctx, n, s.d_first, s.d_cnt, s.d_rcode, s.d_tcode, st );
    submit_results( s, st, n, d_in_kind, k_out, k_chunk, fdesc );
    if( stg ) TX_CHECK( hipStreamWaitEvent( st, s.ev_join, 0 ) );   /* ev_done covers the out dcache writes */
    return;
  }
  submit_results( s, st, n, d_in_kind, d_out, d_out_chunk );
}

/* the frag-batch core for the verify service (fd_txn_hip_int.h): the same
   k_txnm_batch<16> / verify_segs / reduce sequence as submit_frags_body's
   fused path, with per-frag seeds and no host out dcache (the service's
   staging frags are flushed later, fd_verify_svc.hip) */
extern "C" __attribute__((visibility("hidden"))) ulong fd_txn_hip_record_cap( ulong n ) {
  return 12ul * (n + SLOT_SEG_SLACK);
}
extern "C" __attribute__((visibility("hidden"))) ulong fd_txn_hip_misc_bytes( void ) { return SLOT_MISC_BYTES; }

extern "C" __attribute__((visibility("hidden"))) void
fd_txn_hip_batch_core( fd_ed25519_hip_ctx_t * ctx, hipStream_t st, ulong n, u8 const * in, u32 const * in_chunk,
                       u16 const * in_sz, u8 const * in_kind, u8 * out, u32 const * out_chunk, u64 const * seedv,
                       u16 * tsz, u64 * tag, u64 * bid, u32 * first, u8 * cnt, u32 * misc, u8 * rsig, u8 * rpub,
                       u32 * rmoff, u32 * rmsz, ulong rcap, signed char * rcode, signed char * tcode, u64 * fdesc ) {
  if( !n ) return;
  ulong const F = 16ul, nwg = (n + F - 1ul) / F;
  u32 const n_seg = nwg < FB_SEGS ? (u32)nwg : FB_SEGS;
  ulong const seg_cap = 12ul * F * ((nwg + n_seg - 1ul) / n_seg);
  if( (ulong)n_seg * seg_cap > rcap ) {
    fprintf( stderr, "fd_verify_hip: batch core: %lu frags need %lu records, %lu allocated\n", n,
             (ulong)n_seg * seg_cap, rcap );
    abort();
  }
  TX_CHECK( hipMemsetAsync( misc, 0, 4ul*(32ul + (ulong)n_seg*FD_HIP_SEG_STRIDE), st ) );
  hipLaunchKernelGGL( k_txnm_batch<16>, dim3( (unsigned)nwg ), dim3( 64 ), 0, st, n, in, in_chunk, in_sz, in_kind,
                      out, out_chunk, (u64)0, tsz, tag, bid, first, cnt, misc, rsig, rpub, rmoff, rmsz, n_seg, seg_cap,
                      (u8 const *)0, (u32 const *)0, fdesc, seedv );
  TX_CHECK( hipGetLastError() );
  fd_hip_segs_t segs = { misc + 32u, n_seg, seg_cap, misc };
  if( fd_ed25519_hip_verify_segs( ctx, segs, rsig, rpub, out, rmoff, rmsz, rcode, st ) ) {
    fprintf( stderr, "fd_verify_hip: segmented verify refused (%u x %lu records)\n", n_seg, seg_cap );
    abort();
  }
  fd_ed25519_hip_group_reduce_dev( ctx, n, first, cnt, rcode, tcode, st );
}

extern "C" int
fd_verify_hip_tile_submit_frags( fd_verify_hip_tile_t * t, ulong n, uchar const * d_in, uint const * d_in_chunk,
                                 ushort const * d_in_sz, uchar const * d_in_kind, uchar * d_out,
                                 uint const * d_out_chunk ) {
  hipStream_t st; int rc;
  tile_slot * sp = submit_begin( t, n, st, rc );
  if( !sp ) return rc;
  tile_slot & s = *sp;
  s.frags = 1;
  if( !n ) { memset( s.h_res, 0, TILE_RES_HDR ); TX_CHECK( hipEventRecord( s.ev_done, st ) ); return 0; }
  submit_frags_body( t, s, st, n, d_in, d_in_chunk, d_in_sz, d_in_kind, d_out, d_out_chunk );
  TX_CHECK( hipEventRecord( s.ev_done, st ) );
  return 0;
}

/* mcache range mode.  The stem reads a polled link one mcache line at a
   time on the tile's core (fd_stem.c: the line's seq, before_frag, the
   fields, during_frag, the seq again) -- for the quic_verify fan-out every
   verify tile reads every line of the link, a cross-core miss each, which
   bounds the stage at ~15-20 M frags/s on the GPU box whatever the tile
   count.  A tile whose quic_verify link is unpolled
   (FD_TOPOB_UNPOLLED, integration/fd_verify_topo_hip.patch) hands the GPU
   whole published seq ranges of it instead: k_range_gather reads the lines
   (32 B each, from the registered mcache), keeps the tile's round-robin
   share (before_frag, fd_verify_tile.c:37-58), checks each as the stem and
   during_frag do, and writes the frag list k_txnm_batch ingests.

   Per kept seq j (seq = first + j*rr_cnt): the line must still hold seq
   and a chunk in [chunk0, wmark] with sz <= FD_TPU_RAW_MTU; a line that
   does not (overwritten by a producer that lapped the tile, or corrupt) is
   given sz 0xffff, which k_txnm_batch flags as a corrupt frag without
   reading it -- the caller's overrun check after the batch (the oldest
   line, then per frag) tells the two apart: an overrun frag is skipped
   (complete_skip/complete_range), a corrupt one ends the tile as
   during_frag's FD_LOG_ERR does.  The line's fields are read only after
   the caller saw the line hold seq (the producer writes seq last,
   fd_mcache_publish), so they are that frag's unless the line was reused
   since, which the same overrun check catches. */
__global__ __launch_bounds__(256)
void k_range_gather( u32 * __restrict__ misc, u32 misc_words,
                     ulong n, u8 const * __restrict__ mcache, ulong line_mask, ulong first, ulong stride,
                     ulong chunk_off, ulong chunk0, ulong wmark, u32 * __restrict__ in_chunk,
                     u16 * __restrict__ in_sz, u8 * __restrict__ in_kind, u32 * __restrict__ tso ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  /* the slot's misc block for k_txnm_batch (one dispatch fewer on the batch's path) */
  for( ulong w = j; w < (ulong)misc_words; w += (ulong)gridDim.x * blockDim.x ) misc[w] = 0u;
  if( j >= n ) return;
  ulong const seq = first + j * stride;
  u8 const * line = mcache + 32ul * (seq & line_mask);
  uint4 const w1 = *(uint4 const *)(line + 16);                              /* chunk, sz, ctl, tsorig, tspub */
  u64 const found = *(u64 const *)line;
  u32 const chunk = w1.x, sz = w1.y & 0xffffu;
  bool ok = found == seq && (ulong)chunk >= chunk0 && (ulong)chunk <= wmark && sz <= FD_VERIFY_HIP_TPU_RAW_MTU;
  in_chunk[j] = ok ? (u32)((ulong)chunk - chunk_off) : 0u;
  in_sz[j]    = ok ? (u16)sz : (u16)0xffffu;
  in_kind[j]  = (u8)FD_VERIFY_HIP_IN_QUIC;
  tso[j]      = ok ? w1.z : 0u;
}

extern "C" int
fd_verify_hip_tile_submit_range( fd_verify_hip_tile_t * t, fd_verify_hip_range_t const * r, uchar const * d_in,
                                 uchar * d_out, uint const * d_out_chunk ) {
  if( !r || !r->mcache || !d_in || !d_out || !d_out_chunk ) return -1;
  if( !r->depth || (r->depth & (r->depth - 1ul)) || r->seq_cnt > r->depth || !r->rr_cnt || r->rr_idx >= r->rr_cnt ||
      r->chunk0 < r->chunk_off || r->chunk0 > r->wmark || r->wmark - r->chunk_off > 0xffffffffull ) return -1;
  ulong const n = fd_verify_hip_range_frag_cnt( r->seq0, r->seq_cnt, r->rr_cnt, r->rr_idx );
  hipStream_t st; int rc;
  tile_slot * sp = submit_begin( t, n, st, rc );
  if( !sp ) return rc;
  tile_slot & s = *sp;
  s.frags = 1; s.range = 1;
  if( !n ) { memset( s.h_res, 0, TILE_RES_HDR ); TX_CHECK( hipEventRecord( s.ev_done, st ) ); return 0; }
  ulong const first = r->seq0 + (r->rr_idx + r->rr_cnt - r->seq0 % r->rr_cnt) % r->rr_cnt;
  int const fold = !t->ingest_split;                        /* the fused ingest's misc block, zeroed here */
  ulong const F = t->fb == 8 ? 8ul : 16ul, nwg = (n + F - 1ul) / F;
  u32 const misc_words = fold ? 32u + (nwg < FB_SEGS ? (u32)nwg : FB_SEGS) * FD_HIP_SEG_STRIDE : 0u;
  hipLaunchKernelGGL( k_range_gather, dim3( (unsigned)((n + 255ul)/256ul) ), dim3( 256 ), 0, st, s.d_misc, misc_words, n,
                      (u8 const *)r->mcache, r->depth - 1ul, first, r->rr_cnt, r->chunk_off, r->chunk0, r->wmark,
                      s.d_rin, s.d_rsz, s.d_rkind, s.d_tso );
  TX_CHECK( hipGetLastError() );
  submit_frags_body( t, s, st, n, d_in, s.d_rin, s.d_rsz, s.d_rkind, d_out, d_out_chunk, fold );
  TX_CHECK( hipMemcpyAsync( s.h_tso, s.d_tso, 4ul*n, hipMemcpyDeviceToHost, st ) );
  TX_CHECK( hipEventRecord( s.ev_done, st ) );
  return 0;
}

extern "C" int
fd_verify_hip_tile_poll( fd_verify_hip_tile_t const * t ) {
  if( t->completed == t->submitted ) return -1;
  tile_slot const & s = t->slot[t->completed % t->nslot];
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( t->ctx ) ) );
  hipError_t e = hipEventQuery( s.ev_done );
  if( e == hipErrorNotReady ) return 0;
  TX_CHECK( e );
  return 1;
}

extern "C" ulong
fd_verify_hip_tile_inflight( fd_verify_hip_tile_t const * t ) { return t->submitted - t->completed; }

extern "C" int
fd_verify_hip_tile_set_inflight( fd_verify_hip_tile_t * t, ulong k ) {
  if( k < 1ul || k > FD_VERIFY_HIP_INFLIGHT_MAX || t->submitted != t->completed ) return -1;
  int dev = fd_ed25519_hip_ctx_device( t->ctx );
  TX_CHECK( hipSetDevice( dev ) );
  hipStream_t st = (hipStream_t)fd_ed25519_hip_ctx_stream( t->ctx );
  TX_CHECK( hipStreamSynchronize( st ) );
  for( ulong j = t->nalloc; j < k; j++ ) {
    slot_alloc( t->slot[j], t->max_txn ); slot_warm( t->slot[j], t->max_txn, st );
    if( t->staging ) slot_stage_alloc( t->slot[j], t->max_txn );
  }
  if( k > t->nalloc ) t->nalloc = k;
  /* every slot past the first on a context (stream, verify scratch) of its
     own: a batch's GPU time is nearly independent of its size until it
     fills the GPU (~1.1 ms per tile batch of 2-16 K frags), so batches that
     wait on one stream behind each other leave the GPU idle */
  for( ulong j = 1; j < k; j++ ) {
    tile_slot & s = t->slot[j];
    if( s.own_ctx ) continue;
    s.ctx = fd_ed25519_hip_ctx_new( dev, 12ul*(t->max_txn + SLOT_SEG_SLACK) );
    if( !s.ctx ) return -1;
    s.own_ctx = 1;
  }
  for( ulong j = 0; j < t->nalloc; j++ ) if( !t->slot[j].ctx ) t->slot[j].ctx = t->ctx;
  t->nslot = k;
  t->submitted = t->completed = 0;                        /* batch b takes slot b % nslot */
  return 0;
}

static int
tile_complete( fd_verify_hip_tile_t * t, ulong const * bundle_id, uchar const * skip, signed char * result,
               ulong * tag_out, ushort * txn_t_sz, ushort * payload_sz = 0, uint * tsorig = 0 ) {
  if( t->completed == t->submitted ) return -1;
  tile_slot & s = t->slot[t->completed % t->nslot];
  if( tsorig && !s.range ) return -1;                       /* a range batch's lines only */
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( t->ctx ) ) );
  TX_CHECK( hipEventSynchronize( s.ev_done ) );
  u32 const * hdr = (u32 const *)s.h_res;
  tile_res const * R = (tile_res const *)(s.h_res + TILE_RES_HDR);
  int skipped = 0;
  if( skip ) for( ulong j = 0; j < s.n; j++ ) skipped |= !!skip[j];
  /* during_frag's FD_LOG_ERR (fd_verify_tile.c:75-85): a corrupt frag kills
     the tile.  With frags skipped as overruns the flag may be theirs: the
     per-frag bit (out staging) still finds a corrupt frag that was not
     skipped; without staging only the batch flag exists and a skipped
     frag's corruption cannot be told from another's */
  bool corrupt = s.frags && s.n && hdr[1] && !skipped;
  if( s.frags && s.n && hdr[1] && skipped )
    for( ulong j = 0; j < s.n; j++ ) corrupt |= !skip[j] && (R[j].kind & TILE_RES_BAD);
  if( corrupt ) {
    fprintf( stderr, "fd_verify_hip: corrupt frag in batch (size beyond FD_TPU_RAW_MTU / 2048 or payload_sz "
                     "beyond FD_TPU_MTU)\n" );
    abort();
  }
  s.nsig = s.n ? hdr[0] : 0u;
  if( tsorig && s.n ) memcpy( tsorig, s.h_tso, 4ul*s.n );
  float gpu_ms = 0.f;
  TX_CHECK( hipEventElapsedTime( &gpu_ms, s.ev_start, s.ev_done ) );
  auto h0 = std::chrono::steady_clock::now();

  /* ordered pass: after_frag (fd_verify_tile.c:101-161) per frag */
  ulong const n = s.n;
  ulong * const map = t->map; ulong const mask = t->map_cnt - 1;
  ulong * const ring = t->ring;
  ulong const depth = t->depth;
  const ulong PF = 8;
  for( ulong j = 0; j < n && j < PF; j++ ) __builtin_prefetch( map + (R[j].tag & mask) );
  for( ulong j = 0; j < n; j++ ) {
    if( payload_sz ) payload_sz[j] = (ushort)R[j].pad;
    if( skip && skip[j] ) {                                  /* overrun: the stem never calls after_frag */
      if( txn_t_sz ) txn_t_sz[j] = 0;
      if( tag_out ) tag_out[j] = 0;
      result[j] = FD_VERIFY_HIP_FRAG_OVERRUN;
      continue;
    }
    if( s.frags ) {                                          /* after_frag's first statement (:112) */
      u32 k = R[j].kind & ~(FD_VERIFY_HIP_IN_HOSTCOPY | TILE_RES_BAD);
      t->m_gossip += (k == FD_VERIFY_HIP_IN_GOSSIP) | (k == FD_VERIFY_HIP_IN_SEND);
    }
    if( j + PF < n ) {
      __builtin_prefetch( map + (R[j + PF].tag & mask) );
      ulong o = *t->oldest + PF; if( o >= depth ) o -= depth;
      if( o < depth ) __builtin_prefetch( map + (ring[o] & mask) );
    }
    u32 tsz = R[j].tsz;
    if( txn_t_sz ) txn_t_sz[j] = (ushort)tsz;
    if( tag_out ) tag_out[j] = 0;
    ulong bid = s.frags ? R[j].bid : bundle_id ? bundle_id[j] : 0ul;   /* frag mode: from the fd_txn_m_t header */
    int is_bundle = bid != 0ul;
    if( is_bundle && bid != t->bundle_id ) { t->bundle_failed = 0; t->bundle_id = bid; }
    if( is_bundle && t->bundle_failed ) { t->m_bundle++; result[j] = FD_VERIFY_HIP_FRAG_BUNDLE_PEER; continue; }
    if( !tsz ) {
      if( is_bundle ) t->bundle_failed = 1;
      t->m_parse++; result[j] = FD_VERIFY_HIP_FRAG_PARSE_FAIL; continue;
    }
    /* fd_txn_verify with dedup = !is_bundle */
    ulong tag = R[j].tag;
    int res;
    if( !is_bundle && fd_verify_hip_tcache_query( map, t->map_cnt, tag ) )       res = FD_TXN_VERIFY_DEDUP;
    else if( R[j].tcode != FD_ED25519_SUCCESS )                                   res = FD_TXN_VERIFY_FAILED;
    else if( !is_bundle && fd_verify_hip_tcache_insert( t->oldest, ring, depth, map, t->map_cnt, tag ) )
                                                                                  res = FD_TXN_VERIFY_DEDUP;
    else                                                                          res = FD_TXN_VERIFY_SUCCESS;
    if( res != FD_TXN_VERIFY_SUCCESS ) {
      if( is_bundle ) t->bundle_failed = 1;
      if( res == FD_TXN_VERIFY_DEDUP ) t->m_dedup++; else t->m_verify++;
      result[j] = (signed char)res; continue;
    }
    if( tag_out ) tag_out[j] = tag;
    t->m_pub++;
    result[j] = FD_VERIFY_HIP_FRAG_PUBLISH;
  }
  auto h1 = std::chrono::steady_clock::now();
  if( s.frags && !t->ingest_split ) {
    float ims = 0.f;
    if( s.ing_timed && n ) TX_CHECK( hipEventElapsedTime( &ims, s.ev_ing0, s.ev_ing1 ) );
    u64 const * hb = (u64 const *)s.h_res;
    double txnt = 0.0;
    for( ulong j = 0; j < n; j++ ) txnt += (double)R[j].tsz + 2.0;
    t->last_ingest[0] = (double)ims;
    t->last_ingest[1] = (double)n;
    t->last_ingest[2] = n ? (double)hb[2] + (double)hb[3] + txnt + 104.0 * (double)s.nsig + 34.0 * (double)n : 0.0;
    t->last_ingest[3] = (double)s.nsig;
  }
  t->m_sigs += s.nsig;
  t->last_gpu_ms  = gpu_ms;
  t->last_host_ms = std::chrono::duration<double, std::milli>( h1 - h0 ).count();
  t->last_sigs    = (double)s.nsig;
  hist_sample( t->hist[0], (ulong)((double)gpu_ms * 1e6 + 0.5) );
  hist_sample( t->hist[1], (ulong)std::chrono::duration_cast<std::chrono::nanoseconds>( h1 - h0 ).count() );
  s.busy = 0; t->completed++;
  return 0;
}

extern "C" int
fd_verify_hip_tile_complete( fd_verify_hip_tile_t * t, ulong const * bundle_id, signed char * result,
                             ulong * tag_out, ushort * txn_t_sz ) {
  return tile_complete( t, bundle_id, NULL, result, tag_out, txn_t_sz );
}

extern "C" int
fd_verify_hip_tile_complete_skip( fd_verify_hip_tile_t * t, uchar const * skip, signed char * result,
                                  ulong * tag_out, ushort * txn_t_sz, ushort * payload_sz ) {
  if( !t->slot[t->completed % t->nslot].frags && t->completed != t->submitted ) return -1;   /* frag batches only */
  return tile_complete( t, NULL, skip, result, tag_out, txn_t_sz, payload_sz );
}

extern "C" int
fd_verify_hip_tile_complete_range( fd_verify_hip_tile_t * t, uchar const * skip, signed char * result,
                                   ushort * txn_t_sz, ushort * payload_sz, uint * tsorig ) {
  if( !result ) return -1;
  if( t->completed != t->submitted && !t->slot[t->completed % t->nslot].frags ) return -1;
  return tile_complete( t, NULL, skip, result, NULL, txn_t_sz, payload_sz, tsorig );
}

extern "C" int
fd_verify_hip_tile_set_cu_mask( fd_verify_hip_tile_t * t, uint const * mask, uint words ) {
  if( t->submitted != t->completed ) return -1;
  for( ulong j = 0; j < t->nalloc; j++ ) {
    fd_ed25519_hip_ctx_t * c = t->slot[j].ctx;
    bool seen = false;                                       /* slots sharing the tile's context: once */
    for( ulong k = 0; k < j; k++ ) seen |= t->slot[k].ctx == c;
    if( !seen && fd_ed25519_hip_ctx_set_cu_mask( c, mask, words ) ) return -1;
    /* the slot's out-flush stream runs on the same CUs: the new stream is
       made first and the old one destroyed only then, so a refused mask
       leaves the slot its working stream */
    tile_slot & s = t->slot[j];
    hipStream_t ns = 0;
    if( words ) { if( hipExtStreamCreateWithCUMask( &ns, words, mask ) != hipSuccess ) return -1; }
    else        TX_CHECK( hipStreamCreateWithFlags( &ns, hipStreamNonBlocking ) );
    TX_CHECK( hipStreamSynchronize( s.st_flush ) );
    TX_CHECK( hipStreamDestroy( s.st_flush ) );
    s.st_flush = ns;
  }
  return 0;
}

extern "C" int
fd_verify_hip_tile_set_staging( fd_verify_hip_tile_t * t, int on ) {
  if( t->submitted != t->completed || (on && t->ingest_split) ) return -1;
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( t->ctx ) ) );
  if( on ) for( ulong j = 0; j < t->nalloc; j++ ) slot_stage_alloc( t->slot[j], t->max_txn );
  t->staging = !!on;
  return 0;
}

extern "C" void fd_verify_hip_tile_set_ingest_timing( fd_verify_hip_tile_t * t, int on ) { t->ingest_timing = !!on; }

extern "C" void fd_verify_hip_tile_ingest_stats( fd_verify_hip_tile_t const * t, double out[4] ) {
  for( int k = 0; k < 4; k++ ) out[k] = t->last_ingest[k];
}

extern "C" void fd_verify_hip_tile_metrics( fd_verify_hip_tile_t const * t, ulong out[6] ) {
  out[0] = t->m_parse; out[1] = t->m_verify; out[2] = t->m_dedup; out[3] = t->m_bundle;
  out[4] = t->m_pub; out[5] = t->m_sigs;
}

extern "C" void fd_verify_hip_tile_metrics2( fd_verify_hip_tile_t const * t, ulong out[7] ) {
  fd_verify_hip_tile_metrics( t, out );
  out[6] = t->m_gossip;
}

/* before_frag (fd_verify_tile.c:37-58): 1 = skip the frag */
extern "C" int fd_verify_hip_before_frag( uint in_kind, ulong seq, ulong sig, ulong round_robin_cnt,
                                          ulong round_robin_idx ) {
  int is_bundle_packet = in_kind == FD_VERIFY_HIP_IN_BUNDLE && !sig;
  if( is_bundle_packet || in_kind == FD_VERIFY_HIP_IN_QUIC ) return (seq % round_robin_cnt) != round_robin_idx;
  if( in_kind == FD_VERIFY_HIP_IN_BUNDLE ) return round_robin_idx != 0ul;
  if( in_kind == FD_VERIFY_HIP_IN_GOSSIP )
    return (seq % round_robin_cnt) != round_robin_idx || sig != FD_VERIFY_HIP_GOSSIP_UPDATE_TAG_VOTE;
  return 0;
}

extern "C" void fd_verify_hip_tile_last_timing( fd_verify_hip_tile_t const * t, double out[3] ) {
  out[0] = t->last_gpu_ms; out[1] = t->last_host_ms; out[2] = t->last_sigs;
}

/**********************************************************************/
/* replay and shred callers (include/fd_replay_hip.h)                  */

static_assert( sizeof(fd_txn_hip_desc_t) == 16, "fd_txn_hip_desc_t layout" );

/* caller-parsed txn -> the signature span k_txn_expand consumes.
   fd_executor_txn_verify (fd_executor.c:1607-1623) passes signature_cnt as
   batch_sz: 0 or > 16 is ERR_SIG before any signature is read
   (fd_ed25519_user.c:238-241), so such a txn gets no records (cnt 0, which
   the group reduce turns into ERR_SIG). */
__global__ __launch_bounds__(256)
void k_desc_spans( ulong n, fd_txn_hip_desc_t const * __restrict__ desc, u8 * __restrict__ nsig,
                   u32 * __restrict__ sig_at, u32 * __restrict__ acct_at, u32 * __restrict__ msg_at,
                   u32 * __restrict__ msg_sz ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  fd_txn_hip_desc_t d = desc[j];
  u32 c = d.signature_cnt;
  nsig[j]    = (u8)((c >= 1u && c <= 16u) ? c : 0u);
  sig_at[j]  = d.payload_off + d.signature_off;
  acct_at[j] = d.payload_off + d.acct_addr_off;
  msg_at[j]  = d.payload_off + d.message_off;
  msg_sz[j]  = d.payload_sz >= d.message_off ? (u32)(d.payload_sz - d.message_off) : 0u;
}

/* fd_executor.c:1619-1621 */
__global__ __launch_bounds__(256)
void k_exec_codes( ulong n, signed char const * __restrict__ tcode, int * __restrict__ res ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  res[j] = tcode[j] == FD_ED25519_SUCCESS ? FD_RUNTIME_HIP_EXECUTE_SUCCESS : FD_RUNTIME_HIP_TXN_ERR_SIGNATURE_FAILURE;
}

struct fd_replay_hip {
  fd_ed25519_hip_ctx_t * ctx;
  ulong   max_txn, rcap;
  u8 *    d_nsig; u32 * d_sig_at; u32 * d_acct_at; u32 * d_msg_at; u32 * d_msg_sz;
  u32 *   d_first; u8 * d_cnt; signed char * d_tcode; u32 * d_counter; u32 * h_counter;
  u8 *    d_rsig; u8 * d_rpub; u32 * d_rmoff; u32 * d_rmsz; signed char * d_rcode;
  u8 *    d_hpool; fd_txn_hip_desc_t * d_hdesc; int * d_hres;   /* fd_replay_hip_txn_verify_host staging */
  ulong   hpool_cap;
  hipEvent_t ev_last; int ev_used;   /* calls on different streams run in call order over this scratch */
};

extern "C" fd_replay_hip_t *
fd_replay_hip_new( fd_ed25519_hip_ctx_t * ctx, ulong max_txn ) {
  if( !ctx || !max_txn ) return 0;
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( ctx ) ) );
  fd_ed25519_hip_ctx_reserve( ctx, 16ul*max_txn );
  fd_replay_hip_t * r = (fd_replay_hip_t *)calloc( 1, sizeof(fd_replay_hip_t) );
  ulong n = max_txn, rc = 16ul*max_txn;                    /* at most 16 records per txn */
  r->ctx = ctx; r->max_txn = n; r->rcap = rc;
  TX_CHECK( hipMalloc( &r->d_nsig, n ) );       TX_CHECK( hipMalloc( &r->d_sig_at, 4*n ) );
  TX_CHECK( hipMalloc( &r->d_acct_at, 4*n ) );  TX_CHECK( hipMalloc( &r->d_msg_at, 4*n ) );
  TX_CHECK( hipMalloc( &r->d_msg_sz, 4*n ) );   TX_CHECK( hipMalloc( &r->d_first, 4*n ) );
  TX_CHECK( hipMalloc( &r->d_cnt, n ) );        TX_CHECK( hipMalloc( &r->d_tcode, n ) );
  TX_CHECK( hipMalloc( &r->d_counter, 4 ) );    TX_CHECK( hipHostMalloc( &r->h_counter, 4, 0 ) );
  TX_CHECK( hipMalloc( &r->d_rsig, 64*rc ) );   TX_CHECK( hipMalloc( &r->d_rpub, 32*rc ) );
  TX_CHECK( hipMalloc( &r->d_rmoff, 4*rc ) );   TX_CHECK( hipMalloc( &r->d_rmsz, 4*rc ) );
  TX_CHECK( hipMalloc( &r->d_rcode, rc ) );
  r->hpool_cap = (ulong)FD_REPLAY_HIP_TXN_MTU * n;
  TX_CHECK( hipMalloc( &r->d_hpool, r->hpool_cap + 16ul ) );
  TX_CHECK( hipMemset( r->d_hpool, 0, r->hpool_cap + 16ul ) );   /* the 16-byte read-past tail is defined */
  TX_CHECK( hipMalloc( &r->d_hdesc, sizeof(fd_txn_hip_desc_t)*n ) );
  TX_CHECK( hipMalloc( &r->d_hres, 4*n ) );
  TX_CHECK( hipEventCreateWithFlags( &r->ev_last, hipEventDisableTiming ) );
  return r;
}

extern "C" void
fd_replay_hip_delete( fd_replay_hip_t * r ) {
  if( !r ) return;
  (void)hipSetDevice( fd_ed25519_hip_ctx_device( r->ctx ) );
  (void)hipStreamSynchronize( (hipStream_t)fd_ed25519_hip_ctx_stream( r->ctx ) );
  if( r->ev_used ) (void)hipEventSynchronize( r->ev_last );
  (void)hipEventDestroy( r->ev_last );
  (void)hipFree( r->d_nsig ); (void)hipFree( r->d_sig_at ); (void)hipFree( r->d_acct_at ); (void)hipFree( r->d_msg_at );
  (void)hipFree( r->d_msg_sz ); (void)hipFree( r->d_first ); (void)hipFree( r->d_cnt ); (void)hipFree( r->d_tcode );
  (void)hipFree( r->d_counter ); (void)hipHostFree( r->h_counter );
  (void)hipFree( r->d_rsig ); (void)hipFree( r->d_rpub ); (void)hipFree( r->d_rmoff ); (void)hipFree( r->d_rmsz );
  (void)hipFree( r->d_rcode );
  (void)hipFree( r->d_hpool ); (void)hipFree( r->d_hdesc ); (void)hipFree( r->d_hres );
  free( r );
}

extern "C" int
fd_replay_hip_txn_verify_dev( fd_replay_hip_t * r, ulong n, uchar const * d_pool, fd_txn_hip_desc_t const * d_desc,
                              int * d_result, void * stream ) {
  if( n > r->max_txn ) return -1;
  if( !n ) return 0;
  hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)fd_ed25519_hip_ctx_stream( r->ctx );
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( r->ctx ) ) );
  dim3 grid( (unsigned)((n + 255)/256) ), blk( 256 );
  if( r->ev_used ) TX_CHECK( hipStreamWaitEvent( st, r->ev_last, 0 ) );
  hipLaunchKernelGGL( k_desc_spans, grid, blk, 0, st, n, d_desc, r->d_nsig, r->d_sig_at, r->d_acct_at, r->d_msg_at,
                      r->d_msg_sz );
  TX_CHECK( hipGetLastError() );
  TX_CHECK( hipMemsetAsync( r->d_counter, 0, 4, st ) );
  hipLaunchKernelGGL( k_txn_expand, grid, blk, 0, st, n, d_pool, r->d_nsig, r->d_sig_at, r->d_acct_at, r->d_msg_at,
                      r->d_msg_sz, r->d_counter, r->d_first, r->d_cnt, r->d_rsig, r->d_rpub, r->d_rmoff, r->d_rmsz,
                      r->rcap );
  TX_CHECK( hipGetLastError() );
  fd_ed25519_hip_verify_dev_count( r->ctx, 16ul*n, r->d_counter, r->d_rsig, r->d_rpub, d_pool, r->d_rmoff,
                                   r->d_rmsz, r->d_rcode, NULL, st );
  fd_ed25519_hip_group_reduce_dev( r->ctx, n, r->d_first, r->d_cnt, r->d_rcode, r->d_tcode, st );
  hipLaunchKernelGGL( k_exec_codes, grid, blk, 0, st, n, r->d_tcode, d_result );
  TX_CHECK( hipGetLastError() );
  TX_CHECK( hipEventRecord( r->ev_last, st ) );
  r->ev_used = 1;
  return 0;
}

extern "C" int
fd_replay_hip_txn_verify_host( fd_replay_hip_t * r, ulong n, uchar const * h_pool, ulong pool_sz,
                               fd_txn_hip_desc_t const * h_desc, int * h_result, void * stream ) {
  if( n > r->max_txn || pool_sz > r->hpool_cap ) return -1;
  for( ulong j=0; j<n; j++ ) {        /* every span inside the staged pool (k_desc_spans trusts them) */
    fd_txn_hip_desc_t const * d = h_desc + j;
    if( (ulong)d->payload_off + d->payload_sz > pool_sz ) return -1;
    ulong c = d->signature_cnt;
    if( c >= 1ul && c <= 16ul &&        /* the records read: signatures, pubkeys, the message (cnt 0 or > 16 read nothing) */
        ( (ulong)d->signature_off + 64ul*c > d->payload_sz || (ulong)d->acct_addr_off + 32ul*c > d->payload_sz ||
          (ulong)d->message_off > d->payload_sz ) ) return -1;
  }
  if( !n ) return 0;
  hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)fd_ed25519_hip_ctx_stream( r->ctx );
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( r->ctx ) ) );
  if( r->ev_used ) TX_CHECK( hipStreamWaitEvent( st, r->ev_last, 0 ) );
  TX_CHECK( hipMemcpyAsync( r->d_hpool, h_pool, pool_sz, hipMemcpyHostToDevice, st ) );
  TX_CHECK( hipMemcpyAsync( r->d_hdesc, h_desc, sizeof(fd_txn_hip_desc_t)*n, hipMemcpyHostToDevice, st ) );
  int rc = fd_replay_hip_txn_verify_dev( r, n, r->d_hpool, r->d_hdesc, r->d_hres, st );
  if( rc ) return rc;
  TX_CHECK( hipMemcpyAsync( h_result, r->d_hres, 4*n, hipMemcpyDeviceToHost, st ) );
  TX_CHECK( hipEventRecord( r->ev_last, st ) );
  return 0;
}

extern "C" int
fd_replay_hip_wait( fd_replay_hip_t * r ) {
  if( !r->ev_used ) return 0;
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( r->ctx ) ) );
  TX_CHECK( hipEventSynchronize( r->ev_last ) );
  return 0;
}

extern "C" int
fd_replay_hip_poll( fd_replay_hip_t const * r ) {
  if( !r->ev_used ) return -1;
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( r->ctx ) ) );
  hipError_t e = hipEventQuery( r->ev_last );
  if( e == hipErrorNotReady ) return 0;
  TX_CHECK( e );
  return 1;
}

extern "C" int
fd_fec_hip_verify_roots_dev( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_roots, uchar const * d_sigs,
                             uchar const * d_pubs, signed char * d_codes, void * stream ) {
  return fd_ed25519_hip_verify_fixed_dev( ctx, n, d_sigs, d_pubs, d_roots, 32u, d_codes, NULL, stream );
}

/**********************************************************************/
/* ed25519 program instructions (include/fd_replay_hip.h)             */

static_assert( sizeof(fd_precompile_hip_desc_t) == 16, "fd_precompile_hip_desc_t layout" );
static_assert( sizeof(fd_precompile_hip_instr_t) == 8, "fd_precompile_hip_instr_t layout" );

#define PC_ERR_SIGNATURE    2u   /* fd_precompiles.h:16-18 */
#define PC_ERR_DATA_OFFSET  3u
#define PC_ERR_DATA_SIZE    4u
#define PC_ERR_DESC         0xFFFFFFFFu

/* fd_precompile_ed25519_verify :130-154: the instruction-level size checks
   and the signature count (the offset records then lie inside the data) */
__global__ __launch_bounds__(256)
void k_pc_count( ulong n, u8 const * __restrict__ pool, fd_precompile_hip_desc_t const * __restrict__ desc,
                 u8 * __restrict__ cnt, u32 * __restrict__ early ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  fd_precompile_hip_desc_t d = desc[j];
  u32 sz = d.data_sz, e = 0u, c = 0u;
  u8 const * data = pool + d.data_off;
  if( sz > FD_PRECOMPILE_HIP_DATA_MAX ) e = PC_ERR_DESC;
  else if( sz < 16u ) e = (sz == 2u && data[0] == 0u) ? 0u : PC_ERR_DATA_SIZE;   /* the [0,0] edge case */
  else {
    c = data[0];
    if( !c || sz < 14u*c + 2u ) { e = PC_ERR_DATA_SIZE; c = 0u; }
  }
  cnt[j] = (u8)c; early[j] = e;
}

/* fd_precompile_get_instr_data (:76-107) */
DEVI u32 pc_resolve( fd_precompile_hip_desc_t const & d, fd_precompile_hip_instr_t const * __restrict__ tab,
                     u32 index, u32 offset, u32 sz, u32 & at ) {
  u32 base, dsz;
  if( index == 0xFFFFu ) { base = d.data_off; dsz = d.data_sz; }
  else {
    if( index >= d.instr_cnt ) return PC_ERR_DATA_OFFSET;
    fd_precompile_hip_instr_t t = tab[d.instr_base + index];
    base = t.data_off; dsz = t.data_sz;
  }
  if( offset + sz > dsz ) return PC_ERR_SIGNATURE;
  at = base + offset;
  return 0u;
}

/* One record per offset record (signature i of instruction j), allocated as
   k_txn_expand allocates (wave prefix sums, one atomic per wave, records of a
   wave contiguous and in order, first[] says where).  A record whose spans
   fail the fetch checks keeps the error (pre[r]) and a zero signature; the
   others get their signature and public key copied out and their message
   span, for one verify pass over every record. */
__global__ __launch_bounds__(256)
void k_pc_expand( ulong n, u8 const * __restrict__ pool, fd_precompile_hip_desc_t const * __restrict__ desc,
                  fd_precompile_hip_instr_t const * __restrict__ tab, u8 * __restrict__ cnt,
                  u32 * __restrict__ early, u32 * __restrict__ counter, u32 * __restrict__ first,
                  u8 * __restrict__ rsig, u8 * __restrict__ rpub, u32 * __restrict__ rmoff, u32 * __restrict__ rmsz,
                  u8 * __restrict__ rpre, ulong cap ) {
  __shared__ u32 l_excl[256], l_c[256];
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  u32 c = j < n ? cnt[j] : 0u;
  u32 excl = 0, tot = 0;
  #pragma unroll
  for( int b = 0; b < 7; b++ ) {                               /* c <= 87 */
    unsigned long long m = __ballot( (c >> b) & 1u );
    u32 below = __builtin_amdgcn_mbcnt_hi( (u32)(m >> 32), __builtin_amdgcn_mbcnt_lo( (u32)m, 0u ) );
    excl += below << b;
    tot  += (u32)__popcll( m ) << b;
  }
  u32 base = 0;
  if( (threadIdx.x & 63u) == 0u && tot ) base = atomicAdd( counter, tot );
  base = __shfl( base, 0 );
  u32 lc = c;
  if( j < n ) {
    u32 f = base + excl;
    first[j] = f;
    if( (ulong)f + c > cap ) { cnt[j] = 0; early[j] = PC_ERR_DESC; lc = 0; }   /* never taken: cap = 87 per instruction */
  }
  l_excl[threadIdx.x] = excl; l_c[threadIdx.x] = lc;
  __syncthreads();
  u32 w0 = threadIdx.x & ~63u;
  for( u32 t = threadIdx.x & 63u; t < tot; t += 64u ) {
    u32 lo = 0, hi = 63;                                       /* last lane with excl <= t */
    #pragma unroll
    for( int s = 0; s < 6; s++ ) {
      u32 mid = (lo + hi + 1u) >> 1;
      bool le = l_excl[w0 + mid] <= t;
      lo = le ? mid : lo; hi = le ? hi : mid - 1u;
    }
    u32 L = w0 + lo, k = t - l_excl[L];
    if( k >= l_c[L] ) continue;
    fd_precompile_hip_desc_t d = desc[(ulong)blockIdx.x * blockDim.x + L];
    u8 const * o = pool + d.data_off + 2u + 14u*k;             /* fd_ed25519_signature_offsets_t, packed LE */
    u32 f[7];
    #pragma unroll
    for( int q = 0; q < 7; q++ ) f[q] = (u32)o[2*q] | ((u32)o[2*q+1] << 8);
    u32 sig_at = 0, pub_at = 0, msg_at = 0;
    u32 e = pc_resolve( d, tab, f[1], f[0], 64u, sig_at );               /* :164-172 */
    if( !e ) e = pc_resolve( d, tab, f[3], f[2], 32u, pub_at );          /* :179-187 */
    if( !e ) e = pc_resolve( d, tab, f[6], f[4], f[5], msg_at );         /* :194-203 */
    u32 r = base + t;
    u32 w[16];
    if( !e ) ld_words_u<16>( w, pool + sig_at );
    else {
      #pragma unroll
      for( int q = 0; q < 16; q++ ) w[q] = 0u;
    }
    uint4 * ds = (uint4 *)(rsig + 64ul*r);
    #pragma unroll
    for( int q = 0; q < 4; q++ ) ds[q] = make_uint4( w[4*q], w[4*q+1], w[4*q+2], w[4*q+3] );
    if( !e ) ld_words_u<8>( w, pool + pub_at );
    uint4 * dp = (uint4 *)(rpub + 32ul*r);
    #pragma unroll
    for( int q = 0; q < 2; q++ ) dp[q] = make_uint4( w[4*q], w[4*q+1], w[4*q+2], w[4*q+3] );
    rmoff[r] = e ? 0u : msg_at; rmsz[r] = e ? 0u : f[5];
    rpre[r] = (u8)e;
  }
}

/* :156-211: the first offset record in order that fails its fetch checks or
   its verify decides the instruction's result */
__global__ __launch_bounds__(256)
void k_pc_reduce( ulong n, u8 const * __restrict__ cnt, u32 const * __restrict__ first, u32 const * __restrict__ early,
                  u8 const * __restrict__ rpre, signed char const * __restrict__ rcode, int * __restrict__ err,
                  u32 * __restrict__ custom ) {
  ulong j = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= n ) return;
  u32 e = early[j];
  if( e == PC_ERR_DESC ) { err[j] = FD_PRECOMPILE_HIP_ERR_DESC; custom[j] = e; return; }
  if( !e ) {
    u32 c = cnt[j], f = first[j];
    for( u32 k = 0; k < c; k++ ) {
      u32 p = rpre[f + k];
      if( p ) { e = p; break; }
      if( rcode[f + k] != FD_ED25519_SUCCESS ) { e = PC_ERR_SIGNATURE; break; }   /* :205-208 */
    }
  }
  err[j] = e ? FD_PRECOMPILE_HIP_INSTR_ERR_CUSTOM_ERR : FD_PRECOMPILE_HIP_INSTR_SUCCESS;
  custom[j] = e;
}

struct fd_precompile_hip {
  fd_ed25519_hip_ctx_t * ctx;
  ulong   max_instr, rcap;
  u8 *    d_cnt; u32 * d_early; u32 * d_first; u32 * d_counter;
  u8 *    d_rsig; u8 * d_rpub; u32 * d_rmoff; u32 * d_rmsz; u8 * d_rpre; signed char * d_rcode;
  hipEvent_t ev_last; int ev_used;
};

extern "C" fd_precompile_hip_t *
fd_precompile_hip_new( fd_ed25519_hip_ctx_t * ctx, ulong max_instr ) {
  if( !ctx || !max_instr ) return 0;
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( ctx ) ) );
  fd_precompile_hip_t * p = (fd_precompile_hip_t *)calloc( 1, sizeof(fd_precompile_hip_t) );
  ulong n = max_instr, rc = (ulong)FD_PRECOMPILE_HIP_SIG_MAX * max_instr;
  p->ctx = ctx; p->max_instr = n; p->rcap = rc;
  TX_CHECK( hipMalloc( &p->d_cnt, n ) );      TX_CHECK( hipMalloc( &p->d_early, 4*n ) );
  TX_CHECK( hipMalloc( &p->d_first, 4*n ) );  TX_CHECK( hipMalloc( &p->d_counter, 4 ) );
  TX_CHECK( hipMalloc( &p->d_rsig, 64*rc ) ); TX_CHECK( hipMalloc( &p->d_rpub, 32*rc ) );
  TX_CHECK( hipMalloc( &p->d_rmoff, 4*rc ) ); TX_CHECK( hipMalloc( &p->d_rmsz, 4*rc ) );
  TX_CHECK( hipMalloc( &p->d_rpre, rc ) );    TX_CHECK( hipMalloc( &p->d_rcode, rc ) );
  TX_CHECK( hipEventCreateWithFlags( &p->ev_last, hipEventDisableTiming ) );
  return p;
}

extern "C" void
fd_precompile_hip_delete( fd_precompile_hip_t * p ) {
  if( !p ) return;
  (void)hipSetDevice( fd_ed25519_hip_ctx_device( p->ctx ) );
  (void)hipStreamSynchronize( (hipStream_t)fd_ed25519_hip_ctx_stream( p->ctx ) );
  if( p->ev_used ) (void)hipEventSynchronize( p->ev_last );
  (void)hipEventDestroy( p->ev_last );
  (void)hipFree( p->d_cnt ); (void)hipFree( p->d_early ); (void)hipFree( p->d_first ); (void)hipFree( p->d_counter );
  (void)hipFree( p->d_rsig ); (void)hipFree( p->d_rpub ); (void)hipFree( p->d_rmoff ); (void)hipFree( p->d_rmsz );
  (void)hipFree( p->d_rpre ); (void)hipFree( p->d_rcode );
  free( p );
}

extern "C" int
fd_precompile_hip_ed25519_verify_dev( fd_precompile_hip_t * p, ulong n, uchar const * d_pool,
                                      fd_precompile_hip_desc_t const * d_desc,
                                      fd_precompile_hip_instr_t const * d_instr_tab, int * d_err,
                                      uint * d_custom_err, void * stream ) {
  if( n > p->max_instr ) return -1;
  if( !n ) return 0;
  hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)fd_ed25519_hip_ctx_stream( p->ctx );
  TX_CHECK( hipSetDevice( fd_ed25519_hip_ctx_device( p->ctx ) ) );
  dim3 grid( (unsigned)((n + 255)/256) ), blk( 256 );
  if( p->ev_used ) TX_CHECK( hipStreamWaitEvent( st, p->ev_last, 0 ) );
  hipLaunchKernelGGL( k_pc_count, grid, blk, 0, st, n, d_pool, d_desc, p->d_cnt, p->d_early );
  TX_CHECK( hipGetLastError() );
  TX_CHECK( hipMemsetAsync( p->d_counter, 0, 4, st ) );
  hipLaunchKernelGGL( k_pc_expand, grid, blk, 0, st, n, d_pool, d_desc, d_instr_tab, p->d_cnt, p->d_early,
                      p->d_counter, p->d_first, p->d_rsig, p->d_rpub, p->d_rmoff, p->d_rmsz, p->d_rpre, p->rcap );
  TX_CHECK( hipGetLastError() );
  fd_ed25519_hip_verify_dev_count( p->ctx, p->rcap < (ulong)FD_PRECOMPILE_HIP_SIG_MAX*n ? p->rcap
                                                                                           : (ulong)FD_PRECOMPILE_HIP_SIG_MAX*n,
                                   p->d_counter, p->d_rsig, p->d_rpub, d_pool, p->d_rmoff, p->d_rmsz, p->d_rcode, NULL,
                                   st );
  hipLaunchKernelGGL( k_pc_reduce, grid, blk, 0, st, n, p->d_cnt, p->d_first, p->d_early, p->d_rpre, p->d_rcode,
                      d_err, d_custom_err );
  TX_CHECK( hipGetLastError() );
  TX_CHECK( hipEventRecord( p->ev_last, st ) );
  p->ev_used = 1;
  return 0;
}
