/* fd_ed25519_hip.hip -- gfx950 ed25519 batch verify engine: kernels and the
   C ABI declared in include/fd_ed25519_hip.h.

   Pipeline per chunk of up to ctx->chunk signatures (one signature per lane,
   256-thread workgroups = 4 wave64):

     k_msg_hist,    txn paths only: records counting-sorted by SHA-512 block
     k_msg_order    count, so that prep's waves hash equal-length messages
     k_verify_prep  S<L check, decode A and R (sqrt chains), small-order
                    checks, k = SHA-512(R||A||M) mod L (wave-cooperative
                    LDS-staged message blocks) -> 192-B state record at the
                    lane's slot; survivor compaction: final codes of
                    pre-check failures, survivor slots -> idx[] (k_verify_dsm
                    runs only them)
     k_verify_dsm   persistent: resident workgroups pull 64-survivor tasks;
                    half-size scalars k1 = k*k2 (mod 8L), k2 odd, ~128 bits
                    each (sc_halfsize); tables [1..8](+-A) and [1..8](-R) ->
                    per-lane HBM scratch, one 128-B line per entry (the
                    identity is one shared entry); [k1](+-A) + [k2](-R) by
                    fixed signed radix-16 windows, [k2*S mod L]B in signed
                    radix 2^12 from two L2-resident global tables ([0..2048]B
                    and [0..2048]2^132 B): every lane adds at the
                    same positions, one window count per wave; identity
                    check; int8 code
     k_bitmap       verdict bitmap from codes (64-bit ballot per wave)
     k_group_reduce batch_single_msg / per-txn semantics over sig codes

   Small calls (count on the host, <= ctx->lat_max records, default 32) take
   k_verify_lat instead: one 256-thread workgroup per signature (and per
   racing copy), three working waves that decode A / decode R / hash, then run
   the [k1]A, [k2]R and B chains with each chain's group law on four lanes,
   joined in LDS.

   Reference semantics: fd_ed25519_user.c:135-310 (see fd_ed25519_dev.h for
   the per-function citations). */

#include "fd_ed25519_dev.h"
#include "fd_hip_order.h"
#include "../../include/fd_ed25519_hip.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <condition_variable>
#include <mutex>

#define FD_CHECK( x ) do {                                                            \
    hipError_t e_ = (x);                                                               \
    if( e_ != hipSuccess ) {                                                           \
      fprintf( stderr, "fd_ed25519_hip: %s failed at %s:%d: %s\n", #x, __FILE__,     \
               __LINE__, hipGetErrorString( e_ ) );                                    \
      abort();                                                                         \
    }                                                                                  \
  } while( 0 )

/* flags in the state record */
#define F_S_BAD      (1u<<0)
#define F_A_NOTSQ    (1u<<1)
#define F_A_ZX       (1u<<2)
#define F_R_NOTSQ    (1u<<3)
#define F_R_ZX       (1u<<4)
#define F_A_SMALL    (1u<<5)
#define F_R_SMALL    (1u<<6)

/* Signing's radix-256 B tables (k_sign, in LDS): [j]B and [j](2^128 B) for
   j in 0..128, 1/2-scaled affine cached, 3 x 9 limbs + pad per entry. */
#define BTAB_N      129
#define BTAB_STRIDE 28
#define BTAB_WORDS  (BTAB_N*BTAB_STRIDE)   /* one table; d_btab holds [j]B then [j](2^128 B) */
/* A/R table entries: each element packed from 9 limbs to 8 words
   (fe_pack), so an entry (Y-X, Y+X, 2dT, 2Z) is one 128-B line.  Measured
   against the 9-limb layout (144 B, two or three lines): k_verify_dsm 7.35
   vs 7.65 ms, C2 113.2 vs 108.2 M verifies/s (round 1) -- the kernel is
   power-limited and the fetch traffic it saves buys clock. */
#define ATAB_ENT    32
#define RTAB_OFF    (8*ATAB_ENT)   /* per lane: [1..8](+-A), then [1..8](-R) */
#define ATAB_WORDS  (2*RTAB_OFF)
/* the identity entry (digit 0) is shared by every lane: one line in d_btab
   after the two B tables (128-B aligned), hot in cache, never written per
   signature */
#define IDENT_OFF   ((2*BTAB_WORDS + 31) & ~31)
/* k_verify_dsm takes the [k2*S mod L]B term in signed radix 2^12 (11 + 11
   digits against [0..2048]B and [0..2048](2^132 B), 22 affine additions)
   from global tables that stay resident in each XCD's L2 (2 x 2049 entries
   of one 128-B line, 525 KB).  Measured against radix 2^8 (16 + 16 digits,
   32 additions) from two 129-entry LDS tables (profiles/r02r_ab_w12):
   k_verify_dsm 6.59-6.62 vs 6.79-6.87 ms, C2 128.7-129.4 vs 126.3-126.4 M
   verifies/s; against radix 2^16 (8.4 MB of tables, served by MALL,
   profiles/r02r_ab_gw16): +0.7% on C2 for ~1.9 GB more fabric reads per
   launch. */
#define BTG_GW      12             /* bits per digit */
#define BTG_ND      11             /* digits per half */
#define BTG_HB      (BTG_ND*BTG_GW)            /* the high table holds multiples of 2^BTG_HB B */
#define BTG_STEP    (BTG_GW/4)                 /* radix-16 windows between B additions */
#define BT12_N      ((1 << (BTG_GW-1)) + 1)
#define BT12_ENT    32             /* YmX, YpX, T2d: 9 limbs each + pad to one 128-B line */
#define BT12_OFF    ((IDENT_OFF + ATAB_ENT + 31) & ~31)
#define BTAB_ALLOC  (BT12_OFF + 2*BT12_N*BT12_ENT)

/* state record: 32 u32 words per field group, laid out SoA per chunk for
   coalescing: word w of signature i lives at st[ w*chunk + i ].
   i is k_verify_prep's processing slot t (lane t takes record order[t]),
   not the record index, and idx[] holds survivor slots.
   On the txn paths the block-count order scatters records over the chunk:
   indexed by record, a wave's 48 state stores in prep and 48 loads in
   k_verify_dsm each touched 64 separate lines.  By slot they are
   contiguous; the DSM looks up order[slot] once for the code it writes.
   Batches without an order (order[t] = t) are unchanged. */
#define ST_K     0
#define ST_S     8
#define ST_AX   16
#define ST_AY   24
#define ST_RX   32
#define ST_RY   40
#define ST_WORDS 48

struct fd_ed25519_hip_ctx {
  int          device;
  hipStream_t  stream;
  ulong        chunk;       /* signatures per launch */
  u32 *        d_btab;      /* BTAB_WORDS */
  u32 *        d_state;     /* ST_WORDS * chunk */
  u32 *        d_atab;      /* ATAB_WORDS * chunk */
  u32 *        d_idx;       /* chunk: compacted survivor indices */
  u32 *        d_count;     /* [0] survivor count; [16..47] k_msg_order's histogram and cursors */
  ulong        dsm_wgs;     /* resident k_verify_dsm workgroups (its persistent grid) */
  ulong        dsm_wgs_all; /* the same with no slots reserved */
  ulong        dsm_share;   /* the grid is dsm_wgs / dsm_share (contexts sharing the GPU) */
  u32 *        d_order;     /* chunk: k_verify_prep's record order (variable-size message paths) */
  int          errmode;
  int          halfsize;    /* 1: half-size scalars (default); 0: full-length (k, 1) */
  ulong        lat_max;     /* calls of at most this many records (no device count) take k_verify_lat */
  u32          lat_copies;  /* k_verify_lat racing copies per signature at most (LAT_COPIES_MAX) */
  ulong        ncu;         /* CUs: a call's copies stop at one workgroup per CU */
  ulong        lat_cus;     /* k_verify_lat workgroup slots a launch may fill with copies (CUs x 4; the
                               drop-in's batch slots share the GPU: each gets its part) */
  ulong        lat_seq;     /* call number, the k_verify_lat early-exit tag (64-bit: never wraps) */
  ulong *      d_lat_done;  /* LAT_MAX_N: call number of the copy that finished each signature */
  /* optional per-kernel timing (HIP events around each launch, on the launch stream) */
  int          timing;
  double       prep_ms, dsm_ms;
  ulong        prep_launches, dsm_launches, dsm_units;
  hipEvent_t   ev[4];
  /* staging for the host-memory entry points (grown on demand) */
  ulong        h_cap_n, h_cap_pool, h_cap_groups;
  uchar *      d_sigs; uchar * d_pubs; uchar * d_pool; uint * d_moff; uint * d_msz;
  signed char * d_codes; ulong * d_bitmap;
  uint *       d_gfirst; uchar * d_gcnt; signed char * d_gcodes;
  /* stream ordering of the context's scratch: every verify launch sequence
     waits for the previous one (on whatever stream it ran) and records its
     own end, so calls on different streams never overlap on d_state/d_idx/
     d_count/d_atab */
  hipEvent_t   ev_last;
  int          ev_used;
};

/**********************************************************************/
/* Kernels                                                             */

DEV void load_words( u32 * w, uchar const * p, int nw ) {   /* 16-byte aligned p */
  uint4 const * q = (uint4 const *)p;
  #pragma unroll
  for( int i=0; i<nw/4; i++ ) { uint4 v = q[i]; w[4*i]=v.x; w[4*i+1]=v.y; w[4*i+2]=v.z; w[4*i+3]=v.w; }
}

/* Base point B (encoding 0x58666...66, fd_curve25519_table_ref.c:7-14) */
DEV void ge_base( ge_p3 & B ) {
  u32 w[8];
  #pragma unroll
  for( int i=0; i<8; i++ ) w[i] = 0x66666666u;
  w[0] = 0x66666658u;
  ge_decode( B, w );
}

/* affine cached form scaled by 1/2: ((y-x)/2, (y+x)/2, d*x*y), canonical */
DEV void ge_to_affc_half( ge_affc & a, ge_p3 const & p ) {
  fe zi, x, y, t, d, h;
  fe_invert( zi, p.Z ); fe_mul( x, p.X, zi ); fe_mul( y, p.Y, zi );
  fe_d( d ); fe_inv2( h );
  fe_mul( t, x, y ); fe_mul( t, t, d );
  fe_sub( a.YmX, y, x ); fe_mul( a.YmX, a.YmX, h );
  fe_add( a.YpX, y, x ); fe_mul( a.YpX, a.YpX, h );
  fe_canon( a.YmX, a.YmX ); fe_canon( a.YpX, a.YpX ); fe_canon( a.T2d, t );
}

/* j*B for j in [0,128] in affine cached form, then j*(2^128 B) (the
   reference's verify uses a 128-entry odd-multiple B table,
   fd_curve25519_table_ref.c:32; ours holds all multiples 0..128 for signed
   radix-256 windows, and a second table for the high half of the
   half-size-scalar B coefficient, see sc_halfsize). */
DEV void store_cached( u32 * t, ge_cached const & c );   /* A/R table entry layout, below */
DEV void store_affc( u32 * e, ge_affc const & a );       /* B table entry layout, below */

__global__ __launch_bounds__(64) void k_btab_init( u32 * btab ) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= 2*BTAB_N ) return;
  u32 * e = btab + j*BTAB_STRIDE;
  ge_p3 B, P; ge_base( B ); ge_identity( P );
  if( j >= BTAB_N ) {
    j -= BTAB_N;
    for( int q=0; q<128; q++ ) ge_dbl( B, B, true );
  }
  ge_cached Bc; ge_to_cached( Bc, B );
  for( int bit=7; bit>=0; bit-- ) {
    ge_dbl( P, P, true );
    if( (j >> bit) & 1 ) ge_add_cached( P, P, Bc, 0u, true );
  }
  ge_affc a; ge_to_affc_half( a, P );
  store_affc( e, a );
  if( j == 0 && blockIdx.x == 0 ) {             /* the shared identity entry of the A/R tables */
    ge_cached c;
    fe_1( c.YmX ); fe_1( c.YpX ); fe_0( c.T2d ); fe_set( c.Z2, 2,0,0,0,0,0,0,0,0 );
    store_cached( btab + IDENT_OFF, c );
  }
}

/* [j]B and [j](2^132 B) for j in [0,2048], 1/2-scaled affine cached, one
   128-B line each at BT12_OFF */
__global__ __launch_bounds__(64) void k_btab12_init( u32 * btab ) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if( j >= 2*BT12_N ) return;
  u32 * e = btab + BT12_OFF + j*BT12_ENT;
  ge_p3 B, P; ge_base( B ); ge_identity( P );
  if( j >= BT12_N ) {
    j -= BT12_N;
    for( int q=0; q<BTG_HB; q++ ) ge_dbl( B, B, true );
  }
  ge_cached Bc; ge_to_cached( Bc, B );
  for( int bit=BTG_GW-1; bit>=0; bit-- ) {
    ge_dbl( P, P, true );
    if( (j >> bit) & 1 ) ge_add_cached( P, P, Bc, 0u, true );
  }
  ge_affc a; ge_to_affc_half( a, P );
  #pragma unroll
  for( int i=0; i<9; i++ ) { e[i] = a.YmX.v[i]; e[9+i] = a.YpX.v[i]; e[18+i] = a.T2d.v[i]; }
  #pragma unroll
  for( int i=27; i<32; i++ ) e[i] = 0u;
}

DEV int code_of( u32 f, int errmode, bool eq ) {
  if( errmode == FD_ED25519_HIP_ERRMODE_AVX512 ) {
    if( f & F_S_BAD ) return FD_ED25519_ERR_SIG;
    if( f & (F_A_NOTSQ|F_A_ZX|F_R_NOTSQ|F_R_ZX) ) return FD_ED25519_ERR_SIG;  /* decode2 -> -1/-2 -> ERR_SIG */
    if( f & F_A_SMALL ) return FD_ED25519_ERR_PUBKEY;
    if( f & F_R_SMALL ) return FD_ED25519_ERR_SIG;
  } else {
    if( f & F_S_BAD ) return FD_ED25519_ERR_SIG;
    if( f & F_A_NOTSQ ) return FD_ED25519_ERR_PUBKEY;                          /* frombytes_2x -> 1 */
    if( f & F_R_NOTSQ ) return FD_ED25519_ERR_SIG;                             /*             -> 2 */
    if( f & (F_A_SMALL|F_A_ZX) ) return FD_ED25519_ERR_PUBKEY;
    if( f & (F_R_SMALL|F_R_ZX) ) return FD_ED25519_ERR_SIG;
  }
  return eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
}

/* Records ordered by SHA-512 block count (variable-size message paths: the
   txn stream, replay).  A wave hashes for its longest message, and a txn
   stream mixes 2..10-block messages (≤1232-B payloads): in record order a
   wave's maximum is ~9.3 blocks against a mean of ~3.8.  A counting sort on
   the block count (keys clamped to 15) gives k_verify_prep an order[] in
   which waves are uniform; records, state and codes keep their indices.
   Shortest messages first: longest-first shortens a tile batch's prep alone
   (0.68-0.74 vs 0.77-0.78 ms) but C4 with six tiles loses 2-3% (110.6/111.9
   vs 113.7/114.3 M, profiles/r03q_ab_order).
   hist = count[16..31], cursor = count[32..47] (zeroed with count[0]). */
#define ORD_KEYS FD_HIP_ORD_KEYS
DEV u32 msg_key( u32 sz ) { return fd_hip_msg_key( sz ); }

DEV ulong dev_count_n( ulong n, u32 const * d_n, ulong rec0 ) {
  if( !d_n ) return n;
  ulong c = *d_n;
  return c > rec0 ? (c - rec0 < n ? c - rec0 : n) : 0ul;
}

__global__ __launch_bounds__(256)
void k_msg_hist( ulong n, uint const * __restrict__ msz, u32 * __restrict__ count, u32 const * __restrict__ d_n,
                 ulong rec0 ) {
  __shared__ u32 h[ORD_KEYS];
  if( threadIdx.x < ORD_KEYS ) h[threadIdx.x] = 0u;
  __syncthreads();
  n = dev_count_n( n, d_n, rec0 );
  ulong t = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( t < n ) atomicAdd( &h[msg_key( msz[t] )], 1u );
  __syncthreads();
  if( threadIdx.x < ORD_KEYS && h[threadIdx.x] ) atomicAdd( count + 16 + threadIdx.x, h[threadIdx.x] );
}

/* Segmented records (fd_hip_order.h): the segments' histograms summed into
   count[16..31] (k_msg_order's hist) and their record counts into *total
   (prep's device count).  One workgroup. */
__global__ __launch_bounds__(256)
void k_seg_reduce( u32 const * __restrict__ seg, u32 n_seg, u32 * __restrict__ count, u32 * __restrict__ total ) {
  u32 k = threadIdx.x;
  if( k < ORD_KEYS ) {
    u32 h = 0u;
    for( u32 x = 0; x < n_seg; x++ ) h += seg[x*FD_HIP_SEG_STRIDE + FD_HIP_SEG_HIST_W + k];
    count[16 + k] = h;
  } else if( k == ORD_KEYS ) {
    u32 c = 0u;
    for( u32 x = 0; x < n_seg; x++ ) c += seg[x*FD_HIP_SEG_STRIDE + FD_HIP_SEG_CNT_W];
    *total = c;
  }
}

/* count[16..31] = histogram, count[32..47] = cursors.  Record t of the
   launch is active if t < the device count, or, for segmented records
   (seg_cap != 0), if t's place in its segment is below that segment's count;
   order[] receives record indices, densely by block count.  A position past
   the chunk (a histogram that disagrees with msz[]: never, both sides key
   with fd_hip_msg_key) is dropped rather than written out of bounds. */
__global__ __launch_bounds__(256)
void k_msg_order( ulong n, uint const * __restrict__ msz, u32 * __restrict__ count, u32 const * __restrict__ d_n,
                  ulong rec0, u32 * __restrict__ order, ulong chunk, u32 const * __restrict__ seg, ulong seg_cap ) {
  __shared__ u32 h[ORD_KEYS], base[ORD_KEYS];
  if( threadIdx.x < ORD_KEYS ) h[threadIdx.x] = 0u;
  __syncthreads();
  ulong t = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  bool act;
  if( seg_cap ) {
    ulong sx = t / seg_cap;
    act = t < n && t - sx*seg_cap < (ulong)seg[sx*FD_HIP_SEG_STRIDE + FD_HIP_SEG_CNT_W];
  } else {
    act = t < dev_count_n( n, d_n, rec0 );
  }
  u32 key = 0u, r = 0u;
  if( act ) { key = msg_key( msz[t] ); r = atomicAdd( &h[key], 1u ); }   /* rank within the block */
  __syncthreads();
  if( threadIdx.x < ORD_KEYS ) {
    u32 k = threadIdx.x, start = 0u;
    for( u32 j=0; j<k; j++ ) start += count[16 + j];                      /* bucket start: prefix of hist */
    base[k] = h[k] ? start + atomicAdd( count + 32 + k, h[k] ) : 0u;      /* this block's range */
  }
  __syncthreads();
  if( act ) {
    ulong pos = (ulong)base[key] + r;
    if( pos < chunk ) order[pos] = (u32)t;
  }
}

/* SHA-512(R||A||M) with wave-cooperative, LDS-staged message blocks
   (sha512_prefixed_coop; measured against each lane loading its own message
   with dword loads, profiles/r02e_lds_ab: prep 1.879 vs 1.909 ms at C2, C4
   104.2 vs 102.3 M verifies/s) */
#define PREP_MSG_WORDS (64*36)           /* per wave: 64 windows of 144 B */

/* one record slot t of the chunk (n records): checks, decodes, hash, and the
   wave's survivor compaction (all 64 lanes of the wave take part) */
DEV void prep_slot( ulong t, ulong n, ulong chunk, uchar const * __restrict__ sigs, uchar const * __restrict__ pubs,
                    uchar const * __restrict__ pool, uint const * __restrict__ moff, uint const * __restrict__ msz,
                    u32 fixed_sz, u32 * __restrict__ st, int errmode, u32 * __restrict__ idx,
                    u32 * __restrict__ count, signed char * __restrict__ codes, u32 const * __restrict__ order,
                    u32 * lds_msg, u64 * lds_meta ) {
  bool active = t < n;
  /* order (k_msg_order): lane t takes record order[t], so a wave's lanes
     hash messages of the same SHA-512 block count */
  ulong i = active ? (order ? (ulong)order[t] : t) : 0ul;
  ulong const sl = t;                        /* state column and survivor entry: the slot */
  u32 flags = 0u;
  if( active ) {
  u32 * s = st + sl;
  /* decode A then R (user.c:165), one at a time: a rolled loop keeps the two
     pow22523 chains from being interleaved into one register-hungry block
     (measured: pairing the two chains instruction by instruction is slower,
     it costs a wave per SIMD of occupancy) */
  {
    u32 sv[8];
    load_words( sv, sigs + 64*i + 32, 8 );
    flags = sc_is_canonical( sv ) ? 0u : F_S_BAD;                          /* user.c:159-161 */
    #pragma unroll 1
    for( int pt=0; pt<2; pt++ ) {
      u32 w[8];                      /* loaded per point: nothing stays live across the decodes */
      load_words( w, pt ? sigs + 64*i : pubs + 32*i, 8 );
      ge_p3 P;
      u32 f = ge_decode( P, w );
      bool small = !(f & 1u) && ge_affine_is_small_order( P );            /* user.c:194-199 */
      if( pt == 0 ) flags |= ((f & 1u) ? F_A_NOTSQ : 0u) | ((f & 2u) ? F_A_ZX : 0u) | (small ? F_A_SMALL : 0u);
      else          flags |= ((f & 1u) ? F_R_NOTSQ : 0u) | ((f & 2u) ? F_R_ZX : 0u) | (small ? F_R_SMALL : 0u);
      u32 xw[8], yw[8];
      fe_to_words( xw, P.X ); fe_to_words( yw, P.Y );
      u32 base = pt ? ST_RX : ST_AX;
      #pragma unroll
      for( int q=0; q<8; q++ ) { s[(base+q)*chunk] = xw[q]; s[(base+8+q)*chunk] = yw[q]; }
    }
  }
  }
  {
    /* the whole wave hashes together (inactive lanes with an empty message) */
    u32 x[16], k[8];
    uchar const * sp = sigs + 64*i, * pp = pubs + 32*i;  /* inactive lanes: record 0's (valid) R, A */
    asm volatile( "" : "+v"(sp), "+v"(pp) );
    u32 mo = 0u, ms = 0u;
    if( active ) {
      u32 sv[8];                                                           /* S to the state before the */
      load_words( sv, sp + 32, 8 );                                        /* hash: not live across it  */
      u32 * s = st + sl;
      #pragma unroll
      for( int w=0; w<8; w++ ) s[(ST_S+w)*chunk] = sv[w];
      mo = moff ? moff[i] : (u32)i * fixed_sz;
      ms = msz  ? msz[i]  : fixed_sz;
    }
    sha512_prefixed_coop<64u>( x, sp, pp, pool + mo, ms, lds_msg, lds_meta, threadIdx.x & 63u );   /* user.c:205-206 */
    if( active ) {
      sc_reduce512( k, x );                                                /* user.c:207 */
      u32 * s = st + sl;
      #pragma unroll
      for( int w=0; w<8; w++ ) s[(ST_K+w)*chunk] = k[w];
    }
  }
  /* Survivor compaction: a signature that fails a pre-check gets its final
     code here; the others are appended (wave-aggregated atomic, spread over
     the whole prep launch) to idx[] so that k_verify_dsm spends no lanes on
     them (the DSM is VALU-issue bound: a masked lane costs as much as a live
     one). */
  bool pass = active && code_of( flags, FD_ED25519_HIP_ERRMODE_AVX512, true ) == FD_ED25519_SUCCESS;
  if( active && !pass ) codes[i] = (signed char)code_of( flags, errmode, false );
  unsigned long long m = __ballot( pass );
  u32 lane = threadIdx.x & 63u;
  u32 base = 0;
  if( lane == 0u && m ) base = atomicAdd( count, (u32)__popcll( m ) );
  base = __shfl( base, 0 );
  u32 below = (u32)__popcll( m & ((1ULL << lane) - 1ULL) );
  if( pass ) idx[base + below] = (u32)sl;
}

/* one workgroup per 256 records (a persistent grid pulling 64-record tasks,
   as k_verify_dsm does, measured slower on C2: prep 1.98-2.07 vs 1.96-1.98
   ms; C4 within noise) */
/* 4 waves per SIMD (128 VGPRs, ~10 spilled; the LDS windows allow exactly
   4 workgroups per CU) against 3 at the natural 132: C2 134.05 vs 132.92 M
   verifies/s over 6 alternating pairs on two boxes, C4 112.7 vs 112.8
   (profiles/r03ae, profiles/r03af) */
#define PREP_OCCUPANCY __attribute__((amdgpu_waves_per_eu(4, 4)))
__global__ __launch_bounds__(256) PREP_OCCUPANCY
void k_verify_prep( ulong n, ulong chunk, uchar const * __restrict__ sigs, uchar const * __restrict__ pubs,
                    uchar const * __restrict__ pool, uint const * __restrict__ moff, uint const * __restrict__ msz,
                    u32 fixed_sz, u32 * __restrict__ st, int errmode, u32 * __restrict__ idx,
                    u32 * __restrict__ count, signed char * __restrict__ codes, u32 const * __restrict__ d_n,
                    ulong rec0, u32 const * __restrict__ order ) {
  n = dev_count_n( n, d_n, rec0 );            /* device-side count: this chunk starts at record rec0 */
  if( (ulong)blockIdx.x * blockDim.x >= n ) return;
  __shared__ __attribute__((aligned(16))) u32 lds_msg_all[4*PREP_MSG_WORDS];
  __shared__ u64 lds_meta_all[4*64];
  u32 * lds_msg = lds_msg_all + PREP_MSG_WORDS*(threadIdx.x >> 6);
  u64 * lds_meta = lds_meta_all + 64*(threadIdx.x >> 6);
  prep_slot( (ulong)blockIdx.x * blockDim.x + threadIdx.x, n, chunk, sigs, pubs, pool, moff, msz, fixed_sz, st,
             errmode, idx, count, codes, order, lds_msg, lds_meta );
}


/* 9 limbs <-> 8 words.  Every table element is an fe_norm output (limb 0 <
   2^29 + 2^14, limbs 1..7 < 2^29, limb 8 < 2^23) or a product (limb 1 < 2^29 +
   2^17, the others as fe_norm's): one 30-bit limb, seven of 29 bits and one of
   23 = 256 bits.  W30 names the wide limb (0 or 1); offsets are compile-time. */
template<int W30> struct fe_pack_layout {
  static constexpr int off( int j ) { return j == 0 ? 0 : (j <= W30 ? 0 : 1) + 29*j; }
  static constexpr int wid( int j ) { return j == 8 ? 23 : (j == W30 ? 30 : 29); }
};
template<int W30> DEV void fe_pack( u32 w[8], fe const & a ) {
  typedef fe_pack_layout<W30> Lo;
  #pragma unroll
  for( int k=0; k<8; k++ ) w[k] = 0u;
  #pragma unroll
  for( int j=0; j<9; j++ ) {
    int o = Lo::off( j ), k = o >> 5, sh = o & 31;
    w[k] |= a.v[j] << sh;
    if( sh && sh + Lo::wid( j ) > 32 ) w[k+1] |= a.v[j] >> (32 - sh);
  }
}
template<int W30> DEV void fe_unpack( fe & a, u32 const w[8] ) {
  typedef fe_pack_layout<W30> Lo;
  #pragma unroll
  for( int j=0; j<9; j++ ) {
    int o = Lo::off( j ), b = Lo::wid( j ), k = o >> 5, sh = o & 31;
    u32 m = (1u << b) - 1u;
    if( sh + b <= 32 ) a.v[j] = __builtin_amdgcn_ubfe( w[k], (u32)sh, (u32)b );
    else               a.v[j] = __builtin_amdgcn_alignbit( w[k+1], w[k], (u32)sh ) & m;
  }
}
DEV void store_cached( u32 * t, ge_cached const & c ) {   /* 32 words, one 128-B line */
  u32 w[32];
  fe_pack<0>( w, c.YmX ); fe_pack<0>( w + 8, c.YpX ); fe_pack<1>( w + 16, c.T2d ); fe_pack<0>( w + 24, c.Z2 );
  uint4 * q = (uint4 *)t;
  #pragma unroll
  for( int k=0; k<8; k++ ) q[k] = make_uint4( w[4*k], w[4*k+1], w[4*k+2], w[4*k+3] );
}
DEV void load_cached( ge_cached & c, u32 const * t ) {
  uint4 const * q = (uint4 const *)t;
  u32 w[32];
  #pragma unroll
  for( int k=0; k<8; k++ ) { uint4 v = q[k]; w[4*k] = v.x; w[4*k+1] = v.y; w[4*k+2] = v.z; w[4*k+3] = v.w; }
  fe_unpack<0>( c.YmX, w ); fe_unpack<0>( c.YpX, w + 8 ); fe_unpack<1>( c.T2d, w + 16 ); fe_unpack<0>( c.Z2, w + 24 );
}
/* load_cached with Y-X and Y+X exchanged where neg (a per-lane mask): the
   two elements share one packing layout, so negating the entry's point is a
   choice of load address, not a 27-instruction swap (ge_add_cached<true>) */
DEV void load_cached_signed( ge_cached & c, u32 const * t, u32 neg ) {
  uint4 const * q = (uint4 const *)t;
  u32 o = neg & 2u;                                          /* first element at line quad 0 or 2 */
  u32 w[32];
  uint4 v;
  v = q[o];      w[0]  = v.x; w[1]  = v.y; w[2]  = v.z; w[3]  = v.w;
  v = q[o+1u];   w[4]  = v.x; w[5]  = v.y; w[6]  = v.z; w[7]  = v.w;
  v = q[2u-o];   w[8]  = v.x; w[9]  = v.y; w[10] = v.z; w[11] = v.w;
  v = q[3u-o];   w[12] = v.x; w[13] = v.y; w[14] = v.z; w[15] = v.w;
  #pragma unroll
  for( int k=4; k<8; k++ ) { v = q[k]; w[4*k] = v.x; w[4*k+1] = v.y; w[4*k+2] = v.z; w[4*k+3] = v.w; }
  fe_unpack<0>( c.YmX, w ); fe_unpack<0>( c.YpX, w + 8 ); fe_unpack<1>( c.T2d, w + 16 ); fe_unpack<0>( c.Z2, w + 24 );
}
/* one 1/2-scaled affine B-table entry (7 x 16-B loads) */
DEV void store_affc( u32 * e, ge_affc const & a ) {      /* canonical elements: any packing layout fits */
  #pragma unroll
  for( int i=0; i<9; i++ ) { e[i] = a.YmX.v[i]; e[9+i] = a.YpX.v[i]; e[18+i] = a.T2d.v[i]; }
  e[27] = 0u;
}
DEV void load_affc( ge_affc & b, u32 const * bt ) {
  uint4 const * q = (uint4 const *)bt;
  u32 w[28];
  #pragma unroll
  for( int k=0; k<7; k++ ) { uint4 v = q[k]; w[4*k] = v.x; w[4*k+1] = v.y; w[4*k+2] = v.z; w[4*k+3] = v.w; }
  #pragma unroll
  for( int i=0; i<9; i++ ) { b.YmX.v[i] = w[i]; b.YpX.v[i] = w[9+i]; b.T2d.v[i] = w[18+i]; }
}

/* shift a packed 256-bit digit vector left by `bits` (4 or 8) */
DEV void digits_shl( u32 d[8], u32 bits ) {
  #pragma unroll
  for( int i=7; i>0; i-- ) d[i] = __builtin_amdgcn_alignbit( d[i], d[i-1], 32u - bits );
  d[0] <<= bits;
}

/* verdict bitmap from codes: bit i%64 of word i/64 set iff codes[i]==0 */
__global__ __launch_bounds__(256)
void k_bitmap( ulong n, signed char const * __restrict__ codes, ulong * __restrict__ bitmap,
               u32 const * __restrict__ d_n, ulong rec0 ) {
  ulong i = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( d_n ) { ulong c = *d_n; n = c > rec0 ? (c - rec0 < n ? c - rec0 : n) : 0ul; }
  bool ok = i < n && codes[i] == FD_ED25519_SUCCESS;
  unsigned long long b = __ballot( ok );
  if( (threadIdx.x & 63u) == 0u && i < n ) {
    /* the word holding record n-1: with a device-side count, bits at or past
       *d_n belong to no record of this call and keep their value; with a
       host count they are zero, as the ballot leaves them
       (include/fd_ed25519_hip.h) */
    ulong left = n - i;
    if( d_n && left < 64ul ) {
      unsigned long long m = (1ULL << left) - 1ULL;
      b = (bitmap[i >> 6] & ~m) | (b & m);
    }
    bitmap[i >> 6] = b;
  }
}

/* table [1..8]Q in cached form for Q = (qx, qy) affine (fd_curve25519.c:
   130-143), entry j at (j-1)*ATAB_ENT (the identity is the shared entry at
   IDENT_OFF): Q, 2Q, then (j+1)Q = jQ + Q -- a chain keeps one point and Q's
   cached form live */
DEV void build_cached_table( u32 * tab, fe const & qx, fe const & qy ) {
  ge_p3 Q; Q.X = qx; Q.Y = qy; fe_1( Q.Z ); fe_mul( Q.T, Q.X, Q.Y );
  ge_cached c;
  ge_cached c1; ge_to_cached( c1, Q ); store_cached( tab + 0*ATAB_ENT, c1 );
  ge_p3 Pj;
  ge_dbl( Pj, Q, true ); ge_to_cached( c, Pj ); store_cached( tab + 1*ATAB_ENT, c );
  #pragma unroll 1
  for( int j=3; j<=8; j++ ) {
    ge_add_cached_z1( Pj, Pj, c1 ); ge_to_cached( c, Pj ); store_cached( tab + (j-1)*ATAB_ENT, c );
  }
}

/* entry for digit magnitude mag in 0..8: the lane's table, or the shared
   identity for 0 (a select by mask, no v_cndmask) */
DEV u32 const * tab_entry( u32 const * tab, u32 const * ident, u32 mag ) {
  u32 m = (u32)((int)(0u - mag) >> 31);                 /* mag != 0 ? ~0 : 0 */
  u64 t = (u64)(tab + ((mag - 1u) & m) * ATAB_ENT), id = (u64)ident;
  u64 mm = ((u64)m << 32) | m;
  return (u32 const *)(id ^ ((t ^ id) & mm));
}

/* biased signed digit -> (negate mask, magnitude) */
DEV void digit_split( u32 d, u32 bias, u32 & neg, u32 & mag ) {
  int v = (int)d - (int)bias;
  neg = (u32)(v >> 31);
  mag = ((u32)v ^ neg) - neg;
}

/* shift 16 packed radix-256 digits left by one digit */
DEV void digits_shl4( u32 d[4] ) {
  d[3] = __builtin_amdgcn_alignbit( d[3], d[2], 24u );
  d[2] = __builtin_amdgcn_alignbit( d[2], d[1], 24u );
  d[1] = __builtin_amdgcn_alignbit( d[1], d[0], 24u );
  d[0] <<= 8;
}

/* maximum of v < 128 over the wave's active lanes (wave-uniform result) */
DEV u32 wave_max7( u32 v ) {
  u32 m = 0u;
  #pragma unroll
  for( int b=6; b>=0; b-- ) { u32 c = m | (1u << b); if( __ballot( v >= c ) ) m = c; }
  return m;
}

/* k_verify_dsm's register allocation is held to 3 waves per SIMD (the task
   loop alone takes the compiler to 172 VGPRs, 2 waves) */
#define DSM_OCCUPANCY __attribute__((amdgpu_waves_per_eu(3, 3)))

/* signed radix-2^GW digits of sp (< 2^253) for the two global B tables:
   digit i = r_i + c_i - 2^GW c_{i+1}, r_i = bits [GW i, GW i + GW), carry
   bits c in bmask; digits 0..ND-1 against [j]B, ND..2ND-1 against
   [j](2^HB B).  Both halves are held as 160-bit groups whose top GW bits are
   the next digit (consumed top-down): bl = sp << (160-HB) (bits 0..HB-1),
   bh = sp >> (2HB-160) (bits HB.. on top; the bits below are never read). */
DEV void b12_digits( u32 bl[5], u32 bh[5], u32 & bmask, u32 const sp[8] ) {
  constexpr int GW = BTG_GW, ND = BTG_ND, HB = BTG_HB;
  u32 c = 0u; bmask = 0u;
  #pragma unroll
  for( int i=0; i<2*ND; i++ ) {
    int b = GW*i, wi = b >> 5, sh = b & 31;
    u32 x = (sh + GW <= 32) ? (sp[wi] >> sh)
                            : __builtin_amdgcn_alignbit( wi < 7 ? sp[wi+1] : 0u, sp[wi], (u32)sh );
    u32 d = (x & ((1u << GW) - 1u)) + c;
    c = d >= (1u << (GW-1)) ? 1u : 0u;
    bmask |= c << (i+1);
  }
  /* lo = (sp mod 2^HB) << (160-HB): sp bit HB would land at group bit 160,
     so nothing above the low half enters; hi = sp >> (2HB-160): its top
     ND*GW bits are sp's bits from HB up (the bits below are never read) */
  constexpr int LS = 160 - HB, HS = 2*HB - 160;
  #pragma unroll
  for( int q=0; q<5; q++ ) {
    int b = 32*q - LS;                           /* sp bit at the group word's bit 0 */
    u32 lo_w = b + 32 <= 0 ? 0u : b < 0 ? (sp[0] << (-b)) :
               (b & 31) ? __builtin_amdgcn_alignbit( sp[(b>>5)+1], sp[b>>5], (u32)(b & 31) ) : sp[b>>5];
    bl[q] = lo_w;
    int hb = 32*q + HS, hw = hb >> 5, hsh = hb & 31;
    u32 hx = hw + 1 <= 7 ? sp[hw+1] : 0u, hy = hw <= 7 ? sp[hw] : 0u;
    bh[q] = hsh ? __builtin_amdgcn_alignbit( hx, hy, (u32)hsh ) : hy;
  }
}

/* lane-parallel group law for k_verify_lat (see there).  Its products use
   open sums (fe_mul_free / fe_sq_free): a wave alone on its SIMD gains from
   the extra independent chains (single verify p50 299-303 vs 320-323 us,
   profiles/r02zd_latency_lp/ab_free) */
DEV void lp_mul( fe & r, fe const & a, fe const & b ) { fe_mul_free( r, a, b ); }
DEV void lp_sq( fe & r, fe const & a ) { fe_sq_free( r, a ); }

DEV u32 lp_lane( void ) { return threadIdx.x & 63u; }

/* every lane of the quad gets lane K's value of x (DPP quad_perm [K,K,K,K]) */
template<int K>
DEV void fe_bcast( fe & r, fe const & x ) {
  #pragma unroll
  for( int q=0; q<9; q++ ) r.v[q] = (u32)__builtin_amdgcn_mov_dpp( (int)x.v[q], K * 0x55, 0xf, 0xf, false );
}

/* lane l (0..3) picks operand l: three bit-selects (v_bfi) per limb, no branches */
DEV void fe_pick4( fe & r, fe const & a0, fe const & a1, fe const & a2, fe const & a3, u32 l ) {
  u32 m0 = 0u - (u32)(l == 0u), m1 = 0u - (u32)(l == 1u), m2 = 0u - (u32)(l == 2u);
  #pragma unroll
  for( int q=0; q<9; q++ ) {
    u32 t = (m2 & a2.v[q]) | (~m2 & a3.v[q]);
    t = (m1 & a1.v[q]) | (~m1 & t);
    r.v[q] = (m0 & a0.v[q]) | (~m0 & t);
  }
}

/* X3 = E*F, Y3 = G*H, Z3 = F*G, T3 = E*H, one product per lane */
DEV void lp_efgh( ge_p3 & r, fe const & E, fe const & F, fe const & G, fe const & H ) {
  u32 l = lp_lane();
  fe a, b, p;
  fe_pick4( a, E, G, F, E, l );
  fe_pick4( b, F, H, G, H, l );
  lp_mul( p, a, b );
  fe_bcast<0>( r.X, p ); fe_bcast<1>( r.Y, p ); fe_bcast<2>( r.Z, p ); fe_bcast<3>( r.T, p );
}

/* ge_dbl on lanes 0..3 (p uniform over them; r uniform on return, T always) */
DEV void ge_dbl_lp( ge_p3 & r, ge_p3 const & p ) {
  fe S, o, s, A, B, C, S2, H, G, F, E;
  fe_add( S, p.X, p.Y );
  fe_pick4( o, p.X, p.Y, p.Z, S, lp_lane() );
  lp_sq( s, o );
  fe_bcast<0>( A, s ); fe_bcast<1>( B, s ); fe_bcast<2>( C, s ); fe_bcast<3>( S2, s );
  fe_add( C, C, C );          /* 2Z^2            */
  fe_add( H, A, B );          /* A+B             */
  fe_sub( G, A, B );          /* A-B             */
  fe_add( F, C, G );          /* 2Z^2+A-B        */
  fe_norm( F, F );
  fe_sub( E, H, S2 );         /* A+B-(X+Y)^2     */
  fe_norm( E, E );
  lp_efgh( r, E, F, G, H );
}

/* ge_add_cached on lanes 0..3 (T always produced) */
DEV void ge_add_cached_lp( ge_p3 & r, ge_p3 const & p, ge_cached q, u32 neg ) {
  fe a, b, x, y, m, A, B, C, D, E, F, G, H;
  fe_cswap( q.YmX, q.YpX, neg );
  fe_sub( a, p.Y, p.X ); fe_add( b, p.Y, p.X );
  u32 l = lp_lane();
  fe_pick4( x, a, b, p.T, p.Z, l );
  fe_pick4( y, q.YmX, q.YpX, q.T2d, q.Z2, l );
  lp_mul( m, x, y );
  fe_bcast<0>( A, m ); fe_bcast<1>( B, m ); fe_bcast<2>( C, m ); fe_bcast<3>( D, m );
  fe_sub( E, B, A ); fe_norm( E, E ); fe_add( H, B, A );
  fe_sub( F, D, C ); fe_add( G, D, C );
  fe_cswap( F, G, neg );
  lp_efgh( r, E, F, G, H );
}

/* ge_add_affc on lanes 0..3 (T always produced): products a*YmX, b*YpX,
   T*T2d (lane 3 repeats lane 2's), then D = Z1 */
DEV void ge_add_affc_lp( ge_p3 & r, ge_p3 const & p, ge_affc q, u32 neg ) {
  fe a, b, x, y, m, A, B, C, E, F, G, H;
  fe_cswap( q.YmX, q.YpX, neg );
  fe_sub( a, p.Y, p.X ); fe_add( b, p.Y, p.X );
  u32 l = lp_lane();
  fe_pick4( x, a, b, p.T, p.T, l );
  fe_pick4( y, q.YmX, q.YpX, q.T2d, q.T2d, l );
  lp_mul( m, x, y );
  fe_bcast<0>( A, m ); fe_bcast<1>( B, m ); fe_bcast<2>( C, m );
  fe_sub( E, B, A ); fe_norm( E, E ); fe_add( H, B, A );
  fe_sub( F, p.Z, C ); fe_add( G, p.Z, C );
  fe_cswap( F, G, neg );
  lp_efgh( r, E, F, G, H );
}

/* build_cached_table on lanes 0..3 (k_verify_lat): 2Q and the additions of
   Q's cached form (2*Z = 2, the general cached addition) lane-parallel */
DEV void build_cached_table_lp( u32 * tab, fe const & qx, fe const & qy ) {
  ge_p3 Q; Q.X = qx; Q.Y = qy; fe_1( Q.Z ); fe_mul( Q.T, Q.X, Q.Y );
  ge_cached c, c1; ge_to_cached( c1, Q ); store_cached( tab + 0*ATAB_ENT, c1 );
  ge_p3 Pj;
  ge_dbl_lp( Pj, Q ); ge_to_cached( c, Pj ); store_cached( tab + 1*ATAB_ENT, c );
  #pragma unroll 1
  for( int j=3; j<=8; j++ ) {
    ge_add_cached_lp( Pj, Pj, c1, 0u ); ge_to_cached( c, Pj ); store_cached( tab + (j-1)*ATAB_ENT, c );
  }
}

/* P += [digit bi]B + [digit bi+ND](2^HB B) from the global tables, digits
   taken off the top of bl / bh (b12_digits); T of the result if needT */
template<bool LP = false>
DEV void b12_step( ge_p3 & P, u32 bl[5], u32 bh[5], u32 bmask, u32 bi, u32 const * __restrict__ btab,
                   bool needT ) {
  constexpr u32 GW = BTG_GW, ND = BTG_ND;
  u32 negb, ib, negc, ic;
  {
    int v = (int)((bl[4] >> (32u-GW)) + ((bmask >> bi) & 1u)) - (int)(((bmask >> (bi+1u)) & 1u) << GW);
    negb = (u32)(v >> 31); ib = ((u32)v ^ negb) - negb;
    v = (int)((bh[4] >> (32u-GW)) + ((bmask >> (bi+ND)) & 1u)) - (int)(((bmask >> (bi+ND+1u)) & 1u) << GW);
    negc = (u32)(v >> 31); ic = ((u32)v ^ negc) - negc;
  }
  #pragma unroll
  for( int q=4; q>0; q-- ) {
    bl[q] = __builtin_amdgcn_alignbit( bl[q], bl[q-1], 32u-GW );
    bh[q] = __builtin_amdgcn_alignbit( bh[q], bh[q-1], 32u-GW );
  }
  bl[0] <<= GW; bh[0] <<= GW;
  u32 const * bt = btab + BT12_OFF;
  ge_affc b; load_affc( b, bt + ib*BT12_ENT );
  if( LP ) ge_add_affc_lp( P, P, b, negb ); else ge_add_affc( P, P, b, negb, true );
  load_affc( b, bt + (BT12_N + ic)*BT12_ENT );
  if( LP ) ge_add_affc_lp( P, P, b, negc ); else ge_add_affc( P, P, b, negc, needT );
}

/* one survivor: DSM slot t (tables at slot t), state column idx[t] (prep's
   slot), record order[idx[t]] */
DEV void dsm_verify_slot( ulong t, ulong chunk, u32 const * __restrict__ st, u32 const * __restrict__ btab,
                          u32 * __restrict__ atab, u32 const * __restrict__ idx, signed char * __restrict__ codes,
                          int halfsize, u32 const * __restrict__ order ) {
  ulong p = idx[t];
  ulong i = order ? (ulong)order[p] : p;
  ulong ii = t;                                            /* table slot: dense in t */
  u32 const * s = st + p;
  bool eq = false;
  {
    /* ---- half-size scalars (sc_halfsize): the reference's check
       [S]B - [k]A == R (user.c:216-226) becomes
       [k2*S mod L]B - [k1]A - [k2]R == O with k1, k2 ~ 2^128 ---- */
    u32 kd1[8], kd2[8], bl[5], bh[5], bmask, k1neg, D;
    {
      u32 k[8], S[8], k1[8], k2[8], sp[8];
      #pragma unroll
      for( int w=0; w<8; w++ ) { k[w] = s[(ST_K+w)*chunk]; S[w] = s[(ST_S+w)*chunk]; }
      u32 bits;
      if( halfsize ) bits = sc_halfsize( k1, k1neg, k2, k );
      else {                        /* full-length pair (k, 1): the same equation, 64 windows */
        #pragma unroll
        for( int w=0; w<8; w++ ) { k1[w] = k[w]; k2[w] = w ? 0u : 1u; }
        k1neg = 0u; bits = 253u;
      }
      sc_mul( sp, k2, S );
      sc_recode16s( kd1, k1 ); sc_recode16s( kd2, k2 );
      b12_digits( bl, bh, bmask, sp );                       /* signed radix-2^12 digits of sp */
      D = max( (bits >> 2) + 1u, 31u );   /* windows; >= 31 so all 11 B digit pairs (windows 30, 27, .., 0) are reached */
    }
    D = wave_max7( D );             /* one window count per wave: no divergence in the loop */
    #pragma unroll 1
    for( u32 q = D; q < 64u; q++ ) { digits_shl( kd1, 4u ); digits_shl( kd2, 4u ); }

    /* ---- tables [0..8](+-A) and [0..8](-R) (fd_curve25519.c:130-143) ---- */
    u32 * tabA = atab + ii * ATAB_WORDS, * tabR = tabA + RTAB_OFF;
    u32 const * ident = btab + IDENT_OFF;
    {
      fe x, y, nx;
      u32 xw[8], yw[8];
      #pragma unroll
      for( int w=0; w<8; w++ ) { xw[w] = s[(ST_AX+w)*chunk]; yw[w] = s[(ST_AY+w)*chunk]; }
      fe_from_words( x, xw ); fe_from_words( y, yw );
      fe_neg( nx, x ); fe_norm( nx, nx ); fe_cmov( nx, x, k1neg );      /* k1 < 0: [|k1|](+A) */
      build_cached_table( tabA, nx, y );
      #pragma unroll
      for( int w=0; w<8; w++ ) { xw[w] = s[(ST_RX+w)*chunk]; yw[w] = s[(ST_RY+w)*chunk]; }
      fe_from_words( x, xw ); fe_from_words( y, yw );
      fe_neg( nx, x ); fe_norm( nx, nx );
      build_cached_table( tabR, nx, y );
    }

    /* ---- [k1](+-A) + [k2](-R) + [s']B, signed radix-16 windows for k1, k2
       and radix-2^12 digit pairs for s' every third window ---- */
    ge_p3 P; ge_identity( P );
    #pragma unroll 1
    for( int w=(int)D-1; w>=0; w-- ) {
      u32 nega, ia, negr, ir;
      digit_split( kd1[7] >> 28, 7u, nega, ia ); digits_shl( kd1, 4u );
      digit_split( kd2[7] >> 28, 7u, negr, ir ); digits_shl( kd2, 4u );
      /* issued before the window's 4 doublings, which hide its latency */
      ge_cached e; load_cached_signed( e, tab_entry( tabA, ident, ia ), nega );
      if( w != (int)D-1 ) {
        #pragma unroll 1
        for( int j=0; j<3; j++ ) ge_dbl( P, P, false );
        ge_dbl( P, P, true );
      }
      ge_add_cached<true>( P, P, e, nega, true );
      load_cached_signed( e, tab_entry( tabR, ident, ir ), negr );
      /* windows (ND-1)*STEP, .., STEP, 0: lo digits ND-1..0, hi digits 2ND-1..ND */
      bool bw = w <= (BTG_ND-1)*BTG_STEP && w % BTG_STEP == 0;
      ge_add_cached<true>( P, P, e, negr, bw );
      if( bw ) b12_step( P, bl, bh, bmask, (u32)w / (u32)BTG_STEP, btab, false );
    }

    /* ---- P == O: X == 0 and Y == Z (Z != 0: complete formulas) ---- */
    fe x, y, z;
    fe_canon( x, P.X ); fe_canon( y, P.Y ); fe_canon( z, P.Z );
    eq = fe_is_zero_c( x ) && fe_eq_c( y, z );
  }
  codes[i] = (signed char)(eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG);   /* user.c:226-229 */
}

/* Persistent grid: resident workgroups (ctx->dsm_wgs, ~3 per CU) pull
   64-survivor tasks from a counter (count[1]) until none is left, instead of
   one workgroup per 256 survivors: no partial last round of waves (measured
   against the one-shot grid at C4: 103.2-103.7 vs 100.0 M verifies/s).
   Every wave leaves the loop when the counter passes m, so the grid drains. */

__global__ __launch_bounds__(256) DSM_OCCUPANCY
void k_verify_dsm( ulong chunk, u32 const * __restrict__ st, u32 const * __restrict__ btab,
                   u32 * __restrict__ atab, u32 const * __restrict__ idx, u32 * __restrict__ count,
                   signed char * __restrict__ codes, int halfsize, u32 const * __restrict__ order ) {
  u32 m = count[0];
  if( (ulong)blockIdx.x * blockDim.x >= m ) return;        /* whole workgroup past the survivors */
  for( ;; ) {
    u32 task = 0u;
    if( (threadIdx.x & 63u) == 0u ) task = atomicAdd( count + 1, 1u );
    task = __shfl( task, 0 );
    if( (ulong)task * 64ul >= (ulong)m ) break;                       /* wave-uniform exit */
    ulong t = (ulong)task * 64ul + (threadIdx.x & 63u);
    if( t < m ) dsm_verify_slot( t, chunk, st, btab, atab, idx, codes, halfsize, order );
  }
}

/**********************************************************************/
/* Latency path (small batches, the drop-in's single calls): one signature
   per workgroup of three waves, each wave running one lane.  The bulk
   kernels spend one lane per signature for the whole verify, which is what
   throughput wants and what makes a lone call slow (one wave issuing the
   decodes, the hash and every doubling in sequence).  Here the independent
   pieces run side by side:
     phase 1  wave 0 decodes A, wave 1 decodes R (each a pow22523 chain),
              wave 2 checks S, hashes R||A||M, reduces mod L, splits k into
              half-size scalars (sc_halfsize) and recodes all digits;
     phase 2  wave 0 [k1](+-A) and wave 1 [k2](-R) (each its own table and
              doubling chain), wave 2 [k2*S mod L]B from the two global
              radix-2^12 tables (10 x 12 doublings, 22 additions);
     phase 3  one lane adds the three points and checks P == O.
   The equation, the pre-check order and the codes are k_verify_prep's and
   k_verify_dsm's (fd_ed25519_user.c:135-230). */

#define LAT_MAX_N 256ul      /* the largest call fd_ed25519_hip_set_small_batch can send down this path */
#define LAT_DEFAULT_N 32ul   /* default: calls of up to 32 records (tools/bench_batch_latency.py with the
                                lane-parallel chains: this path 334-493 us vs 770-781 us at 1-32
                                records; the bulk kernels win from 64 up, 686 vs 721 us,
                                profiles/r02zd_latency_lp) */
/* Four waves: three working, one that only waits through the barriers.  At
   k_verify_lat's 120 VGPRs a CU holds four such workgroups.  A lone working
   wave is latency-bound, so workgroups sharing a CU barely slow each other
   (192 signatures x 4 copies on 768 workgroups: 771 us vs 698 us for one copy,
   profiles/r03l); and the copies are what matter: a lone workgroup runs
   ~270 us on some CU slots and ~600 us on the others (profiles/r03k).  Against
   768-thread workgroups (one per CU): 16 C callers x 12 signatures through the
   drop-in 0.32-0.33 vs 0.23 M signatures/s, lone calls the same
   (profiles/r03n). */
#define LAT_WG 256
#define LAT_WG_PER_CU 4
#define LAT_COPIES_MAX 16u   /* racing copies of a signature (a lone call's 8..16: p50 323 vs 437 us at 12 signatures) */

struct lat_shared {
  u32 ax[8], ay[8], rx[8], ry[8];   /* canonical decoded coordinates */
  u32 fa, fr, fs;                   /* pre-check flags per wave */
  u32 kd1[8], kd2[8];               /* signed radix-16 digits of |k1|, k2 */
  u32 k1neg, D;                     /* k1 < 0; windows of the A and R chains */
  u32 bl[5], bh[5], bmask;          /* radix-2^12 digits of k2*S mod L */
  u32 P[3][36];                     /* the three partial points (X, Y, Z, T) */
};

DEV void lat_put( u32 * d, ge_p3 const & P ) {
  #pragma unroll
  for( int q=0; q<9; q++ ) { d[q] = P.X.v[q]; d[9+q] = P.Y.v[q]; d[18+q] = P.Z.v[q]; d[27+q] = P.T.v[q]; }
}
DEV void lat_get( ge_p3 & P, u32 const * d ) {
  #pragma unroll
  for( int q=0; q<9; q++ ) { P.X.v[q] = d[q]; P.Y.v[q] = d[9+q]; P.Z.v[q] = d[18+q]; P.T.v[q] = d[27+q]; }
}

/* The latency kernel's chains run their group law on lanes 0..3 of the
   wave instead of lane 0 alone.  Each formula is two rounds of four
   independent products (dbl: X^2, Y^2, Z^2, (X+Y)^2, then E*F, G*H, F*G,
   E*H; add: the four operand products, then the same four); lane l computes
   product l of a round and a DPP quad broadcast hands the four results to every lane,
   which then holds the whole point.  The values and their normalisation
   points are those of ge_dbl / ge_add_cached (same bounds), so a chain issues
   about 2.2x fewer instructions for the same result (single verify p50
   320-322 vs 472-473 us, profiles/r02zd_latency_lp/ab_full). */

/* another copy of signature i already finished this call (seq); the first
   active lane's reading, so that a lane-parallel chain leaves its loop as a
   whole */
DEV bool lat_done( ulong const * done, ulong i, ulong seq ) {
  ulong v = __hip_atomic_load( done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  u32 lo = (u32)__builtin_amdgcn_readfirstlane( (int)(u32)v );
  u32 hi = (u32)__builtin_amdgcn_readfirstlane( (int)(u32)(v >> 32) );
  return (((ulong)hi << 32) | lo) == seq;
}

/* [k](Q) by fixed signed radix-16 windows over a lane's table (digits kd,
   biased by 7, D windows from the top); T of the result is produced.  With
   copies, it stops early once another copy has finished (the result is then
   never used). */
DEV void lat_chain( ge_p3 & P, u32 const * tab, u32 const * ident, u32 kd[8], u32 D, ulong const * done, ulong i,
                    ulong seq, u32 copies ) {
  #pragma unroll 1
  for( u32 q = D; q < 64u; q++ ) digits_shl( kd, 4u );
  ge_identity( P );
  #pragma unroll 1
  for( int w=(int)D-1; w>=0; w-- ) {
    u32 neg, mag;
    digit_split( kd[7] >> 28, 7u, neg, mag ); digits_shl( kd, 4u );
    ge_cached e; load_cached( e, tab_entry( tab, ident, mag ) );
    if( w != (int)D-1 ) {
      #pragma unroll 1
      for( int j=0; j<4; j++ ) ge_dbl_lp( P, P );
    }
    ge_add_cached_lp( P, P, e, neg );
    if( copies > 1u && lat_done( done, i, seq ) ) break;
  }
}

/* copies > 1: each signature gets that many consecutive workgroups (the
   dispatcher deals consecutive workgroups to the XCDs in turn, so they land
   on different CUs), all computing the same verdict; the first to finish
   writes the code and tags done[i] with this call's seq, and the others stop
   at their next window.  A lone workgroup is fast or slow by the state of
   the CU it lands on (415-1068 us per call for one copy; the shader clock is
   the same 2.39 GHz on every launch, tools/xcd_clock; profiles/r03k, r03x),
   so racing copies takes the fastest: up to ctx->lat_copies
   (LAT_COPIES_MAX, 16) per signature, at most one workgroup per CU over the
   whole call and within the context's lat_cus budget (verify_impl).  Every
   copy writes the same code, so a tie is harmless, and done[] is only an
   early-exit hint: the host reads the codes after the whole launch. */
__global__ __launch_bounds__(LAT_WG)
void k_verify_lat( ulong n, uchar const * __restrict__ sigs, uchar const * __restrict__ pubs,
                   uchar const * __restrict__ pool, uint const * __restrict__ moff, uint const * __restrict__ msz,
                   u32 fixed_sz, u32 const * __restrict__ btab, u32 * __restrict__ atab, int errmode,
                   int halfsize, signed char * __restrict__ codes, u32 copies, ulong * __restrict__ done, ulong seq ) {
  __shared__ lat_shared L;
  ulong i = blockIdx.x / copies;
  if( i >= n ) return;                                     /* workgroup-uniform */
  /* wave 3 does no work but stays through both barriers */
  u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  u32 * tabA = atab + (ulong)blockIdx.x * ATAB_WORDS, * tabR = tabA + RTAB_OFF;   /* per copy */
  u32 const * ident = btab + IDENT_OFF;

  /* ---- phase 1 ---- */
  if( lane == 0u && wave < 3u ) {
    if( wave < 2u ) {                                    /* decode A (wave 0) or R (wave 1), user.c:165-199 */
      u32 w[8];
      load_words( w, wave ? sigs + 64*i : pubs + 32*i, 8 );
      ge_p3 Q;
      u32 f = ge_decode<true>( Q, w );                     /* open-sum products (lp_mul) */
      bool small = !(f & 1u) && ge_affine_is_small_order( Q );
      u32 xw[8], yw[8];
      fe_to_words( xw, Q.X ); fe_to_words( yw, Q.Y );
      if( wave == 0u ) {
        L.fa = ((f & 1u) ? F_A_NOTSQ : 0u) | ((f & 2u) ? F_A_ZX : 0u) | (small ? F_A_SMALL : 0u);
        #pragma unroll
        for( int q=0; q<8; q++ ) { L.ax[q] = xw[q]; L.ay[q] = yw[q]; }
      } else {
        L.fr = ((f & 1u) ? F_R_NOTSQ : 0u) | ((f & 2u) ? F_R_ZX : 0u) | (small ? F_R_SMALL : 0u);
        #pragma unroll
        for( int q=0; q<8; q++ ) { L.rx[q] = xw[q]; L.ry[q] = yw[q]; }
      }
    } else {                                             /* S < L, k = H(R||A||M) mod L, half-size split */
      u32 sig[16], pub[8], k[8], k1[8], k2[8], sp[8], k1neg, bits;
      load_words( sig, sigs + 64*i, 16 );
      load_words( pub, pubs + 32*i, 8 );
      L.fs = sc_is_canonical( sig + 8 ) ? 0u : F_S_BAD;                   /* user.c:159-161 */
      u32 mo = moff ? moff[i] : (u32)i * fixed_sz;
      u32 ms = msz  ? msz[i]  : fixed_sz;
      hram_mod_l( k, sig, pub, pool + mo, ms );                            /* user.c:205-207 */
      if( halfsize ) bits = sc_halfsize( k1, k1neg, k2, k );
      else {
        #pragma unroll
        for( int w=0; w<8; w++ ) { k1[w] = k[w]; k2[w] = w ? 0u : 1u; }
        k1neg = 0u; bits = 253u;
      }
      sc_mul( sp, k2, sig + 8 );
      u32 kd1[8], kd2[8], bl[5], bh[5], bmask;
      sc_recode16s( kd1, k1 ); sc_recode16s( kd2, k2 );
      b12_digits( bl, bh, bmask, sp );
      #pragma unroll
      for( int q=0; q<8; q++ ) { L.kd1[q] = kd1[q]; L.kd2[q] = kd2[q]; }
      #pragma unroll
      for( int q=0; q<5; q++ ) { L.bl[q] = bl[q]; L.bh[q] = bh[q]; }
      L.bmask = bmask; L.k1neg = k1neg; L.D = (bits >> 2) + 1u;
    }
  }
  __syncthreads();
  u32 flags = L.fa | L.fr | L.fs;
  if( code_of( flags, FD_ED25519_HIP_ERRMODE_AVX512, true ) != FD_ED25519_SUCCESS ) {   /* workgroup-uniform */
    if( threadIdx.x == 0u ) {
      codes[i] = (signed char)code_of( flags, errmode, false );
      if( copies > 1u ) __hip_atomic_store( done + i, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
    }
    return;
  }

  /* ---- phase 2 (lanes 0..3 of waves 0..2) ---- */
  if( lane < 4u && wave < 3u ) {
    ge_p3 P;
    if( wave < 2u ) {
      u32 xw[8], yw[8], kd[8];
      #pragma unroll
      for( int q=0; q<8; q++ ) {
        xw[q] = wave ? L.rx[q] : L.ax[q]; yw[q] = wave ? L.ry[q] : L.ay[q];
        kd[q] = wave ? L.kd2[q] : L.kd1[q];
      }
      fe x, y, nx;
      fe_from_words( x, xw ); fe_from_words( y, yw );
      fe_neg( nx, x ); fe_norm( nx, nx );
      if( wave == 0u ) fe_cmov( nx, x, L.k1neg );                          /* k1 < 0: [|k1|](+A) */
      u32 * tab = wave ? tabR : tabA;
      build_cached_table_lp( tab, nx, y );
      lat_chain( P, tab, ident, kd, L.D, done, i, seq, copies );
    } else {
      u32 bl[5], bh[5];
      #pragma unroll
      for( int q=0; q<5; q++ ) { bl[q] = L.bl[q]; bh[q] = L.bh[q]; }
      u32 bmask = L.bmask;
      ge_identity( P );
      #pragma unroll 1
      for( int bi=(int)BTG_ND-1; bi>=0; bi-- ) {
        if( bi != (int)BTG_ND-1 ) {
          #pragma unroll 1
          for( int j=0; j<BTG_GW; j++ ) ge_dbl_lp( P, P );
        }
        b12_step<true>( P, bl, bh, bmask, (u32)bi, btab, true );
        if( copies > 1u && lat_done( done, i, seq ) ) break;
      }
    }
    if( lane == 0u ) lat_put( L.P[wave], P );
  }
  __syncthreads();

  /* ---- phase 3: P_A + P_R + P_B == O (user.c:216-229) ----
     done is monotonic within a call: a chain that stopped early saw it set,
     so this check sees it too and the partial points are never used */
  if( threadIdx.x == 0u && !(copies > 1u && lat_done( done, i, seq )) ) {
    ge_p3 P, Q; ge_cached c;
    lat_get( P, L.P[0] );
    lat_get( Q, L.P[1] ); ge_to_cached( c, Q ); ge_add_cached( P, P, c, 0u, true );
    lat_get( Q, L.P[2] ); ge_to_cached( c, Q ); ge_add_cached( P, P, c, 0u, false );
    fe x, y, z;
    fe_canon( x, P.X ); fe_canon( y, P.Y ); fe_canon( z, P.Z );
    bool eq = fe_is_zero_c( x ) && fe_eq_c( y, z );
    codes[i] = (signed char)(eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG);
    if( copies > 1u ) __hip_atomic_store( done + i, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  }
}

/* fd_ed25519_verify_batch_single_msg (user.c:232-310) over per-sig codes */
__global__ void k_group_reduce( ulong ng, uint const * first, uchar const * cnt, signed char const * sc,
                                signed char * gc ) {
  ulong g = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( g >= ng ) return;
  uint f = first[g], c = cnt[g];
  int r;
  if( c == 0u || c > 16u ) r = FD_ED25519_ERR_SIG;
  else {
    r = FD_ED25519_SUCCESS;
    int msg_fail = 0;
    for( uint j=0; j<c; j++ ) {
      int x = sc[f+j];
      if( x == FD_ED25519_ERR_SIG || x == FD_ED25519_ERR_PUBKEY ) { r = x; break; }
      if( x == FD_ED25519_ERR_MSG ) msg_fail = 1;
    }
    if( r == FD_ED25519_SUCCESS && msg_fail ) r = FD_ED25519_ERR_MSG;
  }
  gc[g] = (signed char)r;
}

/* [s]B for s < 2^253 with the radix-256 B table (signing) */
DEV void ge_scalarmult_base( ge_p3 & P, u32 const s[8], u32 const * lds_btab ) {
  u32 sd[8]; sc_recode256( sd, s );
  ge_identity( P );
  #pragma unroll 1
  for( int j=31; j>=0; j-- ) {
    if( j != 31 ) {
      #pragma unroll 1
      for( int q=0; q<7; q++ ) ge_dbl( P, P, false );
      ge_dbl( P, P, true );
    }
    u32 db = sd[7] >> 24; digits_shl( sd, 8u );
    int sb = (int)db - 128;
    u32 negb = sb < 0 ? ~0u : 0u;
    u32 ib = (u32)(sb < 0 ? -sb : sb);
    ge_affc b; load_affc( b, lds_btab + ib*BTAB_STRIDE );
    ge_add_affc( P, P, b, negb, true );
  }
}

/* fd_ed25519_point_tobytes (fd_curve25519.c:63-74) as 8 LE words */
DEV void ge_encode( u32 out[8], ge_p3 const & P ) {
  fe zi, x, y;
  fe_invert( zi, P.Z ); fe_mul( x, P.X, zi ); fe_mul( y, P.Y, zi );
  fe_canon( x, x ); fe_canon( y, y );
  fe_to_words( out, y );
  out[7] |= (x.v[0] & 1u) << 31;
}

/* keygen + sign: fd_ed25519_user.c:4-133 */
__global__ __launch_bounds__(256)
void k_sign( ulong n, uchar const * __restrict__ prvs, uchar const * __restrict__ pool,
             uint const * __restrict__ moff, uint const * __restrict__ msz, u32 const * __restrict__ btab,
             uchar * __restrict__ pubs, uchar * __restrict__ sigs ) {
  __shared__ __attribute__((aligned(16))) u32 lds_btab[BTAB_WORDS];
  for( int t = threadIdx.x; t < BTAB_WORDS/4; t += blockDim.x )
    ((uint4 *)lds_btab)[t] = ((uint4 const *)btab)[t];
  __syncthreads();
  ulong i = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  u32 pre[16], h[16];
  load_words( pre, prvs + 32*i, 8 );
  #pragma unroll
  for( int q=8; q<16; q++ ) pre[q] = 0;
  sha512_prefixed( h, pre, 32u, pool, 0u );                     /* h = SHA512(prv) */
  u32 s[8];
  #pragma unroll
  for( int q=0; q<8; q++ ) s[q] = h[q];
  s[0] &= 0xfffffff8u; s[7] &= 0x7fffffffu; s[7] |= 0x40000000u;   /* clamp (user.c:30-32) */
  /* [s]B == [s mod L]B (B has order L); the reduced scalar is < 2^253 so its
     top radix-256 digit cannot carry out of the table range */
  u32 sx[16], sr[8];
  #pragma unroll
  for( int q=0; q<16; q++ ) sx[q] = q < 8 ? s[q] : 0u;
  sc_reduce512( sr, sx );
  ge_p3 P; u32 A[8], R[8];
  ge_scalarmult_base( P, sr, lds_btab ); ge_encode( A, P );
  uchar const * msg = pool + moff[i]; u32 mlen = msz[i];
  #pragma unroll
  for( int q=0; q<8; q++ ) pre[q] = h[8+q];
  u32 x[16], r[8];
  sha512_prefixed( x, pre, 32u, msg, mlen ); sc_reduce512( r, x );   /* r = H(prefix||M) mod L */
  ge_scalarmult_base( P, r, lds_btab ); ge_encode( R, P );
  u32 k[8]; hram_mod_l( k, R, A, msg, mlen );
  /* S = (r + k*s) mod L */
  u32 prod[16];
  {
    u64 lo = 0, hi = 0;
    #pragma unroll
    for( int c=0; c<16; c++ ) {
      #pragma unroll
      for( int a=0; a<8; a++ ) {
        int b = c - a; if( b < 0 || b > 7 ) continue;
        u64 p = (u64)k[a] * s[b]; lo += p; hi += (lo < p) ? 1u : 0u;
      }
      if( c < 8 ) { u64 q = lo + r[c]; hi += (q < lo) ? 1u : 0u; lo = q; }
      prod[c] = (u32)lo; lo = (lo >> 32) | (hi << 32); hi >>= 32;
    }
  }
  u32 S[8]; sc_reduce512( S, prod );
  uint4 * o = (uint4 *)(sigs + 64*i);
  o[0] = make_uint4( R[0],R[1],R[2],R[3] ); o[1] = make_uint4( R[4],R[5],R[6],R[7] );
  o[2] = make_uint4( S[0],S[1],S[2],S[3] ); o[3] = make_uint4( S[4],S[5],S[6],S[7] );
  uint4 * pa = (uint4 *)(pubs + 32*i);
  pa[0] = make_uint4( A[0],A[1],A[2],A[3] ); pa[1] = make_uint4( A[4],A[5],A[6],A[7] );
}

/**********************************************************************/
/* Host side                                                           */

extern "C" {

/* A reserve of at most half the resident slots: more would starve the
   DSM it is meant to share the GPU with (a reserve at or above
   the grid silently left one workgroup).  A clamped value is said once. */
int
fd_ed25519_hip_ctx_set_dsm_reserve( fd_ed25519_hip_ctx_t * ctx, ulong reserve ) {
  if( !ctx ) return -1;
  ulong const cap = ctx->dsm_wgs_all / 2ul;
  int clamped = reserve > cap;
  if( clamped ) {
    static int warned;
    if( !warned ) {
      warned = 1;
      fprintf( stderr, "fd_ed25519_hip: DSM reserve %lu clamped to %lu (half of %lu resident workgroup slots)\n", reserve,
               cap, ctx->dsm_wgs_all );
    }
    reserve = cap;
  }
  ctx->dsm_wgs = ctx->dsm_wgs_all - reserve > 0ul ? ctx->dsm_wgs_all - reserve : 1ul;
  return clamped;
}

fd_ed25519_hip_ctx_t *
fd_ed25519_hip_ctx_new( int device, ulong chunk_sigs ) {
  if( !chunk_sigs ) chunk_sigs = 1UL << 20;
  chunk_sigs = (chunk_sigs + 255UL) & ~255UL;
  fd_ed25519_hip_ctx_t * ctx = (fd_ed25519_hip_ctx_t *)calloc( 1, sizeof(*ctx) );
  if( !ctx ) { fprintf( stderr, "fd_ed25519_hip: out of host memory\n" ); abort(); }
  ctx->device   = device;
  ctx->chunk    = chunk_sigs;
  ctx->halfsize = 1;
  ctx->lat_max = LAT_DEFAULT_N;
  FD_CHECK( hipSetDevice( device ) );
  FD_CHECK( hipStreamCreateWithFlags( &ctx->stream, hipStreamNonBlocking ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_btab,  BTAB_ALLOC * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_state, (size_t)ST_WORDS * chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_atab,  (size_t)ATAB_WORDS * chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_idx, chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_order, chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_count, 256 ) );
  for( int e=0; e<4; e++ ) FD_CHECK( hipEventCreate( &ctx->ev[e] ) );
  FD_CHECK( hipEventCreateWithFlags( &ctx->ev_last, hipEventDisableTiming ) );
  {
    int ncu = 0, per = 0;
    FD_CHECK( hipDeviceGetAttribute( &ncu, hipDeviceAttributeMultiprocessorCount, device ) );
    FD_CHECK( hipOccupancyMaxActiveBlocksPerMultiprocessor( &per, k_verify_dsm, 256, 0 ) );
    ctx->dsm_wgs = (ulong)(ncu > 0 ? ncu : 1) * (ulong)(per > 0 ? per : 1);
    ctx->lat_cus = (ulong)(ncu > 0 ? ncu : 1);                /* x k_verify_lat workgroups per CU, below */
    /* the copy budget counts k_verify_lat workgroup slots: a register-count
       change that moved the per-CU fit would change the budget, not the
       results -- say so once */
    static int lat_warned;
    per = 0;
    FD_CHECK( hipOccupancyMaxActiveBlocksPerMultiprocessor( &per, k_verify_lat, LAT_WG, 0 ) );
    ctx->lat_cus *= (ulong)(per > 0 ? per : 1);
    if( per != LAT_WG_PER_CU && !lat_warned ) {
      lat_warned = 1;
      fprintf( stderr, "fd_ed25519_hip: k_verify_lat fits %d workgroups per CU (expected %d)\n", per, LAT_WG_PER_CU );
    }
  }
  hipLaunchKernelGGL( k_btab_init, dim3( (2*BTAB_N + 63)/64 ), dim3( 64 ), 0, ctx->stream, ctx->d_btab );
  FD_CHECK( hipGetLastError() );
  hipLaunchKernelGGL( k_btab12_init, dim3( (2*BT12_N + 63)/64 ), dim3( 64 ), 0, ctx->stream, ctx->d_btab );
  FD_CHECK( hipGetLastError() );
  {
    /* Racing copies pay off per CU, not per XCD: a lone workgroup is fast or
       slow by the state of the CU it lands on (profiles/r03k, r03x), so up to
       LAT_COPIES_MAX copies of a signature run (consecutive workgroups go to
       the XCDs in turn), bounded by one workgroup per CU in verify_impl.
       Against one copy per XCD (8): a lone 12-signature drop-in call p50
       323 vs 437 us, 16 concurrent callers unchanged (profiles/r03aa). */
    int ncu_ = 0;
    FD_CHECK( hipDeviceGetAttribute( &ncu_, hipDeviceAttributeMultiprocessorCount, device ) );
    ctx->lat_copies = LAT_COPIES_MAX;
    { char const * lc = getenv( "FD_ED25519_HIP_LAT_COPIES" ); if( lc && atoi( lc ) > 0 ) ctx->lat_copies = (u32)atoi( lc ); }
    /* A/B: every context's DSM grid 1/share of the resident slots (contexts sharing the GPU;
       fd_ed25519_hip_set_dsm_share sets it per context) */
    { char const * ds = getenv( "FD_ED25519_HIP_DSM_SHARE" ); if( ds && atoi( ds ) > 0 ) ctx->dsm_share = (ulong)atoi( ds ); }
    /* leave this many resident DSM workgroup slots free (room on some CUs
       for kernels of other streams while a DSM runs): per context with
       fd_ed25519_hip_ctx_set_dsm_reserve; FD_ED25519_HIP_DSM_RESERVE sets it
       for every context of the process (A/Bs) */
    ctx->dsm_wgs_all = ctx->dsm_wgs;
    { char const * dr = getenv( "FD_ED25519_HIP_DSM_RESERVE" );
      if( dr ) fd_ed25519_hip_ctx_set_dsm_reserve( ctx, strtoul( dr, 0, 0 ) ); }
    ctx->ncu = (ulong)(ncu_ > 0 ? ncu_ : 1);
    FD_CHECK( hipMalloc( (void **)&ctx->d_lat_done, LAT_MAX_N * sizeof(ulong) ) );
    FD_CHECK( hipMemsetAsync( ctx->d_lat_done, 0, LAT_MAX_N * sizeof(ulong), ctx->stream ) );
  }
  FD_CHECK( hipStreamSynchronize( ctx->stream ) );
  return ctx;
}

void
fd_ed25519_hip_ctx_reserve( fd_ed25519_hip_ctx_t * ctx, ulong chunk_sigs ) {
  chunk_sigs = (chunk_sigs + 255UL) & ~255UL;
  if( chunk_sigs <= ctx->chunk ) return;
  FD_CHECK( hipSetDevice( ctx->device ) );
  FD_CHECK( hipDeviceSynchronize() );                      /* the scratch may be in use on any stream */
  (void)hipFree( ctx->d_state ); (void)hipFree( ctx->d_atab ); (void)hipFree( ctx->d_idx );
  (void)hipFree( ctx->d_order );
  FD_CHECK( hipMalloc( (void **)&ctx->d_state, (size_t)ST_WORDS * chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_atab,  (size_t)ATAB_WORDS * chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_idx, chunk_sigs * sizeof(u32) ) );
  FD_CHECK( hipMalloc( (void **)&ctx->d_order, chunk_sigs * sizeof(u32) ) );
  ctx->chunk = chunk_sigs;
}

static void free_staging( fd_ed25519_hip_ctx_t * ctx ) {
  (void)hipFree( ctx->d_sigs ); (void)hipFree( ctx->d_pubs ); (void)hipFree( ctx->d_pool ); (void)hipFree( ctx->d_moff );
  (void)hipFree( ctx->d_msz ); (void)hipFree( ctx->d_codes ); (void)hipFree( ctx->d_bitmap );
  (void)hipFree( ctx->d_gfirst ); (void)hipFree( ctx->d_gcnt ); (void)hipFree( ctx->d_gcodes );
}

void
fd_ed25519_hip_ctx_delete( fd_ed25519_hip_ctx_t * ctx ) {
  if( !ctx ) return;
  (void)hipSetDevice( ctx->device );
  (void)hipStreamSynchronize( ctx->stream );
  if( ctx->ev_used ) (void)hipEventSynchronize( ctx->ev_last );   /* last call may have run on a caller stream */
  (void)hipFree( ctx->d_btab ); (void)hipFree( ctx->d_state ); (void)hipFree( ctx->d_atab );
  (void)hipFree( ctx->d_idx ); (void)hipFree( ctx->d_order ); (void)hipFree( ctx->d_count );
  (void)hipFree( ctx->d_lat_done );
  free_staging( ctx );
  for( int e=0; e<4; e++ ) (void)hipEventDestroy( ctx->ev[e] );
  (void)hipEventDestroy( ctx->ev_last );
  (void)hipStreamDestroy( ctx->stream );
  free( ctx );
}

int   fd_ed25519_hip_ctx_device( fd_ed25519_hip_ctx_t const * ctx ) { return ctx->device; }
int   fd_ed25519_hip_device_cnt( void ) { int n = 0; return hipGetDeviceCount( &n ) == hipSuccess ? n : 0; }
void *fd_ed25519_hip_ctx_stream( fd_ed25519_hip_ctx_t const * ctx ) { return (void *)ctx->stream; }
void  fd_ed25519_hip_set_errmode( fd_ed25519_hip_ctx_t * ctx, int m ) { ctx->errmode = m; }
void  fd_ed25519_hip_set_halfsize( fd_ed25519_hip_ctx_t * ctx, int on ) { ctx->halfsize = on ? 1 : 0; }
void  fd_ed25519_hip_set_dsm_share( fd_ed25519_hip_ctx_t * ctx, ulong share ) { ctx->dsm_share = share ? share : 1ul; }
void  fd_ed25519_hip_set_lat_cus( fd_ed25519_hip_ctx_t * ctx, ulong cus ) { ctx->lat_cus = cus ? cus : 1ul; }

int
fd_ed25519_hip_ctx_set_cu_mask( fd_ed25519_hip_ctx_t * ctx, uint const * mask, uint words ) {
  /* the context's stream, recreated on the CUs the mask names (bit i of
     word w = the runtime's CU 32w+i): work queued on it before is drained */
  FD_CHECK( hipSetDevice( ctx->device ) );
  FD_CHECK( hipStreamSynchronize( ctx->stream ) );
  if( ctx->ev_used ) FD_CHECK( hipEventSynchronize( ctx->ev_last ) );
  hipStream_t s = 0;
  hipError_t e = words ? hipExtStreamCreateWithCUMask( &s, words, mask )
                       : hipStreamCreateWithFlags( &s, hipStreamNonBlocking );
  if( e != hipSuccess ) return -1;
  FD_CHECK( hipStreamDestroy( ctx->stream ) );
  ctx->stream = s;
  return 0;
}
void  fd_ed25519_hip_set_small_batch( fd_ed25519_hip_ctx_t * ctx, ulong max_n ) {
  ctx->lat_max = max_n < LAT_MAX_N ? max_n : LAT_MAX_N;
}

/* test hook: sc_halfsize on n scalars k < L (8 LE words each); out per
   scalar: k1 (8 words), k2 (8 words), k1neg (0 or ~0), bits */
__global__ void k_test_halfsize( ulong n, u32 const * k, u32 * out ) {
  ulong i = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  u32 kk[8], k1[8], k2[8], neg;
  #pragma unroll
  for( int w=0; w<8; w++ ) kk[w] = k[8*i+w];
  u32 bits = sc_halfsize( k1, neg, k2, kk );
  u32 * o = out + 18*i;
  #pragma unroll
  for( int w=0; w<8; w++ ) { o[w] = k1[w]; o[8+w] = k2[w]; }
  o[16] = neg; o[17] = bits;
}

int
fd_ed25519_hip_test_halfsize( fd_ed25519_hip_ctx_t * ctx, ulong n, uint const * d_k, uint * d_out, void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( !n ) return 0;
  hipLaunchKernelGGL( k_test_halfsize, dim3( (unsigned)((n + 63)/64) ), dim3( 64 ), 0, s, n, d_k, d_out );
  FD_CHECK( hipGetLastError() );
  return 0;
}

/* test hook: one device primitive over n items, 32 u32 words in and 32 out
   per item (include/fd_ed25519_hip.h FD_ED25519_HIP_PRIM_*).  Field inputs
   are 9 limbs (value = sum v[i] 2^(29 i)) within the bounds each primitive
   assumes; field outputs are 9 limbs as the primitive leaves them (products:
   tight) or canonical where the op says so. */
__global__ void k_test_prim( int op, ulong n, u32 const * in, u32 * out ) {
  ulong t = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  if( t >= n ) return;
  u32 const * x = in + 32*t;
  u32 o[32];
  #pragma unroll
  for( int q=0; q<32; q++ ) o[q] = 0u;
  fe a, b, r, s;
  #pragma unroll
  for( int q=0; q<9; q++ ) { a.v[q] = x[q]; b.v[q] = x[9+q]; }
  switch( op ) {
  case 0: fe_mul( r, a, b ); break;                                  /* FE_MUL     */
  case 1: fe_sq( r, a ); break;                                      /* FE_SQ      */
  case 2: fe_mul2( r, a, b, s, b, a ); break;                        /* FE_MUL2: a*b, b*a */
  case 3: fe_sq2( r, a, s, b ); break;                               /* FE_SQ2: a^2, b^2 */
  case 4: fe_canon( r, a ); break;                                   /* FE_CANON   */
  case 5: { u32 w[8];                                                /* FE_FROMWORDS */
            #pragma unroll
            for( int q=0; q<8; q++ ) w[q] = x[q];
            fe_from_words( r, w ); } break;
  case 6: fe_sub( r, a, b ); fe_canon( r, r ); break;                /* FE_SUB (b tight) */
  case 7: fe_pow22523( r, a ); fe_canon( r, r ); break;              /* FE_POW22523 */
  case 8: fe_invert( r, a ); fe_canon( r, r ); break;                /* FE_INVERT  */
  case 9: {                                                          /* GE_DECODE  */
            u32 w[8];
            #pragma unroll
            for( int q=0; q<8; q++ ) w[q] = x[q];
            ge_p3 P;
            u32 f = ge_decode( P, w );
            o[0] = f;
            o[1] = (!(f & 1u) && ge_affine_is_small_order( P )) ? 1u : 0u;
            u32 xw[8], yw[8];
            fe_to_words( xw, P.X ); fe_to_words( yw, P.Y );
            #pragma unroll
            for( int q=0; q<8; q++ ) { o[2+q] = xw[q]; o[10+q] = yw[q]; }
          } break;
  case 10: { u32 w[16], k[8];                                        /* SC_REDUCE  */
             #pragma unroll
             for( int q=0; q<16; q++ ) w[q] = x[q];
             sc_reduce512( k, w );
             #pragma unroll
             for( int q=0; q<8; q++ ) o[q] = k[q]; } break;
  case 11: { u32 w[8];                                               /* SC_CANONICAL */
             #pragma unroll
             for( int q=0; q<8; q++ ) w[q] = x[q];
             o[0] = sc_is_canonical( w ) ? 1u : 0u; } break;
  default: break;
  }
  if( op <= 8 ) {
    #pragma unroll
    for( int q=0; q<9; q++ ) o[q] = r.v[q];
    if( op == 2 || op == 3 ) {
      #pragma unroll
      for( int q=0; q<9; q++ ) o[9+q] = s.v[q];
    }
  }
  #pragma unroll
  for( int q=0; q<32; q++ ) out[32*t+q] = o[q];
}

int
fd_ed25519_hip_test_prim( fd_ed25519_hip_ctx_t * ctx, int op, ulong n, uint const * d_in, uint * d_out,
                          void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( op < 0 || op > 11 ) return -1;
  if( !n ) return 0;
  hipLaunchKernelGGL( k_test_prim, dim3( (unsigned)((n + 63)/64) ), dim3( 64 ), 0, s, op, n, d_in, d_out );
  FD_CHECK( hipGetLastError() );
  return 0;
}

/* test hook: plain SHA-512 of n messages with the device hash core used by
   k_verify_prep (sha512_prefixed with an empty prefix); out: 64-byte digests */
__global__ __launch_bounds__(64) void k_test_sha512( ulong n, uchar const * pool, uint const * moff,
                                                      uint const * msz, uchar * out, int coop ) {
  __shared__ __attribute__((aligned(16))) u32 lds_msg[PREP_MSG_WORDS];
  __shared__ u64 lds_meta[64];
  ulong i = (ulong)blockIdx.x * blockDim.x + threadIdx.x;
  u32 pre[16], x[16];
  #pragma unroll
  for( int q=0; q<16; q++ ) pre[q] = 0u;
  if( coop ) {            /* the k_verify_prep path: the whole wave, lanes past n hash nothing */
    sha512_prefixed_coop<0u>( x, nullptr, nullptr, pool + (i < n ? moff[i] : 0u), i < n ? msz[i] : 0u, lds_msg, lds_meta,
                              threadIdx.x & 63u );
    if( i >= n ) return;
  } else {
    if( i >= n ) return;
    sha512_prefixed( x, pre, 0u, pool + moff[i], msz[i] );
  }
  uint4 * o = (uint4 *)(out + 64ul*i);
  #pragma unroll
  for( int q=0; q<4; q++ ) o[q] = make_uint4( x[4*q], x[4*q+1], x[4*q+2], x[4*q+3] );
}

int
fd_ed25519_hip_test_sha512( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_pool, uint const * d_msg_off,
                            uint const * d_msg_sz, uchar * d_out, void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( !n ) return 0;
  for( int coop=0; coop<2; coop++ ) {    /* per-lane path into d_out, cooperative path into d_out + 64*n */
    hipLaunchKernelGGL( k_test_sha512, dim3( (unsigned)((n + 63)/64) ), dim3( 64 ), 0, s, n, d_pool, d_msg_off,
                        d_msg_sz, d_out + (coop ? 64ul*n : 0ul), coop );
    FD_CHECK( hipGetLastError() );
  }
  return 0;
}

void
fd_ed25519_hip_set_timing( fd_ed25519_hip_ctx_t * ctx, int on ) {
  ctx->timing = on; ctx->prep_ms = ctx->dsm_ms = 0.0; ctx->prep_launches = ctx->dsm_launches = 0UL;
  ctx->dsm_units = 0UL;
}

ulong
fd_ed25519_hip_get_dsm_units( fd_ed25519_hip_ctx_t const * ctx ) { return ctx->dsm_units; }

void
fd_ed25519_hip_get_timing( fd_ed25519_hip_ctx_t const * ctx, double * prep_ms, double * dsm_ms, ulong * launches ) {
  if( prep_ms ) *prep_ms = ctx->prep_ms;
  if( dsm_ms ) *dsm_ms = ctx->dsm_ms;
  if( launches ) *launches = ctx->dsm_launches;
}

/* d_msg_off NULL: fixed-size messages, message i = d_pool[ i*fixed_sz, +fixed_sz ) */
static int
verify_impl( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_sigs, uchar const * d_pubs,
             uchar const * d_pool, uint const * d_msg_off, uint const * d_msg_sz, uint fixed_sz,
             signed char * d_codes, ulong * d_bitmap, u32 const * d_n, void * stream,
             fd_hip_segs_t const * segs = (fd_hip_segs_t const *)0 ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( !n ) return 0;
  if( segs && (n > ctx->chunk || !segs->n_seg || segs->n_seg > FD_HIP_SEG_MAX || !segs->total) ) return -1;
  if( segs ) d_n = segs->total;                            /* written by k_seg_reduce below */
  if( ctx->ev_used ) FD_CHECK( hipStreamWaitEvent( s, ctx->ev_last, 0 ) );   /* previous call's scratch use */
  if( !d_n && n <= ctx->lat_max && n <= ctx->chunk && !ctx->timing ) {
    /* small batch: one workgroup per signature (k_verify_lat), racing as
       many copies as the context's workgroup-slot budget holds, up to
       lat_copies and one workgroup per CU */
    u32 copies = 1u;
    {
      ulong c = ctx->lat_cus / n;
      c = c < (ulong)ctx->lat_copies ? c : (ulong)ctx->lat_copies;
      c = c < ctx->ncu / n ? c : ctx->ncu / n;              /* copies beyond one per CU pile up (profiles/r03aa) */
      while( c > 1ul && n * c > ctx->chunk ) c--;           /* each copy builds its tables in d_atab */
      copies = c ? (u32)c : 1u;
    }
    ulong seq = ++ctx->lat_seq;                            /* from 1: 0 is done[]'s initial value */
    hipLaunchKernelGGL( k_verify_lat, dim3( (unsigned)(n * copies) ), dim3( LAT_WG ), 0, s, n, d_sigs, d_pubs,
                        d_pool, d_msg_off, d_msg_sz, fixed_sz, ctx->d_btab, ctx->d_atab, ctx->errmode,
                        ctx->halfsize, d_codes, copies, ctx->d_lat_done, seq );
    FD_CHECK( hipGetLastError() );
    if( d_bitmap ) {
      hipLaunchKernelGGL( k_bitmap, dim3( (unsigned)((n + 255) / 256) ), dim3( 256 ), 0, s, n, d_codes, d_bitmap,
                          (u32 const *)0, 0ul );
      FD_CHECK( hipGetLastError() );
    }
    FD_CHECK( hipEventRecord( ctx->ev_last, s ) );
    ctx->ev_used = 1;
    return 0;
  }
  for( ulong off = 0; off < n; off += ctx->chunk ) {
    ulong m = n - off < ctx->chunk ? n - off : ctx->chunk;
    dim3 grid( (unsigned)((m + 255) / 256) ), blk( 256 );
    /* the txn paths (device-side count, variable-size messages) hash in
       block-count order; fixed or uniform batches keep record order */
    bool ordered = d_n && d_msg_off;
    FD_CHECK( hipMemsetAsync( ctx->d_count, 0, (ordered ? 48 : 3)*sizeof(u32), s ) );
    if( ctx->timing ) FD_CHECK( hipEventRecord( ctx->ev[0], s ) );
    if( ordered ) {
      /* the block-count histogram: summed from the segments' (k_txnm_batch
         built them while expanding the records) or k_msg_hist's */
      if( segs ) {
        hipLaunchKernelGGL( k_seg_reduce, dim3( 1 ), dim3( 256 ), 0, s, segs->seg, segs->n_seg, ctx->d_count,
                            segs->total );
      } else {
        hipLaunchKernelGGL( k_msg_hist, grid, blk, 0, s, m, d_msg_sz + off, ctx->d_count, d_n, off );
      }
      FD_CHECK( hipGetLastError() );
      hipLaunchKernelGGL( k_msg_order, grid, blk, 0, s, m, d_msg_sz + off, ctx->d_count, d_n, off, ctx->d_order,
                          ctx->chunk, segs ? segs->seg : (u32 const *)0, segs ? segs->seg_cap : 0ul );
      FD_CHECK( hipGetLastError() );
    }
    uchar const * pool = d_msg_off ? d_pool : d_pool + off*(ulong)fixed_sz;
    dim3 gprep( grid.x );
    hipLaunchKernelGGL( k_verify_prep, gprep, blk, 0, s, m, ctx->chunk, d_sigs + 64*off, d_pubs + 32*off,
                        pool, d_msg_off ? d_msg_off + off : (uint const *)0,
                        d_msg_off ? d_msg_sz + off : (uint const *)0, fixed_sz, ctx->d_state, ctx->errmode,
                        ctx->d_idx, ctx->d_count, d_codes + off, d_n, off, ordered ? ctx->d_order : (u32 const *)0 );
    FD_CHECK( hipGetLastError() );
    if( ctx->timing ) FD_CHECK( hipEventRecord( ctx->ev[1], s ) );
    if( ctx->timing ) FD_CHECK( hipEventRecord( ctx->ev[3], s ) );
    ulong dsm_grid = ctx->dsm_wgs / (ctx->dsm_share ? ctx->dsm_share : 1ul);
    if( !dsm_grid ) dsm_grid = 1ul;
    dim3 gdsm( grid.x > dsm_grid ? (unsigned)dsm_grid : grid.x );
    hipLaunchKernelGGL( k_verify_dsm, gdsm, blk, 0, s, ctx->chunk, ctx->d_state, ctx->d_btab, ctx->d_atab,
                        ctx->d_idx, ctx->d_count, d_codes + off, ctx->halfsize,
                        ordered ? ctx->d_order : (u32 const *)0 );
    FD_CHECK( hipGetLastError() );
    if( d_bitmap ) {
      hipLaunchKernelGGL( k_bitmap, grid, blk, 0, s, m, d_codes + off, d_bitmap + off/64, d_n, off );
      FD_CHECK( hipGetLastError() );
    }
    if( ctx->timing ) {
      /* timing mode serialises the host with each chunk; it is meant for the
         measured bench leg only */
      FD_CHECK( hipEventRecord( ctx->ev[2], s ) );
      FD_CHECK( hipEventSynchronize( ctx->ev[2] ) );
      float a, b;
      FD_CHECK( hipEventElapsedTime( &a, ctx->ev[0], ctx->ev[1] ) );
      FD_CHECK( hipEventElapsedTime( &b, ctx->ev[3], ctx->ev[2] ) );   /* k_verify_dsm (+ k_bitmap) */
      u32 survivors = 0;
      FD_CHECK( hipMemcpy( &survivors, ctx->d_count, sizeof(u32), hipMemcpyDeviceToHost ) );
      ctx->prep_ms += a; ctx->dsm_ms += b; ctx->prep_launches++; ctx->dsm_launches++; ctx->dsm_units += survivors;
    }
  }
  FD_CHECK( hipEventRecord( ctx->ev_last, s ) );
  ctx->ev_used = 1;
  return 0;
}

int
fd_ed25519_hip_verify_dev( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_sigs, uchar const * d_pubs,
                           uchar const * d_pool, uint const * d_msg_off, uint const * d_msg_sz,
                           signed char * d_codes, ulong * d_bitmap, void * stream ) {
  return verify_impl( ctx, n, d_sigs, d_pubs, d_pool, d_msg_off, d_msg_sz, 0u, d_codes, d_bitmap, NULL, stream );
}

int
fd_ed25519_hip_verify_dev_count( fd_ed25519_hip_ctx_t * ctx, ulong n_max, uint const * d_n, uchar const * d_sigs,
                                 uchar const * d_pubs, uchar const * d_pool, uint const * d_msg_off,
                                 uint const * d_msg_sz, signed char * d_codes, ulong * d_bitmap, void * stream ) {
  return verify_impl( ctx, n_max, d_sigs, d_pubs, d_pool, d_msg_off, d_msg_sz, 0u, d_codes, d_bitmap, d_n, stream );
}

int
fd_ed25519_hip_verify_segs( fd_ed25519_hip_ctx_t * ctx, fd_hip_segs_t segs, uchar const * d_sigs,
                            uchar const * d_pubs, uchar const * d_pool, uint const * d_msg_off,
                            uint const * d_msg_sz, signed char * d_codes, void * stream ) {
  if( !d_msg_off || !d_msg_sz || !segs.seg_cap ) return -1;
  return verify_impl( ctx, (ulong)segs.n_seg * segs.seg_cap, d_sigs, d_pubs, d_pool, d_msg_off, d_msg_sz, 0u,
                      d_codes, NULL, NULL, stream, &segs );
}

int
fd_ed25519_hip_verify_fixed_dev( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_sigs, uchar const * d_pubs,
                                 uchar const * d_msgs, uint msg_sz, signed char * d_codes, ulong * d_bitmap,
                                 void * stream ) {
  return verify_impl( ctx, n, d_sigs, d_pubs, d_msgs, (uint const *)0, (uint const *)0, msg_sz, d_codes, d_bitmap,
                      NULL, stream );
}

int
fd_ed25519_hip_group_reduce_dev( fd_ed25519_hip_ctx_t * ctx, ulong ng, uint const * d_first, uchar const * d_cnt,
                                 signed char const * d_sig_codes, signed char * d_group_codes, void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( !ng ) return 0;
  hipLaunchKernelGGL( k_group_reduce, dim3( (unsigned)((ng + 255)/256) ), dim3( 256 ), 0, s,
                      ng, d_first, d_cnt, d_sig_codes, d_group_codes );
  FD_CHECK( hipGetLastError() );
  return 0;
}

int
fd_ed25519_hip_sign_dev( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * d_prvs, uchar const * d_pool,
                         uint const * d_msg_off, uint const * d_msg_sz, uchar * d_pubs, uchar * d_sigs,
                         void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( !n ) return 0;
  hipLaunchKernelGGL( k_sign, dim3( (unsigned)((n + 255)/256) ), dim3( 256 ), 0, s,
                      n, d_prvs, d_pool, d_msg_off, d_msg_sz, ctx->d_btab, d_pubs, d_sigs );
  FD_CHECK( hipGetLastError() );
  return 0;
}

void *
fd_ed25519_hip_host_alloc( ulong sz ) {
  void * p = NULL;
  FD_CHECK( hipHostMalloc( &p, sz ? sz : 1ul, hipHostMallocMapped | hipHostMallocPortable ) );
  return p;
}

void
fd_ed25519_hip_host_free( void * p ) {
  if( p ) FD_CHECK( hipHostFree( p ) );
}

void *
fd_ed25519_hip_host_register( void * p, ulong sz ) {
  if( !p || !sz ) return NULL;
  FD_CHECK( hipHostRegister( p, sz, hipHostRegisterMapped | hipHostRegisterPortable ) );
  void * d = NULL;
  FD_CHECK( hipHostGetDevicePointer( &d, p, 0 ) );
  return d;
}

void
fd_ed25519_hip_host_unregister( void * p ) {
  if( p ) FD_CHECK( hipHostUnregister( p ) );
}

int
fd_ed25519_hip_stage_async( fd_ed25519_hip_ctx_t * ctx, void * d_dst, void const * h_src, ulong sz, void * stream ) {
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( sz ) FD_CHECK( hipMemcpyAsync( d_dst, h_src, sz, hipMemcpyHostToDevice, s ) );
  return 0;
}

int
fd_ed25519_hip_sync( fd_ed25519_hip_ctx_t * ctx ) {
  FD_CHECK( hipSetDevice( ctx->device ) );
  FD_CHECK( hipStreamSynchronize( ctx->stream ) );
  return 0;
}

static void ensure_staging( fd_ed25519_hip_ctx_t * ctx, ulong n, ulong pool_sz, ulong ng ) {
  if( n > ctx->h_cap_n ) {
    ulong c = n < 4096 ? 4096 : n;
    (void)hipFree( ctx->d_sigs ); (void)hipFree( ctx->d_pubs ); (void)hipFree( ctx->d_moff ); (void)hipFree( ctx->d_msz );
    (void)hipFree( ctx->d_codes ); (void)hipFree( ctx->d_bitmap );
    FD_CHECK( hipMalloc( (void **)&ctx->d_sigs, 64*c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_pubs, 32*c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_moff, 4*c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_msz, 4*c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_codes, c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_bitmap, 8*((c+63)/64) ) );
    ctx->h_cap_n = c;
  }
  if( pool_sz + 16 > ctx->h_cap_pool ) {
    ulong c = pool_sz + 16 < 65536 ? 65536 : pool_sz + 16;
    (void)hipFree( ctx->d_pool );
    FD_CHECK( hipMalloc( (void **)&ctx->d_pool, c ) );
    FD_CHECK( hipMemset( ctx->d_pool, 0, c ) );
    ctx->h_cap_pool = c;
  }
  if( ng > ctx->h_cap_groups ) {
    ulong c = ng < 4096 ? 4096 : ng;
    (void)hipFree( ctx->d_gfirst ); (void)hipFree( ctx->d_gcnt ); (void)hipFree( ctx->d_gcodes );
    FD_CHECK( hipMalloc( (void **)&ctx->d_gfirst, 4*c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_gcnt, c ) );
    FD_CHECK( hipMalloc( (void **)&ctx->d_gcodes, c ) );
    ctx->h_cap_groups = c;
  }
}

int
fd_ed25519_hip_verify_host( fd_ed25519_hip_ctx_t * ctx, ulong n, uchar const * sigs, uchar const * pubs,
                            uchar const * pool, ulong pool_sz, uint const * msg_off, uint const * msg_sz,
                            signed char * codes, ulong * bitmap ) {
  if( !n ) return 0;
  for( ulong i=0; i<n; i++ ) if( (ulong)msg_off[i] + msg_sz[i] > pool_sz ) return -1;   /* device reads stay in the copy */
  FD_CHECK( hipSetDevice( ctx->device ) );
  ensure_staging( ctx, n, pool_sz, 0 );
  hipStream_t s = ctx->stream;
  FD_CHECK( hipMemcpyAsync( ctx->d_sigs, sigs, 64*n, hipMemcpyHostToDevice, s ) );
  FD_CHECK( hipMemcpyAsync( ctx->d_pubs, pubs, 32*n, hipMemcpyHostToDevice, s ) );
  if( pool_sz ) FD_CHECK( hipMemcpyAsync( ctx->d_pool, pool, pool_sz, hipMemcpyHostToDevice, s ) );
  FD_CHECK( hipMemcpyAsync( ctx->d_moff, msg_off, 4*n, hipMemcpyHostToDevice, s ) );
  FD_CHECK( hipMemcpyAsync( ctx->d_msz, msg_sz, 4*n, hipMemcpyHostToDevice, s ) );
  fd_ed25519_hip_verify_dev( ctx, n, ctx->d_sigs, ctx->d_pubs, ctx->d_pool, ctx->d_moff, ctx->d_msz,
                             ctx->d_codes, ctx->d_bitmap, s );
  FD_CHECK( hipMemcpyAsync( codes, ctx->d_codes, n, hipMemcpyDeviceToHost, s ) );
  if( bitmap ) FD_CHECK( hipMemcpyAsync( bitmap, ctx->d_bitmap, 8*((n+63)/64), hipMemcpyDeviceToHost, s ) );
  FD_CHECK( hipStreamSynchronize( s ) );
  return 0;
}

/* ---- reference API on process-wide contexts ---------------------------

   The reference API is re-entrant with no global mutable state
   (fd_ed25519.h:89-94) and replay calls it per transaction from many
   threads (fd_executor.c:1608-1617).  Concurrent drop-in calls are therefore
   combined: each caller appends its records and message to the open staging
   batch (one pinned host block, with a device copy).  A batch runs as soon as
   one of the batch slots is free: whichever caller finds a free slot closes
   the open batch and runs it for everyone in it -- one DMA in, one launch
   sequence (k_verify_lat up to the slot's lat_max records, the bulk kernels
   above), one DMA of the codes back.  There are g_slots slots (default
   DROPIN_SLOTS, FD_ED25519_HIP_DROPIN_SLOTS), each with its own context:
   stream, scratch and k_verify_lat tables, so that many batches are on the
   GPU at once and a call never waits behind a whole earlier batch while the
   GPU has room.  Callers arriving while every slot is busy gather in the
   open batch.  A lone caller gets a launch of its own right away.

   Each slot's latency kernel may fill 1/g_slots of the k_verify_lat
   workgroup slots with racing copies (lat_cus), so the slots' batches fit on
   the GPU side by side.  More slots than the process's 4 hardware queues only
   queue launches behind each other (16 C callers x 12 signatures: 0.32 M/s
   at 4 slots, 0.18 M/s at 8, 0.09 M/s at 16, profiles/r03m).

   Staging block layout, 16-byte aligned: sigs[256*64] pubs[256*32]
   off[256] sz[256] codes[256], then the callers' messages, each followed
   by 16 zero bytes (the kernels' message loads may read past the end). */

#define DROPIN_REC_MAX 256ul
#define STAGE_SIGS   0ul
#define STAGE_PUBS   (STAGE_SIGS + 64ul*DROPIN_REC_MAX)
#define STAGE_OFF    (STAGE_PUBS + 32ul*DROPIN_REC_MAX)
#define STAGE_SZ     (STAGE_OFF + 4ul*DROPIN_REC_MAX)
#define STAGE_CODES  (STAGE_SZ + 4ul*DROPIN_REC_MAX)
#define STAGE_MSG    (STAGE_CODES + DROPIN_REC_MAX)
#define DROPIN_SLOTS     4         /* default batches on the GPU at once (the process's hardware queues) */
#define DROPIN_SLOTS_MAX 16
#define DROPIN_NBUF  (DROPIN_SLOTS_MAX + 2)
#define DROPIN_POOL0 65536ul       /* initial message bytes per staging block */

enum { DSTAGE_FREE = 0, DSTAGE_OPEN, DSTAGE_RUNNING, DSTAGE_DONE };

struct dropin_stage {
  uchar * h;           /* pinned host block */
  uchar * d;           /* its device copy */
  ulong   cap;         /* bytes of each */
  ulong   n, pool;     /* records and message bytes taken */
  int     users;       /* callers attached (read their codes before the block is reused) */
  int     state;
  ulong   gen;         /* batch number */
  std::condition_variable cv;   /* its callers wait here: the batch is done, or a slot is free to run it */
};

static fd_ed25519_hip_ctx_t *   g_ctx;           /* slot 0's context, also the library's default context */
static std::mutex               g_ctx_lock;      /* creation of g_ctx */
static std::mutex               g_dl;            /* the staging ring and slots below */
static std::condition_variable  g_dcv;           /* a block freed or closed, or a slot freed (callers without a block) */
static dropin_stage             g_stage[ DROPIN_NBUF ];
static fd_ed25519_hip_ctx_t *   g_slot_ctx[ DROPIN_SLOTS_MAX ];
static int                      g_slot_busy[ DROPIN_SLOTS_MAX ];
static int                      g_slots;         /* 0: not configured yet */
static int                      g_open = -1;     /* the open block, -1: none */
static int                      g_running;       /* batches on the GPU */
static ulong                    g_gen;
static ulong                    g_batches, g_batch_calls;   /* launches and the calls they served */

static fd_ed25519_hip_ctx_t * default_ctx_new( int device ) {
  fd_ed25519_hip_ctx_t * ctx = fd_ed25519_hip_ctx_new( device, 4096 );
  char const * m = getenv( "FD_ED25519_HIP_ERRMODE" );
  if( m && !strcmp( m, "ref" ) ) ctx->errmode = FD_ED25519_HIP_ERRMODE_REF;
  return ctx;
}

static fd_ed25519_hip_ctx_t * default_ctx( void ) {
  std::lock_guard<std::mutex> lk( g_ctx_lock );
  if( !g_ctx ) {
    char const * e = getenv( "FD_ED25519_HIP_DEVICE" );
    g_ctx = default_ctx_new( e ? atoi( e ) : 0 );
  }
  return g_ctx;
}

/* the process-wide context for the library's other host-memory APIs
   (fd_sha512_hip.hip batching); not part of the public ABI */
__attribute__((visibility("hidden"))) fd_ed25519_hip_ctx_t *
fd_ed25519_hip_private_default_ctx( void ) {
  return default_ctx();
}

static void stage_grow( fd_ed25519_hip_ctx_t * ctx, dropin_stage * b, ulong cap ) {
  FD_CHECK( hipSetDevice( ctx->device ) );
  if( b->h ) FD_CHECK( hipHostFree( b->h ) );
  if( b->d ) FD_CHECK( hipFree( b->d ) );
  FD_CHECK( hipHostMalloc( (void **)&b->h, cap, hipHostMallocDefault ) );
  FD_CHECK( hipMalloc( (void **)&b->d, cap ) );
  b->cap = cap;
}

/* slot count and slot contexts (caller holds g_dl; g_ctx exists).  Slot 0
   runs on g_ctx; the others get contexts of their own on its device.  Every
   slot's latency kernel keeps to its share of the CUs. */
static void slots_setup( void ) {
  if( !g_slots ) {
    char const * e = getenv( "FD_ED25519_HIP_DROPIN_SLOTS" );
    int k = e ? atoi( e ) : DROPIN_SLOTS;
    g_slots = k < 1 ? 1 : k > DROPIN_SLOTS_MAX ? DROPIN_SLOTS_MAX : k;
  }
  for( int j=0; j<g_slots; j++ ) {
    if( g_slot_ctx[j] ) continue;
    fd_ed25519_hip_ctx_t * c = j ? default_ctx_new( g_ctx->device ) : g_ctx;
    char const * lc = getenv( "FD_ED25519_HIP_DROPIN_LAT_CUS" );   /* A/B override of the share */
    c->lat_cus = lc ? (ulong)atol( lc ) : c->lat_cus / (ulong)g_slots;
    if( !c->lat_cus ) c->lat_cus = 1ul;
    /* combined drop-in batches of up to lat_cus records (256 on a 256-CU
       part with 4 slots) take the latency path; FD_ED25519_HIP_DROPIN_LAT_MAX
       overrides (A/B against LAT_DEFAULT_N: INTEGRATION.md §1) */
    char const * lm = getenv( "FD_ED25519_HIP_DROPIN_LAT_MAX" );
    c->lat_max = lm ? (ulong)atol( lm ) : c->lat_cus;
    if( c->lat_max > LAT_MAX_N ) c->lat_max = LAT_MAX_N;
    g_slot_ctx[j] = c;
  }
}

int
fd_ed25519_hip_dropin_init( int device ) {
  {
    std::lock_guard<std::mutex> lk( g_ctx_lock );
    if( g_ctx ) { if( g_ctx->device != device ) return -1; }
    else g_ctx = default_ctx_new( device );
  }
  std::lock_guard<std::mutex> lk( g_dl );
  slots_setup();
  for( int j=0; j<DROPIN_NBUF; j++ )
    if( !g_stage[j].h ) stage_grow( g_ctx, &g_stage[j], STAGE_MSG + DROPIN_POOL0 );
  return 0;
}

void
fd_ed25519_hip_dropin_stats( ulong out[ 2 ] ) {
  std::lock_guard<std::mutex> lk( g_dl );
  out[0] = g_batches; out[1] = g_batch_calls;
}

/* The engine addresses messages with 32-bit offsets and sizes.  A longer
   message cannot be hashed here; verifying a truncated prefix instead would
   be a silent divergence from the reference (which hashes all of it), so the
   process aborts loudly (SURVEY.md 8(b) "Errors": never a silent reject or
   accept). */
#define DROPIN_MSG_MAX ((ulong)UINT32_MAX - 256ul - STAGE_MSG)
static void dropin_check_msg_sz( ulong msg_sz, char const * fn ) {
  if( msg_sz > DROPIN_MSG_MAX ) {
    fprintf( stderr, "fd_ed25519_hip: %s: msg_sz %lu exceeds the engine's 32-bit message limit (%lu)\n", fn,
             msg_sz, DROPIN_MSG_MAX );
    abort();
  }
}

/* run the staging block on a free slot (caller holds g_dl through lk and has
   seen g_running < g_slots; the lock is released while the GPU works) */
static void dropin_launch( dropin_stage * b, std::unique_lock<std::mutex> & lk ) {
  int sl = 0;
  while( g_slot_busy[sl] ) sl++;
  g_slot_busy[sl] = 1; g_running++;
  b->state = DSTAGE_RUNNING; g_open = -1;
  g_batches++; g_batch_calls += (ulong)b->users;
  g_dcv.notify_all();                                      /* callers may open the next block now */
  fd_ed25519_hip_ctx_t * ctx = g_slot_ctx[sl];
  ulong n = b->n, bytes = STAGE_MSG + b->pool;
  lk.unlock();
  FD_CHECK( hipSetDevice( ctx->device ) );
  FD_CHECK( hipMemcpyAsync( b->d, b->h, bytes, hipMemcpyHostToDevice, ctx->stream ) );
  verify_impl( ctx, n, b->d + STAGE_SIGS, b->d + STAGE_PUBS, b->d + STAGE_MSG, (uint const *)(b->d + STAGE_OFF),
               (uint const *)(b->d + STAGE_SZ), 0u, (signed char *)(b->d + STAGE_CODES), NULL, NULL, NULL );
  FD_CHECK( hipMemcpyAsync( b->h + STAGE_CODES, b->d + STAGE_CODES, n, hipMemcpyDeviceToHost, ctx->stream ) );
  FD_CHECK( hipStreamSynchronize( ctx->stream ) );
  lk.lock();
  b->state = DSTAGE_DONE; g_slot_busy[sl] = 0; g_running--;
  b->cv.notify_all();                                      /* this batch's callers */
  if( g_open >= 0 ) g_stage[g_open].cv.notify_one();       /* one caller of the open batch runs it on the freed slot */
  g_dcv.notify_all();                                      /* callers waiting to close a full batch */
}

/* verify n (sig, pub) pairs over one message through the combining staging
   ring; codes[j] gets the per-signature code */
static void
dropin_run( uchar const * msg, ulong msg_sz, uchar const * sigs, uchar const * pubs, ulong n, signed char * codes ) {
  fd_ed25519_hip_ctx_t * ctx = default_ctx();
  ulong need = (msg_sz + 16ul + 15ul) & ~15ul;             /* message + 16 zero bytes, 16-B aligned */
  std::unique_lock<std::mutex> lk( g_dl );
  if( !g_slot_ctx[0] ) slots_setup();                      /* no dropin_init: the first call sets up */
  dropin_stage * b;
  for( ;; ) {
    if( g_open < 0 ) {
      int f = -1;
      for( int j=0; j<DROPIN_NBUF; j++ ) if( g_stage[j].state == DSTAGE_FREE ) { f = j; break; }
      if( f < 0 ) { g_dcv.wait( lk ); continue; }
      dropin_stage * o = &g_stage[f];
      if( !o->h ) stage_grow( ctx, o, STAGE_MSG + DROPIN_POOL0 );
      o->state = DSTAGE_OPEN; o->n = 0; o->pool = 0; o->users = 0; o->gen = ++g_gen;
      g_open = f;
    }
    b = &g_stage[g_open];
    /* the records' message offsets are 32-bit (off[] below): a block's pool
       stays under 2^32 bytes, and a caller that would pass it closes the
       block (an empty block always fits: need <= DROPIN_MSG_MAX + 31) */
    if( b->n + n <= DROPIN_REC_MAX && STAGE_MSG + b->pool + need <= b->cap && b->pool + need <= (ulong)UINT32_MAX ) break;
    if( !b->n ) {                                          /* empty and too small: grow it */
      ulong cap = STAGE_MSG + need, dbl = 2ul*b->cap;
      if( dbl > STAGE_MSG + (ulong)UINT32_MAX ) dbl = STAGE_MSG + (ulong)UINT32_MAX;
      stage_grow( ctx, b, cap > dbl ? cap : dbl );
      break;
    }
    /* full: it runs as soon as a slot is free (one of its callers starts
       it, or we do), then this caller opens the next block */
    if( g_running < g_slots ) { dropin_launch( b, lk ); continue; }
    g_dcv.wait( lk );
  }
  ulong r0 = b->n, p0 = b->pool, gen = b->gen;
  b->n += n; b->pool += need; b->users++;
  uchar * h = b->h;
  memcpy( h + STAGE_SIGS + 64ul*r0, sigs, 64ul*n );
  memcpy( h + STAGE_PUBS + 32ul*r0, pubs, 32ul*n );
  uint * off = (uint *)(h + STAGE_OFF), * sz = (uint *)(h + STAGE_SZ);
  for( ulong j=0; j<n; j++ ) { off[r0+j] = (uint)p0; sz[r0+j] = (uint)msg_sz; }
  if( msg_sz ) memcpy( h + STAGE_MSG + p0, msg, msg_sz );
  memset( h + STAGE_MSG + p0 + msg_sz, 0, need - msg_sz );
  for( ;; ) {
    if( b->gen == gen && b->state == DSTAGE_DONE ) break;
    if( g_running < g_slots && b->state == DSTAGE_OPEN ) { dropin_launch( b, lk ); break; }
    b->cv.wait( lk );
  }
  memcpy( codes, h + STAGE_CODES + r0, n );
  if( !--b->users ) { b->state = DSTAGE_FREE; g_dcv.notify_all(); }
}

int
fd_ed25519_verify( uchar const msg[], ulong msg_sz, uchar const sig[64], uchar const public_key[32],
                   struct fd_sha512_private * sha ) {
  (void)sha;
  dropin_check_msg_sz( msg_sz, "fd_ed25519_verify" );
  signed char code;
  dropin_run( msg, msg_sz, sig, public_key, 1ul, &code );
  return (int)code;
}

int
fd_ed25519_verify_batch_single_msg( uchar const msg[], ulong const msg_sz, uchar const signatures[64],
                                    uchar const pubkeys[32], struct fd_sha512_private * shas[1],
                                    uchar const batch_sz ) {
  (void)shas;
  if( batch_sz == 0 || batch_sz > 16 ) return FD_ED25519_ERR_SIG;         /* user.c:238-241 */
  dropin_check_msg_sz( msg_sz, "fd_ed25519_verify_batch_single_msg" );
  signed char codes[16];
  dropin_run( msg, msg_sz, signatures, pubkeys, (ulong)batch_sz, codes );
  int msg_fail = 0;
  for( int j=0; j<batch_sz; j++ ) {                                        /* pass-1 order, then pass 2 */
    if( codes[j] == FD_ED25519_ERR_SIG || codes[j] == FD_ED25519_ERR_PUBKEY ) return codes[j];
    if( codes[j] == FD_ED25519_ERR_MSG ) msg_fail = 1;
  }
  return msg_fail ? FD_ED25519_ERR_MSG : FD_ED25519_SUCCESS;
}

char const *
fd_ed25519_strerror( int err ) {
  switch( err ) {
  case FD_ED25519_SUCCESS:    return "success";
  case FD_ED25519_ERR_SIG:    return "bad signature";
  case FD_ED25519_ERR_PUBKEY: return "bad public key";
  case FD_ED25519_ERR_MSG:    return "bad message";
  default: break;
  }
  return "unknown";
}

} /* extern "C" */
