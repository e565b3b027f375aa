/* fd_ed25519_dev.h -- device-side building blocks of the gfx950 ed25519
   verify engine: GF(2^255-19) arithmetic, extended-coordinate group law,
   point decode, SHA-512 and scalar mod L.

   Every function restates the semantics of the reference verify path
   (anoushk1234/firedancer src/ballet/ed25519/, cited per function); the
   arithmetic is organised for one signature per 64-wide-wave lane.

   Field representation (unsaturated, 9 limbs of u32):
     value = sum_{i<8} v[i] 2^(29 i) + v[8] 2^232
   A product column of 29-bit limbs is < 2^62, so a 64-bit accumulator
   (v_mad_u64_u32 with 64-bit addend) takes a whole column with no carry
   tracking, squaring doubles an operand limb instead of the product, and
   add is 9 plain v_add_u32.  Bounds (proved worst case by
   tools/fe29_bounds.py, which mirrors every formula here; run by
   tests/test_fe_bounds.py):
     "tight"  (every fe_mul / fe_sq output): v[i] <= 2^29-1, except
              v[1] < 2^29 + 2^17 and v[8] <= 2^23-1
     fe_add   no carry: limb-wise sums (< 2^32)
     fe_sub   a + 2p - b, b must be tight (2p's limbs dominate tight limbs)
     fe_norm  one carry pass, restores ~tight limbs; used where a product's
              operands would otherwise overflow a column (dbl: F, and E when T
              is needed; add: E)
   fe_canon gives the unique representative in [0, p) with limbs in range. */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32;
typedef uint64_t u64;
typedef uint8_t  u8;

#define DEV __device__ __forceinline__

/**********************************************************************/
/* Field elements                                                      */

#define FE_M29 0x1fffffffu
#define FE_M23 0x007fffffu

struct fe { u32 v[9]; };

/* Scheduling fence after every multiply: left free, the machine scheduler
   overlaps consecutive multiplies of a long chain (pow22523, the ladder) until
   the kernel runs out of VGPRs and spills to AGPRs; fencing each multiply
   keeps the live set to ~one product column pair plus the operands. */
#define FE_SCHED_FENCE() __builtin_amdgcn_sched_barrier( 0 )

DEV void fe_set( fe & r, u32 c0, u32 c1, u32 c2, u32 c3, u32 c4, u32 c5, u32 c6, u32 c7, u32 c8 ) {
  r.v[0]=c0; r.v[1]=c1; r.v[2]=c2; r.v[3]=c3; r.v[4]=c4; r.v[5]=c5; r.v[6]=c6; r.v[7]=c7; r.v[8]=c8;
}
DEV void fe_0( fe & r ) { fe_set( r, 0,0,0,0,0,0,0,0,0 ); }
DEV void fe_1( fe & r ) { fe_set( r, 1,0,0,0,0,0,0,0,0 ); }
/* d = -121665/121666, 2d, sqrt(-1) (fd_f25519_table_ref.c:28-47), 1/2 */
DEV void fe_d( fe & r )      { fe_set( r, 0x135978a3u,0x0f5a6e50u,0x10762addu,0x00149a82u,0x1e898007u,0x003cbbbcu,0x19ce331du,0x1dc56dffu,0x0052036cu ); }
DEV void fe_d2( fe & r )     { fe_set( r, 0x06b2f159u,0x1eb4dca1u,0x00ec55bau,0x00293505u,0x1d13000eu,0x00797779u,0x139c663au,0x1b8adbffu,0x002406d9u ); }
DEV void fe_sqrtm1( fe & r ) { fe_set( r, 0x0a0ea0b0u,0x0770d93au,0x0bf91e31u,0x06300d5au,0x1d7a72f4u,0x004c9efdu,0x1c2cad34u,0x1009f83bu,0x002b8324u ); }
DEV void fe_inv2( fe & r )   { fe_set( r, 0x1ffffff7u,0x1fffffffu,0x1fffffffu,0x1fffffffu,0x1fffffffu,0x1fffffffu,0x1fffffffu,0x1fffffffu,0x003fffffu ); }

/* 64-bit multiply-accumulate kept in program order: the empty asm makes
   each partial sum opaque, so the compiler cannot re-associate a column into
   two half-chains joined by v_lshl_add_u64 (one extra 64-bit op per column). */
/* split limbs pass through an empty asm so the compiler keeps the masked
   limb instead of re-deriving 2*limb from the unmasked column as
   (col << 1) & 0x3ffffffe (an extra v_and per limb in squaring chains) */
#define FE_OPAQUE( x ) asm( "" : "+v"( x ) )

DEV u64 fe_mad64( u32 a, u32 b, u64 c ) { u64 r = c + (u64)a * b; asm( "" : "+v"(r) ); return r; }
DEV u64 fe_mul64( u32 a, u32 b )        { u64 r = (u64)a * b;     asm( "" : "+v"(r) ); return r; }
/* FREE = true leaves the sums open to re-association (more independent
   chains per product for a wave alone on its SIMD, at an extra 64-bit add
   per split column): the latency kernel's lane-parallel products */
template<bool FREE> DEV u64 fe_madT( u32 a, u32 b, u64 c ) { return FREE ? c + (u64)a * b : fe_mad64( a, b, c ); }
template<bool FREE> DEV u64 fe_mulT( u32 a, u32 b )        { return FREE ? (u64)a * b : fe_mul64( a, b ); }

/* Product columns (column k = sum over i+j=k, 0<=i,j<=8):
     high column 9+j is kept as an unsplit 64-bit sum H_{9+j} (< 2^63): a
       fresh, independent chain of 8-j multiply-adds;
     low column j = carry + its products + 1216*lo32(H_{9+j})
       + 9728*hi32(H_{8+j})  (2^261 == 19*2^6 == 1216 mod p, and the high
       word of H_{8+j} sits 32 bits up = 3 bits into the next limb: 1216*8),
       then split at 29 bits (v_and + v_lshrrev_b64).
   H_{9+j} is computed interleaved with low column j, so only two H sums are
   live per product.  Column 8 splits at bit 255 and its overflow folds into
   limb 0 with 19.
   fe_mulN / fe_sqN run N independent products interleaved instruction by
   instruction (2N chains): back-to-back dependent v_mad_u64_u32 need a wait
   state, which another chain's multiply-add fills.  Formulas pair (N = 2)
   their independent products; N = 3 measured slower in k_verify_dsm. */
DEV void fe_fin( fe & r, u32 o[9], u64 l ) {   /* column-8 split + fold, output copy */
  o[8] = (u32)l & FE_M23;
  u64 t = (l >> 23) * 19u + o[0];
  o[0] = (u32)t & FE_M29;
  o[1] += (u32)(t >> 29);
  #pragma unroll
  for( int i=0; i<9; i++ ) r.v[i] = o[i];
}

template<int N, bool FREE = false>
DEV void fe_mulN( fe * const r[N], fe const * const a[N], fe const * const b[N] ) {
  u32 o[N][9];
  u64 l[N], hp[N], h[N];
  #pragma unroll
  for( int j=0; j<=8; j++ ) {
    int c = 9 + j;
    #pragma unroll
    for( int i=0; i<=8; i++ ) {
      if( j < 8 && i <= 7-j ) {
        #pragma unroll
        for( int n=0; n<N; n++ ) h[n] = (i == 0) ? fe_mulT<FREE>( a[n]->v[c-8+i], b[n]->v[8-i] ) : fe_madT<FREE>( a[n]->v[c-8+i], b[n]->v[8-i], h[n] );
      }
      if( i <= j ) {
        #pragma unroll
        for( int n=0; n<N; n++ ) l[n] = (j == 0) ? fe_mulT<FREE>( a[n]->v[0], b[n]->v[0] ) : fe_madT<FREE>( a[n]->v[i], b[n]->v[j-i], l[n] );
      }
    }
    #pragma unroll
    for( int n=0; n<N; n++ ) {
      if( j < 8 ) l[n] = fe_madT<FREE>( (u32)h[n], 1216u, l[n] );
      if( j > 0 ) l[n] = fe_madT<FREE>( (u32)(hp[n] >> 32), 9728u, l[n] );
      if( j < 8 ) { o[n][j] = (u32)l[n] & FE_M29; FE_OPAQUE( o[n][j] ); l[n] >>= 29; }
      hp[n] = h[n];
    }
  }
  #pragma unroll
  for( int n=0; n<N; n++ ) fe_fin( *r[n], o[n], l[n] );
  FE_SCHED_FENCE();
}

/* 2*x as v_add_u32_e32 (x + x): the compiler's v_lshlrev_b32 form issues
   at the full-cost rate on gfx950, the add at the fast VOP2 rate
   (profiles/r02zd_valu_issue_calibration.json: lshl_e32 vs add_e32); with
   the address-swapped cached loads, C2 +1.0%, k_verify_dsm -1.1% against the
   round-2 forms on one box (profiles/r03e/ab_micro) */
DEV u32 fe_x2( u32 x ) {
  u32 r; asm( "v_add_u32_e32 %0, %1, %1" : "=v"( r ) : "v"( x ) ); return r;
}

/* squares: off-diagonal products taken once against 2*a_i */
template<int N, bool FREE = false>
DEV void fe_sqN( fe * const r[N], fe const * const a[N] ) {
  u32 d[N][9], o[N][9];
  u64 l[N], hp[N], h[N];
  #pragma unroll
  for( int n=0; n<N; n++ ) {
    #pragma unroll
    for( int i=0; i<9; i++ ) d[n][i] = fe_x2( a[n]->v[i] );
  }
  #pragma unroll
  for( int j=0; j<=8; j++ ) {
    int c = 9 + j;
    #pragma unroll
    for( int i=0; i<=8; i++ ) {
      int hi = c - 8 + i;                             /* high: d[hi]*a[c-hi], 2*hi < c */
      if( j < 8 && 2*hi < c ) {
        #pragma unroll
        for( int n=0; n<N; n++ ) h[n] = (i == 0) ? fe_mulT<FREE>( d[n][hi], a[n]->v[c-hi] ) : fe_madT<FREE>( d[n][hi], a[n]->v[c-hi], h[n] );
      }
      if( 2*i < j ) {                                 /* j >= 1: onto the carry */
        #pragma unroll
        for( int n=0; n<N; n++ ) l[n] = fe_madT<FREE>( d[n][i], a[n]->v[j-i], l[n] );
      }
    }
    #pragma unroll
    for( int n=0; n<N; n++ ) {
      if( j < 8 && (c & 1) == 0 ) h[n] = (c == 16) ? fe_mulT<FREE>( a[n]->v[8], a[n]->v[8] ) : fe_madT<FREE>( a[n]->v[c/2], a[n]->v[c/2], h[n] );
      if( (j & 1) == 0 ) l[n] = (j == 0) ? fe_mulT<FREE>( a[n]->v[0], a[n]->v[0] ) : fe_madT<FREE>( a[n]->v[j/2], a[n]->v[j/2], l[n] );
    }
    #pragma unroll
    for( int n=0; n<N; n++ ) {
      if( j < 8 ) l[n] = fe_madT<FREE>( (u32)h[n], 1216u, l[n] );
      if( j > 0 ) l[n] = fe_madT<FREE>( (u32)(hp[n] >> 32), 9728u, l[n] );
      if( j < 8 ) { o[n][j] = (u32)l[n] & FE_M29; FE_OPAQUE( o[n][j] ); l[n] >>= 29; }
      hp[n] = h[n];
    }
  }
  #pragma unroll
  for( int n=0; n<N; n++ ) fe_fin( *r[n], o[n], l[n] );
  FE_SCHED_FENCE();
}

DEV void fe_mul( fe & r, fe const & a, fe const & b ) {
  fe * const R[1] = { &r }; fe const * const A[1] = { &a }; fe const * const B[1] = { &b };
  fe_mulN<1>( R, A, B );
}
DEV void fe_mul2( fe & r, fe const & a, fe const & b, fe & s, fe const & c, fe const & d ) {
  fe * const R[2] = { &r, &s }; fe const * const A[2] = { &a, &c }; fe const * const B[2] = { &b, &d };
  fe_mulN<2>( R, A, B );
}
/* one product / square with open sums (FREE, see fe_madT) */
DEV void fe_mul_free( fe & r, fe const & a, fe const & b ) {
  fe * const R[1] = { &r }; fe const * const A[1] = { &a }; fe const * const B[1] = { &b };
  fe_mulN<1, true>( R, A, B );
}
DEV void fe_sq_free( fe & r, fe const & a ) {
  fe * const R[1] = { &r }; fe const * const A[1] = { &a };
  fe_sqN<1, true>( R, A );
}
DEV void fe_sq( fe & r, fe const & a ) {
  fe * const R[1] = { &r }; fe const * const A[1] = { &a };
  fe_sqN<1>( R, A );
}
DEV void fe_sq2( fe & r, fe const & a, fe & s, fe const & c ) {
  fe * const R[2] = { &r, &s }; fe const * const A[2] = { &a, &c };
  fe_sqN<2>( R, A );
}

DEV void fe_add( fe & r, fe const & a, fe const & b ) {
  #pragma unroll
  for( int i=0; i<9; i++ ) r.v[i] = a.v[i] + b.v[i];
}

/* 2a, limb-wise (the fast VOP2 add, fe_x2) */
DEV void fe_dbl( fe & r, fe const & a ) {
  #pragma unroll
  for( int i=0; i<9; i++ ) r.v[i] = fe_x2( a.v[i] );
}

/* a - b + 2p (b tight) */
DEV void fe_sub( fe & r, fe const & a, fe const & b ) {
  r.v[0] = (a.v[0] - b.v[0]) + 0x3fffffdau;
  #pragma unroll
  for( int i=1; i<8; i++ ) r.v[i] = (a.v[i] - b.v[i]) + 0x3ffffffeu;
  r.v[8] = (a.v[8] - b.v[8]) + 0x00fffffeu;
}

/* one carry pass (no overflow for limbs < 2^32 - 8) */
DEV void fe_norm( fe & r, fe const & a ) {
  u32 c = 0;
  #pragma unroll
  for( int i=0; i<8; i++ ) { u32 x = a.v[i] + c; c = x >> 29; r.v[i] = x & FE_M29; }
  u32 x = a.v[8] + c;
  r.v[8] = x & FE_M23;
  r.v[0] += 19u * (x >> 23);
}

/* FREE: the open-sum products (fe_mul_free / fe_sq_free), for a wave alone
   on its SIMD (k_verify_lat); the bulk kernels use the default */
template<bool FREE> DEV void fe_mulF( fe & r, fe const & a, fe const & b ) { if( FREE ) fe_mul_free( r, a, b ); else fe_mul( r, a, b ); }
template<bool FREE> DEV void fe_sqF( fe & r, fe const & a ) { if( FREE ) fe_sq_free( r, a ); else fe_sq( r, a ); }

template<bool FREE = false>
DEV void fe_sqn( fe & r, fe const & a, int n ) {
  fe_sqF<FREE>( r, a );
  #pragma unroll 1
  for( int i=1; i<n; i++ ) fe_sqF<FREE>( r, r );
}

/* any bounded a -> canonical [0,p): two carry passes leave limbs in range and
   the value < 2^255; then subtract p once iff value + 19 >= 2^255. */
DEV void fe_canon( fe & r, fe const & a ) {
  fe t; fe_norm( t, a ); fe_norm( t, t );
  u32 c = (t.v[0] + 19u) >> 29;
  #pragma unroll
  for( int i=1; i<8; i++ ) c = (t.v[i] + c) >> 29;
  u32 q = (t.v[8] + c) >> 23;              /* t >= p */
  u32 x = t.v[0] + 19u*q;
  r.v[0] = x & FE_M29; c = x >> 29;
  #pragma unroll
  for( int i=1; i<8; i++ ) { x = t.v[i] + c; r.v[i] = x & FE_M29; c = x >> 29; }
  r.v[8] = (t.v[8] + c) & FE_M23;
}

DEV bool fe_is_zero_c( fe const & c ) {   /* c canonical */
  return (c.v[0]|c.v[1]|c.v[2]|c.v[3]|c.v[4]|c.v[5]|c.v[6]|c.v[7]|c.v[8]) == 0u;
}
DEV bool fe_eq_c( fe const & a, fe const & b ) {   /* both canonical */
  return ((a.v[0]^b.v[0])|(a.v[1]^b.v[1])|(a.v[2]^b.v[2])|(a.v[3]^b.v[3])|(a.v[4]^b.v[4])|
          (a.v[5]^b.v[5])|(a.v[6]^b.v[6])|(a.v[7]^b.v[7])|(a.v[8]^b.v[8])) == 0u;
}

/* r = -a for tight a (result 2p-bounded; fe_norm it before use as tight) */
DEV void fe_neg( fe & r, fe const & a ) { fe z; fe_0( z ); fe_sub( r, z, a ); }

/* conditional swap / move (mask is 0 or ~0 per lane; xor form: v_cndmask_b32
   issues at 1/8 the rate of v_xor_b32 on gfx950, profiles/r01_valu_rates_b.txt) */
DEV void fe_cswap( fe & a, fe & b, u32 mask ) {
  #pragma unroll
  for( int i=0; i<9; i++ ) { u32 t = (a.v[i] ^ b.v[i]) & mask; a.v[i] ^= t; b.v[i] ^= t; }
}
DEV void fe_cmov( fe & r, fe const & a, u32 mask ) {   /* r = mask ? a : r */
  #pragma unroll
  for( int i=0; i<9; i++ ) r.v[i] ^= (r.v[i] ^ a.v[i]) & mask;
}

/* z^(2^252-3): fd_f25519.c:25-74 (same exponent; this addition chain) */
template<bool FREE = false>
DEV void fe_pow22523( fe & out, fe const & z ) {
  fe z2, z9, z11, a, b, c, t;
  fe_sqF<FREE>( z2, z );                                  /* 2 */
  fe_sqn<FREE>( t, z2, 2 ); fe_mulF<FREE>( z9, t, z );   /* 9 */
  fe_mulF<FREE>( z11, z9, z2 );                           /* 11 */
  fe_sqF<FREE>( t, z11 ); fe_mulF<FREE>( a, t, z9 );      /* a = z^(2^5-1) */
  fe_sqn<FREE>( t, a, 5 );   fe_mulF<FREE>( b, t, a );   /* 2^10-1 */
  fe_sqn<FREE>( t, b, 10 );  fe_mulF<FREE>( c, t, b );   /* 2^20-1 */
  fe_sqn<FREE>( t, c, 20 );  fe_mulF<FREE>( t, t, c );   /* 2^40-1 */
  fe_sqn<FREE>( t, t, 10 );  fe_mulF<FREE>( b, t, b );   /* b = 2^50-1 */
  fe_sqn<FREE>( t, b, 50 );  fe_mulF<FREE>( c, t, b );   /* c = 2^100-1 */
  fe_sqn<FREE>( t, c, 100 ); fe_mulF<FREE>( t, t, c );   /* 2^200-1 */
  fe_sqn<FREE>( t, t, 50 );  fe_mulF<FREE>( t, t, b );   /* 2^250-1 */
  fe_sqn<FREE>( t, t, 2 );   fe_mulF<FREE>( out, t, z ); /* 2^252-3 */
}

/* z^(p-2) = (z^(2^252-3))^8 * z^3 */
DEV void fe_invert( fe & out, fe const & z ) {
  fe a, z3;
  fe_pow22523( a, z ); fe_sqn( a, a, 3 );
  fe_sq( z3, z ); fe_mul( z3, z3, z );
  fe_mul( out, a, z3 );
}

/* 32 little-endian bytes (as 8 LE u32 words) -> fe, masking bit 255
   (fd_f25519.h frombytes accepts non-canonical y in [p, 2^255)) */
DEV void fe_from_words( fe & r, u32 const w[8] ) {
  r.v[0] = w[0] & FE_M29;
  #pragma unroll
  for( int i=1; i<8; i++ ) {
    int b = 29*i, j = b >> 5, s = b & 31;
    u32 x = (s + 29 <= 32) ? (w[j] >> s) : __builtin_amdgcn_alignbit( w[j+1], w[j], (u32)s );
    r.v[i] = x & FE_M29;
  }
  r.v[8] = (w[7] >> 8) & FE_M23;
}

/* canonical fe -> 8 LE u32 words */
DEV void fe_to_words( u32 w[8], fe const & a ) {
  w[0] = a.v[0]        | (a.v[1] << 29);
  w[1] = (a.v[1] >> 3)  | (a.v[2] << 26);
  w[2] = (a.v[2] >> 6)  | (a.v[3] << 23);
  w[3] = (a.v[3] >> 9)  | (a.v[4] << 20);
  w[4] = (a.v[4] >> 12) | (a.v[5] << 17);
  w[5] = (a.v[5] >> 15) | (a.v[6] << 14);
  w[6] = (a.v[6] >> 18) | (a.v[7] << 11);
  w[7] = (a.v[7] >> 21) | (a.v[8] << 8);
}

/**********************************************************************/
/* Group: twisted Edwards a=-1, extended coordinates, HWCD'08 formulas
   (ref/fd_curve25519.c:25-92 add, ref/fd_curve25519.h:190-211 dbl).
   Normalisation points are the ones tools/fe29_bounds.py proves.        */

struct ge_p3     { fe X, Y, Z, T; };
struct ge_cached { fe YmX, YpX, T2d, Z2; };   /* (Y-X, Y+X, 2d*T, 2*Z), each normalised */
/* affine cached point scaled by 1/2: ((y-x)/2, (y+x)/2, d*x*y); the implied
   2*Z is 1, so the addition's D = Z1*2*Z2 is just Z1 (the result is the same
   projective point, every output coordinate scaled by 1/4) */
struct ge_affc   { fe YmX, YpX, T2d; };

DEV void ge_identity( ge_p3 & r ) { fe_0( r.X ); fe_1( r.Y ); fe_1( r.Z ); fe_0( r.T ); }

/* r = 2p.  partial_dbl + final mul; T produced only when asked. */
DEV void ge_dbl( ge_p3 & r, ge_p3 const & p, bool needT ) {
  fe A, B, C, S, H, G, F, E;
  fe_add( S, p.X, p.Y );
  fe_sq2( A, p.X, B, p.Y ); fe_sq2( C, p.Z, S, S );
  fe_dbl( C, C );             /* 2Z^2            */
  fe_add( H, A, B );          /* A+B             */
  fe_sub( G, A, B );          /* A-B             */
  fe_add( F, C, G );          /* 2Z^2+A-B        */
  fe_norm( F, F );
  fe_sub( E, H, S );          /* A+B-(X+Y)^2     */
  if( needT ) fe_norm( E, E );
  fe_mul2( r.X, E, F, r.Y, G, H );
  if( needT ) fe_mul2( r.Z, F, G, r.T, E, H );
  else        fe_mul( r.Z, F, G );
}

/* r = p +/- q (q in cached form).  neg is a per-lane mask (0 or ~0).
   YX_SWAPPED: the caller loaded q with Y-X / Y+X already exchanged where neg
   (load_cached_signed), so only 2dT's sign is left to apply here. */
template<bool YX_SWAPPED = false>
DEV void ge_add_cached( ge_p3 & r, ge_p3 const & p, ge_cached q, u32 neg, bool needT ) {
  fe a, b, A, B, C, D, E, F, G, H;
  if( !YX_SWAPPED ) fe_cswap( q.YmX, q.YpX, neg );   /* -q: swap Y-X / Y+X ... */
  fe_sub( a, p.Y, p.X ); fe_add( b, p.Y, p.X );
  fe_mul2( A, a, q.YmX, B, b, q.YpX );
  fe_mul2( C, p.T, q.T2d, D, p.Z, q.Z2 );
  fe_sub( E, B, A ); fe_norm( E, E ); fe_add( H, B, A );
  fe_sub( F, D, C ); fe_add( G, D, C );
  fe_cswap( F, G, neg );                   /* ... and negate 2dT: C -> -C swaps F and G */
  fe_mul2( r.X, E, F, r.Y, G, H );
  if( needT ) fe_mul2( r.Z, F, G, r.T, E, H );
  else        fe_mul( r.Z, F, G );
}

/* r = p + q with q the cached form of an affine point (2*Z = 2): D = 2*Z1
   is an add, not a multiply (table chains, whose addend is the base point) */
DEV void ge_add_cached_z1( ge_p3 & r, ge_p3 const & p, ge_cached const & q ) {
  fe a, b, A, B, C, D, E, F, G, H;
  fe_sub( a, p.Y, p.X ); fe_add( b, p.Y, p.X );
  fe_mul2( A, a, q.YmX, B, b, q.YpX );
  fe_mul( C, p.T, q.T2d );
  fe_add( D, p.Z, p.Z ); fe_norm( D, D );
  fe_sub( E, B, A ); fe_norm( E, E ); fe_add( H, B, A );
  fe_sub( F, D, C ); fe_add( G, D, C );
  fe_mul2( r.X, E, F, r.Y, G, H );
  fe_mul2( r.Z, F, G, r.T, E, H );
}

/* r = p +/- q with q an affine cached point scaled by 1/2 (D = Z1) */
DEV void ge_add_affc( ge_p3 & r, ge_p3 const & p, ge_affc q, u32 neg, bool needT ) {
  fe a, b, A, B, C, E, F, G, H;
  fe_cswap( q.YmX, q.YpX, neg );
  fe_sub( a, p.Y, p.X ); fe_add( b, p.Y, p.X );
  fe_mul2( A, a, q.YmX, B, b, q.YpX );
  fe_mul( C, p.T, q.T2d );
  fe_sub( E, B, A ); fe_norm( E, E ); fe_add( H, B, A );
  fe_sub( F, p.Z, C ); fe_add( G, p.Z, C );
  fe_cswap( F, G, neg );
  fe_mul2( r.X, E, F, r.Y, G, H );
  if( needT ) fe_mul2( r.Z, F, G, r.T, E, H );
  else        fe_mul( r.Z, F, G );
}

/* fd_curve25519_into_precomputed (ref/fd_curve25519.h:141-151) with Z doubled */
DEV void ge_to_cached( ge_cached & c, ge_p3 const & p ) {
  fe d2; fe_d2( d2 );
  fe_sub( c.YmX, p.Y, p.X ); fe_norm( c.YmX, c.YmX );
  fe_add( c.YpX, p.Y, p.X ); fe_norm( c.YpX, c.YpX );
  fe_mul( c.T2d, p.T, d2 );
  fe_add( c.Z2, p.Z, p.Z );  fe_norm( c.Z2, c.Z2 );
}

/* Point decompression: fd_curve25519.c:34-61 + fd_f25519.c:122-158, with the
   AVX-512 backend's failure split (avx512/fd_r43x6_ge.c:163-254).
   Returns bit0 = not on curve (u/v not a square), bit1 = x==0 with sign bit
   set (AVX-512 rejects in decode; the ref backend keeps x=0 and rejects it
   as small order).  On success r = (x, y, 1, xy) with x, y canonical. */
template<bool FREE = false>
DEV u32 ge_decode( ge_p3 & r, u32 const w[8] ) {
  fe y, y2, u, v, v3, v7, t, x, chk, one, d;
  u32 sign = w[7] >> 31;
  fe_from_words( y, w );
  fe_1( one ); fe_d( d );
  fe_sqF<FREE>( y2, y );
  fe_sub( u, y2, one );                 /* u = y^2 - 1 */
  fe_mulF<FREE>( v, y2, d ); fe_add( v, v, one ); /* v = d y^2 + 1 */
  fe_sqF<FREE>( v3, v ); fe_mulF<FREE>( v3, v3, v );  /* v^3 */
  fe_sqF<FREE>( v7, v3 ); fe_mulF<FREE>( v7, v7, v ); /* v^7 */
  fe_mulF<FREE>( t, u, v7 ); fe_pow22523<FREE>( t, t );
  fe_mulF<FREE>( x, u, v3 ); fe_mulF<FREE>( x, x, t ); /* x = u v^3 (u v^7)^((p-5)/8) */
  fe_sqF<FREE>( chk, x ); fe_mulF<FREE>( chk, chk, v ); /* v x^2 */
  fe cu, cc, nu;
  fe_canon( cu, u ); fe_canon( cc, chk );
  fe_neg( nu, cu ); fe_canon( nu, nu );
  bool ok1 = fe_eq_c( cc, cu );
  bool ok2 = fe_eq_c( cc, nu );
  fe xs, sq; fe_sqrtm1( sq ); fe_mul( xs, x, sq );
  fe_cmov( x, xs, ok1 ? 0u : ~0u );     /* v x^2 == -u: x *= sqrt(-1) */
  fe_canon( x, x );
  u32 xz = fe_is_zero_c( x ) ? 1u : 0u;
  u32 flags = ((ok1 || ok2) ? 0u : 1u) | ((xz & sign) << 1);
  /* choose the root with parity == sign (neg(0) stays 0) */
  fe nx; fe_neg( nx, x ); fe_canon( nx, nx );
  fe_cmov( x, nx, ((x.v[0] & 1u) != sign) ? ~0u : 0u );
  fe_canon( r.Y, y );
  r.X = x; fe_1( r.Z ); fe_mul( r.T, x, r.Y );
  return flags;
}

/* fd_curve25519.h:88-118: x==0 | y==0 | y==y0 | y==y1 (affine, canonical x,y) */
DEV bool ge_affine_is_small_order( ge_p3 const & p ) {
  fe y0, y1;
  fe_set( y0, 0x0f95e826u,0x013d9614u,0x1d30d16cu,0x11dfe513u,0x0dfd5f09u,0x036982d6u,0x02c4e4cfu,0x0db10047u,0x0005fc53u );
  fe_set( y1, 0x106a17c7u,0x1ec269ebu,0x02cf2e93u,0x0e201aecu,0x1202a0f6u,0x1c967d29u,0x1d3b1b30u,0x124effb8u,0x007a03acu );
  return fe_is_zero_c( p.X ) | fe_is_zero_c( p.Y ) | fe_eq_c( p.Y, y0 ) | fe_eq_c( p.Y, y1 );
}


/**********************************************************************/
/* Scalars mod L (fd_curve25519_scalar.h / .c)                         */

/* S <= L-1 (fd_curve25519_scalar.h:57-73) */
DEV bool sc_is_canonical( u32 const s[8] ) {
  const u32 L[8] = { 0x5cf5d3edu,0x5812631au,0xa2f79cd6u,0x14def9deu,0u,0u,0u,0x10000000u };
  /* s < L  <=>  s - L borrows */
  u64 bw = 0;
  #pragma unroll
  for( int i=0; i<8; i++ ) { u64 d = (u64)s[i] - L[i] - bw; bw = (d >> 63) & 1u; }
  return bw != 0;
}

/* 512-bit little-endian x (16 limbs) mod L, Barrett (HAC 14.42, b=2^32, k=8,
   mu = floor(2^512/L)).  Restates fd_curve25519_scalar_reduce
   (fd_curve25519_scalar.c:3-110) as a different algorithm with the same
   result. */
DEV void sc_reduce512( u32 r[8], u32 const x[16] ) {
  const u32 MU[9] = { 0x0a2c131bu,0xed9ce5a3u,0x086329a7u,0x2106215du,0xffffffebu,0xffffffffu,0xffffffffu,0xffffffffu,0x0000000fu };
  const u32 L[8]  = { 0x5cf5d3edu,0x5812631au,0xa2f79cd6u,0x14def9deu,0u,0u,0u,0x10000000u };
  /* q3 = floor( floor(x / b^7) * mu / b^9 ) : columns 9..17 of q1*mu (q1 = x[7..15]) */
  u32 q3[9];
  u64 lo = 0, hi = 0;   /* 128-bit column accumulator (lo, hi) */
  #pragma unroll
  for( int k=0; k<18; k++ ) {
    #pragma unroll
    for( int i=0; i<9; i++ ) {
      int j = k - i;
      if( j < 0 || j > 8 ) continue;
      u64 p = (u64)x[7+i] * MU[j];
      lo += p; hi += (lo < p) ? 1u : 0u;
    }
    if( k >= 9 ) q3[k-9] = (u32)lo;
    lo = (lo >> 32) | (hi << 32); hi >>= 32;
  }
  /* r2 = q3 * L mod b^9 ; r = x mod b^9 - r2 (mod b^9) */
  u32 r2[9];
  lo = 0; hi = 0;
  #pragma unroll
  for( int k=0; k<9; k++ ) {
    #pragma unroll
    for( int i=0; i<9; i++ ) {
      int j = k - i;
      if( j < 0 || j > 7 ) continue;
      if( j >= 4 && j < 7 ) continue;     /* L limbs 4..6 are zero */
      u64 p = (u64)q3[i] * L[j];
      lo += p; hi += (lo < p) ? 1u : 0u;
    }
    r2[k] = (u32)lo;
    lo = (lo >> 32) | (hi << 32); hi >>= 32;
  }
  u32 t[9]; u64 bw = 0;
  #pragma unroll
  for( int i=0; i<9; i++ ) { u64 d = (u64)x[i] - r2[i] - bw; t[i] = (u32)d; bw = (d >> 63) & 1u; }
  /* t < 3L: subtract L at most twice */
  #pragma unroll
  for( int rep=0; rep<2; rep++ ) {
    u32 s[9]; bw = 0;
    #pragma unroll
    for( int i=0; i<9; i++ ) { u64 d = (u64)t[i] - (i<8 ? L[i] : 0u) - bw; s[i] = (u32)d; bw = (d >> 63) & 1u; }
    u32 m = bw ? 0u : ~0u;                 /* no borrow: t >= L, take s */
    #pragma unroll
    for( int i=0; i<9; i++ ) t[i] = (s[i] & m) | (t[i] & ~m);
  }
  #pragma unroll
  for( int i=0; i<8; i++ ) r[i] = t[i];
}

/* Signed radix-16 digits of k < 2^253 packed (biased by 8) 8 per u32:
   nibble i of out[i/8] = d_i + 8, d_i in [-8,7] except d_63 in [0,2]. */
DEV void sc_recode16( u32 out[8], u32 const k[8] ) {
  u32 carry = 0;
  #pragma unroll
  for( int w=0; w<8; w++ ) {
    u32 o = 0;
    #pragma unroll
    for( int n=0; n<8; n++ ) {
      u32 d = ((k[w] >> (4*n)) & 15u) + carry;
      carry = (d + 8u) >> 4;
      d = d + 8u - (carry << 4);          /* biased digit in [0,15] (d_63 may be 10) */
      o |= d << (4*n);
    }
    out[w] = o;
  }
}

/* Signed radix-256 digits of s < 2^253 packed (biased by 128) 4 per u32 */
DEV void sc_recode256( u32 out[8], u32 const s[8] ) {
  u32 carry = 0;
  #pragma unroll
  for( int w=0; w<8; w++ ) {
    u32 o = 0;
    #pragma unroll
    for( int n=0; n<4; n++ ) {
      u32 d = ((s[w] >> (8*n)) & 255u) + carry;
      carry = (d + 128u) >> 8;
      d = d + 128u - (carry << 8);
      o |= d << (8*n);
    }
    out[w] = o;
  }
}

/* Signed radix-16 digits in [-7,8] of k < 2^252 packed (biased by 7) 8 per
   u32: nibble i of out[i/8] = d_i + 7.  With digit 8 allowed, a k of b bits
   has all digits from floor(b/4)+1 up zero (the carry out of the top nibble
   needs it >= 8 plus a carry in, i.e. b % 4 == 0). */
DEV void sc_recode16s( u32 out[8], u32 const k[8] ) {
  u32 carry = 0;
  #pragma unroll
  for( int w=0; w<8; w++ ) {
    u32 o = 0;
    #pragma unroll
    for( int n=0; n<8; n++ ) {
      u32 d = ((k[w] >> (4*n)) & 15u) + carry;
      carry = (d + 7u) >> 4;               /* d >= 9 */
      d = d + 7u - (carry << 4);
      o |= d << (4*n);
    }
    out[w] = o;
  }
}

/* ---- multiword integers, little-endian u32 words ---- */

/* m ? a : b for a mask m (0 or ~0), as v_bfi_b32: the compiler would
   otherwise turn a compare-derived mask into v_cndmask, which issues at ~1/5
   the rate on gfx950 (profiles/r01_valu_rates_b.txt) */
DEV u32 mw_sel( u32 m, u32 a, u32 b ) {
  u32 r;
  asm( "v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b) );
  return r;
}

/* o = a - q*b mod 2^(32N); returns 1 when a < q*b (a, b unsigned, the
   difference above -2^(32N)) */
/* carry chains through v_add_co / v_addc_co (v_sub_co / v_subb_co) */
template<int N>
DEV u32 mw_submul( u32 o[N], u32 const a[N], u32 const b[N], u32 q ) {
  u32 c = 0, bw = 0;
  #pragma unroll
  for( int i=0; i<N; i++ ) {
    u64 p = (u64)b[i] * q + c; c = (u32)(p >> 32);
    o[i] = __builtin_subc( a[i], (u32)p, bw, &bw );
  }
  return (c | bw) != 0u;
}
template<int N>
DEV void mw_add( u32 o[N], u32 const a[N], u32 const b[N] ) {
  u32 c = 0;
  #pragma unroll
  for( int i=0; i<N; i++ ) o[i] = __builtin_addc( a[i], b[i], c, &c );
}
template<int N>
DEV u32 mw_sub( u32 o[N], u32 const a[N], u32 const b[N] ) {   /* returns the borrow (a < b unsigned) */
  u32 bw = 0;
  #pragma unroll
  for( int i=0; i<N; i++ ) o[i] = __builtin_subc( a[i], b[i], bw, &bw );
  return bw;
}
template<int N>
DEV void mw_cneg( u32 x[N], u32 m ) {       /* x = m ? -x : x (two's complement), m 0 or ~0 */
  u32 c = m & 1u;
  #pragma unroll
  for( int i=0; i<N; i++ ) x[i] = __builtin_addc( x[i] ^ m, 0u, c, &c );
}
template<int N>
DEV u32 mw_bitlen( u32 const x[N] ) {       /* unsigned bit length */
  u32 b = 0;
  #pragma unroll
  for( int i=0; i<N; i++ ) b = x[i] ? 32u*(u32)i + 32u - (u32)__builtin_clz( x[i] ) : b;
  return b;
}
template<int N>
DEV u32 mw_abs_bitlen( u32 const x[N] ) {   /* bit length of |x|, x two's complement */
  u32 a[N];
  #pragma unroll
  for( int i=0; i<N; i++ ) a[i] = x[i];
  mw_cneg<N>( a, (u32)((int)x[N-1] >> 31) );
  return mw_bitlen<N>( a );
}
DEV double mw_to_f64( u32 const a[8] ) {   /* approximation, relative error < 2^-49 */
  double d = (double)a[7];
  #pragma unroll
  for( int i=6; i>=0; i-- ) d = fma( d, 4294967296.0, (double)a[i] );
  return d;
}

/* r = a*b mod L for a, b < 2^256 */
DEV void sc_mul( u32 r[8], u32 const a[8], u32 const b[8] ) {
  u32 prod[16];
  u64 lo = 0, hi = 0;
  #pragma unroll
  for( int c=0; c<16; c++ ) {
    #pragma unroll
    for( int i=0; i<8; i++ ) {
      int j = c - i; if( j < 0 || j > 7 ) continue;
      u64 p = (u64)a[i] * b[j]; lo += p; hi += (lo < p) ? 1u : 0u;
    }
    prod[c] = (u32)lo; lo = (lo >> 32) | (hi << 32); hi >>= 32;
  }
  sc_reduce512( r, prod );
}

/* ---- half-size scalars -------------------------------------------------

   For k < L find k1, k2 with k1 == k*k2 (mod 8L), k2 odd and 0 < k2 < L,
   both near 2^128.  Then with D = [S]B - [k]A - R (the point whose being
   the identity is the reference's accept condition, fd_ed25519_user.c:
   216-226):

     [k2]D = [k2*S mod L]B - [k1]A - [k2]R

   (B has order L; A and R lie in the group of order 8L, so k2*k may be
   replaced by anything congruent to it mod 8L), and [k2]D == O iff D == O
   since k2 is prime to 8L.  The cofactorless verdict is unchanged bit for
   bit, while the double-scalar multiplication needs ~128 doublings instead
   of ~252.  The technique is the half-size-scalar EdDSA verification of
   T. Pornin, "Optimized Lattice Basis Reduction In Dimension 2, and Fast
   Schnorr and EdDSA Signature Verification" (IACR eprint 2020/454); the
   reduction here is truncated Euclid on (8L, k) with cofactors (remainder
   r_i == k*t_i mod 8L), float-estimated 32-bit quotients corrected exactly,
   stopped when the remainder falls below 2^128; the result is the shortest
   odd-t vector among three consecutive (r_i, t_i) and their sums and
   differences.  A lane that meets a quotient >= 2^32 (probability ~2^-30
   for a hashed k) keeps the full-length pair (k, 1).  tools/halfsize_model.py
   models it.

   Out: k1 = |k1| (< 2^251), k1neg = k1 < 0 (0 or ~0), k2 > 0 (< 2^160);
   returns max(bitlen k1, bitlen k2). */
DEV void hs_pick( u32 br[9], u32 bt[5], u32 & bc, u32 const r[9], u32 const t[5] ) {
  u32 c = max( mw_abs_bitlen<9>( r ), mw_abs_bitlen<5>( t ) ) | ((~t[0] & 1u) << 10);   /* even t: 1024+ */
  u32 take = (u32)((int)(c - bc) >> 31);       /* c < bc (both < 2^11) */
  #pragma unroll
  for( int i=0; i<9; i++ ) br[i] = mw_sel( take, r[i], br[i] );
  #pragma unroll
  for( int i=0; i<5; i++ ) bt[i] = mw_sel( take, t[i], bt[i] );
  bc = mw_sel( take, c, bc );
}
DEV void hs_pick2( u32 br[9], u32 bt[5], u32 & bc, u32 const ra[9], u32 const ta[5], u32 const rb[9],
                   u32 const tb[5] ) {
  u32 r[9], t[5];
  mw_add<9>( r, ra, rb ); mw_add<5>( t, ta, tb ); hs_pick( br, bt, bc, r, t );
  mw_sub<9>( r, ra, rb ); mw_sub<5>( t, ta, tb ); hs_pick( br, bt, bc, r, t );
}

/* One Euclid step in place: x = x mod y, t_x -= q*t_y, for remainders
   x >= y >= 2^128.  q comes from the float quotient (relative error < 2^-47,
   so it is the exact quotient or one off either way); the rare corrections
   run behind wave-wide votes so the common path carries no selects.
   Returns false when q >= 2^32. */
DEV bool hs_step( u32 x[8], u32 tx[5], double & dx, u32 const y[8], u32 const ty[5], double dy ) {
  double r = __builtin_amdgcn_rcp( dy );
  r = fma( r, fma( -dy, r, 1.0 ), r );
  r = fma( r, fma( -dy, r, 1.0 ), r );
  double qd = floor( dx * r );
  if( !(qd < 4294967296.0) ) return false;
  u32 q = (u32)qd;
  u32 neg = mw_submul<8>( x, x, y, q );
  mw_submul<5>( tx, tx, ty, q );
  if( __ballot( neg ) ) {                        /* estimate one too high */
    if( neg ) { mw_add<8>( x, x, y ); mw_add<5>( tx, tx, ty ); }
  }
  #pragma unroll 1
  for( ;; ) {                                    /* estimate too low */
    u32 tmp[8];
    bool ge = mw_sub<8>( tmp, x, y ) == 0u;
    if( !__ballot( ge ) ) break;
    if( ge ) {
      #pragma unroll
      for( int i=0; i<8; i++ ) x[i] = tmp[i];
      mw_sub<5>( tx, tx, ty );
    }
  }
  dx = mw_to_f64( x );
  return true;
}

DEV bool mw_below128( u32 const x[8] ) { return (x[4] | x[5] | x[6] | x[7]) == 0u; }

DEV u32 sc_halfsize( u32 k1[8], u32 & k1neg, u32 k2[8], u32 const k[8] ) {
  /* Euclid on (a, b) = (8L, k), remainders alternating between a and b so
     the step needs no swap; on exit (rp, tp) is the last remainder >= 2^128
     and (rc, tc) the first one below */
  u32 a[8] = { 0xe7ae9f68u,0xc09318d2u,0x17bce6b2u,0xa6f7cef5u,0u,0u,0u,0x80000000u };   /* 8L */
  u32 b[8], ta[5] = { 0u,0u,0u,0u,0u }, tb[5] = { 1u,0u,0u,0u,0u };
  #pragma unroll
  for( int i=0; i<8; i++ ) b[i] = k[i];
  double da = mw_to_f64( a ), db = mw_to_f64( b );
  bool fb = false, in_a = false;                 /* in_a: the newest remainder is a */
  #pragma unroll 1
  for( int it=0; ; it++ ) {
    if( mw_below128( b ) ) break;
    if( it >= 256 || !hs_step( a, ta, da, b, tb, db ) ) { fb = true; break; }
    if( mw_below128( a ) ) { in_a = true; break; }
    if( !hs_step( b, tb, db, a, ta, da ) ) { fb = true; break; }
  }
  u32 im = in_a ? ~0u : 0u;
  u32 rp[8], rc[8], tp[5], tc[5];
  #pragma unroll
  for( int i=0; i<8; i++ ) { rp[i] = mw_sel( im, b[i], a[i] ); rc[i] = mw_sel( im, a[i], b[i] ); }
  #pragma unroll
  for( int i=0; i<5; i++ ) { tp[i] = mw_sel( im, tb[i], ta[i] ); tc[i] = mw_sel( im, ta[i], tb[i] ); }
  double dp = in_a ? db : da, dc = in_a ? da : db;
  u32 bc = 999u, br[9], bt[5];
  #pragma unroll
  for( int i=0; i<9; i++ ) br[i] = 0u;
  #pragma unroll
  for( int i=0; i<5; i++ ) bt[i] = 0u;
  if( !fb ) {
    /* one more Euclid step (q = 0 when r_c == 0 or q >= 2^30: v2 then
       repeats v0).  |t_c| <= 8L/r_p <= 2^128, so q < 2^30 keeps |t_n| below
       2^159, inside the 5-word two's complement cofactors. */
    u32 rn[8], tn[5];
    double qd = floor( dp / dc );
    bool ok = (rc[0] | rc[1] | rc[2] | rc[3]) != 0u && qd < 1073741824.0;
    u32 q = ok ? (u32)qd : 0u;
    u32 neg = mw_submul<8>( rn, rp, rc, q );
    mw_submul<5>( tn, tp, tc, q );
    if( neg ) { mw_add<8>( rn, rn, rc ); mw_add<5>( tn, tn, tc ); }
    u32 v0[9], v1[9], v2[9];
    #pragma unroll
    for( int i=0; i<8; i++ ) { v0[i] = rp[i]; v1[i] = rc[i]; v2[i] = rn[i]; }
    v0[8] = v1[8] = v2[8] = 0u;
    hs_pick( br, bt, bc, v0, tp ); hs_pick( br, bt, bc, v1, tc ); hs_pick( br, bt, bc, v2, tn );
    hs_pick2( br, bt, bc, v0, tp, v1, tc );
    hs_pick2( br, bt, bc, v0, tp, v2, tn );
    hs_pick2( br, bt, bc, v1, tc, v2, tn );
  }
  if( bc > 250u ) {                           /* fallback: (k, 1) */
    #pragma unroll
    for( int i=0; i<8; i++ ) br[i] = k[i];
    br[8] = 0u;
    bt[0] = 1u; bt[1] = bt[2] = bt[3] = bt[4] = 0u;
    bc = mw_bitlen<8>( k );
  }
  u32 tneg = (u32)((int)bt[4] >> 31);         /* make k2 > 0: negate the pair */
  mw_cneg<9>( br, tneg ); mw_cneg<5>( bt, tneg );
  k1neg = (u32)((int)br[8] >> 31);
  mw_cneg<9>( br, k1neg );
  #pragma unroll
  for( int i=0; i<8; i++ ) { k1[i] = br[i]; k2[i] = i < 5 ? bt[i] : 0u; }
  return bc;
}

/**********************************************************************/
/* SHA-512 (fd_sha512.c:264-399 semantics), one message per lane.      */

/* 64-bit rotate / shift / 3-input logic on the 32-bit ALU, spelled out: the
   compiler lowers (x >> n) | (x << (64-n)) to two 64-bit shifts and two ORs,
   where a rotate is two v_alignbit_b32; and x ^ y ^ z to two XORs per half,
   where gfx950's v_bitop3_b32 takes any 3-input function in one */
DEV u32 lo32( u64 x ) { return (u32)x; }
DEV u32 hi32( u64 x ) { return (u32)(x >> 32); }
typedef u32 v2u32 __attribute__((ext_vector_type(2)));
DEV u64 mk64( u32 lo, u32 hi ) { v2u32 v = { lo, hi }; return __builtin_bit_cast( u64, v ); }
DEV u64 ror64( u64 x, int n ) {                 /* n a compile-time constant in (0, 64) */
  u32 lo = lo32( x ), hi = hi32( x );
  if( n >= 32 ) { u32 t = lo; lo = hi; hi = t; n -= 32; }
  if( n == 0 ) return mk64( lo, hi );
  return mk64( __builtin_amdgcn_alignbit( hi, lo, (u32)n ), __builtin_amdgcn_alignbit( lo, hi, (u32)n ) );
}
DEV u64 shr64( u64 x, int n ) {                 /* n a compile-time constant in (0, 32) */
  return mk64( __builtin_amdgcn_alignbit( hi32( x ), lo32( x ), (u32)n ), hi32( x ) >> n );
}
DEV u64 xor3_64( u64 a, u64 b, u64 c ) {
  return mk64( __builtin_amdgcn_bitop3_b32( lo32( a ), lo32( b ), lo32( c ), 0x96 ),
               __builtin_amdgcn_bitop3_b32( hi32( a ), hi32( b ), hi32( c ), 0x96 ) );
}
DEV u64 maj64( u64 a, u64 b, u64 c ) {          /* majority: (a&b) ^ (a&c) ^ (b&c) */
  return mk64( __builtin_amdgcn_bitop3_b32( lo32( a ), lo32( b ), lo32( c ), 0xe8 ),
               __builtin_amdgcn_bitop3_b32( hi32( a ), hi32( b ), hi32( c ), 0xe8 ) );
}

/* round constants in constant memory: the round index is wave-uniform, so
   each K[t] is a scalar load rather than 160 VGPRs of hoisted literals */
__constant__ u64 SHA512_K[80] = {
    0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL,0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL,0x12835b0145706fbeULL,0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL,0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,0x06ca6351e003826fULL,0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,0x53380d139d95b3dfULL,
    0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL,0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,
    0xca273eceea26619cULL,0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,0x113f9804bef90daeULL,0x1b710b35131c471bULL,
    0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL };

DEV void sha512_round( u64 & a, u64 & b, u64 & c, u64 & d, u64 & e, u64 & f, u64 & g, u64 & h, u64 w, u64 k ) {
  u64 S1 = xor3_64( ror64( e, 14 ), ror64( e, 18 ), ror64( e, 41 ) );
  u64 ch = (e & f) ^ (~e & g);
  u64 t1 = h + S1 + ch + k + w;
  u64 S0 = xor3_64( ror64( a, 28 ), ror64( a, 34 ), ror64( a, 39 ) );
  u64 mj = maj64( a, b, c );
  d += t1; h = t1 + S0 + mj;
}

/* 80 rounds as 5 x 16: inside a 16-round group the W ring index and the
   a..h rotation are static (no register moves); the groups stay rolled. */
DEV void sha512_block( u64 st[8], u64 W[16] ) {
  u64 a=st[0],b=st[1],c=st[2],d=st[3],e=st[4],f=st[5],g=st[6],h=st[7];
  #pragma unroll 1
  for( int t0=0; t0<80; t0+=16 ) {
    #pragma unroll
    for( int j=0; j<16; j++ ) {
      if( t0 ) {
        u64 w15 = W[(j+1)&15], w2 = W[(j+14)&15];
        u64 s0 = xor3_64( ror64( w15, 1 ), ror64( w15, 8 ), shr64( w15, 7 ) );
        u64 s1 = xor3_64( ror64( w2, 19 ), ror64( w2, 61 ), shr64( w2, 6 ) );
        W[j] += s0 + W[(j+9)&15] + s1;
      }
      u64 k = SHA512_K[t0+j];
      switch( j & 7 ) {
        case 0: sha512_round( a,b,c,d,e,f,g,h, W[j], k ); break;
        case 1: sha512_round( h,a,b,c,d,e,f,g, W[j], k ); break;
        case 2: sha512_round( g,h,a,b,c,d,e,f, W[j], k ); break;
        case 3: sha512_round( f,g,h,a,b,c,d,e, W[j], k ); break;
        case 4: sha512_round( e,f,g,h,a,b,c,d, W[j], k ); break;
        case 5: sha512_round( d,e,f,g,h,a,b,c, W[j], k ); break;
        case 6: sha512_round( c,d,e,f,g,h,a,b, W[j], k ); break;
        case 7: sha512_round( b,c,d,e,f,g,h,a, W[j], k ); break;
      }
    }
  }
  st[0]+=a; st[1]+=b; st[2]+=c; st[3]+=d; st[4]+=e; st[5]+=f; st[6]+=g; st[7]+=h;
}

DEV u32 bswap32( u32 x ) { return __builtin_bswap32( x ); }
DEV u64 be64_of_le_words( u32 lo, u32 hi ) {   /* bytes b0..b7 (lo = b0..b3 LE) -> big-endian word */
  return ((u64)bswap32( lo ) << 32) | (u64)bswap32( hi );
}

/* 8 message bytes starting at message offset m (m a multiple of 8, m < msz),
   as two little-endian words, zero-masked past msz and with the 0x80 pad
   byte at msz if it falls inside.  The pool must be readable up to
   msg + msz + 12 (the host pads every pool by 16 bytes). */
DEV void msg_load8( u32 & lo, u32 & hi, u8 const * msg, u32 msz, u32 m ) {
  u32 c = msz - m; if( c > 8u ) c = 8u;               /* valid bytes, >= 1 */
  uintptr_t a = (uintptr_t)(msg + m);
  u32 const * p = (u32 const *)(a & ~(uintptr_t)3);
  u32 sh = (u32)(a & 3u) * 8u;
  u32 w0 = p[0], w1 = p[1], w2 = p[2];
  lo = __builtin_amdgcn_alignbit( w1, w0, sh );
  hi = __builtin_amdgcn_alignbit( w2, w1, sh );
  if( c < 8u ) {
    u32 pad_lo = 0, pad_hi = 0;
    if( c < 4u ) { lo &= (1u << (8u*c)) - 1u; pad_lo = 0x80u << (8u*c); hi = 0; }
    else         { hi &= (c == 4u) ? 0u : ((1u << (8u*(c-4u))) - 1u); pad_hi = 0x80u << (8u*(c-4u)); }
    lo |= pad_lo; hi |= pad_hi;
  }
}

/* SHA-512( pre || M ) where pre is 32 or 64 bytes given as LE words and
   M = msg[0..msz); the 64-byte digest is returned reinterpreted as a 512-bit
   little-endian integer (16 LE limbs), the form fd_curve25519_scalar_reduce
   consumes. */
DEV void sha512_prefixed( u32 x[16], u32 const pre[16], u32 plen, u8 const * msg, u32 msz ) {
  u64 st[8] = { 0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,0xa54ff53a5f1d36f1ULL,
                0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL };
  u32 tot = plen + msz;
  u32 nb = (tot + 17u + 127u) >> 7;           /* ceil((plen + msz + 1 + 16) / 128) */
  u64 bitlen = (u64)tot << 3;
  #pragma unroll 1
  for( u32 b=0; b<nb; b++ ) {
    u64 W[16];
    bool last = (b + 1u == nb);
    #pragma unroll
    for( int t=0; t<16; t++ ) {
      u32 g = b*128u + 8u*(u32)t;             /* byte offset in pre||M||pad */
      u64 w;
      if( t < 8 && b == 0u && 8u*(u32)t < plen ) {   /* prefix words: static index (no scratch) */
        w = be64_of_le_words( pre[(2*t)&15], pre[(2*t+1)&15] );
      } else {
        u32 m = g - plen;
        u32 lo = 0, hi = 0;
        if( m < msz )       msg_load8( lo, hi, msg, msz, m );
        else if( m == msz ) lo = 0x80u;
        w = be64_of_le_words( lo, hi );
      }
      if( last && t == 14 ) w = 0;
      if( last && t == 15 ) w = bitlen;
      W[t] = w;
    }
    sha512_block( st, W );
  }
  #pragma unroll
  for( int j=0; j<8; j++ ) { x[2*j] = bswap32( (u32)(st[j] >> 32) ); x[2*j+1] = bswap32( (u32)st[j] ); }
}

/* ---- SHA-512(R||A||M) with LDS-staged, wave-cooperative message blocks ----

   The same hash as sha512_prefixed(pre = R||A, 64), for all 64 lanes of a
   wave at once (wave-uniform control flow: every lane of the wave calls it;
   a lane with nothing to hash passes msz = 0).  For each 128-byte block b
   (up to the wave's largest block count):
     1. each lane publishes its record's message window for the block -- the
        16-B-aligned base of message bytes [max(0,128b-64), min(msz,128b+64))
        and the number of 16-B chunks covering it (<= 9) -- in LDS;
     2. the wave loads all 64 windows cooperatively: piece p = lane + 64*i
        (i < 9) is chunk p%9 of record p/9, so lanes 9r..9r+8 read record r's
        window as contiguous 16-B loads (coalesced: one record's 144 B per 9
        lanes instead of 64 lanes each walking its own message with dword
        loads); chunks past a window are stored as zeros;
     3. each lane fixes its own window in LDS where the message ends (bytes
        past msz zero, the 0x80 pad byte at msz: fd_sha512.c:365-385);
     4. each lane reads its window back at its byte offset, forms the block's
        big-endian words and runs the compression in registers.
   Lanes whose (message, size) repeats the previous lane's (the signatures of
   one txn, a batch_single_msg group) skip steps 1-3 and read the first
   lane's window of their run: a shared message is loaded once per wave.
   buf: this wave's 64 x 36 words of LDS; meta: its 64 u64.  The pool must be
   readable up to the 16-B boundary after each message's last byte. */
DEV void wave_lds_sync( void ) {
  __builtin_amdgcn_fence( __ATOMIC_SEQ_CST, "wavefront" );
  __builtin_amdgcn_wave_barrier();
}

DEV u32 wave_max_u32( u32 v ) {                 /* max of v over all lanes of the wave (butterfly) */
  #pragma unroll
  for( int d=32; d>=1; d>>=1 ) v = max( v, (u32)__shfl_xor( (int)v, d ) );
  return v;
}

template<u32 PLEN>   /* prefix bytes: 64 (R||A, the verify path) or 0 (plain SHA-512, the test hook) */
DEV void sha512_prefixed_coop( u32 x[16], u8 const * pre_r, u8 const * pre_a, u8 const * msg, u32 msz, u32 * buf,
                               u64 * meta, u32 lane ) {
  /* pre_r / pre_a: the 32-byte R and A (16-B aligned) hashed ahead of M when
     PLEN = 64, read in block 0 only (not held in registers across blocks);
     unused (may be null) when PLEN = 0 */
  u64 st[8] = { 0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,0xa54ff53a5f1d36f1ULL,
                0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL };
  u32 nb = (PLEN + msz + 17u + 127u) >> 7;
  u32 nbmax = wave_max_u32( nb );
  u64 bitlen = (u64)(PLEN + msz) << 3;
  /* records sharing a message (a txn's signatures, expanded side by side;
     batch_single_msg groups) load it once: a lane whose (message, size)
     equals the previous lane's publishes an empty window and reads its
     run leader's copy */
  u64 mp = (u64)(uintptr_t)msg;
  u32 plo = __shfl_up( (u32)mp, 1u ), phi = __shfl_up( (u32)(mp >> 32), 1u ), pms = __shfl_up( msz, 1u );
  bool dup = lane > 0u && plo == (u32)mp && phi == (u32)(mp >> 32) && pms == msz;
  unsigned long long dmask = __ballot( dup );
  unsigned long long below = lane == 63u ? ~0ULL : ((2ULL << lane) - 1ULL);
  u32 leader = 63u - (u32)__clzll( ~dmask & below );
  u32 * own = buf + 36u*lane;
  u32 const * src = buf + 36u*leader;
  #pragma unroll 1
  for( u32 b=0; b<nbmax; b++ ) {
    u32 m0 = b ? 128u*b - PLEN : 0u;                      /* message offset of the window */
    u32 wlen = b ? 128u : 128u - PLEN;                    /* message bytes the block holds */
    bool act = b < nb;
    u32 hi = min( msz, m0 + wlen );
    u32 nbytes = (act && hi > m0) ? hi - m0 : 0u;
    uintptr_t addr = (uintptr_t)(msg + m0);
    u32 o = (u32)(addr & 15u);
    u32 nch = nbytes ? (o + nbytes + 15u) >> 4 : 0u;
    meta[lane] = dup ? 0ul : ((u64)(addr >> 4) & 0xfffffffffffULL) | ((u64)nch << 44);
    wave_lds_sync();
    #pragma unroll
    for( u32 i=0; i<9u; i++ ) {                            /* 576 pieces = 64 records x 9 chunks */
      u32 pc = lane + 64u*i, r = pc / 9u, c = pc - 9u*r;
      u64 mr = meta[r];
      uint4 v = make_uint4( 0u, 0u, 0u, 0u );
      if( c < (u32)(mr >> 44) ) v = ((uint4 const *)(uintptr_t)((mr & 0xfffffffffffULL) << 4))[c];
      ((uint4 *)(buf + 36u*r))[c] = v;
    }
    wave_lds_sync();
    u32 P = msz - m0;                                     /* pad position in the window (unsigned: */
    if( act && !dup && msz >= m0 && P < wlen ) {          /* messages up to 4 GB)                 */
      u32 e = o + P, q = e >> 4;
      uint4 * cp = (uint4 *)own + q;
      uint4 v = *cp;
      u32 w[4] = { v.x, v.y, v.z, v.w };
      #pragma unroll
      for( u32 k=0; k<4u; k++ ) {
        int rel = (int)(e - 16u*q) - (int)(4u*k);        /* bytes of word k before the pad */
        u32 keep = rel >= 4 ? ~0u : rel <= 0 ? 0u : (1u << (8*rel)) - 1u;
        u32 pad = (rel >= 0 && rel < 4) ? 0x80u << (8*rel) : 0u;
        w[k] = (w[k] & keep) | pad;
      }
      *cp = make_uint4( w[0], w[1], w[2], w[3] );
    }
    wave_lds_sync();
    u32 mw[33];
    u32 const * rp = src + (o >> 2);
    #pragma unroll
    for( int k=0; k<33; k++ ) mw[k] = rp[k];
    u32 sh = (o & 3u) * 8u;
    u32 mm[32];                                           /* message bytes [m0 + 4k, +4) */
    #pragma unroll
    for( int k=0; k<32; k++ ) mm[k] = __builtin_amdgcn_alignbit( mw[k+1], mw[k], sh );
    u64 W[16];
    if( PLEN && b == 0u ) {                               /* wave-uniform branch */
      u32 pre[16];
      uint4 const * qr = (uint4 const *)pre_r, * qa = (uint4 const *)pre_a;
      #pragma unroll
      for( int k=0; k<2; k++ ) {
        uint4 v = qr[k]; pre[4*k] = v.x; pre[4*k+1] = v.y; pre[4*k+2] = v.z; pre[4*k+3] = v.w;
        v = qa[k]; pre[8+4*k] = v.x; pre[8+4*k+1] = v.y; pre[8+4*k+2] = v.z; pre[8+4*k+3] = v.w;
      }
      #pragma unroll
      for( int t=0; t<8; t++ ) W[t] = be64_of_le_words( pre[2*t], pre[2*t+1] );
      #pragma unroll
      for( int t=8; t<16; t++ ) W[t] = be64_of_le_words( mm[2*t-16], mm[2*t-15] );
    } else {
      #pragma unroll
      for( int t=0; t<16; t++ ) W[t] = be64_of_le_words( mm[2*t], mm[2*t+1] );
    }
    if( b + 1u == nb ) { W[14] = 0ul; W[15] = bitlen; }
    if( act ) sha512_block( st, W );
    wave_lds_sync();                                      /* the next block reuses the buffers */
  }
  #pragma unroll
  for( int j=0; j<8; j++ ) { x[2*j] = bswap32( (u32)(st[j] >> 32) ); x[2*j+1] = bswap32( (u32)st[j] ); }
}

/* k = SHA512( R || A || M ) mod L as 8 LE limbs (fd_ed25519_user.c:205-207). */
DEV void hram_mod_l( u32 kout[8], u32 const R[8], u32 const A[8], u8 const * msg, u32 msz ) {
  u32 pre[16], x[16];
  #pragma unroll
  for( int i=0; i<8; i++ ) { pre[i] = R[i]; pre[8+i] = A[i]; }
  sha512_prefixed( x, pre, 64u, msg, msz );
  sc_reduce512( kout, x );
}
