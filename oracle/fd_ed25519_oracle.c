/* fd_ed25519_oracle.c -- TEST INFRASTRUCTURE ONLY (see fd_ed25519_oracle.h).

   A plain-C restatement of the reference's ed25519 verify path.  Every
   function names the reference code it restates.  Reference paths are
   relative to anoushk1234/firedancer src/.  Field elements use 5x51-bit
   limbs with 128-bit products (the same radix as the reference's portable
   backend, ballet/ed25519/ref/fd_f25519.h:14-23, but written here
   independently); nothing here is performance-critical. */

#include "fd_ed25519_oracle.h"
#include <string.h>
#include <stdlib.h>

static unsigned long strtoul_hex( char const * t ) { return strtoul( t, NULL, 16 ); }

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint8_t  u8;

/**********************************************************************/
/* SHA-512 (FIPS 180-4).  Restates ballet/sha512/fd_sha512.c:264-399
   (init / append / fini with 0x80 pad and 128-bit big-endian bit count). */

static const u64 SHA512_K[80] = {
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

static inline u64 ror64( u64 x, int n ) { return (x>>n) | (x<<(64-n)); }
static inline u64 load_be64( u8 const * p ) {
  u64 r = 0; for( int i=0; i<8; i++ ) r = (r<<8) | p[i]; return r;
}

static void sha512_block( u64 st[8], u8 const blk[128] ) {
  u64 w[80];
  for( int t=0; t<16; t++ ) w[t] = load_be64( blk + 8*t );
  for( int t=16; t<80; t++ ) {
    u64 s0 = ror64( w[t-15], 1 ) ^ ror64( w[t-15], 8 ) ^ (w[t-15]>>7);
    u64 s1 = ror64( w[t-2], 19 ) ^ ror64( w[t-2], 61 ) ^ (w[t-2]>>6);
    w[t] = w[t-16] + s0 + w[t-7] + s1;
  }
  u64 a=st[0],b=st[1],c=st[2],d=st[3],e=st[4],f=st[5],g=st[6],h=st[7];
  for( int t=0; t<80; t++ ) {
    u64 S1 = ror64(e,14) ^ ror64(e,18) ^ ror64(e,41);
    u64 ch = (e & f) ^ (~e & g);
    u64 t1 = h + S1 + ch + SHA512_K[t] + w[t];
    u64 S0 = ror64(a,28) ^ ror64(a,34) ^ ror64(a,39);
    u64 mj = (a & b) ^ (a & c) ^ (b & c);
    u64 t2 = S0 + mj;
    h=g; g=f; f=e; e=d+t1; d=c; c=b; b=a; a=t1+t2;
  }
  st[0]+=a; st[1]+=b; st[2]+=c; st[3]+=d; st[4]+=e; st[5]+=f; st[6]+=g; st[7]+=h;
}

typedef struct { u64 st[8]; u8 buf[128]; size_t used; u64 total; } sha512_ctx;

static void sha512_init( sha512_ctx * c ) {
  static const u64 iv[8] = {
    0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL };
  memcpy( c->st, iv, sizeof(iv) ); c->used = 0; c->total = 0;
}

static void sha512_append( sha512_ctx * c, u8 const * p, size_t sz ) {
  c->total += sz;
  while( sz ) {
    size_t take = 128 - c->used; if( take > sz ) take = sz;
    memcpy( c->buf + c->used, p, take ); c->used += take; p += take; sz -= take;
    if( c->used == 128 ) { sha512_block( c->st, c->buf ); c->used = 0; }
  }
}

static void sha512_fini( sha512_ctx * c, u8 out[64] ) {
  u64 bits = c->total << 3;
  c->buf[ c->used++ ] = 0x80;
  if( c->used > 112 ) { memset( c->buf + c->used, 0, 128 - c->used ); sha512_block( c->st, c->buf ); c->used = 0; }
  memset( c->buf + c->used, 0, 120 - c->used );
  for( int i=0; i<8; i++ ) c->buf[120+i] = (u8)(bits >> (56-8*i));   /* high 64 bits of the 128-bit count are 0 */
  sha512_block( c->st, c->buf );
  for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (u8)(c->st[i] >> (56-8*j));
}

void oracle_sha512( u8 out[64], u8 const * in, size_t sz ) {
  sha512_ctx c; sha512_init( &c ); sha512_append( &c, in, sz ); sha512_fini( &c, out );
}

/**********************************************************************/
/* Scalars mod L = 2^252 + 27742317777372353535851937790883648493.
   Restates ballet/ed25519/fd_curve25519_scalar.h:25-73 (validate: S <= L-1)
   and fd_curve25519_scalar.c:3-110 (reduce a 512-bit value mod L) /
   muladd.  Reduction here is plain binary long division: slow, obviously
   correct, independent of the reference's ref10 limb schedule. */

static const u8 L_BYTES[32] = {
  0xed,0xd3,0xf5,0x5c,0x1a,0x63,0x12,0x58,0xd6,0x9c,0xf7,0xa2,0xde,0xf9,0xde,0x14,
  0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0x10 };

static void le_to_words( u64 * w, u8 const * b, int nw ) {
  for( int i=0; i<nw; i++ ) { w[i]=0; for( int j=7; j>=0; j-- ) w[i] = (w[i]<<8) | b[8*i+j]; }
}
static void words_to_le( u8 * b, u64 const * w, int nw ) {
  for( int i=0; i<nw; i++ ) for( int j=0; j<8; j++ ) b[8*i+j] = (u8)(w[i] >> (8*j));
}

/* r (4 words, < L) <- x (nw words) mod L */
static void mod_l( u64 r[4], u64 const * x, int nw ) {
  u64 L[4]; le_to_words( L, L_BYTES, 4 );
  u64 acc[5] = {0,0,0,0,0};
  for( int bit = 64*nw-1; bit >= 0; bit-- ) {
    /* acc = 2*acc + bit (acc < L < 2^253 so 2*acc+1 < 2^254 fits) */
    for( int i=4; i>0; i-- ) acc[i] = (acc[i]<<1) | (acc[i-1]>>63);
    acc[0] = (acc[0]<<1) | ((x[bit>>6] >> (bit&63)) & 1);
    /* if acc >= L: acc -= L */
    int ge = 1;
    if( acc[4] ) ge = 1;
    else for( int i=3; i>=0; i-- ) { if( acc[i] != L[i] ) { ge = acc[i] > L[i]; break; } }
    if( ge ) {
      u64 bw = 0;
      for( int i=0; i<4; i++ ) { u128 d = (u128)acc[i] - L[i] - bw; acc[i] = (u64)d; bw = (u64)(d>>64) & 1; }
      acc[4] -= bw;
    }
  }
  for( int i=0; i<4; i++ ) r[i] = acc[i];
}

void oracle_scalar_reduce( u8 out[32], u8 const in[64] ) {
  u64 x[8], r[4]; le_to_words( x, in, 8 ); mod_l( r, x, 8 ); words_to_le( out, r, 4 );
}

/* fd_curve25519_scalar.h:57-73: S valid iff S <= L-1 (lexicographic on LE words) */
static int scalar_is_canonical( u8 const s[32] ) {
  for( int i=31; i>=0; i-- ) {
    u8 lm1 = (i==0) ? (u8)(L_BYTES[0]-1) : L_BYTES[i];
    if( s[i] != lm1 ) return s[i] < lm1;
  }
  return 1; /* s == L-1 */
}

/* out = (a*b + c) mod L  (fd_curve25519_scalar.h muladd, used by sign) */
static void scalar_muladd( u8 out[32], u8 const a[32], u8 const b[32], u8 const c[32] ) {
  u64 A[4], B[4], C[4], P[9] = {0};
  le_to_words( A, a, 4 ); le_to_words( B, b, 4 ); le_to_words( C, c, 4 );
  for( int i=0; i<4; i++ ) {
    u64 carry = 0;
    for( int j=0; j<4; j++ ) {
      u128 t = (u128)A[i]*B[j] + P[i+j] + carry; P[i+j] = (u64)t; carry = (u64)(t>>64);
    }
    P[i+4] += carry;
  }
  u64 carry = 0;
  for( int i=0; i<9; i++ ) { u128 t = (u128)P[i] + (i<4 ? C[i] : 0) + carry; P[i] = (u64)t; carry = (u64)(t>>64); }
  u64 r[4]; mod_l( r, P, 9 ); words_to_le( out, r, 4 );
}

/**********************************************************************/
/* GF(2^255-19), 5x51-bit limbs.  Restates ballet/ed25519/fd_f25519.h API
   (frombytes masks bit 255 and accepts non-canonical y; tobytes is
   canonical; is_zero / eq compare canonical encodings). */

typedef struct { u64 v[5]; } fe;
#define M51 ((1ULL<<51)-1)

static void fe_carry( fe * h ) {
  u64 c;
  for( int pass=0; pass<2; pass++ ) {
    c = h->v[0]>>51; h->v[0] &= M51; h->v[1] += c;
    c = h->v[1]>>51; h->v[1] &= M51; h->v[2] += c;
    c = h->v[2]>>51; h->v[2] &= M51; h->v[3] += c;
    c = h->v[3]>>51; h->v[3] &= M51; h->v[4] += c;
    c = h->v[4]>>51; h->v[4] &= M51; h->v[0] += 19*c;
  }
}
static void fe_frombytes( fe * h, u8 const s[32] ) {
  u64 w[4]; le_to_words( w, s, 4 );
  w[3] &= 0x7fffffffffffffffULL;                       /* mask bit 255 (x sign) */
  h->v[0] =  w[0]                & M51;
  h->v[1] = (w[0]>>51 | w[1]<<13) & M51;
  h->v[2] = (w[1]>>38 | w[2]<<26) & M51;
  h->v[3] = (w[2]>>25 | w[3]<<39) & M51;
  h->v[4] = (w[3]>>12)            & M51;
}
static void fe_tobytes( u8 s[32], fe const * a ) {
  fe t = *a; fe_carry( &t );
  /* t < 2^255 + small; subtract p if t >= p */
  u64 q = (t.v[0] + 19) >> 51; q = (t.v[1]+q)>>51; q = (t.v[2]+q)>>51; q = (t.v[3]+q)>>51; q = (t.v[4]+q)>>51;
  t.v[0] += 19*q;
  u64 c;
  c = t.v[0]>>51; t.v[0] &= M51; t.v[1] += c;
  c = t.v[1]>>51; t.v[1] &= M51; t.v[2] += c;
  c = t.v[2]>>51; t.v[2] &= M51; t.v[3] += c;
  c = t.v[3]>>51; t.v[3] &= M51; t.v[4] += c;
  t.v[4] &= M51;
  u64 w[4];
  w[0] = t.v[0]       | t.v[1]<<51;
  w[1] = t.v[1]>>13   | t.v[2]<<38;
  w[2] = t.v[2]>>26   | t.v[3]<<25;
  w[3] = t.v[3]>>39   | t.v[4]<<12;
  words_to_le( s, w, 4 );
}
static void fe_set( fe * h, u64 x ) { memset( h, 0, sizeof(*h) ); h->v[0] = x; }
static void fe_add( fe * h, fe const * a, fe const * b ) { for( int i=0;i<5;i++ ) h->v[i] = a->v[i]+b->v[i]; fe_carry( h ); }
static void fe_sub( fe * h, fe const * a, fe const * b ) {
  /* a + 4p - b, 4p limbs: 4*(2^51-19), 4*(2^51-1) */
  h->v[0] = a->v[0] + 0x1fffffffffffb4ULL - b->v[0];
  for( int i=1;i<5;i++ ) h->v[i] = a->v[i] + 0x1ffffffffffffcULL - b->v[i];
  fe_carry( h );
}
static void fe_neg( fe * h, fe const * a ) { fe z; fe_set( &z, 0 ); fe_sub( h, &z, a ); }
static void fe_mul( fe * h, fe const * a, fe const * b ) {
  u64 const * f = a->v; u64 const * g = b->v;
  u128 r0 = (u128)f[0]*g[0] + (u128)19*((u128)f[1]*g[4] + (u128)f[2]*g[3] + (u128)f[3]*g[2] + (u128)f[4]*g[1]);
  u128 r1 = (u128)f[0]*g[1] + (u128)f[1]*g[0] + (u128)19*((u128)f[2]*g[4] + (u128)f[3]*g[3] + (u128)f[4]*g[2]);
  u128 r2 = (u128)f[0]*g[2] + (u128)f[1]*g[1] + (u128)f[2]*g[0] + (u128)19*((u128)f[3]*g[4] + (u128)f[4]*g[3]);
  u128 r3 = (u128)f[0]*g[3] + (u128)f[1]*g[2] + (u128)f[2]*g[1] + (u128)f[3]*g[0] + (u128)19*((u128)f[4]*g[4]);
  u128 r4 = (u128)f[0]*g[4] + (u128)f[1]*g[3] + (u128)f[2]*g[2] + (u128)f[3]*g[1] + (u128)f[4]*g[0];
  u64 c;
  c = (u64)(r0>>51); r1 += c; h->v[0] = (u64)r0 & M51;
  c = (u64)(r1>>51); r2 += c; h->v[1] = (u64)r1 & M51;
  c = (u64)(r2>>51); r3 += c; h->v[2] = (u64)r2 & M51;
  c = (u64)(r3>>51); r4 += c; h->v[3] = (u64)r3 & M51;
  c = (u64)(r4>>51);          h->v[4] = (u64)r4 & M51;
  h->v[0] += 19*c; fe_carry( h );
}
static void fe_sq( fe * h, fe const * a ) { fe_mul( h, a, a ); }
static void fe_sqn( fe * h, fe const * a, int n ) { fe_sq( h, a ); for( int i=1;i<n;i++ ) fe_sq( h, h ); }
static int  fe_is_zero( fe const * a ) { u8 s[32]; fe_tobytes( s, a ); u8 o=0; for(int i=0;i<32;i++) o|=s[i]; return o==0; }
static int  fe_eq( fe const * a, fe const * b ) { u8 x[32], y[32]; fe_tobytes( x, a ); fe_tobytes( y, b ); return !memcmp( x, y, 32 ); }
static int  fe_sgn( fe const * a ) { u8 s[32]; fe_tobytes( s, a ); return s[0] & 1; }

/* z^(2^252-3): ballet/ed25519/fd_f25519.c:25-74 (same exponent, own chain) */
static void fe_pow22523( fe * out, fe const * z ) {
  fe z2, z9, z11, z_5_0, z_10_0, z_20_0, z_40_0, z_50_0, z_100_0, z_200_0, z_250_0, t;
  fe_sq( &z2, z );                                   /* 2 */
  fe_sqn( &t, &z2, 2 ); fe_mul( &z9, &t, z );        /* 9 */
  fe_mul( &z11, &z9, &z2 );                          /* 11 */
  fe_sq( &t, &z11 ); fe_mul( &z_5_0, &t, &z9 );      /* 2^5-1 */
  fe_sqn( &t, &z_5_0, 5 );    fe_mul( &z_10_0, &t, &z_5_0 );
  fe_sqn( &t, &z_10_0, 10 );  fe_mul( &z_20_0, &t, &z_10_0 );
  fe_sqn( &t, &z_20_0, 20 );  fe_mul( &z_40_0, &t, &z_20_0 );
  fe_sqn( &t, &z_40_0, 10 );  fe_mul( &z_50_0, &t, &z_10_0 );
  fe_sqn( &t, &z_50_0, 50 );  fe_mul( &z_100_0, &t, &z_50_0 );
  fe_sqn( &t, &z_100_0, 100 ); fe_mul( &z_200_0, &t, &z_100_0 );
  fe_sqn( &t, &z_200_0, 50 ); fe_mul( &z_250_0, &t, &z_50_0 );
  fe_sqn( &t, &z_250_0, 2 );  fe_mul( out, &t, z );  /* 2^252 - 4 + 1 = 2^252-3 */
}
/* z^(p-2): ballet/ed25519/fd_f25519.c:77-119 */
static void fe_invert( fe * out, fe const * z ) {
  /* p-2 = 2^255-21 = (2^252-3)*8 + 3  ->  z^(p-2) = (z^(2^252-3))^8 * z^3 */
  fe a, z3;
  fe_pow22523( &a, z ); fe_sqn( &a, &a, 3 );
  fe_sq( &z3, z ); fe_mul( &z3, &z3, z );
  fe_mul( out, &a, &z3 );
}

static fe FE_D, FE_D2, FE_SQRTM1, FE_ONE, FE_Y0, FE_Y1;

static void fe_from_hex_le( fe * h, char const * hex ) {
  u8 b[32];
  for( int i=0;i<32;i++ ) { unsigned v; char t[3] = { hex[2*i], hex[2*i+1], 0 }; v = (unsigned)strtoul_hex( t ); b[i]=(u8)v; }
  fe_frombytes( h, b );
}

/**********************************************************************/
/* Group: twisted Edwards a=-1, extended coordinates (X:Y:Z:T), complete
   HWCD'08 formulas as in ballet/ed25519/ref/fd_curve25519.c:25-92
   (add) and ref/fd_curve25519.h:190-211 (dbl). */

typedef struct { fe X, Y, Z, T; } ge;

static void ge_zero( ge * r ) { fe_set( &r->X, 0 ); fe_set( &r->Y, 1 ); fe_set( &r->Z, 1 ); fe_set( &r->T, 0 ); }
static void ge_add( ge * r, ge const * p, ge const * q ) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub( &a, &p->Y, &p->X ); fe_sub( &t, &q->Y, &q->X ); fe_mul( &a, &a, &t );
  fe_add( &b, &p->Y, &p->X ); fe_add( &t, &q->Y, &q->X ); fe_mul( &b, &b, &t );
  fe_mul( &c, &p->T, &q->T ); fe_mul( &c, &c, &FE_D2 );
  fe_mul( &d, &p->Z, &q->Z ); fe_add( &d, &d, &d );
  fe_sub( &e, &b, &a ); fe_sub( &f, &d, &c ); fe_add( &g, &d, &c ); fe_add( &h, &b, &a );
  fe_mul( &r->X, &e, &f ); fe_mul( &r->Y, &g, &h ); fe_mul( &r->T, &e, &h ); fe_mul( &r->Z, &f, &g );
}
static void ge_neg( ge * r, ge const * p ) { fe_neg( &r->X, &p->X ); r->Y = p->Y; r->Z = p->Z; fe_neg( &r->T, &p->T ); }
static void ge_sub( ge * r, ge const * p, ge const * q ) { ge n; ge_neg( &n, q ); ge_add( r, p, &n ); }
static void ge_dbl( ge * r, ge const * p ) {
  fe a, b, c, h, e, g, f, t;
  fe_sq( &a, &p->X ); fe_sq( &b, &p->Y ); fe_sq( &c, &p->Z ); fe_add( &c, &c, &c );
  fe_add( &h, &a, &b ); fe_add( &t, &p->X, &p->Y ); fe_sq( &t, &t ); fe_sub( &e, &h, &t );
  fe_sub( &g, &a, &b ); fe_add( &f, &c, &g );
  fe_mul( &r->X, &e, &f ); fe_mul( &r->Y, &g, &h ); fe_mul( &r->T, &e, &h ); fe_mul( &r->Z, &f, &g );
}
/* projective equality: ref/fd_curve25519.h:132-139 / avx512 fd_r43x6_ge.h:52-82 */
static int ge_eq( ge const * p, ge const * q ) {
  fe a, b;
  fe_mul( &a, &p->X, &q->Z ); fe_mul( &b, &q->X, &p->Z ); if( !fe_eq( &a, &b ) ) return 0;
  fe_mul( &a, &p->Y, &q->Z ); fe_mul( &b, &q->Y, &p->Z ); return fe_eq( &a, &b );
}
static void ge_tobytes( u8 s[32], ge const * p ) {   /* ballet/ed25519/fd_curve25519.c:63-74 */
  fe zi, x, y; fe_invert( &zi, &p->Z ); fe_mul( &x, &p->X, &zi ); fe_mul( &y, &p->Y, &zi );
  fe_tobytes( s, &y ); s[31] ^= (u8)(fe_sgn( &x ) << 7);
}

/* Point decompression, ballet/ed25519/fd_curve25519.c:34-61 with
   fd_f25519.c:122-158 (sqrt_ratio).  Returns 0 ok, 1 not on curve (u/v is
   not a square), 2 x==0 with sign bit set: the AVX-512 backend rejects
   case 2 in decode (avx512/fd_r43x6_ge.c:231-232), the ref backend keeps
   the point and rejects it later as small order. */
static int ge_frombytes( ge * r, u8 const s[32] ) {
  fe y, u, v, v3, v7, x, chk, t;
  fe_frombytes( &y, s );
  int x_sign = s[31] >> 7;
  fe_sq( &u, &y ); fe_mul( &v, &u, &FE_D );
  fe_sub( &u, &u, &FE_ONE ); fe_add( &v, &v, &FE_ONE );         /* u = y^2-1, v = dy^2+1 */
  fe_sq( &v3, &v ); fe_mul( &v3, &v3, &v );                      /* v^3 */
  fe_sq( &v7, &v3 ); fe_mul( &v7, &v7, &v );                     /* v^7 */
  fe_mul( &t, &u, &v7 ); fe_pow22523( &t, &t );                  /* (uv^7)^((p-5)/8) */
  fe_mul( &x, &u, &v3 ); fe_mul( &x, &x, &t );                   /* uv^3 (uv^7)^((p-5)/8) */
  fe_sq( &chk, &x ); fe_mul( &chk, &chk, &v );                   /* v x^2 */
  fe nu; fe_neg( &nu, &u );
  if( fe_eq( &chk, &u ) ) { /* root */ }
  else if( fe_eq( &chk, &nu ) ) fe_mul( &x, &x, &FE_SQRTM1 );
  else return 1;
  if( fe_is_zero( &x ) && x_sign ) {
    /* keep x = 0 (ref semantics); caller decides */
    fe_set( &r->X, 0 ); r->Y = y; fe_set( &r->Z, 1 ); fe_set( &r->T, 0 );
    return 2;
  }
  if( fe_sgn( &x ) != x_sign ) fe_neg( &x, &x );
  r->X = x; r->Y = y; fe_set( &r->Z, 1 ); fe_mul( &r->T, &x, &y );
  return 0;
}

/* fd_curve25519.h:88-118: affine small-order test (Z==1) */
static int ge_affine_is_small_order( ge const * p ) {
  return fe_is_zero( &p->X ) | fe_is_zero( &p->Y ) | fe_eq( &p->Y, &FE_Y0 ) | fe_eq( &p->Y, &FE_Y1 );
}

/**********************************************************************/
/* Scalar multiplication.  fd_curve25519_scalar.c:277-360 (wNAF recoding)
   and fd_curve25519.c:121-165 (double-base Straus with a w=4 table of
   odd multiples of A and a w=8 table of odd multiples of B). */

static void scalar_wnaf( short t[256], u8 const s[32], int bits ) {
  int max = (1<<bits) - 1;
  for( int i=0;i<256;i++ ) t[i] = (i<255) ? (short)((s[i>>3] >> (i&7)) & 1) : 0;
  int i = 0;
  while( i<256 && !t[i] ) i++;
  while( i<256 ) {
    int ti = 1, j;
    for( j=i+1; j<256; j++ ) {
      if( !t[j] ) continue;
      int delta = 1 << ((j-i) < 14 ? (j-i) : 14);
      if( delta > 2*max ) break;
      if( ti + delta <= max ) { ti += delta; t[j] = 0; continue; }
      if( ti - delta >= -max ) {
        ti -= delta; t[j] = 0;
        for(;;) { j++; if( !t[j] ) { t[j] = 1; break; } t[j] = 0; }
        break;
      }
      break;
    }
    t[i] = (short)ti;
    i = j;
  }
}

static ge GE_B;
static ge B_ODD[128];   /* B, 3B, 5B, ..., 255B */

/* r = [n1]a + [n2]B */
static void ge_double_scalar_mul_base( ge * r, u8 const n1[32], ge const * a, u8 const n2[32] ) {
  short s1[256], s2[256];
  scalar_wnaf( s1, n1, 4 ); scalar_wnaf( s2, n2, 8 );
  ge ai[8], a2; ai[0] = *a; ge_dbl( &a2, a );
  for( int i=1;i<8;i++ ) ge_add( &ai[i], &ai[i-1], &a2 );
  ge_zero( r );
  int i; for( i=255; i>=0; i-- ) if( s1[i] || s2[i] ) break;
  for( ; i>=0; i-- ) {
    ge_dbl( r, r );
    if( s1[i] > 0 ) ge_add( r, r, &ai[  s1[i] /2] ); else if( s1[i] < 0 ) ge_sub( r, r, &ai[(-s1[i])/2] );
    if( s2[i] > 0 ) ge_add( r, r, &B_ODD[  s2[i] /2] ); else if( s2[i] < 0 ) ge_sub( r, r, &B_ODD[(-s2[i])/2] );
  }
}

/* r = [n]B for a 256-bit n (keygen / sign; no secrecy requirement here) */
static void ge_scalar_mul_base( ge * r, u8 const n[32] ) {
  ge_zero( r );
  for( int i=255; i>=0; i-- ) { ge_dbl( r, r ); if( (n[i>>3]>>(i&7)) & 1 ) ge_add( r, r, &GE_B ); }
}

/**********************************************************************/


static int g_init = 0;
static void oracle_init( void ) {
  if( __atomic_load_n( &g_init, __ATOMIC_ACQUIRE ) ) return;
  #pragma omp critical(oracle_init)
  {
    if( !g_init ) {
      /* d = -121665/121666, sqrt(-1), order-8 y's: fd_f25519_table_ref.c:38-47,
         fd_curve25519_table_ref.c:18-27 (encodings as LE hex). */
      fe_from_hex_le( &FE_D,      "a3785913ca4deb75abd841414d0a700098e879777940c78c73fe6f2bee6c0352" );
      fe_from_hex_le( &FE_SQRTM1, "b0a00e4a271beec478e42fad0618432fa7d7fb3d99004d2b0bdfc14f8024832b" );
      fe_from_hex_le( &FE_Y0,     "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05" );
      fe_from_hex_le( &FE_Y1,     "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a" );
      fe_add( &FE_D2, &FE_D, &FE_D );
      fe_set( &FE_ONE, 1 );
      u8 bb[32]; for( int i=0;i<32;i++ ) bb[i] = 0x66; bb[0] = 0x58;   /* base point encoding */
      ge_frombytes( &GE_B, bb );
      ge b2; ge_dbl( &b2, &GE_B ); B_ODD[0] = GE_B;
      for( int i=1;i<128;i++ ) ge_add( &B_ODD[i], &B_ODD[i-1], &b2 );
      __atomic_store_n( &g_init, 1, __ATOMIC_RELEASE );
    }
  }
}

/**********************************************************************/

void oracle_hram( u8 k[32], u8 const R[32], u8 const A[32], u8 const * msg, size_t msg_sz ) {
  sha512_ctx c; u8 h[64];
  sha512_init( &c ); sha512_append( &c, R, 32 ); sha512_append( &c, A, 32 );
  if( msg_sz ) sha512_append( &c, msg, msg_sz );
  sha512_fini( &c, h ); oracle_scalar_reduce( k, h );
}

int oracle_point_decode( u8 xy[64], u8 const buf[32] ) {
  oracle_init();
  ge p; int rc = ge_frombytes( &p, buf );
  if( rc != 1 ) { fe_tobytes( xy, &p.X ); fe_tobytes( xy+32, &p.Y ); }
  return rc;
}

int oracle_point_is_small_order( u8 const buf[32] ) {
  oracle_init();
  ge p; if( ge_frombytes( &p, buf ) == 1 ) return -1;
  return ge_affine_is_small_order( &p );
}

/* Pass-1 checks of fd_ed25519_user.c:159-199 (and :270-287 in the batch).
   Returns 0 when every check passed and fills A, R; else the error code. */
static int verify_prechecks( ge * A, ge * R, u8 const sig[64], u8 const pub[32], int errmode ) {
  if( !scalar_is_canonical( sig+32 ) ) return ORACLE_ERR_SIG;            /* :159-161 */
  int ra = ge_frombytes( A, pub );                                          /* :165 (A first) */
  int rr = ge_frombytes( R, sig );
  if( errmode == ORACLE_ERRMODE_AVX512 ) {
    /* decode2 returns -1/-2; user.c:192 maps anything but 1 to ERR_SIG */
    if( ra || rr ) return ORACLE_ERR_SIG;
  } else {
    if( ra == 1 ) return ORACLE_ERR_PUBKEY;                                 /* res==1 */
    if( rr == 1 ) return ORACLE_ERR_SIG;                                    /* res==2 */
  }
  if( ge_affine_is_small_order( A ) ) return ORACLE_ERR_PUBKEY;            /* :194-196 */
  if( ge_affine_is_small_order( R ) ) return ORACLE_ERR_SIG;               /* :197-199 */
  return ORACLE_SUCCESS;
}

/* fd_ed25519_user.c:135-230 */
int oracle_verify( u8 const * msg, size_t msg_sz, u8 const sig[64], u8 const pub[32], int errmode ) {
  oracle_init();
  ge A, R;
  int rc = verify_prechecks( &A, &R, sig, pub, errmode );
  if( rc ) return rc;
  u8 k[32]; oracle_hram( k, sig, pub, msg, msg_sz );                       /* :205-207 */
  ge nA, Rc; ge_neg( &nA, &A );                                             /* :216 */
  ge_double_scalar_mul_base( &Rc, k, &nA, sig+32 );                         /* :217 */
  return ge_eq( &Rc, &R ) ? ORACLE_SUCCESS : ORACLE_ERR_MSG;               /* :226-229 */
}

/* fd_ed25519_user.c:232-310 */
int oracle_verify_batch_single_msg( u8 const * msg, size_t msg_sz, u8 const * sigs, u8 const * pubs,
                                    unsigned batch_sz, int errmode ) {
  oracle_init();
  if( batch_sz==0 || batch_sz>16 ) return ORACLE_ERR_SIG;                   /* :238-241 */
  ge A[16], R[16]; u8 k[16][32];
  for( unsigned j=0; j<batch_sz; j++ ) {                                   /* pass 1, :264-294 */
    int rc = verify_prechecks( &A[j], &R[j], sigs+64*j, pubs+32*j, errmode );
    if( rc ) return rc;
    oracle_hram( k[j], sigs+64*j, pubs+32*j, msg, msg_sz );
  }
  for( unsigned j=0; j<batch_sz; j++ ) {                                   /* pass 2, :297-306 */
    ge nA, Rc; ge_neg( &nA, &A[j] );
    ge_double_scalar_mul_base( &Rc, k[j], &nA, sigs+64*j+32 );
    if( !ge_eq( &Rc, &R[j] ) ) return ORACLE_ERR_MSG;
  }
  return ORACLE_SUCCESS;
}

void oracle_verify_many( size_t n, u8 const * sigs, u8 const * pubs, u8 const * msg_pool,
                         uint32_t const * msg_off, uint32_t const * msg_sz, int8_t * codes, int errmode ) {
  oracle_init();
  #pragma omp parallel for schedule(dynamic, 64)
  for( long i=0; i<(long)n; i++ )
    codes[i] = (int8_t)oracle_verify( msg_pool + msg_off[i], msg_sz[i], sigs + 64*i, pubs + 32*i, errmode );
}

/* fd_ed25519_user.c:4-57 */
void oracle_public_from_private( u8 pub[32], u8 const prv[32] ) {
  oracle_init();
  u8 h[64]; oracle_sha512( h, prv, 32 );
  h[0] &= 0xf8; h[31] &= 0x7f; h[31] |= 0x40;
  ge A; ge_scalar_mul_base( &A, h ); ge_tobytes( pub, &A );
}

/* fd_ed25519_user.c:59-133 */
void oracle_sign( u8 sig[64], u8 const * msg, size_t msg_sz, u8 const pub[32], u8 const prv[32] ) {
  oracle_init();
  u8 h[64]; oracle_sha512( h, prv, 32 );
  h[0] &= 0xf8; h[31] &= 0x7f; h[31] |= 0x40;
  sha512_ctx c; u8 rh[64], r[32];
  sha512_init( &c ); sha512_append( &c, h+32, 32 ); if( msg_sz ) sha512_append( &c, msg, msg_sz ); sha512_fini( &c, rh );
  oracle_scalar_reduce( r, rh );
  ge Rp; ge_scalar_mul_base( &Rp, r ); ge_tobytes( sig, &Rp );
  u8 k[32]; oracle_hram( k, sig, pub, msg, msg_sz );
  scalar_muladd( sig+32, k, h, r );
}

void oracle_sign_many( size_t n, u8 const * prvs, u8 * pubs, u8 * sigs, u8 const * msg_pool,
                       uint32_t const * msg_off, uint32_t const * msg_sz ) {
  oracle_init();
  #pragma omp parallel for schedule(dynamic, 16)
  for( long i=0; i<(long)n; i++ ) {
    oracle_public_from_private( pubs + 32*i, prvs + 32*i );
    oracle_sign( sigs + 64*i, msg_pool + msg_off[i], msg_sz[i], pubs + 32*i, prvs + 32*i );
  }
}
