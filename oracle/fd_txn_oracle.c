/* fd_txn_oracle.c -- TEST INFRASTRUCTURE ONLY.  See fd_txn_oracle.h for the
   reference functions restated here and how the restatement is pinned. */

#include "fd_txn_oracle.h"
#include "fd_ed25519_oracle.h"

#include <string.h>

typedef uint8_t  u8;
typedef uint16_t u16;
typedef uint64_t u64;

/* ---- fd_hash: src/util/fd_hash.c:6-72 ------------------------------------ */

#define H_P1 11400714785074694791ULL
#define H_P2 14029467366897019727ULL
#define H_P3  1609587929392839161ULL
#define H_P4  9650029242287828579ULL
#define H_P5  2870177450012600261ULL

static inline u64 rotl64( u64 x, int r ) { return (x<<r) | (x>>(64-r)); }
static inline u64 ld64( u8 const * p ) { u64 v; memcpy( &v, p, 8 ); return v; }
static inline u64 ld32( u8 const * p ) { uint32_t v; memcpy( &v, p, 4 ); return v; }
static inline u64 lane_round( u64 acc, u64 w ) { acc += w*H_P2; acc = rotl64( acc, 31 ); return acc*H_P1; }

uint64_t oracle_fd_hash( uint64_t seed, void const * buf, size_t sz ) {
  u8 const * p = (u8 const *)buf, * end = p + sz;
  u64 h;
  if( sz < 32 ) h = seed + H_P5;                                          /* :21 */
  else {                                                                   /* :22-43 */
    u64 v[4] = { seed + H_P1 + H_P2, seed + H_P2, seed, seed - H_P1 };
    while( (size_t)(end - p) >= 32 ) {
      for( int k=0;k<4;k++ ) v[k] = lane_round( v[k], ld64( p + 8*k ) );
      p += 32;
    }
    h = rotl64( v[0], 1 ) + rotl64( v[1], 7 ) + rotl64( v[2], 12 ) + rotl64( v[3], 18 );
    for( int k=0;k<4;k++ ) { h ^= lane_round( 0, v[k] ); h = h*H_P1 + H_P4; }
  }
  h += (u64)sz;                                                            /* :46 */
  for( ; end - p >= 8; p += 8 ) { h ^= lane_round( 0, ld64( p ) ); h = rotl64( h, 27 )*H_P1 + H_P4; }   /* :48-52 */
  if( end - p >= 4 ) { h ^= ld32( p )*H_P1; h = rotl64( h, 23 )*H_P2 + H_P3; p += 4; }                 /* :54-58 */
  for( ; p < end; p++ ) { h ^= (u64)p[0]*H_P5; h = rotl64( h, 11 )*H_P1; }                              /* :60-64 */
  h ^= h >> 33; h *= H_P2; h ^= h >> 29; h *= H_P3; h ^= h >> 32;         /* :67-71 */
  return h;
}

/* ---- fd_txn_parse_core: src/ballet/txn/fd_txn_parse.c:7-254 --------------
   Output layout is fd_txn_t (fd_txn.h:186-305): 20-byte header, then
   instr_cnt 10-byte fd_txn_instr_t, then lut_cnt 8-byte fd_txn_acct_addr_lut_t.
   Every check below is one CHECK / CHECK_LEFT / READ_CHECKED_COMPACT_U16 of
   the reference, in the same order. */

typedef struct { u8 const * b; size_t sz, i; } rd_t;

static inline int have( rd_t const * r, size_t n ) { return n <= r->sz - r->i; }

/* fd_compact_u16.h:38-92: 1-3 bytes, minimal encoding, value < 2^16 */
static inline int cu16( rd_t * r, u16 * v ) {
  u8 const * q = r->b + r->i; size_t left = r->sz - r->i;
  if( left>=1 && !(q[0]&0x80) ) { *v = q[0]; r->i += 1; return 1; }
  if( left>=2 && !(q[1]&0x80) ) {
    if( !q[1] ) return 0;
    *v = (u16)((q[0]&0x7f) | (q[1]<<7)); r->i += 2; return 1;
  }
  if( left>=3 && !(q[2]&0xfc) ) {
    if( !q[2] ) return 0;
    *v = (u16)((q[0]&0x7f) | ((q[1]&0x7f)<<7) | (q[2]<<14)); r->i += 3; return 1;
  }
  return 0;
}

static inline void st16( u8 * o, size_t off, unsigned v ) { if( o ) { o[off] = (u8)v; o[off+1] = (u8)(v>>8); } }
static inline void st8 ( u8 * o, size_t off, unsigned v ) { if( o ) o[off] = (u8)v; }

size_t oracle_txn_parse( uint8_t const * payload, size_t payload_sz, uint8_t * out ) {
  rd_t r = { payload, payload_sz, 0 };
  if( payload_sz > ORACLE_TXN_MTU ) return 0;                              /* :82  */
  if( !have( &r, 1 ) ) return 0;
  unsigned sig_cnt = payload[r.i++];                                       /* :89  */
  if( sig_cnt<1 || sig_cnt>127 ) return 0;                                 /* :91  */
  if( !have( &r, 64*(size_t)sig_cnt ) ) return 0;
  size_t sig_off = r.i; r.i += 64*(size_t)sig_cnt;
  size_t msg_off = r.i;
  if( !have( &r, 1 ) ) return 0;
  unsigned b0 = payload[r.i++];                                            /* :95  */
  unsigned version;
  if( b0 & 0x80 ) {                                                        /* :98-104 */
    version = b0 & 0x7f;
    if( version != 0 ) return 0;
    if( !have( &r, 1 ) ) return 0;
    if( payload[r.i] != sig_cnt ) return 0;
    r.i++;
  } else {
    version = 0xff;                                                        /* FD_TXN_VLEGACY */
    if( b0 != sig_cnt ) return 0;
  }
  if( !have( &r, 1 ) ) return 0;
  unsigned ro_signed = payload[r.i++];
  if( ro_signed >= sig_cnt ) return 0;                                     /* :111 */
  if( !have( &r, 1 ) ) return 0;
  unsigned ro_unsigned = payload[r.i++];
  u16 acct_cnt;
  if( !cu16( &r, &acct_cnt ) ) return 0;                                   /* :116 */
  if( sig_cnt > acct_cnt || acct_cnt > 128 ) return 0;
  if( sig_cnt + ro_unsigned > (unsigned)acct_cnt ) return 0;               /* :118 */
  if( !have( &r, 32*(size_t)acct_cnt ) ) return 0;
  size_t acct_off = r.i; r.i += 32*(size_t)acct_cnt;
  if( !have( &r, 32 ) ) return 0;
  size_t bh_off = r.i; r.i += 32;
  u16 instr_cnt;
  if( !cu16( &r, &instr_cnt ) ) return 0;                                  /* :126 */
  if( instr_cnt > 64 ) return 0;                                           /* :129, instr_max = FD_TXN_INSTR_MAX */
  if( !have( &r, 3*(size_t)instr_cnt ) ) return 0;
  if( !( acct_cnt > (instr_cnt ? 1u : 0u) ) ) return 0;                    /* :134 */

  st8( out, 0, version ); st8( out, 1, sig_cnt ); st16( out, 2, (unsigned)sig_off ); st16( out, 4, (unsigned)msg_off );
  st8( out, 6, ro_signed ); st8( out, 7, ro_unsigned ); st16( out, 8, acct_cnt ); st16( out, 10, (unsigned)acct_off );
  st16( out, 12, (unsigned)bh_off ); st16( out, 18, instr_cnt );

  unsigned max_acct = 0;
  for( unsigned j=0; j<instr_cnt; j++ ) {                                  /* :153-184 */
    if( !have( &r, 3 ) ) return 0;
    unsigned prog = payload[r.i++];
    u16 ia_cnt, data_sz;
    if( !cu16( &r, &ia_cnt ) ) return 0;
    if( !have( &r, ia_cnt ) ) return 0;
    size_t ia_off = r.i;
    for( unsigned k=0; k<ia_cnt; k++ ) if( payload[ia_off+k] > max_acct ) max_acct = payload[ia_off+k];
    r.i += ia_cnt;
    if( !cu16( &r, &data_sz ) ) return 0;
    if( !have( &r, data_sz ) ) return 0;
    size_t data_off = r.i; r.i += data_sz;
    if( !( prog > 0 && prog < acct_cnt ) ) return 0;                       /* :171 */
    size_t o = 20 + 10*(size_t)j;
    st8( out, o, prog ); st8( out, o+1, 0 ); st16( out, o+2, ia_cnt ); st16( out, o+4, data_sz );
    st16( out, o+6, (unsigned)ia_off ); st16( out, o+8, (unsigned)data_off );
  }

  unsigned lut_cnt = 0, adtl_w = 0, adtl = 0;
  if( version == 0 ) {                                                     /* :193-226 */
    u16 c;
    if( !cu16( &r, &c ) ) return 0;
    lut_cnt = c;
    if( lut_cnt > 127 ) return 0;
    if( !have( &r, 34*(size_t)lut_cnt ) ) return 0;
    for( unsigned j=0; j<lut_cnt; j++ ) {
      if( !have( &r, 32 ) ) return 0;
      size_t a_off = r.i; r.i += 32;
      u16 w, ro;
      if( !cu16( &r, &w ) ) return 0;
      if( !have( &r, w ) ) return 0;
      size_t w_off = r.i; r.i += w;
      if( !cu16( &r, &ro ) ) return 0;
      if( !have( &r, ro ) ) return 0;
      size_t ro_off = r.i; r.i += ro;
      if( w  > 128u - acct_cnt ) return 0;
      if( ro > 128u - acct_cnt ) return 0;
      if( 1u > (unsigned)w + ro ) return 0;
      size_t o = 20 + 10*(size_t)instr_cnt + 8*(size_t)j;
      st16( out, o, (unsigned)a_off ); st8( out, o+2, w ); st8( out, o+3, ro );
      st16( out, o+4, (unsigned)w_off ); st16( out, o+6, (unsigned)ro_off );
      adtl_w += w; adtl += (unsigned)w + ro;
    }
  }
  if( r.i != payload_sz ) return 0;                                        /* :229 */
  if( acct_cnt + adtl > 128 ) return 0;                                    /* :231 */
  if( !( max_acct < acct_cnt + adtl ) ) return 0;                          /* :234 */
  st8( out, 14, lut_cnt ); st8( out, 15, adtl_w ); st8( out, 16, adtl ); st8( out, 17, 0 );
  return 20 + 10*(size_t)instr_cnt + 8*(size_t)lut_cnt;                    /* :244, fd_txn_footprint */
}

void oracle_txn_parse_many( size_t n, uint8_t const * pool, uint32_t const * off, uint16_t const * sz,
                            uint8_t * out, uint16_t * txn_t_sz ) {
  #pragma omp parallel for schedule(static, 256)
  for( long j=0; j<(long)n; j++ )
    txn_t_sz[j] = (uint16_t)oracle_txn_parse( pool + off[j], sz[j], out ? out + ORACLE_TXN_MAX_SZ*(size_t)j : NULL );
}

/* ---- tcache: src/tango/tcache/fd_tcache.h ------------------------------- */

size_t oracle_tcache_map_cnt_default( size_t depth ) {                     /* :115-141 */
  if( !depth || depth == (size_t)-1 ) return 0;
  int lg = 63 - __builtin_clzll( (unsigned long long)depth + 1 ) + 2;     /* SPARSE_DEFAULT 2 */
  if( lg > 63 ) return 0;
  return (size_t)1 << lg;
}

void oracle_tcache_reset( uint64_t * ring, size_t depth, uint64_t * map, size_t map_cnt ) {  /* :237-244 */
  memset( ring, 0, depth*8 ); memset( map, 0, map_cnt*8 );
}

/* FD_TCACHE_QUERY (:281-295): linear probe from tag & (map_cnt-1) until the
   tag or an empty (0) slot; a null query tag "finds" the first empty slot. */
static size_t probe( uint64_t const * map, size_t map_cnt, uint64_t tag, int * found ) {
  size_t i = (size_t)tag & (map_cnt-1);
  for(;;) {
    uint64_t t = map[i];
    if( t == tag ) { *found = 1; return i; }
    if( !t )       { *found = 0; return i; }
    i = (i+1) & (map_cnt-1);
  }
}

int oracle_tcache_query( uint64_t const * map, size_t map_cnt, uint64_t tag ) {
  int f; probe( map, map_cnt, tag, &f ); return f;
}

/* fd_tcache_remove (:309-347): delete with backward shift so every probe
   chain stays unbroken. */
static void tc_remove( uint64_t * map, size_t map_cnt, uint64_t tag ) {
  if( !tag ) return;
  int f; size_t hole = probe( map, map_cnt, tag, &f );
  if( !f ) return;
  size_t m = map_cnt - 1;
  for(;;) {
    map[hole] = 0;
    size_t s = hole;
    for(;;) {
      s = (s+1) & m;
      uint64_t t = map[s];
      if( !t ) return;
      size_t home = (size_t)t & m;
      /* t may move into the hole iff its home is not cyclically in (hole, s] */
      int home_in = hole <= s ? (home > hole && home <= s) : (home > hole || home <= s);
      if( !home_in ) { map[hole] = t; hole = s; break; }
    }
  }
}

int oracle_tcache_insert( uint64_t * oldest, uint64_t * ring, size_t depth,
                          uint64_t * map, size_t map_cnt, uint64_t tag ) {   /* :373-410 */
  int f; size_t slot = probe( map, map_cnt, tag, &f );
  if( f ) return 1;
  map[slot] = tag;
  uint64_t ev = ring[*oldest];
  ring[*oldest] = tag;
  *oldest = *oldest + 1 >= depth ? 0 : *oldest + 1;
  tc_remove( map, map_cnt, ev );
  return 0;
}

/* ---- after_frag + fd_txn_verify ------------------------------------------ */

void oracle_verify_tile_run( oracle_verify_tile_t * t, size_t n, uint8_t const * pool,
                             uint32_t const * off, uint16_t const * sz, uint64_t const * bundle_id,
                             int8_t * result, uint64_t * tag_out, uint16_t * txn_t_sz, int errmode ) {
  u8 txn[ORACLE_TXN_MAX_SZ];
  for( size_t j=0; j<n; j++ ) {
    u8 const * p = pool + off[j];
    size_t tsz = oracle_txn_parse( p, sz[j], txn );                        /* fd_verify_tile.c:116 */
    if( txn_t_sz ) txn_t_sz[j] = (uint16_t)tsz;
    tag_out[j] = 0;
    u64 bid = bundle_id ? bundle_id[j] : 0;
    int is_bundle = bid != 0;                                              /* :118 */
    if( is_bundle && bid != t->bundle_id ) { t->bundle_failed = 0; t->bundle_id = bid; }   /* :120-123 */
    if( is_bundle && t->bundle_failed ) { t->bundle_peer_fail_cnt++; result[j] = ORACLE_FRAG_BUNDLE_PEER; continue; }
    if( !tsz ) {                                                           /* :130-134 */
      if( is_bundle ) t->bundle_failed = 1;
      t->parse_fail_cnt++; result[j] = ORACLE_FRAG_PARSE_FAIL; continue;
    }
    /* fd_txn_verify (fd_verify_tile.h:61-111) with dedup = !is_bundle */
    unsigned sig_cnt = txn[1];
    size_t sig_off = txn[2] | (size_t)txn[3]<<8, msg_off = txn[4] | (size_t)txn[5]<<8;
    size_t acct_off = txn[10] | (size_t)txn[11]<<8;
    u64 tag = oracle_fd_hash( t->hashmap_seed, p + sig_off, 64 );
    int res;
    if( !is_bundle && oracle_tcache_query( t->tcache_map, t->tcache_map_cnt, tag ) ) res = -2;
    else if( oracle_verify_batch_single_msg( p + msg_off, sz[j] - msg_off, p + sig_off, p + acct_off,
                                             sig_cnt, errmode ) != ORACLE_SUCCESS ) res = -1;
    else if( !is_bundle && oracle_tcache_insert( &t->tcache_oldest, t->tcache_ring, t->tcache_depth,
                                                 t->tcache_map, t->tcache_map_cnt, tag ) ) res = -2;
    else res = 0;
    if( res ) {                                                            /* :145-152 */
      if( is_bundle ) t->bundle_failed = 1;
      if( res == -2 ) t->dedup_fail_cnt++; else t->verify_fail_cnt++;
      result[j] = (int8_t)res; continue;
    }
    tag_out[j] = tag; result[j] = ORACLE_FRAG_PUBLISH;
  }
}
