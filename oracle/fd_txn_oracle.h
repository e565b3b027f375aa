/* fd_txn_oracle.h -- TEST INFRASTRUCTURE ONLY.

   CPU restatement of the verify tile's per-frag path around the signature
   check (SURVEY.md 8(f) "verify-tile integration" / "GPU txn parse"):

     fd_txn_parse_core   src/ballet/txn/fd_txn_parse.c:7-254
                         (+ fd_cu16_dec_sz / _fixed, fd_compact_u16.h:38-92)
     fd_hash             src/util/fd_hash.c:14-72 (xxhash-r39 variant)
     tcache              src/tango/tcache/fd_tcache.h:115-135,237-410
     fd_txn_verify       src/disco/verify/fd_verify_tile.h:61-111
     after_frag          src/disco/verify/fd_verify_tile.c:101-161

   Used as the parity checker for the GPU parse kernel, the GPU tag hash and
   the engine's host tcache pass.  Only tests/, __graft_entry__.smoke() and
   bench.py's cpu_baseline leg load it; firedancer_amd/ never does.

   Pinning: tests/test_txn_oracle.py checks every function here against the
   reference built from its own sources (oracle/_ref/libfdref_txn.so, which
   contains the reference's fd_txn_parse_core, fd_hash and the header-inline
   fd_txn_verify + FD_TCACHE_* macros) and against the reference's own test
   fixtures (src/ballet/txn/fixtures/transaction{1..6}.bin and the
   src/disco/verify/test_verify.c sequences, tests/golden/txn_vectors.json). */

#ifndef FD_TXN_ORACLE_H
#define FD_TXN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#define ORACLE_TXN_MAX_SZ   852u   /* fd_txn.h:60  */
#define ORACLE_TXN_MTU      1232u  /* fd_txn.h:65  */

/* Per-frag outcome of the verify tile (after_frag), as reported here. */
#define ORACLE_FRAG_PUBLISH      ( 0)  /* fd_stem_publish                       */
#define ORACLE_FRAG_VERIFY_FAIL  (-1)  /* FD_TXN_VERIFY_FAILED, verify_fail_cnt */
#define ORACLE_FRAG_DEDUP        (-2)  /* FD_TXN_VERIFY_DEDUP,  dedup_fail_cnt  */
#define ORACLE_FRAG_PARSE_FAIL   (-3)  /* parse_fail_cnt                        */
#define ORACLE_FRAG_BUNDLE_PEER  (-4)  /* bundle_peer_fail_cnt                  */

#ifdef __cplusplus
extern "C" {
#endif

uint64_t oracle_fd_hash( uint64_t seed, void const * buf, size_t sz );

/* Returns the fd_txn_t footprint (20 + 10*instr_cnt + 8*lut_cnt) on success,
   0 on failure.  out (may be NULL) receives the fd_txn_t bytes. */
size_t oracle_txn_parse( uint8_t const * payload, size_t payload_sz, uint8_t * out );

/* tcache on the reference memory layout: ring[depth], map[map_cnt] */
size_t   oracle_tcache_map_cnt_default( size_t depth );
void     oracle_tcache_reset ( uint64_t * ring, size_t depth, uint64_t * map, size_t map_cnt );
int      oracle_tcache_query ( uint64_t const * map, size_t map_cnt, uint64_t tag );
int      oracle_tcache_insert( uint64_t * oldest, uint64_t * ring, size_t depth,
                               uint64_t * map, size_t map_cnt, uint64_t tag );

/* Verify-tile state carried across frags (the fields of fd_verify_ctx_t
   that after_frag / fd_txn_verify touch). */
typedef struct {
  uint64_t   hashmap_seed;
  uint64_t   tcache_oldest;
  uint64_t * tcache_ring;
  size_t     tcache_depth;
  uint64_t * tcache_map;
  size_t     tcache_map_cnt;
  int        bundle_failed;
  uint64_t   bundle_id;
  uint64_t   parse_fail_cnt, verify_fail_cnt, dedup_fail_cnt, bundle_peer_fail_cnt;
} oracle_verify_tile_t;

/* Runs after_frag over n frags in arrival order.  Frag j is the payload
   pool[off[j] .. off[j]+sz[j]) with bundle id bundle_id[j] (NULL: none).
   result[j] gets ORACLE_FRAG_*, tag[j] the dedup tag written to opt_sig on
   publish (0 otherwise), txn_t_sz[j] the parse footprint (NULL to skip). */
void oracle_verify_tile_run( oracle_verify_tile_t * t, size_t n, uint8_t const * pool,
                             uint32_t const * off, uint16_t const * sz, uint64_t const * bundle_id,
                             int8_t * result, uint64_t * tag, uint16_t * txn_t_sz, int errmode );

/* Bulk parse for tests: out stride ORACLE_TXN_MAX_SZ (may be NULL). */
void oracle_txn_parse_many( size_t n, uint8_t const * pool, uint32_t const * off, uint16_t const * sz,
                            uint8_t * out, uint16_t * txn_t_sz );

#ifdef __cplusplus
}
#endif

#endif
