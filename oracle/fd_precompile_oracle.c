/* fd_precompile_oracle.c -- TEST INFRASTRUCTURE ONLY.

   CPU restatement of the ed25519 program (precompile) instruction check,
   fd_precompile_ed25519_verify (src/flamenco/runtime/program/
   fd_precompiles.c:114-211) with its data fetch fd_precompile_get_instr_data
   (:76-107), on top of this oracle's fd_ed25519_verify restatement
   (oracle_verify, fd_ed25519_oracle.c).  The checker for
   fd_precompile_hip_ed25519_verify_dev (include/fd_replay_hip.h).

   Pinning (round 6): the reference's fd_precompiles.c compiles here from
   the file where it lies (headers only; the secp256k1/r1 verifiers it also
   holds are never referenced and are garbage-collected), and
   oracle/ref_precompile_drv.c drives its fd_precompile_ed25519_verify
   through a minimal instruction context (_ref/libfdref_precompile.so).
   tests/test_precompile_ref.py checks this restatement against it, return
   value and custom error, on boundary offsets, random blocks and mutated
   instructions, and against the committed reference answers
   (tests/golden/precompile_ref.npz).  The offset / size rules below are
   restated line by line from the reference's source text. */

#include "fd_ed25519_oracle.h"
#include "fd_precompile_oracle.h"

#include <stdint.h>
#include <string.h>

#define SIG_SZ        64u   /* SIGNATURE_SERIALIZED_SIZE          :44 */
#define OFFS_SZ       14u   /* SIGNATURE_OFFSETS_SERIALIZED_SIZE  :45 */
#define OFFS_START     2u   /* SIGNATURE_OFFSETS_START            :46 */
#define DATA_START    16u   /* DATA_START                         :47 */
#define PUB_SZ        32u   /* ED25519_PUBKEY_SERIALIZED_SIZE     :53 */

#define ERR_SIGNATURE        2u   /* fd_precompiles.h:16 */
#define ERR_DATA_OFFSET      3u   /* fd_precompiles.h:17 */
#define ERR_INSTR_DATA_SIZE  4u   /* fd_precompiles.h:18 */
#define INSTR_SUCCESS        0    /* fd_executor_err.h:14 */
#define INSTR_ERR_CUSTOM   (-26)  /* fd_executor_err.h:40 */

static unsigned ld16( uint8_t const * p ) { return (unsigned)p[0] | ((unsigned)p[1] << 8); }

/* fd_precompile_get_instr_data (:76-107): index 0xFFFF names the current
   instruction; an index past the txn's instructions is DATA_OFFSET; a span
   past the instruction's data is SIGNATURE */
static unsigned
get_instr_data( uint8_t const * cur, size_t cur_sz, uint8_t const * const * instr_data, size_t const * instr_sz,
                size_t instr_cnt, unsigned index, unsigned offset, unsigned sz, uint8_t const ** res ) {
  uint8_t const * data; size_t data_sz;
  if( index == 0xFFFFu ) { data = cur; data_sz = cur_sz; }
  else {
    if( index >= instr_cnt ) return ERR_DATA_OFFSET;
    data = instr_data[index]; data_sz = instr_sz[index];
  }
  if( (size_t)offset + (size_t)sz > data_sz ) return ERR_SIGNATURE;
  *res = data + offset;
  return 0u;
}

int
oracle_precompile_ed25519_verify( uint8_t const * data, size_t data_sz, uint8_t const * const * instr_data,
                                  size_t const * instr_sz, size_t instr_cnt, uint32_t * custom_err ) {
  *custom_err = 0u;
  if( data_sz < DATA_START ) {                                    /* :130-141 */
    if( data_sz == 2 && data[0] == 0 ) return INSTR_SUCCESS;
    *custom_err = ERR_INSTR_DATA_SIZE; return INSTR_ERR_CUSTOM;
  }
  size_t sig_cnt = data[0];
  if( sig_cnt == 0 ) { *custom_err = ERR_INSTR_DATA_SIZE; return INSTR_ERR_CUSTOM; }   /* :143-147 */
  if( data_sz < sig_cnt*OFFS_SZ + OFFS_START ) {                  /* :150-154 */
    *custom_err = ERR_INSTR_DATA_SIZE; return INSTR_ERR_CUSTOM;
  }
  size_t off = OFFS_START;
  for( size_t i=0; i<sig_cnt; i++ ) {                             /* :156-208 */
    uint8_t const * o = data + off;
    off += OFFS_SZ;
    unsigned sig_offset = ld16( o ), sig_idx = ld16( o+2 ), pub_offset = ld16( o+4 ), pub_idx = ld16( o+6 );
    unsigned msg_offset = ld16( o+8 ), msg_sz = ld16( o+10 ), msg_idx = ld16( o+12 );
    uint8_t const * sig = NULL, * pub = NULL, * msg = NULL;
    unsigned err = get_instr_data( data, data_sz, instr_data, instr_sz, instr_cnt, sig_idx, sig_offset, SIG_SZ, &sig );
    if( err ) { *custom_err = err; return INSTR_ERR_CUSTOM; }
    err = get_instr_data( data, data_sz, instr_data, instr_sz, instr_cnt, pub_idx, pub_offset, PUB_SZ, &pub );
    if( err ) { *custom_err = err; return INSTR_ERR_CUSTOM; }
    err = get_instr_data( data, data_sz, instr_data, instr_sz, instr_cnt, msg_idx, msg_offset, msg_sz, &msg );
    if( err ) { *custom_err = err; return INSTR_ERR_CUSTOM; }
    if( oracle_verify( msg, msg_sz, sig, pub, 0 ) != 0 ) { *custom_err = ERR_SIGNATURE; return INSTR_ERR_CUSTOM; }
  }
  return INSTR_SUCCESS;
}

/* Bulk form for tests, on the GPU entry's layout: instruction j's data is
   pool[desc_off[j], +desc_sz[j]); its txn's instruction k is
   pool[tab_off[base[j]+k], +tab_sz[base[j]+k]) for k < cnt[j]. */
void
oracle_precompile_ed25519_verify_many( size_t n, uint8_t const * pool, uint32_t const * desc_off,
                                       uint16_t const * desc_sz, uint16_t const * instr_cnt,
                                       uint32_t const * instr_base, uint32_t const * tab_off,
                                       uint32_t const * tab_sz, int32_t * err, uint32_t * custom_err ) {
  enum { MAXI = 65536 };
  static uint8_t const * ptrs[MAXI];
  static size_t          szs [MAXI];
  for( size_t j=0; j<n; j++ ) {
    size_t c = instr_cnt[j];
    for( size_t k=0; k<c && k<MAXI; k++ ) {
      ptrs[k] = pool + tab_off[instr_base[j] + k];
      szs [k] = tab_sz[instr_base[j] + k];
    }
    err[j] = oracle_precompile_ed25519_verify( pool + desc_off[j], desc_sz[j], ptrs, szs, c, custom_err + j );
  }
}
