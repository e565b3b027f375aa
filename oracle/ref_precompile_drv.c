/* ref_precompile_drv.c -- TEST INFRASTRUCTURE ONLY.

   Drives the reference's own ed25519-program precompile,
   fd_precompile_ed25519_verify (/root/reference/src/flamenco/runtime/
   program/fd_precompiles.c:120-222, with fd_precompile_get_instr_data at
   :78-112), compiled by gcc from that file where it lies (oracle/Makefile,
   target _ref/libfdref_precompile.so).  The driver builds the smallest
   instruction context the function reads:
     ctx->instr                    the precompile's own instruction (data, data_sz)
     ctx->txn_in->txn              TXN(...)->instr_cnt (fd_txn_p.h:46)
     ctx->runtime->instr.infos[i]  every instruction of the transaction
     ctx->txn_out->err.custom_err  the precompile error code
   and exports it with the argument list of our restatement
   (oracle_precompile_ed25519_verify, fd_precompile_oracle.h), so the tests
   pin the restatement -- and through it the GPU path -- to the reference.
   The secp256k1/r1 verifiers in the same object are never referenced and
   are garbage-collected at link time. */

#include "flamenco/runtime/program/fd_precompiles.h"
#include "disco/fd_txn_p.h"

#include <stdlib.h>
#include <string.h>

static fd_runtime_t * drv_rt;
static fd_txn_p_t *   drv_txn;

int
ref_precompile_ed25519_verify( uchar const *         data,
                               ulong                 data_sz,
                               uchar const * const * instr_data,
                               ulong const *         instr_sz,
                               ulong                 instr_cnt,
                               uint *                custom_err ) {
  if( !drv_rt  ) drv_rt  = (fd_runtime_t *)calloc( 1UL, sizeof(fd_runtime_t) );
  if( !drv_txn ) drv_txn = (fd_txn_p_t   *)calloc( 1UL, sizeof(fd_txn_p_t)   );
  ulong const infos_max = sizeof(drv_rt->instr.infos) / sizeof(drv_rt->instr.infos[0]);
  if( !drv_rt || !drv_txn || instr_cnt > infos_max || data_sz > USHORT_MAX ) return -1000;

  for( ulong i=0UL; i<instr_cnt; i++ ) {
    if( instr_sz[ i ] > USHORT_MAX ) return -1000;
    drv_rt->instr.infos[ i ].data    = (uchar *)instr_data[ i ];
    drv_rt->instr.infos[ i ].data_sz = (ushort)instr_sz[ i ];
  }
  TXN( drv_txn )->instr_cnt = (ushort)instr_cnt;

  fd_instr_info_t own[1];
  memset( own, 0, sizeof(own) );
  own->data    = (uchar *)data;
  own->data_sz = (ushort)data_sz;

  fd_txn_in_t  txn_in[1];  memset( txn_in,  0, sizeof(txn_in)  );
  fd_txn_out_t txn_out[1]; memset( txn_out, 0, sizeof(txn_out) );
  txn_in->txn = drv_txn;

  fd_exec_instr_ctx_t ctx[1];
  memset( ctx, 0, sizeof(ctx) );
  ctx->instr   = own;
  ctx->runtime = drv_rt;
  ctx->txn_in  = txn_in;
  ctx->txn_out = txn_out;

  int rc = fd_precompile_ed25519_verify( ctx );
  *custom_err = rc ? txn_out->err.custom_err : 0U;
  return rc;
}
