/* fd_ed25519_oracle.h -- TEST INFRASTRUCTURE ONLY.

   CPU restatement of the reference's ed25519 verify path
   (anoushk1234/firedancer src/ballet/ed25519/fd_ed25519_user.c:135-310),
   used as the parity checker for the HIP engine.  Only tests/,
   __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
   The product path (firedancer_amd/) never links or calls this code.

   Parity pinning: this restatement is checked against the reference's own
   vectors (Wycheproof 133, CCTV 914, malleability 396, fuzz corpus seeds)
   and against the reference built from its own sources
   (oracle/Makefile -> oracle/_ref/), see tests/test_oracle.py.

   Error codes: the reference's two backends agree on the accept/reject
   bitmap but not on the error code of some rejects (SURVEY.md 8(a) A1').
   ERRMODE_AVX512 reproduces the AVX-512 build (fd_r43x6_ge.c:163-254 returns
   -1/-2, so every decode failure maps to ERR_SIG at fd_ed25519_user.c:192);
   ERRMODE_REF reproduces the portable build (ref/fd_curve25519.c:209-224). */

#ifndef FD_ED25519_ORACLE_H
#define FD_ED25519_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#define ORACLE_SUCCESS     ( 0)
#define ORACLE_ERR_SIG     (-1)
#define ORACLE_ERR_PUBKEY  (-2)
#define ORACLE_ERR_MSG     (-3)

#define ORACLE_ERRMODE_AVX512 0
#define ORACLE_ERRMODE_REF    1

#ifdef __cplusplus
extern "C" {
#endif

void oracle_sha512( uint8_t out[64], uint8_t const * in, size_t sz );

int  oracle_verify( uint8_t const * msg, size_t msg_sz, uint8_t const sig[64],
                    uint8_t const pub[32], int errmode );

int  oracle_verify_batch_single_msg( uint8_t const * msg, size_t msg_sz,
                                     uint8_t const * sigs, uint8_t const * pubs,
                                     unsigned batch_sz, int errmode );

/* Bulk helper for tests: record i uses sigs+64*i, pubs+32*i and the
   message pool bytes [msg_off[i], msg_off[i]+msg_sz[i]).  Writes one int8
   code per record.  Uses OpenMP when built with it. */
void oracle_verify_many( size_t n, uint8_t const * sigs, uint8_t const * pubs,
                         uint8_t const * msg_pool, uint32_t const * msg_off,
                         uint32_t const * msg_sz, int8_t * codes, int errmode );

void oracle_public_from_private( uint8_t pub[32], uint8_t const prv[32] );
void oracle_sign( uint8_t sig[64], uint8_t const * msg, size_t msg_sz,
                  uint8_t const pub[32], uint8_t const prv[32] );
void oracle_sign_many( size_t n, uint8_t const * prvs, uint8_t * pubs, uint8_t * sigs,
                       uint8_t const * msg_pool, uint32_t const * msg_off,
                       uint32_t const * msg_sz );

/* k = SHA512(R||A||M) mod L, exposed for unit tests of the kernel stages. */
void oracle_hram( uint8_t k[32], uint8_t const R[32], uint8_t const A[32],
                  uint8_t const * msg, size_t msg_sz );
void oracle_scalar_reduce( uint8_t out[32], uint8_t const in[64] );

/* Point decode with both error semantics reported: returns 0 ok,
   1 not on curve, 2 x==0 with sign bit set (AVX-512 rejects, ref accepts).
   xy receives canonical x||y (64 bytes) when the point decodes. */
int  oracle_point_decode( uint8_t xy[64], uint8_t const buf[32] );
int  oracle_point_is_small_order( uint8_t const buf[32] );

#ifdef __cplusplus
}
#endif

#endif
