/* fd_precompile_oracle.h -- TEST INFRASTRUCTURE ONLY (see fd_precompile_oracle.c). */

#ifndef FD_PRECOMPILE_ORACLE_H
#define FD_PRECOMPILE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* fd_precompile_ed25519_verify (fd_precompiles.c:114-211): returns 0
   (FD_EXECUTOR_INSTR_SUCCESS) or -26 (FD_EXECUTOR_INSTR_ERR_CUSTOM_ERR) with
   *custom_err = 2 (signature), 3 (data offset) or 4 (instruction data size). */
int  oracle_precompile_ed25519_verify( uint8_t const * data, size_t data_sz, uint8_t const * const * instr_data,
                                       size_t const * instr_sz, size_t instr_cnt, uint32_t * custom_err );
void oracle_precompile_ed25519_verify_many( size_t n, uint8_t const * pool, uint32_t const * desc_off,
                                            uint16_t const * desc_sz, uint16_t const * instr_cnt,
                                            uint32_t const * instr_base, uint32_t const * tab_off,
                                            uint32_t const * tab_sz, int32_t * err, uint32_t * custom_err );

#ifdef __cplusplus
}
#endif

#endif /* FD_PRECOMPILE_ORACLE_H */
