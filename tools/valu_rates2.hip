// gfx950 VALU issue-rate microbenchmark (tools/, not product code).
// Measures wave-instructions per cycle per SIMD for the integer instructions a
// GF(2^255-19) limb multiplier can be built from, so the field representation is
// chosen from measured rates rather than guessed ones. Each kernel runs 8
// independent dependency chains per lane (one asm block, so hipcc inserts no
// boundary nops inside it) and 1..8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define ITERS 256
#define BODY(F) F("%0","%16") F("%1","%17") F("%2","%18") F("%3","%19") F("%4","%20") F("%5","%21") F("%6","%22") F("%7","%23")

#define KERN(NAME, T, F, NOPS)                                                          \
__global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned seed) {         \
  T a0=seed+threadIdx.x,a1=a0*3,a2=a0*5,a3=a0*7,a4=a0*9,a5=a0*11,a6=a0*13,a7=a0*15;    \
  unsigned b = seed ^ 0x9e3779b9u, c = seed * 77u;                                        \
  unsigned long long s0,s1,s2,s3,s4,s5,s6,s7;                                           \
  for (int it = 0; it < ITERS; ++it) {                                                  \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                     \
      asm volatile(BODY(F) : "+v"(a0),"+v"(a1),"+v"(a2),"+v"(a3),"+v"(a4),"+v"(a5),"+v"(a6),"+v"(a7) \
                   : "v"(b), "v"(c), "v"(b), "v"(c), "v"(b), "v"(c), "v"(b), "v"(c), \
                     "s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull) : "vcc", "s8", "s9"); \
    }                                                                                   \
  }                                                                                     \
  (void)s0;(void)s1;(void)s2;(void)s3;(void)s4;(void)s5;(void)s6;(void)s7;             \
  out[blockIdx.x*256+threadIdx.x] = (unsigned)(a0^a1^a2^a3^a4^a5^a6^a7);                \
}
// %8 = b, %9 = c ; second arg of F = a per-chain SGPR pair (read-only use as a scratch sdst is not allowed, so mad64 writes vcc)
#define F_add_e32(d,s) "v_add_u32_e32 " d ", " d ", %8\n\t"
#define F_add_e64(d,s) "v_add_u32_e64 " d ", " d ", %8\n\t"
#define F_sub_e32(d,s) "v_sub_u32_e32 " d ", " d ", %8\n\t"
#define F_and_e32(d,s) "v_and_b32_e32 " d ", " d ", %8\n\t"
#define F_xor_e32(d,s) "v_xor_b32_e32 " d ", " d ", %8\n\t"
#define F_or_e32(d,s) "v_or_b32_e32 " d ", " d ", %8\n\t"
#define F_lshl_e32(d,s) "v_lshlrev_b32_e32 " d ", 3, " d "\n\t"
#define F_lshr_e32(d,s) "v_lshrrev_b32_e32 " d ", 3, " d "\n\t"
#define F_mov_e32(d,s) "v_mov_b32_e32 " d ", %8\n\t"
#define F_addco_e32(d,s) "v_add_co_u32_e32 " d ", vcc, " d ", %8\n\t"
#define F_addc_e32(d,s) "v_addc_co_u32_e32 " d ", vcc, " d ", %8, vcc\n\t"
#define F_subco_e32(d,s) "v_sub_co_u32_e32 " d ", vcc, " d ", %8\n\t"
#define F_mul24_e32(d,s) "v_mul_u32_u24_e32 " d ", " d ", %8\n\t"
#define F_mulhi24_e32(d,s) "v_mul_hi_u32_u24_e32 " d ", " d ", %8\n\t"
#define F_cndmask_e32(d,s) "v_cndmask_b32_e32 " d ", " d ", %8, vcc\n\t"
#define F_fmac_e32(d,s) "v_fmac_f32_e32 " d ", %8, %9\n\t"
#define F_add_f32_e32(d,s) "v_add_f32_e32 " d ", " d ", %8\n\t"
#define F_pk_fma_f32(d,s) "v_pk_fma_f32 " d ", " d ", " d ", " d "\n\t"
#define F_pk_add_f32(d,s) "v_pk_add_f32 " d ", " d ", " d "\n\t"
#define F_lshl_or(d,s) "v_lshl_or_b32 " d ", %8, 3, " d "\n\t"
#define F_and_or(d,s) "v_and_or_b32 " d ", %8, %9, " d "\n\t"
#define F_perm(d,s) "v_perm_b32 " d ", " d ", %8, %9\n\t"
#define F_xad(d,s) "v_xad_u32 " d ", " d ", %8, %9\n\t"
#define F_mov_b64(d,s) "v_mov_b64 " d ", " d "\n\t"
#define F_mad64_addc_mix(d,s) "v_mad_u64_u32 " d ", vcc, %8, %9, " d "\n\tv_addc_co_u32_e32 %9, vcc, 0, %9, vcc\n\t"
#define F_mad64_add_mix(d,s) "v_mad_u64_u32 " d ", vcc, %8, %9, " d "\n\tv_add_u32_e32 %8, %8, %9\n\t"
#define F_addco_e64_sgpr(d,s) "v_add_co_u32_e64 " d ", s[8:9], " d ", %8\n\t"
KERN(add_e32, unsigned, F_add_e32, 1)
KERN(add_e64, unsigned, F_add_e64, 1)
KERN(sub_e32, unsigned, F_sub_e32, 1)
KERN(and_e32, unsigned, F_and_e32, 1)
KERN(xor_e32, unsigned, F_xor_e32, 1)
KERN(or_e32, unsigned, F_or_e32, 1)
KERN(lshl_e32, unsigned, F_lshl_e32, 1)
KERN(lshr_e32, unsigned, F_lshr_e32, 1)
KERN(mov_e32, unsigned, F_mov_e32, 1)
KERN(addco_e32, unsigned, F_addco_e32, 1)
KERN(addc_e32, unsigned, F_addc_e32, 1)
KERN(subco_e32, unsigned, F_subco_e32, 1)
KERN(mul24_e32, unsigned, F_mul24_e32, 1)
KERN(mulhi24_e32, unsigned, F_mulhi24_e32, 1)
KERN(cndmask_e32, unsigned, F_cndmask_e32, 1)
KERN(fmac_e32, unsigned, F_fmac_e32, 1)
KERN(add_f32_e32, unsigned, F_add_f32_e32, 1)
KERN(pk_fma_f32, unsigned long long, F_pk_fma_f32, 1)
KERN(pk_add_f32, unsigned long long, F_pk_add_f32, 1)
KERN(lshl_or, unsigned, F_lshl_or, 1)
KERN(and_or, unsigned, F_and_or, 1)
KERN(perm, unsigned, F_perm, 1)
KERN(xad, unsigned, F_xad, 1)
KERN(mov_b64, unsigned long long, F_mov_b64, 1)
KERN(mad64_addc_mix, unsigned long long, F_mad64_addc_mix, 1)
KERN(mad64_add_mix, unsigned long long, F_mad64_add_mix, 1)
KERN(addco_e64_sgpr, unsigned, F_addco_e64_sgpr, 1)

typedef void (*kfn)(unsigned*, unsigned);
struct Case { const char* name; kfn fn; };

int main() {
  CHK(hipSetDevice(0));
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  double clk_ghz = p.clockRate / 1e6;
  printf("device %s gcn %s CUs %d clockRate %.3f GHz\n", p.name, p.gcnArchName, cus, clk_ghz);
  Case cases[] = {
    {"add_e32", k_add_e32},
    {"add_e64", k_add_e64},
    {"sub_e32", k_sub_e32},
    {"and_e32", k_and_e32},
    {"xor_e32", k_xor_e32},
    {"or_e32", k_or_e32},
    {"lshl_e32", k_lshl_e32},
    {"lshr_e32", k_lshr_e32},
    {"mov_e32", k_mov_e32},
    {"addco_e32", k_addco_e32},
    {"addc_e32", k_addc_e32},
    {"subco_e32", k_subco_e32},
    {"mul24_e32", k_mul24_e32},
    {"mulhi24_e32", k_mulhi24_e32},
    {"cndmask_e32", k_cndmask_e32},
    {"fmac_e32", k_fmac_e32},
    {"add_f32_e32", k_add_f32_e32},
    {"pk_fma_f32", k_pk_fma_f32},
    {"pk_add_f32", k_pk_add_f32},
    {"lshl_or", k_lshl_or},
    {"and_or", k_and_or},
    {"perm", k_perm},
    {"xad", k_xad},
    {"mov_b64", k_mov_b64},
    {"mad64_addc_mix", k_mad64_addc_mix},
    {"mad64_add_mix", k_mad64_add_mix},
    {"addco_e64_sgpr", k_addco_e64_sgpr},
  };
  unsigned* out; CHK(hipMalloc(&out, (size_t)cus * 64 * 256 * sizeof(unsigned)));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  int occs[] = {1, 2, 4, 8};  // waves per SIMD (256-thread blocks = 1 wave per SIMD each)
  printf("%-28s", "wave-instr/cycle/SIMD @");
  for (int o : occs) printf("  w/SIMD=%d", o);
  printf("   best lane-ops/s (at clockRate)\n");
  for (auto& c : cases) {
    printf("%-28s", c.name);
    double best = 0;
    for (int o : occs) {
      int blocks = cus * o;
      hipLaunchKernelGGL(c.fn, dim3(blocks), dim3(256), 0, 0, out, 1u);
      CHK(hipDeviceSynchronize());
      const int reps = 5;
      CHK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(c.fn, dim3(blocks), dim3(256), 0, 0, out, 1u);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double waveinstr = (double)reps * blocks * 4 * ITERS * 8 * 8;
      double ipc = waveinstr / (cus * 4.0) / (ms * 1e-3) / (clk_ghz * 1e9);
      double laneops = waveinstr * 64 / (ms * 1e-3);
      if (laneops > best) best = laneops;
      printf("  %10.3f", ipc);
    }
    printf("   %.3e\n", best);
  }
  return 0;
}
