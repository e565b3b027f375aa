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
                     "s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull),"s"(0ull) : "vcc"); \
    }                                                                                   \
  }                                                                                     \
  (void)s0;(void)s1;(void)s2;(void)s3;(void)s4;(void)s5;(void)s6;(void)s7;             \
  out[blockIdx.x*256+threadIdx.x] = (unsigned)(a0^a1^a2^a3^a4^a5^a6^a7);                \
}
// %8 = b, %9 = c ; second arg of F = a per-chain SGPR pair (read-only use as a scratch sdst is not allowed, so mad64 writes vcc)
#define F_add(d,s)      "v_add_u32 " d ", " d ", %8\n\t"
#define F_add3(d,s)     "v_add3_u32 " d ", " d ", %8, %9\n\t"
#define F_mad24(d,s)    "v_mad_u32_u24 " d ", %8, %9, " d "\n\t"
#define F_mulhi24(d,s)  "v_mul_hi_u32_u24 " d ", " d ", %8\n\t"
#define F_mullo(d,s)    "v_mul_lo_u32 " d ", " d ", %8\n\t"
#define F_mulhi(d,s)    "v_mul_hi_u32 " d ", " d ", %8\n\t"
#define F_dot2(d,s)     "v_dot2_u32_u16 " d ", %8, %9, " d "\n\t"
#define F_lshladd(d,s)  "v_lshl_add_u32 " d ", %8, 3, " d "\n\t"
#define F_align(d,s)    "v_alignbit_b32 " d ", " d ", %8, 7\n\t"
#define F_fma32(d,s)    "v_fma_f32 " d ", %8, %9, " d "\n\t"
#define F_mad16(d,s)    "v_mad_u32_u16 " d ", %8, %9, " d "\n\t"
#define F_bfe(d,s)      "v_bfe_u32 " d ", " d ", 3, 20\n\t"
#define F_addco(d,s)    "v_add_co_u32 " d ", vcc, " d ", %8\n\t"
#define F_addc(d,s)     "v_addc_co_u32 " d ", vcc, " d ", %8, vcc\n\t"
#define F_mad64(d,s)    "v_mad_u64_u32 " d ", vcc, %8, %9, " d "\n\t"
#define F_fma64(d,s)    "v_fma_f64 " d ", " d ", " d ", " d "\n\t"
#define F_lshladd64(d,s) "v_lshl_add_u64 " d ", " d ", 2, " d "\n\t"
#define F_lshr64(d,s)   "v_lshrrev_b64 " d ", 3, " d "\n\t"
#define F_add64f(d,s)   "v_add_f64 " d ", " d ", " d "\n\t"
#define F_pkadd16(d,s)  "v_pk_add_u16 " d ", " d ", %8\n\t"
#define F_pkmad16(d,s)  "v_pk_mad_u16 " d ", %8, %9, " d "\n\t"

KERN(add, unsigned, F_add, 1)
KERN(add3, unsigned, F_add3, 1)
KERN(mad24, unsigned, F_mad24, 1)
KERN(mulhi24, unsigned, F_mulhi24, 1)
KERN(mullo, unsigned, F_mullo, 1)
KERN(mulhi, unsigned, F_mulhi, 1)
KERN(dot2, unsigned, F_dot2, 1)
KERN(lshladd, unsigned, F_lshladd, 1)
KERN(align, unsigned, F_align, 1)
KERN(fma32, unsigned, F_fma32, 1)
KERN(mad16, unsigned, F_mad16, 1)
KERN(bfe, unsigned, F_bfe, 1)
KERN(addco, unsigned, F_addco, 1)
KERN(addc, unsigned, F_addc, 1)
KERN(pkadd16, unsigned, F_pkadd16, 1)
KERN(pkmad16, unsigned, F_pkmad16, 1)
KERN(mad64, unsigned long long, F_mad64, 1)
KERN(fma64, unsigned long long, F_fma64, 1)
KERN(lshladd64, unsigned long long, F_lshladd64, 1)
KERN(lshr64, unsigned long long, F_lshr64, 1)
KERN(add64f, unsigned long long, F_add64f, 1)

typedef void (*kfn)(unsigned*, unsigned);
struct Case { const char* name; kfn fn; };

int main() {
  CHK(hipSetDevice(0));
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  double clk_ghz = p.clockRate / 1e6;
  printf("device %s gcn %s CUs %d clockRate %.3f GHz\n", p.name, p.gcnArchName, cus, clk_ghz);
  Case cases[] = {
    {"v_add_u32", k_add}, {"v_add3_u32", k_add3}, {"v_mad_u32_u24", k_mad24},
    {"v_mul_hi_u32_u24", k_mulhi24}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
    {"v_dot2_u32_u16", k_dot2}, {"v_lshl_add_u32", k_lshladd}, {"v_alignbit_b32", k_align},
    {"v_fma_f32", k_fma32}, {"v_mad_u32_u16", k_mad16}, {"v_bfe_u32", k_bfe},
    {"v_add_co_u32 (vcc)", k_addco}, {"v_addc_co_u32 (vcc chain)", k_addc},
    {"v_pk_add_u16", k_pkadd16}, {"v_pk_mad_u16", k_pkmad16},
    {"v_mad_u64_u32", k_mad64}, {"v_fma_f64", k_fma64}, {"v_lshl_add_u64", k_lshladd64},
    {"v_lshrrev_b64", k_lshr64}, {"v_add_f64", k_add64f},
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
