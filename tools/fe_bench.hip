// Field-arithmetic correctness dump + throughput microbenchmark (tools/, dev only).
// mode "dump": writes a, b, mul, add, sub, sqr-chain results for N lanes to a file
//               (checked by tools/check_fe.py with Python big ints).
// mode "bench": dependent fe_mul chains, 1 or 2 independent chains per lane,
//               at 1..8 waves per SIMD; prints fe_mul/s and slow-instr rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "fe25519_asm.h"

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_dump(const uint32_t* in, uint32_t* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t a[8], b[8], r[8];
  for (int i = 0; i < 8; ++i) { a[i] = in[t * 16 + i]; b[i] = in[t * 16 + 8 + i]; }
  fe_mul(r, a, b);   for (int i = 0; i < 8; ++i) out[t * 40 + i] = r[i];
  fe_add(r, a, b);   for (int i = 0; i < 8; ++i) out[t * 40 + 8 + i] = r[i];
  // sub needs tight b: use b' = b*1 (mul output is tight)
  uint32_t one[8] = {1,0,0,0,0,0,0,0}, bt[8];
  fe_mul(bt, b, one);
  fe_sub(r, a, bt);  for (int i = 0; i < 8; ++i) out[t * 40 + 16 + i] = r[i];
  for (int i = 0; i < 8; ++i) out[t * 40 + 24 + i] = bt[i];
  uint32_t x[8]; for (int i = 0; i < 8; ++i) x[i] = a[i];
  for (int k = 0; k < 100; ++k) fe_mul(x, x, b);
  for (int i = 0; i < 8; ++i) out[t * 40 + 32 + i] = x[i];
}

template <int CHAINS>
__global__ __launch_bounds__(256) void k_bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t x[8], y[8], z[8];
  for (int i = 0; i < 8; ++i) { x[i] = seed * (threadIdx.x + 7 * i + 1); y[i] = seed ^ (i * 0x9e3779b9u); z[i] = x[i] ^ 0x5555u; }
  for (int it = 0; it < iters; ++it) {
    fe_mul(x, x, y);
    if (CHAINS > 1) fe_mul(z, z, y);
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s ^= x[i] ^ z[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "bench";
  CHK(hipSetDevice(0));
  if (!strcmp(mode, "dump")) {
    int n = atoi(argv[2]);
    std::vector<uint32_t> in(n * 16);
    FILE* f = fopen(argv[3], "rb"); if (!f) { fprintf(stderr, "cannot open %s\n", argv[3]); return 1; } if (fread(in.data(), 4, n * 16, f) != (size_t)n * 16) return 1; fclose(f);
    uint32_t *din, *dout; CHK(hipMalloc(&din, n * 64)); CHK(hipMalloc(&dout, n * 160));
    CHK(hipMemcpy(din, in.data(), n * 64, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_dump, dim3((n + 255) / 256), dim3(256), 0, 0, din, dout, n);
    CHK(hipDeviceSynchronize());
    std::vector<uint32_t> out(n * 40);
    CHK(hipMemcpy(out.data(), dout, n * 160, hipMemcpyDeviceToHost));
    f = fopen(argv[4], "wb"); fwrite(out.data(), 4, n * 40, f); fclose(f);
    printf("dumped %d\n", n);
    return 0;
  }
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  uint32_t* out; CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  int iters = 2000;
  for (int chains = 1; chains <= 2; ++chains) {
    for (int w : {1, 2, 3, 4, 6, 8}) {
      int blocks = cus * w;
      auto launch = [&]() {
        if (chains == 1) hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
        else hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
      };
      launch(); CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0)); for (int r = 0; r < 3; ++r) launch(); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double muls = 3.0 * blocks * 256 * iters * chains;
      double per_simd_cycles = (ms * 1e-3) * 2.4e9 / (muls / 64.0 / (cus * 4));   // cycles per wave-mul per SIMD
      printf("chains=%d waves/SIMD=%d : %.3e fe_mul/s  %.1f SIMD-cycles per wave-level fe_mul\n", chains, w, muls / (ms * 1e-3), per_simd_cycles);
    }
  }
  return 0;
}
