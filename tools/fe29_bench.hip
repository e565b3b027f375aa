// Candidate field representation microbenchmark (tools/, dev only):
// GF(2^255-19) in 9 unsaturated limbs (8 x 29 bits + a top limb holding bits
// 232..254), product scanning with carry-free 64-bit column accumulators.
// mode "dump": mul / sq results for N lanes (checked by tools/check_fe29.py)
// mode "bench": dependent mul and sq chains at 1..8 waves per SIMD, next to the
//               current 8x32 asm fe_mul.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "fe25519_asm.h"

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
typedef uint32_t u32; typedef uint64_t u64;
#define M29 0x1fffffffu
#define M23 0x7fffffu
#define DEV __device__ __forceinline__

DEV void f29_mul(u32 r[9], const u32 a[9], const u32 b[9]) {
  u32 o[9];
  u32 z[9]; u64 acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; k++) {
    acc = (k == 9) ? 0ull : (acc >> 29);
#pragma unroll
    for (int i = k - 8; i <= 8; i++) acc += (u64)a[i] * b[k - i];
    z[k - 9] = (u32)acc & M29;
  }
  z[8] = (u32)(acc >> 29);
#pragma unroll
  for (int k = 0; k <= 8; k++) {
    acc = (k == 0 ? 0ull : (acc >> 29)) + (u64)z[k] * 1216u;
#pragma unroll
    for (int i = 0; i <= k; i++) acc += (u64)a[i] * b[k - i];
    if (k < 8) o[k] = (u32)acc & M29;
  }
  o[8] = (u32)acc & M23;
  u64 t = (acc >> 23) * 19u + o[0];
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}

DEV void f29_sq(u32 r[9], const u32 a[9]) {
  u32 o[9];
  u32 d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a[i] << 1;
  u32 z[9]; u64 acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; k++) {
    acc = (k == 9) ? 0ull : (acc >> 29);
#pragma unroll
    for (int i = k - 8; 2 * i < k; i++) acc += (u64)d[i] * a[k - i];
    if ((k & 1) == 0) acc += (u64)a[k / 2] * a[k / 2];
    z[k - 9] = (u32)acc & M29;
  }
  z[8] = (u32)(acc >> 29);
#pragma unroll
  for (int k = 0; k <= 8; k++) {
    acc = (k == 0 ? 0ull : (acc >> 29)) + (u64)z[k] * 1216u;
#pragma unroll
    for (int i = 0; 2 * i < k; i++) acc += (u64)d[i] * a[k - i];
    if ((k & 1) == 0) acc += (u64)a[k / 2] * a[k / 2];
    if (k < 8) o[k] = (u32)acc & M29;
  }
  o[8] = (u32)acc & M23;
  u64 t = (acc >> 23) * 19u + o[0];
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}


DEV u64 mad64(u32 a, u32 b, u64 c) {
  u64 r = c + (u64)a * b; asm("" : "+v"(r)); return r;
}
DEV u64 mul64(u32 a, u32 b) {
  u64 r = (u64)a * b; asm("" : "+v"(r)); return r;
}
// serial column chains: every product of a column accumulates into one chain
DEV void f29s_mul(u32 r[9], const u32 a[9], const u32 b[9]) {
  u32 o[9], z[9]; u64 acc = 0;
#pragma unroll
  for (int k = 9; k <= 16; k++) {
#pragma unroll
    for (int i = k - 8; i <= 8; i++) acc = (k == 9 && i == 1) ? mul64(a[i], b[k - i]) : mad64(a[i], b[k - i], acc);
    z[k - 9] = (u32)acc & M29; acc >>= 29;
  }
  z[8] = (u32)acc;
#pragma unroll
  for (int k = 0; k <= 8; k++) {
    acc = (k == 0) ? mul64(z[k], 1216u) : mad64(z[k], 1216u, acc);
#pragma unroll
    for (int i = 0; i <= k; i++) acc = mad64(a[i], b[k - i], acc);
    if (k < 8) { o[k] = (u32)acc & M29; acc >>= 29; }
  }
  o[8] = (u32)acc & M23;
  u64 t = mad64((u32)(acc >> 23), 19u, (u64)o[0]);
  t += (u64)((u32)(acc >> 55) * 19u) << 32;
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}
DEV void f29s_sq(u32 r[9], const u32 a[9]) {
  u32 d[9], o[9], z[9]; u64 acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a[i] << 1;
#pragma unroll
  for (int k = 9; k <= 16; k++) {
    bool first = (k == 9);
#pragma unroll
    for (int i = k - 8; 2 * i < k; i++) { acc = first ? mul64(d[i], a[k - i]) : mad64(d[i], a[k - i], acc); first = false; }
    if ((k & 1) == 0) acc = mad64(a[k / 2], a[k / 2], acc);
    z[k - 9] = (u32)acc & M29; acc >>= 29;
  }
  z[8] = (u32)acc;
#pragma unroll
  for (int k = 0; k <= 8; k++) {
    acc = (k == 0) ? mul64(z[k], 1216u) : mad64(z[k], 1216u, acc);
#pragma unroll
    for (int i = 0; 2 * i < k; i++) acc = mad64(d[i], a[k - i], acc);
    if ((k & 1) == 0) acc = mad64(a[k / 2], a[k / 2], acc);
    if (k < 8) { o[k] = (u32)acc & M29; acc >>= 29; }
  }
  o[8] = (u32)acc & M23;
  u64 t = mad64((u32)(acc >> 23), 19u, (u64)o[0]);
  t += (u64)((u32)(acc >> 55) * 19u) << 32;
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}


// two independent serial chains interleaved: high column 9+k next to low
// column k (products first, then the 1216*z_k fold)
DEV void f29p_mul(u32 r[9], const u32 a[9], const u32 b[9]) {
  u32 o[9], z[9]; u64 h = 0, l = 0;
#pragma unroll
  for (int k = 0; k <= 8; k++) {
    if (k < 8) {
      int c = 9 + k;
#pragma unroll
      for (int i = c - 8; i <= 8; i++) h = (k == 0 && i == 1) ? mul64(a[i], b[c - i]) : mad64(a[i], b[c - i], h);
      z[k] = (u32)h & M29; h >>= 29;
    } else z[8] = (u32)h;
#pragma unroll
    for (int i = 0; i <= k; i++) l = (k == 0) ? mul64(a[0], b[0]) : mad64(a[i], b[k - i], l);
    l = mad64(z[k], 1216u, l);
    if (k < 8) { o[k] = (u32)l & M29; l >>= 29; }
  }
  o[8] = (u32)l & M23;
  u64 t = (l >> 23) * 19u + o[0];
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}
DEV void f29p_sq(u32 r[9], const u32 a[9]) {
  u32 d[9], o[9], z[9]; u64 h = 0, l = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a[i] << 1;
#pragma unroll
  for (int k = 0; k <= 8; k++) {
    if (k < 8) {
      int c = 9 + k; bool first = (k == 0);
#pragma unroll
      for (int i = c - 8; 2 * i < c; i++) { h = first ? mul64(d[i], a[c - i]) : mad64(d[i], a[c - i], h); first = false; }
      if ((c & 1) == 0) h = mad64(a[c / 2], a[c / 2], h);
      z[k] = (u32)h & M29; h >>= 29;
    } else z[8] = (u32)h;
    bool first = (k == 0);
#pragma unroll
    for (int i = 0; 2 * i < k; i++) { l = mad64(d[i], a[k - i], l); }
    if ((k & 1) == 0) l = first ? mul64(a[0], a[0]) : mad64(a[k / 2], a[k / 2], l);
    l = mad64(z[k], 1216u, l);
    if (k < 8) { o[k] = (u32)l & M29; l >>= 29; }
  }
  o[8] = (u32)l & M23;
  u64 t = (l >> 23) * 19u + o[0];
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}


// high columns kept as unsplit 64-bit sums H_k (independent, no carry chain);
// low column j folds 1216*lo32(H_{j+9}) + 9728*hi32(H_{j+8})
DEV void f29q_mul(u32 r[9], const u32 a[9], const u32 b[9]) {
  u64 H[8]; u32 o[9]; u64 l = 0;
#pragma unroll
  for (int k = 9; k <= 16; k++) {
    H[k - 9] = mul64(a[k - 8], b[8]);
#pragma unroll
    for (int i = k - 7; i <= 8; i++) H[k - 9] = mad64(a[i], b[k - i], H[k - 9]);
  }
#pragma unroll
  for (int k = 0; k <= 8; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) l = (k == 0) ? mul64(a[0], b[0]) : mad64(a[i], b[k - i], l);
    if (k < 8) l = mad64((u32)H[k], 1216u, l);
    if (k > 0) l = mad64((u32)(H[k - 1] >> 32), 9728u, l);
    if (k < 8) { o[k] = (u32)l & M29; l >>= 29; }
  }
  o[8] = (u32)l & M23;
  u64 t = (l >> 23) * 19u + o[0];
  o[0] = (u32)t & M29;
  o[1] += (u32)(t >> 29);
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = o[i];
}

template <bool SER>
__global__ void k_dump(const uint32_t* in, uint32_t* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  u32 a[9], b[9], r[9];
  for (int i = 0; i < 9; ++i) { a[i] = in[t * 18 + i]; b[i] = in[t * 18 + 9 + i]; }
  if (SER) f29q_mul(r, a, b); else f29_mul(r, a, b);
  for (int i = 0; i < 9; ++i) out[t * 36 + i] = r[i];
  if (SER) f29p_sq(r, a); else f29_sq(r, a);
  for (int i = 0; i < 9; ++i) out[t * 36 + 9 + i] = r[i];
  u32 x[9]; for (int i = 0; i < 9; ++i) x[i] = r[i];
  for (int k = 0; k < 100; ++k) { if (SER) f29q_mul(x, x, b); else f29_mul(x, x, b); }
  for (int i = 0; i < 9; ++i) out[t * 36 + 18 + i] = x[i];
  for (int i = 0; i < 9; ++i) x[i] = a[i];
  for (int k = 0; k < 100; ++k) { if (SER) f29p_sq(x, x); else f29_sq(x, x); }
  for (int i = 0; i < 9; ++i) out[t * 36 + 27 + i] = x[i];
}

template <int KIND, int CHAINS>
__global__ __launch_bounds__(256) void k_bench(uint32_t* out, int iters, uint32_t seed) {
  u32 x[9], y[9], z[9];
  for (int i = 0; i < 9; ++i) { x[i] = (seed * (threadIdx.x + 7 * i + 1)) & M29; y[i] = (seed ^ (i * 0x9e3779b9u)) & M29; z[i] = x[i] ^ 0x5555u; }
  x[8] &= M23; y[8] &= M23; z[8] &= M23;
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0) { fe_mul(x, x, y); if (CHAINS > 1) fe_mul(z, z, y); }
    if (KIND == 1) { f29_mul(x, x, y); if (CHAINS > 1) f29_mul(z, z, y); }
    if (KIND == 2) { f29_sq(x, x); if (CHAINS > 1) f29_sq(z, z); }
    if (KIND == 3) { f29s_mul(x, x, y); if (CHAINS > 1) f29s_mul(z, z, y); }
    if (KIND == 4) { f29s_sq(x, x); if (CHAINS > 1) f29s_sq(z, z); }
    if (KIND == 5) { f29p_mul(x, x, y); if (CHAINS > 1) f29p_mul(z, z, y); }
    if (KIND == 6) { f29p_sq(x, x); if (CHAINS > 1) f29p_sq(z, z); }
    if (KIND == 7) { f29q_mul(x, x, y); if (CHAINS > 1) f29q_mul(z, z, y); }
  }
  uint32_t s = 0; for (int i = 0; i < 9; ++i) s ^= x[i] ^ z[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND, int CHAINS>
void run(int cus, uint32_t* out, hipEvent_t e0, hipEvent_t e1, const char* name) {
  int iters = 2000;
  for (int w : {1, 2, 4, 8}) {
    int blocks = cus * w;
    auto launch = [&]() { hipLaunchKernelGGL((k_bench<KIND, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, iters, 3u); };
    launch(); CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0)); for (int r = 0; r < 3; ++r) launch(); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    double ops = 3.0 * blocks * 256 * iters * CHAINS;
    double cyc = (ms * 1e-3) * 2.4e9 / (ops / 64.0 / (cus * 4));
    printf("%-10s chains=%d waves/SIMD=%d : %.3e /s  %.1f SIMD-cycles per wave-level op\n", name, CHAINS, w, ops / (ms * 1e-3), cyc);
  }
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "bench";
  CHK(hipSetDevice(0));
  if (!strcmp(mode, "dump")) {
    int n = atoi(argv[2]);
    std::vector<uint32_t> in(n * 18);
    FILE* f = fopen(argv[3], "rb"); if (!f) return 1; if (fread(in.data(), 4, n * 18, f) != (size_t)n * 18) return 1; fclose(f);
    uint32_t *din, *dout; CHK(hipMalloc(&din, n * 72)); CHK(hipMalloc(&dout, n * 144));
    CHK(hipMemcpy(din, in.data(), n * 72, hipMemcpyHostToDevice));
    if (argc > 5) hipLaunchKernelGGL(k_dump<true>, dim3((n + 255) / 256), dim3(256), 0, 0, din, dout, n);
    else hipLaunchKernelGGL(k_dump<false>, dim3((n + 255) / 256), dim3(256), 0, 0, din, dout, n);
    CHK(hipDeviceSynchronize());
    std::vector<uint32_t> out(n * 36);
    CHK(hipMemcpy(out.data(), dout, n * 144, hipMemcpyDeviceToHost));
    f = fopen(argv[4], "wb"); fwrite(out.data(), 4, n * 36, f); fclose(f);
    printf("dumped %d\n", n);
    return 0;
  }
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  uint32_t* out; CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  run<5, 1>(cus, out, e0, e1, "f29p_mul");
  run<5, 2>(cus, out, e0, e1, "f29p_mul");
  run<6, 1>(cus, out, e0, e1, "f29p_sq");
  run<6, 2>(cus, out, e0, e1, "f29p_sq");
  run<7, 1>(cus, out, e0, e1, "f29q_mul");
  run<7, 2>(cus, out, e0, e1, "f29q_mul");
  return 0;
}
