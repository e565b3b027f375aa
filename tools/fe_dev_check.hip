// dev check: device fe_mul/fe_sq/fe_mul2/fe_sq2 vs Python big ints
#include "../firedancer_amd/csrc/fd_ed25519_dev.h"
#include <cstdio>
#include <vector>
__global__ void k(const u32* in, u32* out, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x; if (t >= n) return;
  fe a, b, r, s;
  for (int i = 0; i < 9; i++) { a.v[i] = in[t*18+i]; b.v[i] = in[t*18+9+i]; }
  fe_mul(r, a, b); for (int i = 0; i < 9; i++) out[t*54+i] = r.v[i];
  fe_sq(r, a);     for (int i = 0; i < 9; i++) out[t*54+9+i] = r.v[i];
  fe_mul2(r, a, b, s, b, b); for (int i = 0; i < 9; i++) { out[t*54+18+i] = r.v[i]; out[t*54+27+i] = s.v[i]; }
  fe_sq2(r, a, s, b); for (int i = 0; i < 9; i++) { out[t*54+36+i] = r.v[i]; out[t*54+45+i] = s.v[i]; }
}
int main(int argc, char** argv) {
  int n = atoi(argv[1]); std::vector<u32> in(n*18), out(n*54);
  FILE* f = fopen(argv[2], "rb"); if (fread(in.data(), 4, n*18, f) != (size_t)n*18) return 1; fclose(f);
  u32 *di, *dout; hipMalloc(&di, n*72); hipMalloc(&dout, n*216); hipMemcpy(di, in.data(), n*72, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n+255)/256), dim3(256), 0, 0, di, dout, n); hipDeviceSynchronize();
  hipMemcpy(out.data(), dout, n*216, hipMemcpyDeviceToHost); f = fopen(argv[3], "wb"); fwrite(out.data(), 4, n*54, f); fclose(f);
  printf("ok %d\n", n); return 0;
}
