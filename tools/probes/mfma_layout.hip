// Probe (GPU box): operand/result lane layout of v_mfma_f32_32x32x2_f32 and the
// semantics of v_permlane32_swap on gfx950, as used by the MFMA Cholesky.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f16v __attribute__((ext_vector_type(16)));
__global__ void probe(float* out) {
  int l = threadIdx.x;
  f16v z = {};
  // A[i][k] = i + 100 k (hypothesis: lane l holds A[l % 32][l / 32]); B[k][j] = [k == 0]
  f16v d1 = __builtin_amdgcn_mfma_f32_32x32x2f32((float)(l % 32 + 100 * (l / 32)), l / 32 == 0 ? 1.f : 0.f, z, 0, 0, 0);
  // A[i][k] = [k == 0]; B[k][j] = j + 100 k (hypothesis: lane l holds B[l / 32][l % 32])
  f16v d2 = __builtin_amdgcn_mfma_f32_32x32x2f32(l / 32 == 0 ? 1.f : 0.f, (float)(l % 32 + 100 * (l / 32)), z, 0, 0, 0);
  for (int v = 0; v < 16; v++) { out[v * 64 + l] = d1[v]; out[1024 + v * 64 + l] = d2[v]; }
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint((float)l), __float_as_uint((float)(100 + l)), false, false);
  out[2048 + l] = __uint_as_float(r[0]);
  out[2112 + l] = __uint_as_float(r[1]);
}
int main() {
  float* d; hipMalloc(&d, 4096 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[4096]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  bool rows_ok = true, cols_ok = true;
  for (int l = 0; l < 64; l++)
    for (int v = 0; v < 16; v++) {
      int i = 8 * (v / 4) + 4 * (l / 32) + (v % 4), j = l % 32;
      if (h[v * 64 + l] != (float)i) rows_ok = false;
      if (h[1024 + v * 64 + l] != (float)j) cols_ok = false;
    }
  printf("D[i][j] at lane l, vgpr v with i = 8*(v/4) + 4*(l/32) + v%%4, j = l%%32: rows %s cols %s\n", rows_ok ? "ok" : "MISMATCH", cols_ok ? "ok" : "MISMATCH");
  printf("lane 0..3 v0..3 of d1: %g %g %g %g | lane 32: %g\n", h[0], h[64], h[128], h[192], h[32]);
  printf("permlane32_swap(x=lane, y=100+lane): r0 lanes 0,31,32,63 = %g %g %g %g ; r1 = %g %g %g %g\n",
         h[2048], h[2048 + 31], h[2048 + 32], h[2048 + 63], h[2112], h[2112 + 31], h[2112 + 32], h[2112 + 63]);
  return 0;
}
