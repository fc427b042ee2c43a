// Phase timing of the step kernel's 32 x 32 matrix-core Cholesky solve
// (dx_device.h mfma_chol_solve32) in isolation, at the step kernel's occupancy
// (one 64-lane wave per workgroup, 20 KB of LDS each: 8 per CU).  Each wave solves
// R systems A x = b with a 30 x 30 SPD A held in LDS and reports the mean cycles per
// solve.  Variants:
//   0  the solve with s_memtime stamps (and a wait) between its phases: init, factor,
//      row stores, forward, column loads, backward
//   1  0 with bank-conflict-free row stores and unconditional init loads
//   2  1 with the right-hand side as row / column 31 (forward substitution folded into
//      the factorisation)
//   3  dx_device.h's mfma_chol_solve32 itself, one stamp
//   4  0 with one stamp (what 0 costs without the phase waits)
// The stamps' waits change the schedule: 1 and 2 gain 0.2 k / 0.75 k cycles per solve
// against 0, but the same changes in the real function (3) measured 13.0 k against 4's
// 13.0 k, so they were not kept.
//   hipcc --offload-arch=gfx950 -O3 -I dexterity_amd/csrc tools/probes/chol_bench.hip -o /tmp/chol_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "dx_device.h"

constexpr int NPH = 6;  // init, factor, T stores, forward, column loads, backward

__device__ __forceinline__ void stamp(unsigned long long* acc, int k, unsigned long long& last) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  unsigned long long t = __builtin_amdgcn_s_memtime();
  if (LANE == 0) acc[k] += t - last;
  last = t;
}

// mfma_chol_solve32 with stamps (same code path as dx_device.h, n = 30, dj = 0)
template <int V0>
__device__ void solve_stamped(const float* A, int n, float* x, float* T, unsigned long long* acc) {
  constexpr int V = V0 == 4 ? 0 : V0;
  constexpr bool quiet = V0 == 4;  // one stamp at the end
  unsigned long long last = __builtin_amdgcn_s_memtime();
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  dx_f16v C;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    const int ra = max(i, j), rb = min(i, j);
    const bool in = i < n && j < n;
    if (V == 0) {
      C[v] = in ? A[ti(ra) + rb] : (i == j ? 1.f : 0.f);
    } else {
      const float a = A[in ? ti(ra) + rb : 0];  // unconditional load (padding lanes broadcast slot 0)
      C[v] = in ? a : (i == j ? 1.f : 0.f);
    }
    if (V == 2 && i == 31 && j < n) C[v] = x[j];
    if (V == 2 && j == 31 && i < n) C[v] = x[i];
  }
  float b = l < n ? x[l] : 0.f;
  SYNC();
  if (!quiet) stamp(acc, 0, last);
  float Lr[32];
  float dinv = 0.f;
  float y = 0.f;
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C[vk], up), rk1 = half_dup(C[vk + 1], up);
    const float i11 = __builtin_amdgcn_rsqf(fmaxf(rl(rk, k), 1e-30f));
    const float l21 = rl(rk1, k) * i11;
    const float i22 = __builtin_amdgcn_rsqf(fmaxf(rl(rk1, k + 1) - l21 * l21, 1e-30f));
    dinv = wl(dinv, i11, k);
    dinv = wl(dinv, i22, k + 1);
    const float lk = rk * i11;
    const float lk1 = (rk1 - lk * l21) * i22;
    Lr[k] = j > k ? lk : 0.f;
    Lr[k + 1] = j > k + 1 ? lk1 : 0.f;
    const float p = j > k + 1 ? (hi ? lk1 : lk) : 0.f;
    C = __builtin_amdgcn_mfma_f32_32x32x2f32(-p, p, C, 0, 0, 0);
    if (V == 2) {
      if (k < n) y = wl(y, rl(lk, 31), k);
      if (k + 1 < n) y = wl(y, rl(lk1, 31), k + 1);
    }
  }
  if (!quiet) {
    float z = C[0] + C[15];  // wait for the last MFMA
    asm volatile("" ::"v"(z));
  }
  if (!quiet) stamp(acc, 1, last);
  const int i = l;
  if (V == 0) {
#pragma unroll
    for (int k = 0; k < 32; k++) T[(k < i && i < n) ? ti(i) + k : 0] = Lr[k];
  } else if (i < n) {
    // each lane its own row; entries on / past the diagonal go to the row's own
    // diagonal slot (never read): for a fixed k the 30 rows hit 30 distinct banks
#pragma unroll
    for (int k = 0; k < 32; k++) T[ti(i) + min(k, i)] = Lr[k];
  }
  if (!quiet) stamp(acc, 2, last);
  if (V != 2) {
#pragma unroll
    for (int k = 0; k < 32; k++) {
      float yk = rl(b, k) * rl(dinv, k);
      y = wl(y, yk, k);
      b = fmaf(-Lr[k], yk, b);
    }
  }
  SYNC();
  if (!quiet) stamp(acc, 3, last);
  const int ic = min(i, n - 1);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    float v = T[ti(k) + ic];
    Lr[k] = ic < k && k < n ? v : 0.f;
  }
  if (!quiet) stamp(acc, 4, last);
  float xo = 0.f;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    float xk = rl(y, k) * rl(dinv, k);
    xo = wl(xo, xk, k);
    y = fmaf(-Lr[k], xk, y);
  }
  if (i < n) x[i] = xo;
  SYNC();
  stamp(acc, quiet ? 0 : 5, last);
}

template <int V>
__global__ __launch_bounds__(64) void bench(int reps, unsigned long long* out, float* res) {
  extern __shared__ float smem[];
  const int n = 30;
  float* A0 = smem;          // pristine SPD matrix (packed lower)
  float* A = smem + 512;     // working copy (factor transposes through it)
  float* x = smem + 1024;
  unsigned long long acc[NPH] = {0, 0, 0, 0, 0, 0};
  for (int k = LANE; k < ti(n); k += 64) {
    int r = 0;
    while (ti(r + 1) <= k) r++;
    int c = k - ti(r);
    float h = 0.37f * __sinf(0.7f * r + 1.3f * c + blockIdx.x);
    A0[k] = r == c ? 4.0f + 0.1f * r : 0.1f * h;
  }
  SYNC();
  float sum = 0.f;
  for (int it = 0; it < reps; it++) {
    for (int k = LANE; k < ti(n); k += 64) A[k] = A0[k];
    if (LANE < n) x[LANE] = 1.0f + 0.01f * LANE + it;
    SYNC();
    if (V == 3) {  // the kernel's own mfma_chol_solve32 (dx_device.h), total only
      unsigned long long last = __builtin_amdgcn_s_memtime();
      mfma_chol_solve32(A, n, 0.f, x, A);
      stamp(acc, 0, last);
    } else {
      solve_stamped<V>(A, n, x, A, acc);
    }
    sum += LANE < n ? x[LANE] : 0.f;
  }
  if (LANE == 0)
    for (int k = 0; k < NPH; k++) atomicAdd(out + k, acc[k]);
  res[blockIdx.x * 64 + LANE] = sum;
}

int main() {
  const int grid = 2048, reps = 200;
  unsigned long long* out;
  float* res;
  (void)hipMalloc(&out, NPH * 8);
  (void)hipMalloc(&res, grid * 64 * 4);
  const char* names[NPH] = {"init", "factor", "T stores", "forward", "column loads", "backward"};
  std::vector<float> r0(grid * 64), r1(grid * 64), r2(grid * 64), r3(grid * 64);
  for (int V = 0; V < 5; V++) {
    (void)hipMemset(out, 0, NPH * 8);
    if (V == 0) hipLaunchKernelGGL(bench<0>, dim3(grid), dim3(64), 20 * 1024, 0, reps, out, res);
    else if (V == 1) hipLaunchKernelGGL(bench<1>, dim3(grid), dim3(64), 20 * 1024, 0, reps, out, res);
    else if (V == 2) hipLaunchKernelGGL(bench<2>, dim3(grid), dim3(64), 20 * 1024, 0, reps, out, res);
    else if (V == 3) hipLaunchKernelGGL(bench<3>, dim3(grid), dim3(64), 20 * 1024, 0, reps, out, res);
    else hipLaunchKernelGGL(bench<4>, dim3(grid), dim3(64), 20 * 1024, 0, reps, out, res);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    unsigned long long h[NPH];
    (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipMemcpy(V == 0 ? r0.data() : V == 1 ? r1.data() : V == 2 ? r2.data() : V == 3 ? r3.data() : r0.data(), res, grid * 64 * 4,
                    hipMemcpyDeviceToHost);
    double tot = 0;
    for (int k = 0; k < NPH; k++) tot += (double)h[k] / ((double)grid * reps);
    printf("variant %d\n", V);
    for (int k = 0; k < NPH; k++)
      printf("  %-14s %8.1f cycles per solve (%.1f %%)\n", names[k], (double)h[k] / ((double)grid * reps),
             100.0 * h[k] / ((double)grid * reps) / tot);
    printf("  total          %8.1f\n", tot);
  }
  double md = 0, md2 = 0, md3 = 0;
  for (int k = 0; k < grid * 64; k++) {
    md = fmax(md, fabs((double)r0[k] - r1[k]));
    md2 = fmax(md2, fabs((double)r0[k] - r2[k]) / fmax(1.0, fabs((double)r0[k])));
    md3 = fmax(md3, fabs((double)r0[k] - r3[k]) / fmax(1.0, fabs((double)r0[k])));
  }
  printf("max |variant 0 - variant 1| of the summed solutions: %g; variant 2 relative: %g; variant 3 (dx_device.h) "
         "relative: %g\n", md, md2, md3);
  return 0;
}
