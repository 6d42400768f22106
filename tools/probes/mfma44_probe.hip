// Probe: v_mfma_f64_4x4x4f64 on gfx950 -- (1) its operand layout, from a product of known
// matrices, and (2) its rate under sustained load (PROBE_LAUNCHES back-to-back launches; socket
// power sampled from outside by tools/fp64_energy.sh).  Decides whether levels 1-5 of the fma
// filter bank could run as 4x4x4 blocks on the matrix pipe.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void layout(double* out) {
  const int l = threadIdx.x;
  // A value = 1000 + lane, B value = lane: D = sum_k A[i][k] B[k][j] reveals which lanes feed
  // which output when A or B is a one-hot: run 1: A one-hot at lane a, B = 1 everywhere -> the
  // outputs that receive A[a]'s row; run 2 the same for B.
  for (int a = 0; a < 64; ++a) {
    const double A = l == a ? 1.0 : 0.0;
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(A, 1.0, 0.0, 0, 0, 0);
    out[a * 64 + l] = d;
    const double B = l == a ? 1.0 : 0.0;
    d = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, B, 0.0, 0, 0, 0);
    out[4096 + a * 64 + l] = d;
  }
}

__global__ __launch_bounds__(512) void rate(double* out, int iters) {
  double acc[8];
  const double a = 1.0 + threadIdx.x * 1e-3, b = 0.5;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i];
  if (s == 12345.0) *out = s;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 8192 * 8);
  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, d);
  double h[8192];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // for each source lane, the destination lanes it reaches
  for (int which = 0; which < 2; ++which) {
    printf("%s lane -> output lanes:\n", which ? "B" : "A");
    for (int a = 0; a < 64; ++a) {
      printf("  %2d:", a);
      for (int l = 0; l < 64; ++l)
        if (h[which * 4096 + a * 64 + l] != 0.0) printf(" %d", l);
      printf("\n");
    }
  }
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int iters = 8192, reps = getenv("PROBE_LAUNCHES") ? atoi(getenv("PROBE_LAUNCHES")) : 20;
  const dim3 grid(p.multiProcessorCount * 4), block(512);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rate, grid, block, 0, 0, d, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(rate, grid, block, 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double macs = (double)grid.x * 8 * iters * 8 * 256;
  printf("mfma_f64_4x4x4: %.3f ms per launch, %.2f TF (fp64, 2 flop/MAC)\n", ms, 2 * macs / ms / 1e9);
  return 0;
}
