// Probe: fp64 issue rates on gfx950 -- VALU v_fma_f64, MFMA v_mfma_f64_16x16x4f64, and both
// pipes at once (separate waves of one workgroup, and interleaved inside one wave).  Decides
// whether any of the dwt-8 filter bank can move to the matrix pipe (DESIGN.md "Alternatives").
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 8192;

__device__ __forceinline__ void valu_loop(double seed, double* out, int iters) {
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed + i;
  const double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_fma(a[i], m, c);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  if (s == 12345.0) *out = s;
}

__device__ __forceinline__ void mfma_loop(double seed, double* out, int iters) {
  d4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = (d4){seed, seed, seed, seed};
  const double a = seed * 0.5, b = seed * 0.25;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  if (s == 12345.0) *out = s;
}

// mode 0: all waves VALU; 1: all waves MFMA; 2: waves 0-3 VALU, 4-7 MFMA; 3: each wave both
__global__ __launch_bounds__(512) void probe(int mode, double* out, int iters) {
  const int w = threadIdx.x >> 6;
  const double seed = 1.0 + threadIdx.x * 1e-3;
  if (mode == 4 || mode == 5) {
    double a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed + i;
    const double m = 1.0000001;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = mode == 4 ? a[i] + m : a[i] * m;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    if (s == 12345.0) *out = s;
    return;
  }
  if (mode == 0) valu_loop(seed, out, iters);
  else if (mode == 1) mfma_loop(seed, out, iters);
  else if (mode == 2) {
    if (w < 4) valu_loop(seed, out, iters);
    else mfma_loop(seed, out, iters);
  } else {
    double a[8];
    d4 acc[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed + i;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (d4){seed, seed, seed, seed};
    const double m = 1.0000001, c = 1e-9, x = seed * 0.5, y = seed * 0.25;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_fma(a[i], m, c);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
    if (s == 12345.0) *out = s;
  }
}

int main() {
  double* out;
  (void)hipMalloc(&out, 64);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const dim3 grid(cus * 4), block(512);  // 32 waves / CU: 8 per SIMD
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[6] = {"valu fma_f64", "mfma_f64_16x16x4", "split valu|mfma waves", "interleaved", "valu add_f64", "valu mul_f64"};
  // PROBE_MODE=m: run mode m back to back for PROBE_LAUNCHES launches (socket power / clock
  // sampled from outside, tools/fp64_energy.sh), then report its rate like the sweep below
  const int only = getenv("PROBE_MODE") ? atoi(getenv("PROBE_MODE")) : -1;
  const int reps = getenv("PROBE_LAUNCHES") ? atoi(getenv("PROBE_LAUNCHES")) : 5;
  for (int mode = 0; mode < 6; ++mode) {
    if (only >= 0 && mode != only) continue;
    hipLaunchKernelGGL(probe, grid, block, 0, 0, mode, out, kIters);
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(probe, grid, block, 0, 0, mode, out, kIters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double waves = (double)grid.x * 8;
    // per wave-iteration: VALU 8 x 64 FMA, MFMA 4 x 1024 FMA
    double valu_fma = 0, mfma_fma = 0;
    if (mode == 0 || mode >= 4) valu_fma = waves * kIters * 8 * 64;
    if (mode == 1) mfma_fma = waves * kIters * 4 * 1024;
    if (mode == 2) { valu_fma = waves / 2 * kIters * 8 * 64; mfma_fma = waves / 2 * kIters * 4 * 1024; }
    if (mode == 3) { valu_fma = waves * kIters * 8 * 64; mfma_fma = waves * kIters * 4 * 1024; }
    printf("%-24s %8.3f ms  valu %7.2f TF  mfma %7.2f TF  total %7.2f TF (fp64, 2 flop/FMA)\n",
           names[mode], ms, 2 * valu_fma / ms / 1e9, 2 * mfma_fma / ms / 1e9,
           2 * (valu_fma + mfma_fma) / ms / 1e9);
  }
  return 0;
}
