// Probe: throughput and (with amd-smi sampled by tools/pipe_energy.sh) socket power of the
// instruction mixes an exact-integer matrix-core form of the dwt-8 operator would run
// (DESIGN.md §6): the window kernel's v_fma_f64 against v_pk_fma_f32 (the
// decode residuals), v_mfma_i32_16x16x64_i8 (M_q . v in int8 limbs) and v_mfma_f32_16x16x32_f16
// (M . e in f16 limbs).  Every CU runs 8 waves per SIMD of one mode back to back for a few
// seconds; operands change every iteration (constant operands flatter both pipes' energy).
//   PROBE_MODE=0..3 PROBE_LAUNCHES=N tools/probes/pipe_energy_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int i4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 4096;

__global__ __launch_bounds__(512) void probe(int mode, int iters, int* out) {
  const int t = threadIdx.x + blockIdx.x * 512;
  if (mode == 0) {  // 8 independent fp64 fma chains
    double a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = 1.0 + t * 1e-7 + i;
    double m = 1.0000001, c = 1e-9 * t;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_fma(a[i], m, c);
      m += 1e-17;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    if (s == 12345.0) out[0] = 1;
  } else if (mode == 1) {  // 8 independent packed fp32 fma chains (2 lanes of fp32 each)
    f2 a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (f2){1.0f + t * 1e-7f + i, 2.0f - i};
    f2 m = {1.0000001f, 0.9999999f}, c = {1e-9f * t, 2e-9f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_fma(a[i], m, c);
      m.x += 1e-12f;
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
    if (s == 12345.0f) out[0] = 1;
  } else if (mode == 2) {  // int8 MFMA, 4 independent accumulators, B changes every iteration
    i4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (i4){t, i, 0, 1};
    i4 a = {0x01fe7f80 ^ t, 0x7f017f01, (int)0x80818283 ^ t, 0x11223344};
    i4 b = {0x05060708, 0x090a0b0c ^ t, 0x7e7d7c7b, 0x01020304};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
      b.x += 0x01010101;
      b.z ^= it;
    }
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
    if (s == 12345) out[0] = 1;
  } else {  // f16 MFMA, 4 independent accumulators
    f4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = (f4){(float)t, (float)i, 0.f, 1.f};
    h8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = (_Float16)(0.001f * (t % 97 + i));
      b[i] = (_Float16)(0.002f * (i + 1));
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
      b[0] += (_Float16)0.001f;
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
    if (s == 12345.0f) out[0] = 1;
  }
}

int main() {
  const int mode = getenv("PROBE_MODE") ? atoi(getenv("PROBE_MODE")) : 0;
  const int launches = getenv("PROBE_LAUNCHES") ? atoi(getenv("PROBE_LAUNCHES")) : 200;
  int* d = nullptr;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  const int grid = 256 * 4;  // 4 workgroups of 8 waves per CU: 8 waves per SIMD
  hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, mode, kIters, d);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < launches; ++i)
    hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, mode, kIters, d);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const double waves = (double)grid * 8 * launches;
  // per wave and iteration: mode 0: 8 fma_f64 x 64 lanes; 1: 8 pk_fma x 128 fp32 fma;
  // 2: 4 MFMA x 16x16x64 MACs; 3: 4 MFMA x 16x16x32 MACs
  const double ops[4] = {8.0 * 64, 8.0 * 128, 4.0 * 16 * 16 * 64, 4.0 * 16 * 16 * 32};
  const double instr[4] = {8, 8, 4, 4};
  const double rate = waves * kIters * ops[mode] / s;
  const char* name[4] = {"v_fma_f64", "v_pk_fma_f32", "v_mfma_i32_16x16x64_i8",
                         "v_mfma_f32_16x16x32_f16"};
  printf("mode %d %s: %.3f s, %.4g MAC/s, %.4g wave-instr/s\n", mode, name[mode], s, rate,
         waves * kIters * instr[mode] / s);
  (void)hipFree(d);
  return 0;
}
