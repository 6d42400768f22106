// Probe: throughput of the dwt8 cascade alone (inputs synthesised in registers, no LDS staging,
// no HBM reads) for 1M epochs x 3 channels, exact vs FMA, halo via bpermute vs LDS slots.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../eeg_dataanalysispackage_amd/csrc/dwt8.h"
using namespace eegfx::dev;

template <bool FAST, bool SHFL, int MINW>
__global__ __launch_bounds__(256, MINW) void cascade(double* out, int64_t npairs) {
  __shared__ __attribute__((aligned(16))) double xch[SHFL ? 2 : 4 * 64 * kSlot];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t pair = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int s = lane & 7;
  double x[kIn];
#pragma unroll
  for (int k = 0; k < kIn; ++k) x[k] = (double)(float)((pair * 131 + s * 64 + k) & 1023) * 0.1;
  double a6, d6;
  dwt8_cascade<FAST, SHFL>(x, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
  if (pair < npairs) out[pair * 16 + s] = a6 + d6;
}

template <bool FAST, bool SHFL, int MINW>
float run(double* out, int64_t npairs) {
  const int64_t threads = npairs * 8;
  dim3 grid((unsigned)(threads / 256));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((cascade<FAST, SHFL, MINW>), grid, dim3(256), 0, 0, out, npairs);
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((cascade<FAST, SHFL, MINW>), grid, dim3(256), 0, 0, out, npairs);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const int64_t npairs = 3000000;  // 1M epochs x 3 channels
  double* out; (void)hipMalloc(&out, npairs * 16 * sizeof(double));
  printf("exact shfl minw4: %.3f ms\n", run<false, true, 4>(out, npairs));
  printf("fma   shfl minw4: %.3f ms\n", run<true, true, 4>(out, npairs));
  printf("exact lds  minw3: %.3f ms\n", run<false, false, 3>(out, npairs));
  printf("fma   lds  minw3: %.3f ms\n", run<true, false, 3>(out, npairs));
  printf("exact shfl minw2: %.3f ms\n", run<false, true, 2>(out, npairs));
  printf("fma   shfl minw2: %.3f ms\n", run<true, true, 2>(out, npairs));
  printf("fma   shfl minw3: %.3f ms\n", run<true, true, 3>(out, npairs));
  printf("fma   lds  minw2: %.3f ms\n", run<true, false, 2>(out, npairs));
  printf("fma   shfl minw1: %.3f ms\n", run<true, true, 1>(out, npairs));
  return 0;
}
