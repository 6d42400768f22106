// Probe: achievable HBM rate of the fused path's access pattern with no arithmetic -- per epoch
// the 600-byte baseline span [pos-100, pos) and the 3,072-byte window [pos+175, pos+687) of a
// 3-channel int16 recording (6,000-byte epoch stride), 16-byte loads, plus a 384-byte row store.
// Also a plain contiguous copy for the reference rate.  (DESIGN.md "Roofline".)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// one wave per epoch: 230 quads of window+baseline (misaligned spans rounded out to 16 B)
__global__ __launch_bounds__(256) void pattern(const uint8_t* raw, const int64_t* pos, int64_t n,
                                               double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (e >= n) return;
  const int64_t p = pos[e];
  const int64_t b0 = ((p - 100) * 6) & ~15, b1 = ((p + 175) * 6) & ~15;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // window: 193 quads
    const int q = lane + 64 * k;
    if (q < 193) {
      const u4 v = *(const u4*)(raw + b1 + 16 * q);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (lane < 39) {  // baseline: 39 quads
    const u4 v = *(const u4*)(raw + b0 + 16 * lane);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (lane < 24) {
    double2 d = make_double2((double)acc, (double)lane);
    *(double2*)(out + e * 48 + 2 * lane) = d;
  }
}

// baseline span only (what baseline_kernel reads): one thread per quad, 39 quads per epoch,
// plus one 16-byte store per epoch (baselines + window word)
__global__ __launch_bounds__(256) void baseline_pattern(const uint8_t* raw, const int64_t* pos,
                                                        int64_t n, u4* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e = t / 39;
  const int q = (int)(t - e * 39);
  if (e >= n) return;
  const int64_t b0 = ((pos[e] - 100) * 6) & ~15;
  const u4 v = __builtin_nontemporal_load((const u4*)(raw + b0 + 16 * q));
  const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
  const uint32_t r = __shfl_xor(x, 1, 64) ^ x;
  if (q == 0) out[e] = (u4){r, 0u, 0u, 0u};
}

__global__ __launch_bounds__(256) void copy(const u4* src, u4* dst, int64_t nq) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int main() {
  const int64_t n = 1000000, nf = 1000 * n + 2000;
  uint8_t* raw;
  int64_t* pos;
  double* out;
  (void)hipMalloc(&raw, nf * 6);
  (void)hipMalloc(&pos, n * 8);
  (void)hipMalloc(&out, n * 48 * 8);
  (void)hipMemset(raw, 1, nf * 6);
  int64_t* hp = new int64_t[n];
  for (int64_t i = 0; i < n; ++i) hp[i] = 1000 + 1000 * i;
  (void)hipMemcpy(pos, hp, n * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms;
  const dim3 g((unsigned)((n * 64 + 255) / 256));
  hipLaunchKernelGGL(pattern, g, dim3(256), 0, 0, raw, pos, n, out);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(pattern, g, dim3(256), 0, 0, raw, pos, n, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  const double alg = 4064.0 * n;  // 3,672 in + 8 pos + 384 out
  const double touched = (232.0 * 16 + 8 + 384) * n;
  printf("pattern: %.4f ms  algorithmic %.1f GB/s  touched %.1f GB/s\n", ms, alg / ms / 1e6,
         touched / ms / 1e6);
  {
    const dim3 gb((unsigned)((n * 39 + 255) / 256));
    hipLaunchKernelGGL(baseline_pattern, gb, dim3(256), 0, 0, raw, pos, n, (u4*)out);
    (void)hipEventRecord(a);
    for (int r = 0; r < 20; ++r)
      hipLaunchKernelGGL(baseline_pattern, gb, dim3(256), 0, 0, raw, pos, n, (u4*)out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= 20;
    printf("baseline span only: %.4f ms  algorithmic %.1f GB/s (620 B/epoch)  touched %.1f GB/s\n",
           ms, 620.0 * n / ms / 1e6, (39.0 * 16 + 16 + 8) * n / ms / 1e6);
  }
  const int64_t nq = nf * 6 / 32;  // copy half the recording into the other half
  hipLaunchKernelGGL(copy, dim3(4096), dim3(256), 0, 0, (const u4*)raw, (u4*)(raw + nq * 16), nq);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r)
    hipLaunchKernelGGL(copy, dim3(4096), dim3(256), 0, 0, (const u4*)raw, (u4*)(raw + nq * 16), nq);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  printf("copy:    %.4f ms  %.1f GB/s (read+write)\n", ms, 2.0 * nq * 16 / ms / 1e6);
  return 0;
}
