// Probe: ways for 16 lanes to load one epoch's 3,072-byte window (configs[1] layout: 1M windows,
// 6,000 bytes apart, window byte offsets = 10 mod 16) straight into VGPRs, at HBM scale.
//   mode 0  lane t loads its own 192 bytes from the window's (2-byte aligned) offset: 12 unaligned
//           16-byte loads (what window_direct_kernel does)
//   mode 1  lane t loads 13 aligned quads from floor16 and realigns with v_alignbyte
//   mode 2  lane t loads 12 aligned quads from floor16 (no realignment: the bandwidth ceiling of
//           the per-lane pattern)
//   mode 3  coalesced: load k of lane t reads quad 16k + t of the window (12 loads, 256 contiguous
//           bytes per 16 lanes), i.e. the bytes land in the wrong lanes
// Each lane folds its dwords into one value so the loads stay live.  Prints ms per launch.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u4a2 __attribute__((ext_vector_type(4), aligned(2)));
typedef uint32_t u4a16 __attribute__((ext_vector_type(4), aligned(16)));

template <int MODE>
__global__ __launch_bounds__(256) void load_kernel(const uint8_t* __restrict__ raw, int64_t n,
                                                   uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63, t = lane & 15;
  const int64_t e = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (e >= n) return;
  const int64_t B = 7050 + 6000 * e;
  uint32_t acc = 0;
  if constexpr (MODE == 0) {
    const u4a2* p = (const u4a2*)(raw + B + 192 * t);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const u4a2 v = __builtin_nontemporal_load(p + i);
      acc = acc * 3 + (v.x ^ v.y) + (v.z ^ v.w);
    }
  } else if constexpr (MODE == 1) {
    const int64_t A = B + 192 * t;
    const u4a16* p = (const u4a16*)(raw + (A & ~(int64_t)15));
    const uint32_t sh = (uint32_t)(A & 15);
    uint32_t d[52];
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      const u4a16 v = __builtin_nontemporal_load(p + i);
      d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
    }
    const uint32_t w = sh >> 2, b = (sh & 3) * 8;
#pragma unroll
    for (int k = 0; k < 48; ++k) {
      // dword k of the realigned stream: bytes sh + 4k .. of the aligned block
      const uint32_t lo = w == 0 ? d[k] : w == 1 ? d[k + 1] : w == 2 ? d[k + 2] : d[k + 3];
      const uint32_t hi = w == 0 ? d[k + 1] : w == 1 ? d[k + 2] : w == 2 ? d[k + 3] : d[k + 4];
      const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, b >> 3);
      acc = acc * 3 + v;
    }
  } else if constexpr (MODE == 2) {
    const u4a16* p = (const u4a16*)(raw + ((B + 192 * t) & ~(int64_t)15));
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const u4a16 v = __builtin_nontemporal_load(p + i);
      acc = acc * 3 + (v.x ^ v.y) + (v.z ^ v.w);
    }
  } else {
    const u4a16* p = (const u4a16*)(raw + (B & ~(int64_t)15));
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const u4a16 v = __builtin_nontemporal_load(p + 16 * i + t);
      acc = acc * 3 + (v.x ^ v.y) + (v.z ^ v.w);
    }
  }
  out[e * 16 + t] = acc;
}

int main() {
  const int64_t n = 1000000, bytes = 6000 * n + 16384;
  uint8_t* raw;
  uint32_t* out;
  (void)hipMalloc(&raw, bytes);
  (void)hipMalloc(&out, n * 16 * 4);
  (void)hipMemset(raw, 1, bytes);
  const int iters = getenv("PROBE_ITERS") ? atoi(getenv("PROBE_ITERS")) : 200;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const dim3 g((unsigned)((n + 15) / 16)), blk(256);
  auto run = [&](int mode) {
    switch (mode) {
      case 0: hipLaunchKernelGGL(load_kernel<0>, g, blk, 0, 0, raw, n, out); break;
      case 1: hipLaunchKernelGGL(load_kernel<1>, g, blk, 0, 0, raw, n, out); break;
      case 2: hipLaunchKernelGGL(load_kernel<2>, g, blk, 0, 0, raw, n, out); break;
      default: hipLaunchKernelGGL(load_kernel<3>, g, blk, 0, 0, raw, n, out); break;
    }
  };
  for (int mode = 0; mode < 4; ++mode) {
    for (int r = 0; r < 20; ++r) run(mode);
    (void)hipEventRecord(a);
    for (int r = 0; r < iters; ++r) run(mode);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double per = ms / iters;
    printf("mode %d: %.4f ms per launch, %.2f TB/s of window bytes  %s\n", mode, per,
           3072.0 * n / (per * 1e-3) / 1e12, hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
