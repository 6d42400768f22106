// plan.hip -- marker planning (a4 + a8, OffLineDataProvider.java:200-265) as a parallel scan.
//
// The reference walks the markers in order with one piece of state, the class balance
// D = targets - non-targets accepted so far (:248-260): a target is accepted iff D <= 0 (D += 1),
// a non-target iff D >= 0 (D -= 1), and a marker whose cut would leave the recording
// (position - 100 outside [0, n_frames], the caught AIOOBE of :220-225, :262-264) changes nothing.
// Starting from 0, D never leaves {-1, 0, 1}, so every marker is a map of that 3-element set and
// the walk is a prefix composition of such maps -- associative, so it scans in
// parallel:
//   1. plan_maps_kernel   marker -> map (2 bits per input state), first unparsable index
//   2. rocprim exclusive_scan of the maps under composition -> each marker's input state
//   3. plan_flags_kernel  accept flag from the input state
//   4. rocprim exclusive_scan of the flags -> output slot; plan_scatter_kernel writes
//      position and label (1.0 target / 0.0) of every accepted marker in order.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstring>

#include <rocprim/device/device_scan.hpp>

#include "launch.h"

namespace eegfx {
namespace dev {

// state s in {-1, 0, 1} is coded s + 1; a map packs f(-1), f(0), f(1) in bits 0-1, 2-3, 4-5
constexpr uint8_t kIdentity = 0 | (1 << 2) | (2 << 4);
constexpr uint8_t kTarget = 1 | (2 << 2) | (2 << 4);     // D <= 0 -> D + 1
constexpr uint8_t kNonTarget = 0 | (0 << 2) | (1 << 4);  // D >= 0 -> D - 1

__host__ __device__ __forceinline__ int apply_map(uint8_t m, int code) {
  return (m >> (2 * code)) & 3;
}

struct ComposeMaps {  // (a then b)
  __host__ __device__ __forceinline__ uint8_t operator()(uint8_t a, uint8_t b) const {
    return (uint8_t)(apply_map(b, apply_map(a, 0)) | (apply_map(b, apply_map(a, 1)) << 2) |
                     (apply_map(b, apply_map(a, 2)) << 4));
  }
};

__device__ __forceinline__ bool in_range(int64_t pos, int64_t n_frames) {
  const int64_t lo = pos - 100;
  return lo >= 0 && lo <= n_frames;
}

__global__ void plan_maps_kernel(const int64_t* __restrict__ pos, const int32_t* __restrict__ stim,
                                 int64_t n, int64_t n_frames, int32_t guessed,
                                 uint8_t* __restrict__ maps, unsigned long long* first_bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = stim[i];
    if (s == INT32_MIN) atomicMin(first_bad, (unsigned long long)i);  // Integer.parseInt NFE
    uint8_t m = kIdentity;
    if (in_range(pos[i], n_frames)) m = ((int64_t)s + 1 == (int64_t)guessed) ? kTarget : kNonTarget;
    maps[i] = m;
  }
}

__global__ void plan_flags_kernel(const int64_t* __restrict__ pos, const int32_t* __restrict__ stim,
                                  int64_t n, int64_t n_frames, int32_t guessed, int d0_code,
                                  const uint8_t* __restrict__ prefix, uint32_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t f = 0;
    if (in_range(pos[i], n_frames)) {
      const int d = apply_map(prefix[i], d0_code) - 1;
      const bool target = (int64_t)stim[i] + 1 == (int64_t)guessed;
      f = target ? (d <= 0) : (d >= 0);
    }
    flags[i] = f;
  }
}

__global__ void plan_scatter_kernel(const int64_t* __restrict__ pos,
                                    const int32_t* __restrict__ stim, int64_t n, int32_t guessed,
                                    const uint32_t* __restrict__ flags,
                                    const int64_t* __restrict__ slot, int64_t* __restrict__ pos_out,
                                    double* __restrict__ label_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (!flags[i]) continue;
    const int64_t k = slot[i];
    if (pos_out) pos_out[k] = pos[i];
    if (label_out) label_out[k] = ((int64_t)stim[i] + 1 == (int64_t)guessed) ? 1.0 : 0.0;
  }
}

}  // namespace dev

namespace {
unsigned grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}
}  // namespace

size_t plan_scratch_bytes(int64_t n) {
  size_t a = 0, b = 0;
  (void)rocprim::exclusive_scan(nullptr, a, (const uint8_t*)nullptr, (uint8_t*)nullptr,
                                dev::kIdentity, (size_t)n, dev::ComposeMaps());
  (void)rocprim::exclusive_scan(nullptr, b, (const uint32_t*)nullptr, (int64_t*)nullptr,
                                (int64_t)0, (size_t)n, rocprim::plus<int64_t>());
  const size_t tmp = (a > b ? a : b) + 256;
  // maps, prefix (1 B each), flags (4 B), slots (8 B), first_bad (8 B), scan temp
  return (size_t)n * (1 + 1 + 4 + 8) + 64 + 8 + tmp + 4 * 256;
}

static uint8_t* align256(uint8_t* p) { return (uint8_t*)(((uintptr_t)p + 255) & ~(uintptr_t)255); }

hipError_t launch_plan_markers(hipStream_t st, const int64_t* pos, const int32_t* stim, int64_t n,
                               int64_t n_frames, int32_t guessed, int d0, void* scratch,
                               int64_t* pos_out, double* label_out, PlanResult* result) {
  uint8_t* p = align256((uint8_t*)scratch);
  uint8_t* maps = p;
  p = align256(p + n);
  uint8_t* prefix = p;
  p = align256(p + n);
  uint32_t* flags = (uint32_t*)p;
  p = align256(p + 4 * n);
  int64_t* slot = (int64_t*)p;
  p = align256(p + 8 * n);
  unsigned long long* first_bad = (unsigned long long*)p;
  p = align256(p + 8);
  void* tmp = p;
  size_t a = 0, b = 0;
  hipError_t e;
  if ((e = rocprim::exclusive_scan(nullptr, a, maps, prefix, dev::kIdentity, (size_t)n,
                                   dev::ComposeMaps(), st)) != hipSuccess)
    return e;
  if ((e = rocprim::exclusive_scan(nullptr, b, flags, slot, (int64_t)0, (size_t)n,
                                   rocprim::plus<int64_t>(), st)) != hipSuccess)
    return e;
  const unsigned long long none = ~0ull;
  if ((e = hipMemcpyAsync(first_bad, &none, 8, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(dev::plan_maps_kernel, dim3(grid_for(n)), dim3(256), 0, st, pos, stim, n,
                     n_frames, guessed, maps, first_bad);
  unsigned long long bad = none;
  if ((e = hipMemcpyAsync(&bad, first_bad, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  // an unparsable description aborts the reference's loop there: plan the prefix before it
  const int64_t m = bad == none ? n : (int64_t)bad;
  result->first_unparsable = bad == none ? -1 : (int64_t)bad;
  result->selected = 0;
  result->balance = d0;
  if (m == 0) return hipSuccess;
  if ((e = rocprim::exclusive_scan(tmp, a, maps, prefix, dev::kIdentity, (size_t)m,
                                   dev::ComposeMaps(), st)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(dev::plan_flags_kernel, dim3(grid_for(m)), dim3(256), 0, st, pos, stim, m,
                     n_frames, guessed, d0 + 1, prefix, flags);
  if ((e = rocprim::exclusive_scan(tmp, b, flags, slot, (int64_t)0, (size_t)m,
                                   rocprim::plus<int64_t>(), st)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(dev::plan_scatter_kernel, dim3(grid_for(m)), dim3(256), 0, st, pos, stim, m,
                     guessed, flags, slot, pos_out, label_out);
  uint8_t last_prefix = 0, last_map = 0;
  uint32_t last_flag = 0;
  int64_t last_slot = 0;
  if ((e = hipMemcpyAsync(&last_prefix, prefix + m - 1, 1, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(&last_map, maps + m - 1, 1, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(&last_flag, flags + m - 1, 4, hipMemcpyDeviceToHost, st)) ||
      (e = hipMemcpyAsync(&last_slot, slot + m - 1, 8, hipMemcpyDeviceToHost, st)))
    return e;
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  result->selected = last_slot + last_flag;
  result->balance = dev::apply_map(dev::ComposeMaps()(last_prefix, last_map), d0 + 1) - 1;
  return hipGetLastError();
}

}  // namespace eegfx
