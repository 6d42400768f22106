// launch.h -- host-side launchers of the gfx950 kernels (kernels.hip, fused.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace eegfx {

constexpr int kMaxChannels = 64;

// Selected channels, passed by value as a kernel argument: 0-based column in the multiplexed
// frame and the .vhdr resolution (narrowed to float, as the reference multiplies in fp32).
struct ChanSel {
  int32_t col[kMaxChannels];
  float res[kMaxChannels];
};

hipError_t launch_cut_epochs(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                             const ChanSel& sel, int C, const int64_t* pos, int64_t n, double* out);
hipError_t launch_features_from_epochs(hipStream_t st, const double* ep, int64_t n, int C, int skip,
                                       int nfeat, bool fast, double* out);
hipError_t launch_synth(hipStream_t st, int16_t* dst, int64_t n_frames, int ct, uint64_t seed);

// Fused raw -> features (baseline_kernel + window_kernel, fused.hip).  `scratch` holds
// fused_scratch_bytes(n, C) bytes of device memory (the per-epoch baselines).  Returns
// hipErrorNotSupported (without launching) when no fused kernel covers (fmt, ct, C); the caller
// then runs cut + features through a device scratch buffer.
size_t fused_scratch_bytes(int64_t n, int C);
hipError_t launch_fused_features(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 bool fast, void* scratch, double* out);

}  // namespace eegfx
