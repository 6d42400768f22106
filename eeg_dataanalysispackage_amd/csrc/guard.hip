// guard.hip -- the follow-up launch of the fma numerics' conditioning guard (guard.h) for the
// generic any-layout kernels (wide.hip window_wide_kernel; the 3- and 32-channel window kernels and
// the batch extract recompute their flagged rows themselves, dwt8_exact_row_wave).
//
// The generic kernels append every row whose sum of squares fails the guard to a list; this kernel
// recomputes exactly those rows with the EXACT filter bank (dwt8_cascade<false>: each tap one
// rounded multiply and one rounded add in the reference's order, WaveletTransform.java:126-137)
// and the reference's sequential normalisation (SignalProcessing.java:38-52), overwriting the fma
// rows in place.  The samples are decoded exactly as the fused kernels decode them,
// (double)((float)raw * res - b) with the baseline the baseline kernel wrote (Baseline.java:29-42),
// so a recomputed row is value-identical to the EXACT path's row.
//
// Launched right after the guarded kernel on the same stream with a fixed grid that reads the
// device-side count: no host synchronisation; when nothing was flagged every workgroup exits after
// one load (~4-5 us per launch, profiles/r04d).  Rows are few; each is read straight from memory.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dwt8.h"
#include "guard.h"
#include "launch.h"

namespace eegfx {

// The follow-up launch: kGuardGrid workgroups of kGuardBlock threads loop over the flagged rows
// (one row per workgroup at a time, 8 lanes per signal).  Small, because it runs after every
// guarded launch and nearly always finds the list empty: 128 x 256 measured 4.8 us per launch
// (2.7 us minimum) on the bench step (profiles/r04c); an input that flags many rows is still
// recomputed correctly, at 16 rows at a time.
constexpr int kGuardGrid = 16;
constexpr int kGuardBlock = 128;

namespace dev {

// Window samples of (epoch e, channel c) from the multiplexed recording: frame pos + 175 + k.
template <typename T>
struct RawWindows {
  const uint8_t* raw;
  int64_t n_frames;
  int ct;
  ChanSel sel;
  const int64_t* pos;
  const float* base;  // [n][C] baselines of the baseline kernel
  int C;
  // x[0..72) = samples [64 s, 64 s + 72) mod 512 of the window, decoded
  __device__ __forceinline__ void window(int64_t e, int c, int s, double (&x)[kIn]) const {
    const int64_t p0 = pos[e];
    const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : (int64_t)kPre;  // as the kernels
    const float r = sel.res[c];
    const float b = base[e * C + c];
    const int col = sel.col[c];
#pragma unroll
    for (int k = 0; k < kIn; ++k) {
      const int64_t f = p + 175 + ((kSegLen * s + k) & (kWin - 1));
      // Arrays.copyOfRange zero-pads past the end of the recording (toFloatArray -> 0.0f)
      const float v = f < n_frames ? (float)*(const T*)(raw + (f * ct + col) * (int64_t)sizeof(T))
                                   : 0.0f;
      float y = v * r;
      y = y - b;
      x[k] = (double)y;
    }
  }
};

template <typename Src>
__global__ __launch_bounds__(kGuardBlock) void exact_rows_kernel(Src src, int nfeat, Guard g,
                                                                 double* __restrict__ out) {
  __shared__ double feat[kMaxChannels * 16];
  __shared__ double norm;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, s = lane & 7;
  constexpr int SIG = kGuardBlock / 8;  // signals per pass
  const int cnt = *g.count;  // written by the guarded kernel before this launch
  if (blockIdx.x == 0 && tid == 0 && cnt > 0) guard_count_recomputed(g, (unsigned long long)cnt);
  const int C = src.C;
  const int F = C * nfeat;
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {  // uniform
    const int64_t e = g.list[i];
    for (int c0 = 8 * w; c0 < C; c0 += SIG) {  // uniform per wave
      const int c = c0 + (lane >> 3);
      const bool valid = c < C;
      double x[kIn];
      src.window(e, valid ? c : 0, s, x);
      double a6, d6;
      dwt8_cascade<false, true>(x, nullptr, lane & ~7, s, a6, d6);
      if (valid) {
        if (s < nfeat) feat[c * nfeat + s] = a6;
        if (8 + s < nfeat) feat[c * nfeat + 8 + s] = d6;
      }
    }
    __syncthreads();
    if (tid == 0) {  // Math.pow(f, 2) summed in index order
      double acc = 0.0;
      for (int k = 0; k < F; ++k) acc = acc + feat[k] * feat[k];
      norm = sqrt(acc);
    }
    __syncthreads();
    for (int k = tid; k < F; k += kGuardBlock) out[e * F + k] = feat[k] / norm;
    __syncthreads();
  }
}

}  // namespace dev

hipError_t launch_guard_fixup_raw(hipStream_t st, const void* raw, int fmt, int64_t n_frames,
                                  int ct, const ChanSel& sel, int C, const int64_t* pos,
                                  const void* scratch, const Guard& g, double* out) {
  if (!g.count) return hipSuccess;
  if (fmt == 0) {
    dev::RawWindows<int16_t> src{(const uint8_t*)raw, n_frames, ct, sel, pos,
                                 (const float*)scratch, C};
    hipLaunchKernelGGL(dev::exact_rows_kernel<dev::RawWindows<int16_t>>, dim3(kGuardGrid),
                       dim3(kGuardBlock), 0, st, src, 16, g, out);
  } else {
    dev::RawWindows<float> src{(const uint8_t*)raw, n_frames, ct, sel, pos, (const float*)scratch,
                               C};
    hipLaunchKernelGGL(dev::exact_rows_kernel<dev::RawWindows<float>>, dim3(kGuardGrid),
                       dim3(kGuardBlock), 0, st, src, 16, g, out);
  }
  return hipGetLastError();
}

}  // namespace eegfx
