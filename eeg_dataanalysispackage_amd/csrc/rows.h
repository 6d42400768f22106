// rows.h -- normalisation and store of the feature rows of an 8-epoch sub-tile, shared by the
// fused window kernel (fused.hip) and the one-pass getData + features kernel (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dwt8.h"
#include "guard.h"
#include "launch.h"

namespace eegfx {
namespace dev {

// SignalProcessing.normalize (SignalProcessing.java:38-52) for the <= 8 feature rows of a
// sub-tile, executed by one wave.  `fb` holds the rows in LDS; `norm` is an 8-double LDS scratch
// owned by the calling wave.
//   EXACT: lane e < ne folds Math.pow(f, 2) over row e in index order (the 8 dependent chains run
//          side by side), then the 64 lanes divide and store (16-byte stores).
//   FMA:   (1e-9 contract) the 8 lanes of an epoch each square-sum F/8 features, a 3-step
//          butterfly completes the row sum, and the row is scaled by 1/sqrt (rsqrt_nr: within an
//          ulp or two of x / s; an all-zero row still gives NaN = 0 * inf); the scaled rows go
//          back to LDS and leave as contiguous non-temporal 1 KB wave stores (storing each lane's
//          16-byte pieces 48 B apart cost 1,114 instead of 384 written bytes per row).  A row
//          whose sum of squares fails the conditioning guard (guard.h; gx = the C per-signal X^2)
//          goes to the second stage: recheck(e), a wave-collective call, returns the row's
//          measured sum of X_c^2, and only rows that fail again are recomputed under EXACT by
//          redo(e, row) into their row slots before the store (rare: never on the bench workload),
//          and counted in the guard's running total.  Every recheck runs before the first redo,
//          whose LDS scratch may overwrite the staged windows that a recheck reads.
struct NoRedo {
  __device__ void operator()(int, double*) const {}
};
struct NoRecheck {  // no second stage: every flagged row is recomputed
  __device__ double operator()(int) const { return __builtin_inf(); }
};
template <int F, bool FAST, int C = F / 16, typename Redo = NoRedo, typename Recheck = NoRecheck>
__device__ __forceinline__ void normalise_store(double* fb, double* norm, double* o, int ne,
                                                int lane, const double* gx = nullptr,
                                                Guard g = Guard{nullptr, nullptr, nullptr},
                                                Redo redo = Redo{}, Recheck recheck = Recheck{}) {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  if constexpr (FAST) {
    static_assert(F % 16 == 0, "8 lanes per row, pairs of features");
    constexpr int P = F / 8;
    const int e = lane >> 3, p = lane & 7;
    double v[P];
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      v[i] = e < ne ? fb[e * F + p * P + i] : 0.0;
      acc = __builtin_fma(v[i], v[i], acc);
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    bool fails = false;
    if (EEGFX_GUARD && g.total && p == 0 && e < ne) {
      double sx = 0.0;
#pragma unroll
      for (int c = 0; c < C; ++c) sx += gx[e * C + c];
      fails = guard_fails(acc, kGuardK2Collapsed, sx);
    }
    const double inv = rsqrt_nr(acc);
    if (e < ne) {
#pragma unroll
      for (int i = 0; i < P; i += 2)
        *(double2*)(fb + e * F + p * P + i) = make_double2(v[i] * inv, v[i + 1] * inv);
    }
    wave_sync();
    uint64_t flagged = __ballot(fails);  // bit 8e: row e failed the a-priori test
    if (flagged) {                        // uniform, rare
      uint64_t left = 0;                  // rows that fail the measured test too
      for (uint64_t f = flagged; f; f &= f - 1) {
        const int e1 = __ffsll((unsigned long long)f) - 1;
        const double acc_e = lane_value(acc, e1);  // e1 is wave-uniform
        // the verdict is wave-uniform: a scalar branch keeps `left` in SGPRs
        if (__builtin_amdgcn_readfirstlane(
                guard_fails(acc_e, kGuardK2Collapsed, recheck(e1 >> 3)) ? 1 : 0))
          left |= 1ull << e1;
      }
      if (lane == 0) {
        guard_count_rechecked(g, __popcll(flagged));
        if (left) guard_count_recomputed(g, (unsigned long long)__popcll(left));
      }
      for (; left; left &= left - 1) {
        const int e1 = __ffsll((unsigned long long)left) - 1;
        redo(e1 >> 3, fb + (e1 >> 3) * F);
      }
    }
    for (int i = 2 * lane; i < ne * F; i += 128)
      __builtin_nontemporal_store(*(const f64x2*)(fb + i), (f64x2*)(o + i));
    wave_sync();
    (void)norm;
    return;
  }
  if (lane < ne) {
    double acc = 0.0;
#pragma unroll 16
    for (int i = 0; i < F; ++i) {
      const double f = fb[lane * F + i];
      acc = acc + f * f;
    }
    norm[lane] = sqrt(acc);
  }
  wave_sync();
  for (int i = 2 * lane; i < ne * F; i += 128) {
    const double v0 = fb[i] / norm[i / F];
    const double v1 = fb[i + 1] / norm[(i + 1) / F];
    *(double2*)(o + i) = make_double2(v0, v1);
  }
  wave_sync();
}

// The conditioning guard's second stage (guard.h) for one row of the 3-channel kernels, by one
// wave: lane l reads frames 64 (l >> 3) + 8 (l & 7) .. + 7 of the window, all three channels --
// from the staged window `lds` (the window kernel's layout: segment s at 16 SEGQ s bytes past the
// epoch's misalignment) or, when from_raw, from the recording (zero past its end, the reference's
// padding) -- keeps each channel's min and max raw sample, decodes those six extremes exactly as
// the kernel decodes every sample (x = fl(fl(raw * r) - b) is monotone in raw, so they bound the
// lane's |x|), and takes one wave maximum: X = max_c max |x_c|.  It returns 3 X^2 >= sum_c X_c^2,
// a rigorous bound at most 3x looser than the per-channel sum (which would cost three wave
// reductions: this pass is VALU-bound at the power cap, ~50 instead of ~100 VALU per row).
// One LDS (or memory) round trip for all 24 samples of a lane.
template <int FB, int SEGQ>
__device__ __forceinline__ double recheck_c3(const uint8_t* __restrict__ raw, int64_t n_frames,
                                             const ChanSel& sel, int64_t W,
                                             const float* __restrict__ b, const uint8_t* lds,
                                             bool from_raw, int lane) {
  const int f0 = 8 * lane;  // = 64 (lane >> 3) + 8 (lane & 7)
  int v[3][8];
  if (from_raw) {  // wave-uniform
    const int64_t B = W & ~(int64_t)1;
    const int64_t g0 = B / FB + f0;
    if (B / FB + kWin <= n_frames) {  // wave-uniform: the whole window inside, no per-load test
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          v[c][i] = *(const int16_t*)(raw + B + (int64_t)(f0 + i) * FB + 2 * sel.col[c]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          v[c][i] = g0 + i < n_frames
                        ? *(const int16_t*)(raw + B + (int64_t)(f0 + i) * FB + 2 * sel.col[c])
                        : 0;
    }
  } else {
    const uint8_t* p = lds + ((uint32_t)W & 14u) + 16 * SEGQ * (lane >> 3) +
                       FB * 8 * (lane & 7);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c][i] = *(const int16_t*)(p + FB * i + 2 * sel.col[c]);
  }
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  float xm = 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int mn = v[c][0], mx = v[c][0];
#pragma unroll
    for (int i = 1; i < 8; ++i) {
      mn = min(mn, v[c][i]);
      mx = max(mx, v[c][i]);
    }
    // (lo, hi) decoded as one pair: packed fp32 multiply and add, each lane rounded as the
    // scalar fl(fl(raw * r) - b)
    const float r = sel.res[c], bc = b[c];
    f32x2 x = f32x2{(float)mn, (float)mx} * f32x2{r, r};
    x = x + f32x2{-bc, -bc};
    xm = fmaxf(xm, fmaxf(fabsf(x.x), fabsf(x.y)));
  }
  // |x| >= 0: its bit pattern orders like the value
  const double X = (double)__uint_as_float(wave_max_u32(__float_as_uint(xm)));
  return (X * X) * (3.0 * (1.0 + 0x1p-20));  // the constant is exact: 3 + 3 * 2^-20
}

}  // namespace dev
}  // namespace eegfx
