// guard.h -- the conditioning guard of the fma numerics.
//
// Both numerics filter the SAME decoded doubles x (the fp32 decode and baseline are order-exact in
// both), so an fma row differs from the EXACT (reference-order) row only by fp64 rounding.
// tools/fma_bound.py propagates rigorous bounds through both filter banks, operation by operation
// in the kernels' order: |f_fma - f_exact| <= E * X per coefficient for a signal whose samples
// satisfy |x_i| <= X.  The normalised rows then differ by at most 2 |f_fma - f_exact| / |f_fma|
// (SignalProcessing.java:38-52 divides by the norm), so a row is certified within 0.5e-9 (half of
// the north_star's 1e-9; the normalisations' own rounding, ~1e-15, takes the rest) when
//     |f_fma|^2 >= K2 * sum_c X_c^2,     K2 = (2 / 0.5e-9)^2 * 8 (E_a6^2 + E_d6^2) * 1.25.
// A row that fails the test -- its features are close to rounding noise, e.g. a window in the
// filters' null space (an alternating +-A signal) -- is appended to the guard list, and a
// follow-up launch (guard.hip exact_rows_kernel) recomputes exactly those rows with the EXACT
// filter bank, value-identical to the reference.
//
// X_c: for int16 recordings a bound known without touching the window,
//   |x| = |fl(fl(raw * r) - b)| <= (32768 |r| + |b|)(1 + 2^-23) for every int16 raw (zero padding
//   included), taken with a 2^-20 margin; for float32 recordings and caller-supplied double epochs
//   the measured max |x| of the window (no a-priori bound exists).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace eegfx {

// tools/fma_bound.py (tests/test_taps.py checks these against it): the collapsed four-point filter
// of the fused and batch kernels, and the level-by-level fma cascade of features_small_kernel.
constexpr double kGuardK2Collapsed = 7.02e-05;
constexpr double kGuardK2Cascade = 1.62e-04;

// Device state of a guarded launch: `count` flagged rows so far (zeroed before the launch that
// fills it), their epoch indices in `list` (capacity: the launch's epochs), and the running total
// of recomputed rows since the context was created (eegfx_ctx_guard_stats).  count == nullptr
// disables the guard (EXACT numerics).
struct Guard {
  int* count;
  int64_t* list;
  unsigned long long* total;
};

namespace dev {

// X_c^2 for an int16 signal with resolution r and baseline b (see the header comment).
__device__ __forceinline__ double guard_x2_int16(float r, float b) {
  const double X = (32768.0 * fabs((double)r) + fabs((double)b)) * (1.0 + 0x1p-20);
  return X * X;
}

// Appends epoch e to the guard list (rare: rows whose features are rounding-level).
__device__ __forceinline__ void guard_flag(const Guard& g, int64_t e) {
  const int i = atomicAdd(g.count, 1);
  g.list[i] = e;
}

// sum of squares `acc` against the row's threshold; NaN fails (and is recomputed as EXACT).
__device__ __forceinline__ bool guard_fails(double acc, double k2, double sum_x2) {
  return !(acc >= k2 * sum_x2);
}

}  // namespace dev
}  // namespace eegfx
