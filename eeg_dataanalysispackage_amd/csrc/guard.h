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
// A row that fails the test -- its features are close to rounding noise, or X_c is loose -- goes
// to a second stage: the wave that normalises it measures the row's own max |x| per channel
// (guard_measured_x2_wave) and tests again with that X -- in the 3-channel kernels the cheaper
// 3 max_c X_c^2 >= sum_c X_c^2 (rows.h recheck_c3: one wave reduction instead of three; the pass
// is VALU-bound at the power cap).  Only rows that still fail (e.g. a window
// in the filters' null space, an alternating +-A signal) are recomputed with the EXACT filter bank,
// value-identical to the reference, by the same wave inside the same kernel
// (dwt8_exact_row_wave): the 3-channel window kernel, the 32-channel kernel, the one-pass kernels,
// the batch extract and the per-epoch kernel.  Only the generic any-layout window kernel
// (window_wide_kernel) appends its failing rows to `list` for a follow-up launch
// (guard.hip exact_rows_kernel); `count` / `list` are unused elsewhere.
//
// X_c: for int16 recordings a bound known without touching the window,
//   |x| = |fl(fl(raw * r) - b)| <= (32768 |r| + |b|)(1 + 2^-23) for every int16 raw (zero padding
//   included), taken with a 2^-20 margin -- loose when the samples stay far below full scale (a
//   flat stretch decodes to ~1e-3 against X ~ 6e3), hence the second stage; for float32 recordings
//   and caller-supplied double epochs the measured max |x| of the window from the start (no
//   a-priori bound exists).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace eegfx {

// tools/fma_bound.py (tests/test_taps.py checks these against it): the collapsed four-point filter
// of the batch and 32-channel kernels, the level-by-level fma cascade of features_small_kernel, and
// the six-point form of window4_kernel (4 lanes per signal, A/B builds).
constexpr double kGuardK2Collapsed = 7.02e-05;
constexpr double kGuardK2Cascade = 1.62e-04;
constexpr double kGuardK2Toom6 = 2.16e-04;

// Device state of a guarded launch: `count` flagged rows so far and their epoch indices in `list`
// (window_wide_kernel only: zeroed before the launch that fills it, capacity the launch's epochs),
// the running total of rows recomputed under EXACT since the context was created, and of rows that
// failed the a-priori test and went to the second stage (`rechecked`; may be null)
// (eegfx_ctx_guard_stats / eegfx_ctx_guard_detail).  total == nullptr disables the guard (EXACT).
// `total` and `rechecked` are running counters spread over kGuardSlots slots, one per 128-byte
// line, a workgroup adding into slot blockIdx % kGuardSlots: one shared word took every
// workgroup's atomic in turn, which at a 10 % flag rate cost as much as the kernel itself
// (profiles/r05h: 0.733 -> 1.398 ms).  The host sums the slots.
constexpr int kGuardSlots = 256;
constexpr int kGuardSlotWords = 16;  // 128 B
constexpr size_t kGuardSlotBytes = sizeof(unsigned long long) * kGuardSlots * kGuardSlotWords;
struct Guard {
  int* count;
  int64_t* list;
  unsigned long long* total;
  unsigned long long* rechecked = nullptr;
  // the 3-channel window kernel's guard strategy (fused.hip, EEGFX_TRACK_X): adapt[0] = 1 when
  // the previous launch sent more than 1/16 of its rows to the second stage (every lane then
  // tracks max |x| while decoding, so no row needs the scan), set by baseline_kernel from
  // adapt[1] (the rechecked total it last saw) and adapt[2] (that launch's rows); may be null
  unsigned long long* adapt = nullptr;
  // host-mapped word that baseline_kernel sets to the strategy it chose from adapt (the host picks
  // the window kernel's variant for its next launch from it); may be null
  unsigned int* track_out = nullptr;
};

// The guard's second stage in the fma 3-channel window kernel (fused.hip), two strategies:
//   scan   the a-priori int16 bound for every row, and a scan of the staged windows for the rows
//          it flags (channel_x2_rows): free while few rows are flagged;
//   track  every lane keeps the largest |x| of the samples it decodes (one v_max3_f32 per pair,
//          +3 % per step), so every row has its measured X_c and no flagged row needs the scan
//          (+0.8 % at a 32 % flag rate, where the scan costs +8 %).
// 1 (product) = adaptive: the host launches the tracking variant when the last launch's
// baseline_kernel found that the launch before sent more than 1/16 of its rows to the second
// stage; 0 = always scan, 2 = always track (A/B builds).
#ifndef EEGFX_TRACK_X
#define EEGFX_TRACK_X 1
#endif

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

__device__ __forceinline__ void guard_slot_add(unsigned long long* slots, unsigned long long v) {
  atomicAdd(slots + (blockIdx.x & (kGuardSlots - 1)) * kGuardSlotWords, v);
}
// The window kernel's guard strategy for the launch that follows (Guard::adapt, EEGFX_TRACK_X),
// by the first wave of a baseline pass's block 0 (lane = tid < 64): track when the previous
// launch sent more than 1/16 of its rows to the second stage.  adapt[1] is the rechecked total
// seen last, as a signed offset (a host counter reset subtracts the total it clears, so the
// difference still counts the launches since); the choice also goes to the host-mapped word the
// host reads when it picks the window kernel's variant.
__device__ __forceinline__ void guard_adapt_update(const unsigned long long* rechecked,
                                                   unsigned long long* adapt,
                                                   unsigned int* track_out, int64_t n, int lane) {
  unsigned long long t = 0;
  for (int i = lane; i < kGuardSlots; i += 64) t += rechecked[i * kGuardSlotWords];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
  if (lane == 0) {
    const long long delta = (long long)t - (long long)adapt[1];
    const unsigned long long nprev = adapt[2];
    unsigned long long mode = adapt[0];
    if (delta >= 0) mode = nprev > 0 && (unsigned long long)delta * 16 > nprev ? 1ull : 0ull;
    adapt[0] = mode;
    adapt[1] = t;
    adapt[2] = (unsigned long long)n;
    if (track_out)
      __hip_atomic_store(track_out, (unsigned int)mode, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// rows recomputed with the EXACT cascade
__device__ __forceinline__ void guard_count_recomputed(const Guard& g, unsigned long long rows) {
  guard_slot_add(g.total, rows);
}
// rows that went to the second stage
__device__ __forceinline__ void guard_count_rechecked(const Guard& g, int rows) {
  if (g.rechecked && rows) guard_slot_add(g.rechecked, (unsigned long long)rows);
}

// Wave-wide minimum of packed int16 pairs (every lane gets it): the 16 lanes of a DPP row by
// quad_perm xor 1 / xor 2, row_half_mirror and row_mirror (no LDS), then across the four rows.
__device__ __forceinline__ uint32_t wave_pk_min_i16(uint32_t v) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  auto mn = [](uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(s2, a),
                                                                  __builtin_bit_cast(s2, b)));
  };
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
  v = mn(v, (uint32_t)__shfl_xor((int)v, 16, 64));
  return mn(v, (uint32_t)__shfl_xor((int)v, 32, 64));
}

// lane j's v (j wave-uniform), as a wave-uniform value
__device__ __forceinline__ double lane_value(double v, int j) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), j);
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

// Wave-wide maximum of unsigned words (every lane gets it), the same moves as wave_pk_min_i16.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
  v = max(v, (uint32_t)__shfl_xor((int)v, 16, 64));
  return max(v, (uint32_t)__shfl_xor((int)v, 32, 64));
}

// Packs a lane's (min, max) of int16 samples as (min, ~max) so that one packed minimum reduces
// both (min(~a, ~b) = ~max(a, b), no overflow); unpack with guard_unpack_min / _max.
__device__ __forceinline__ uint32_t guard_pack_minmax(int mn, int mx) {
  return ((uint32_t)mn & 0xFFFFu) | ((uint32_t)~mx << 16);
}
__device__ __forceinline__ int guard_unpack_min(uint32_t p) { return (int)(int16_t)(p & 0xFFFFu); }
__device__ __forceinline__ int guard_unpack_max(uint32_t p) { return ~(int)(int16_t)(p >> 16); }

// The second stage, by one wave (every lane calls it; the result is wave-uniform): sum over the
// row's C signals of X_c^2, X_c = max_k |x_c[k]| over the 512 window samples, measured.
// sample(c, k) returns the int16 raw value of sample k of channel c (0 for the zero padding past
// the recording's end); the decode x = fl(fl(raw * r) - b) is monotone in raw, so X_c =
// max(|x(min raw)|, |x(max raw)|) with decode(c, v) the kernels' own fp32 decode.  16 lanes (one
// DPP row) per channel, four channels per pass; each lane's 32 reads are independent.  The
// 2^-20 margin covers the rounding of the sum.
template <typename Sample, typename Decode>
__device__ __forceinline__ double guard_measured_x2_wave(Sample sample, Decode decode, int C,
                                                         int lane) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  auto mn = [](uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(s2, a),
                                                                  __builtin_bit_cast(s2, b)));
  };
  const int grp = lane >> 4, l = lane & 15;
  double sx = 0.0;
#pragma unroll 1
  for (int c0 = 0; c0 < C; c0 += 4) {
    const int c = c0 + grp < C ? c0 + grp : C - 1;
    int lo = 32767, hi = -32768;
#pragma unroll 8
    for (int k = l; k < 512; k += 16) {
      const int v = sample(c, k);
      lo = min(lo, v);
      hi = max(hi, v);
    }
    uint32_t p = guard_pack_minmax(lo, hi);  // reduced over the DPP row = this channel's lanes
    p = mn(p, (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0xB1, 0xF, 0xF, true));
    p = mn(p, (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0x4E, 0xF, 0xF, true));
    p = mn(p, (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0x141, 0xF, 0xF, true));
    p = mn(p, (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0x140, 0xF, 0xF, true));
    const double X = fmax(fabs(decode(c, (float)guard_unpack_min(p))),
                          fabs(decode(c, (float)guard_unpack_max(p))));
    double x2 = c0 + grp < C ? X * X : 0.0;
    x2 += __shfl_xor(x2, 16, 64);
    x2 += __shfl_xor(x2, 32, 64);
    sx += x2;
  }
  return sx * (1.0 + 0x1p-20);
}

}  // namespace dev
}  // namespace eegfx
