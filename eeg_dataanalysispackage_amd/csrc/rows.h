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
//          goes to the second stage: recheck(flagged, acc), a wave-collective call on the mask of
//          flagged rows (bit 8e = row e) and this lane's row sum of squares, returns the mask of
//          rows that fail the test with their measured X too (per_row_recheck adapts a per-row
//          X^2 functor; recheck_c3_rows tests all of a sub-tile's rows in one pass).  Only those
//          rows are recomputed under EXACT by redo(e, row) into their row slots before the store
//          (rare: never on the bench workload), and counted in the guard's running total.  Every
//          recheck runs before the first redo, whose LDS scratch may overwrite the staged windows
//          that a recheck reads.
struct NoRedo {
  __device__ void operator()(int, double*) const {}
};
struct NoRecheck {  // no second stage: every flagged row is recomputed
  __device__ uint64_t operator()(uint64_t flagged, double) const { return flagged; }
};
// The second stage one row at a time: x2(e), a wave-collective call, returns row e's measured
// sum of X_c^2 (recheck_c3 or guard_measured_x2_wave).
template <typename X2>
struct PerRowRecheck {
  X2 x2;
  __device__ __forceinline__ uint64_t operator()(uint64_t flagged, double acc) const {
    uint64_t left = 0;
    for (uint64_t f = flagged; f; f &= f - 1) {
      const int e1 = __ffsll((unsigned long long)f) - 1;
      const double acc_e = lane_value(acc, e1);  // e1 is wave-uniform
      // the verdict is wave-uniform: a scalar branch keeps `left` in SGPRs
      if (__builtin_amdgcn_readfirstlane(guard_fails(acc_e, kGuardK2Collapsed, x2(e1 >> 3)) ? 1 : 0))
        left |= 1ull << e1;
    }
    return left;
  }
};
template <typename X2>
__device__ __forceinline__ PerRowRecheck<X2> per_row_recheck(X2 x2) {
  return PerRowRecheck<X2>{x2};
}
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
      uint64_t left = recheck(flagged, acc);  // rows that fail the measured test too
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

// The second stage for the flagged rows of a 3-channel window kernel's sub-tile in one pass
// (window_kernel): the rows whose staged windows are still in LDS (epochs 1-7) share the wave,
// 64 / L of them side by side, L = 64, 32, 16 or 8 lanes per row for 1, 2, 3-4, 5-7 rows; each
// lane scans 512 / L consecutive frames of its row in runs of 8 frames with packed int16 minimum /
// maximum.  A run is 24 int16 words, the three columns interleaved; it is read as 13 aligned dwords
// from the dword that holds its first word, so when the run starts mid-dword (per row: the
// window's misalignment mod 4) the first dword also carries the word before the run and otherwise
// the last dword carries the two words after it -- both real samples of the recording next to the
// frames scanned (the staged quads hold them), which can only loosen the bound.  The dwords fall in
// three classes by index mod 3 whose halves hold two columns each -- (0, 1), (2, 0), (1, 2), or
// rotated by one class when the run starts mid-dword -- so one packed operation updates two
// columns' extremes.  Each column's min and max are then decoded for every selected channel
// exactly as the kernel decodes samples (x = fl(fl(raw * r) - b) is monotone in raw), and max |x|
// is reduced over the row's lanes: X = max_c max |x_c|, tested as 3 X^2 >= sum_c X_c^2, as
// recheck_c3 does.  Epoch 0's window lies under the rows: recheck0() tests it from the recording
// (recheck_c3).  win: the sub-tile's LDS windows (epoch e from byte e * EBYTES, 4-byte aligned;
// segment s at 16 SEGQ s bytes past the epoch's misalignment); delta: the misalignment of the
// lane's epoch (lane >> 3); base: the sub-tile's [8][3] baselines.
template <int SEGQ, int EBYTES, typename Recheck0>
__device__ __forceinline__ uint64_t recheck_c3_rows(uint64_t flagged, double acc,
                                                    const ChanSel& sel,
                                                    const float* __restrict__ base,
                                                    const uint8_t* win, int delta, int lane,
                                                    Recheck0 recheck0) {
  constexpr int FB = 6;
  static_assert(EBYTES % 4 == 0 && SEGQ * 16 >= 64 * FB + 16, "dword-aligned epochs, runs fit");
  typedef short s2 __attribute__((ext_vector_type(2)));
  auto pmin = [](uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(s2, a),
                                                                  __builtin_bit_cast(s2, b)));
  };
  auto pmax = [](uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, a),
                                                                  __builtin_bit_cast(s2, b)));
  };
  uint64_t left = 0;
  if (flagged & 1ull) {  // uniform
    if (__builtin_amdgcn_readfirstlane(
            guard_fails(lane_value(acc, 0), kGuardK2Collapsed, recheck0()) ? 1 : 0))
      left |= 1ull;
  }
  // rows 1-7: the slots' epochs, 4 bits each (uniform)
  uint32_t T = 0;
  int k = 0;
#pragma unroll
  for (int e = 1; e < 8; ++e)
    if ((flagged >> (8 * e)) & 1ull) { T |= (uint32_t)e << (4 * k); ++k; }
  if (k == 0) return left;
  const int sh = k <= 1 ? 6 : k <= 2 ? 5 : k <= 4 ? 4 : 3;  // log2(L)
  const int j = lane >> sh, sub = lane & ((1 << sh) - 1);
  const bool valid = j < k;
  const int e = valid ? (int)((T >> (4 * j)) & 15u) : (int)(T & 15u);
  const int de = __shfl(delta, 8 * e, 64);  // even
  const bool mid = (de & 2) != 0;           // runs start mid-dword (6 f, 16 SEGQ s are 0 mod 4)
  const uint32_t* wp = (const uint32_t*)(win + e * EBYTES + (de & ~3));
  const int fpl = 512 >> sh;  // frames per lane: 8, 16, 32, 64
  uint32_t mn[3], mx[3];
  auto run = [&](int f, bool first) {  // frames f .. f+7 (never across a 64-frame segment)
    const uint32_t* p = wp + 4 * SEGQ * (f >> 6) + FB * (f & 63) / 4;  // f: a multiple of 8
    uint32_t d[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) d[i] = p[i];
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      const int c = i % 3;
      if (first && i < 3) { mn[c] = d[i]; mx[c] = d[i]; }
      else { mn[c] = pmin(mn[c], d[i]); mx[c] = pmax(mx[c], d[i]); }
    }
  };
  const int f0 = sub * fpl;
  run(f0, true);
  for (int t = 8; t < fpl; t += 8) run(f0 + t, false);  // uniform trip count
  // class c holds columns (c0, c1) = (0, 1), (2, 0), (1, 2) from a dword boundary; from mid-dword
  // class c holds what class c + 1 holds otherwise
  uint32_t amn[3], amx[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    amn[c] = mid ? mn[(c + 2) % 3] : mn[c];
    amx[c] = mid ? mx[(c + 2) % 3] : mx[c];
  }
  auto lo = [](uint32_t v) { return (int)(int16_t)(uint16_t)v; };
  auto hi = [](uint32_t v) { return (int)(int16_t)(uint16_t)(v >> 16); };
  const int cmn[3] = {min(lo(amn[0]), hi(amn[1])), min(hi(amn[0]), lo(amn[2])),
                      min(lo(amn[1]), hi(amn[2]))};
  const int cmx[3] = {max(lo(amx[0]), hi(amx[1])), max(hi(amx[0]), lo(amx[2])),
                      max(lo(amx[1]), hi(amx[2]))};
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  float xm = 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = __builtin_amdgcn_readfirstlane(sel.col[c]);  // uniform: scalar selects
    int a, z;
    if (col == 0) { a = cmn[0]; z = cmx[0]; }
    else if (col == 1) { a = cmn[1]; z = cmx[1]; }
    else { a = cmn[2]; z = cmx[2]; }
    const float r = sel.res[c], bc = base[e * 3 + c];
    // (lo, hi) decoded as one pair: packed fp32 multiply and add, each lane rounded as the
    // scalar fl(fl(raw * r) - b)
    f32x2 x = f32x2{(float)a, (float)z} * f32x2{r, r};
    x = x + f32x2{-bc, -bc};
    xm = fmaxf(xm, fmaxf(fabsf(x.x), fabsf(x.y)));
  }
  // maximum over the row's L lanes (|x| >= 0: its bit pattern orders like the value)
  uint32_t u = __float_as_uint(xm);
  u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0xB1, 0xF, 0xF, true));
  u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x4E, 0xF, 0xF, true));
  u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x141, 0xF, 0xF, true));
  if (sh >= 4) u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x140, 0xF, 0xF, true));
  if (sh >= 5) u = max(u, (uint32_t)__shfl_xor((int)u, 16, 64));
  if (sh >= 6) u = max(u, (uint32_t)__shfl_xor((int)u, 32, 64));
  const double X = (double)__uint_as_float(u);
  const double acc_e = __shfl(acc, 8 * e, 64);
  const bool fails = valid && sub == 0 &&
                     guard_fails(acc_e, kGuardK2Collapsed, (X * X) * (3.0 * (1.0 + 0x1p-20)));
  for (uint64_t b = __ballot(fails); b; b &= b - 1) {  // uniform
    const int jj = (__ffsll((unsigned long long)b) - 1) >> sh;
    left |= 1ull << (8 * ((T >> (4 * jj)) & 15u));
  }
  return left;
}

}  // namespace dev
}  // namespace eegfx
