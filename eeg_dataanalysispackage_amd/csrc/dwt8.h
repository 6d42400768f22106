// dwt8.h -- the fe=dwt-8 filter bank as a per-lane device routine for gfx950 (wave64).
//
// Reference: FeatureExtraction/WaveletTransform.java:126-137 runs the eegdsp 1.0 DWT
// (names[8]; un-vendored jar, pom.xml:79-83) on x = epoch[c][175..686] and keeps the first 16
// coefficients.  SURVEY.md Appendix A pins that transform: 10-tap Daubechies filter with
// 12-decimal literals, periodic extension, pyramid while n >= 10 (512 -> 256 -> ... -> 16), the
// first 16 coefficients are a6[0..7] ++ d6[0..7].
//
// MI355X mapping.  One (epoch, channel) signal is owned by an aligned group of 8 lanes of one
// wave.  Lane s holds samples [64s, 64s+64) plus an 8-sample halo, and at every level owns the
// matching contiguous slice of the coefficients:
//     level  1   2   3   4   5   6
//     owned 32  16   8   4   2   1(a6) + 1(d6)
// so every lane computes exactly 64 outputs (perfect balance, no idle lanes at the deep
// levels).  The taps of a lane's last outputs reach into the slices of the lanes that follow it
// (periodic wrap inside the group = the reference's periodic extension); that cross-lane data
// moves through ds_bpermute (or, for the kernels that keep an exchange area, a per-lane LDS
// slot).  Everything else stays in VGPRs; only the detail coefficients that reach the output (d6)
// are ever computed (5,120 MAC per channel instead of the reference's 10,080).
//
// Numerics.  EXACT: every tap is one rounded fp64 multiply followed by one rounded fp64 add in
// the reference's j = 0..9 order (the file is compiled with -ffp-contract=off), which makes the
// coefficients bit-identical to the Java/C restatement up to the sign of an exactly-zero sum
// (the reference starts its accumulator at +0.0); the halos carry values.  FMA:
// fused multiply-adds, and the halos of levels 1-5 carry partial sums instead of values (the
// following lanes sum the taps that fall on their slices; dwt8_fast_cascade / levels2to6_ps), so
// the boundary outputs add their taps in two or three chains; within 1e-9 of EXACT, tested.
#pragma once
// classic guard as well: a perf-probe build may include a patched copy of this header first
#ifndef EEGFX_DWT8_H
#define EEGFX_DWT8_H

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dwt8_taps.h"

// FMA numerics' filter bank: levels 1-5 collapsed into one 280-tap filter (dwt8_collapsed_cascade)
// or the level-by-level cascade with partial-sum halos (dwt8_fast_cascade; A/B builds only).
#ifndef EEGFX_COLLAPSED
#define EEGFX_COLLAPSED 1
#endif

// The fma numerics' conditioning guard in the window kernels (guard.h); 0 only in A/B probe builds
// (tools/probes/ablations/noguard.patch) that measure its cost.
#ifndef EEGFX_GUARD
#define EEGFX_GUARD 1
#endif

namespace eegfx {
namespace dev {

constexpr int kPre = 100;   // Const.PREESTIMULUS_VALUES
constexpr int kPost = 750;  // Const.POSTSTIMULUS_VALUES
constexpr int kWin = 512;   // WaveletTransform EPOCH_SIZE for dwt-8
constexpr int kTaps = 10;
constexpr int kLanesPerSignal = 8;
constexpr int kSegLen = kWin / kLanesPerSignal;  // 64 samples per lane
constexpr int kIn = kSegLen + 8;                 // + halo
constexpr int kSlot = 10;  // doubles per lane exchange slot (80 B: conflict-free ds_read_b128)

// Low-pass taps.  High-pass g[j] = (-1)^(j+1) h[9-j].
#define EEGFX_H0 0.160102397974
#define EEGFX_H1 0.603829269797
#define EEGFX_H2 0.724308528438
#define EEGFX_H3 0.138428145901
#define EEGFX_H4 -0.242294887066
#define EEGFX_H5 -0.032244869585
#define EEGFX_H6 0.077571493840
#define EEGFX_H7 -0.006241490213
#define EEGFX_H8 -0.012580751999
#define EEGFX_H9 0.003335725285

__device__ __forceinline__ constexpr double tap_h(int j) {
  return j == 0 ? EEGFX_H0 : j == 1 ? EEGFX_H1 : j == 2 ? EEGFX_H2 : j == 3 ? EEGFX_H3
       : j == 4 ? EEGFX_H4 : j == 5 ? EEGFX_H5 : j == 6 ? EEGFX_H6 : j == 7 ? EEGFX_H7
       : j == 8 ? EEGFX_H8 : EEGFX_H9;
}
__device__ __forceinline__ constexpr double tap_g(int j) {
  return (j & 1) ? tap_h(kTaps - 1 - j) : -tap_h(kTaps - 1 - j);
}

// One output of the analysis filter: sum_j x[j] * f[j], j = 0..9, in order.
template <bool FAST, bool HIGH>
__device__ __forceinline__ double fir10(const double* x) {
  double a = x[0] * (HIGH ? tap_g(0) : tap_h(0));
#pragma unroll
  for (int j = 1; j < kTaps; ++j) {
    const double t = HIGH ? tap_g(j) : tap_h(j);
    if constexpr (FAST) a = __builtin_fma(x[j], t, a);
    else a = a + x[j] * t;
  }
  return a;
}

template <int N, bool FAST>
__device__ __forceinline__ void lowpass(const double* in, double* out) {
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = fir10<FAST, false>(in + 2 * i);
}

// The 16-byte quad a kernel reads in place of an out-of-range one (the value is discarded): the
// last whole aligned quad of the recording.  Never offset 0: the streamed path
// (eegfx_process_recording_streamed) passes a `raw` whose offset 0 lies before its chunk buffer.
// Recordings under 16 bytes fall back to offset 0 of a resident (page-granular) allocation.
__device__ __forceinline__ const uint8_t* safe_quad(const uint8_t* raw, int64_t nbytes) {
  return nbytes >= 16 ? raw + ((nbytes & ~(int64_t)15) - 16) : raw;
}

// XCD-aware tile order (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"): blocks are dealt
// round-robin over the 8 XCDs, so block b runs on the XCD of b % 8.  Renumbering the blocks so that
// each XCD walks one contiguous range of tiles keeps tiles that share input bytes (overlapping
// windows of dense markers) in the same L2.  Bijective for any grid size; a speed choice only.
#ifndef EEGFX_XCD_REMAP
#define EEGFX_XCD_REMAP 1
#endif
// EEGFX_XCD_SUPER = T > 0: the grid is walked in rounds of 8T tiles, XCD x taking the T contiguous
// tiles x*T .. x*T+T-1 of each round (the last, partial round as above), so the eight XCDs' read
// streams stay within 8T tiles of each other however large the grid is.
#ifndef EEGFX_XCD_SUPER
#define EEGFX_XCD_SUPER 0
#endif
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t nb) {
  if (!EEGFX_XCD_REMAP) return b;
  if (EEGFX_XCD_SUPER > 0) {
    constexpr uint32_t T = EEGFX_XCD_SUPER > 0 ? EEGFX_XCD_SUPER : 1;
    const uint32_t full = nb / (8 * T), k = b / 8;
    if (k < full * T) return (k / T) * 8 * T + (b % 8) * T + k % T;
    b -= full * 8 * T;  // b % 8 and b / 8 - full T as before: the remainder remapped alone
    const uint32_t base = full * 8 * T;
    nb -= base;
    const uint32_t q = nb / 8, r = nb % 8, x = b % 8;
    return base + (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
  }
  const uint32_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Orders LDS traffic of the lanes of one wave (DS ops of a wave execute in order; the fences
// keep the compiler from moving them across this point).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Publishes the first min(CNT, 8) owned values v[0..) and gathers the 8 values that follow the
// lane's slice at this level into v[CNT .. CNT+8) from lanes s+1, s+2, ... (mod 8).
template <int CNT>
__device__ __forceinline__ void halo_exchange(double* v, double* xch, int gbase, int s) {
  constexpr int P = CNT < 8 ? CNT : 8;
  double* mine = xch + (gbase + s) * kSlot;
#pragma unroll
  for (int i = 0; i < P; ++i) mine[i] = v[i];
  wave_sync();
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int src = (s + 1 + m / P) & (kLanesPerSignal - 1);
    v[CNT + m] = xch[(gbase + src) * kSlot + (m % P)];
  }
  wave_sync();
}

// Same contract as halo_exchange, through the cross-lane network (ds_bpermute) instead of an
// LDS slot: no LDS allocation and no ordering fences.
template <int CNT>
__device__ __forceinline__ void halo_shuffle(double* v, int gbase, int s) {
  constexpr int P = CNT < 8 ? CNT : 8;
  double h[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) h[m] = __shfl(v[m % P], gbase + ((s + 1 + m / P) & 7), 64);
#pragma unroll
  for (int m = 0; m < 8; ++m) v[CNT + m] = h[m];
}

template <int CNT, bool SHFL>
__device__ __forceinline__ void halo(double* v, double* xch, int gbase, int s) {
  if constexpr (SHFL) halo_shuffle<CNT>(v, gbase, s);
  else halo_exchange<CNT>(v, xch, gbase, s);
}

// The cascade in two parts, so a caller can issue memory traffic between level 1 (which consumes
// the 72 decoded samples) and levels 2..6 (which only need the 40-value level-1 slice).
template <bool FAST, bool SHFL = false>
__device__ __forceinline__ void dwt8_level1(const double (&x)[kIn], double* xch, int gbase, int s,
                                            double (&a1)[40]) {
  lowpass<32, FAST>(x, a1);
  halo<32, SHFL>(a1, xch, gbase, s);
}
template <bool FAST, bool SHFL = false>
__device__ __forceinline__ void dwt8_levels2to6(double (&a1)[40], double* xch, int gbase, int s,
                                                double& a6, double& d6) {
  double a2[16 + 8];
  lowpass<16, FAST>(a1, a2);
  halo<16, SHFL>(a2, xch, gbase, s);
  double a3[8 + 8];
  lowpass<8, FAST>(a2, a3);
  halo<8, SHFL>(a3, xch, gbase, s);
  double a4[4 + 8];
  lowpass<4, FAST>(a3, a4);
  halo<4, SHFL>(a4, xch, gbase, s);
  double a5[2 + 8];
  lowpass<2, FAST>(a4, a5);
  halo<2, SHFL>(a5, xch, gbase, s);
  a6 = fir10<FAST, false>(a5);
  d6 = fir10<FAST, true>(a5);
}

// Level 1 with the decode (DataProviderUtils.java:49-59, Baseline.java:39-41: (double)((float)v *
// res - b), two correctly rounded fp32 operations) fused in: samples are fetched and decoded two
// at a time with packed fp32 math just before the first output that needs them, so only a
// 10-sample window and the outputs are live.  fetch(k) returns sample k (k < 72) as float.
typedef float dwt8_f32x2 __attribute__((ext_vector_type(2)));
template <bool FAST, typename Fetch>
__device__ __forceinline__ void level1_jit(Fetch fetch, float r, float b, double (&a1)[40]) {
  const dwt8_f32x2 rr = {r, r}, bb = {b, b};
  double x[kIn];
#pragma unroll
  for (int i = 0; i < 32; ++i) {  // output i reads x[2i .. 2i+9]
#pragma unroll
    for (int k = (i == 0 ? 0 : 2 * i + 8); k < 2 * i + 10; k += 2) {
      const dwt8_f32x2 v = {fetch(k), fetch(k + 1)};
      const dwt8_f32x2 y = v * rr - bb;
      x[k] = (double)y.x;
      x[k + 1] = (double)y.y;
    }
    a1[i] = fir10<FAST, false>(x + 2 * i);
  }
}

// Level 1 under EXACT numerics with the decode fused in: the lane decodes only its own 64 samples
// and takes the 8 halo samples as decoded doubles from lane s+1 (its x[0..7], identical values),
// instead of decoding them again from the next segment (24 VALU instructions per lane).
template <typename Fetch>
__device__ __forceinline__ void level1_exact(Fetch fetch, float r, float b, int gbase, int s,
                                             double (&a1)[40]) {
  const dwt8_f32x2 rr = {r, r}, bb = {b, b};
  const int src = gbase + ((s + 1) & (kLanesPerSignal - 1));
  double x[kIn];
#pragma unroll
  for (int i = 0; i < 32; ++i) {  // output i reads x[2i .. 2i+9]
#pragma unroll
    for (int k = (i == 0 ? 0 : 2 * i + 8); k < 2 * i + 10; k += 2) {
      if (k < kSegLen) {
        const dwt8_f32x2 v = {fetch(k), fetch(k + 1)};
        const dwt8_f32x2 y = v * rr - bb;
        x[k] = (double)y.x;
        x[k + 1] = (double)y.y;
      } else {
        x[k] = __shfl(x[k - kSegLen], src, 64);
        x[k + 1] = __shfl(x[k + 1 - kSegLen], src, 64);
      }
    }
    a1[i] = fir10<false, false>(x + 2 * i);
  }
}

// FMA numerics: partial-sum halos.  The last 4 outputs of a lane's slice (t = 0..3) reach 2 + 2t
// taps into the next lane's slice.  That lane computes those tap terms from its own first 8 values
// and sends the 4 partial sums; the owner continues each FMA chain from the received partial over
// its own taps.  The multiply / FMA count is fir10's, and 4 doubles cross lanes (8 ds_bpermute)
// instead of the 8 halo values (16).  Only the summation order of those 4 outputs differs from the
// reference's, inside the 1e-9 contract; EXACT keeps the value halos (halo / level1_jit).
template <typename V>
__device__ __forceinline__ void partials_for_left(const V& v, double (&p)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    double a = v(0) * tap_h(8 - 2 * t);
#pragma unroll
    for (int j = 9 - 2 * t; j < kTaps; ++j) a = __builtin_fma(v(j - 8 + 2 * t), tap_h(j), a);
    p[t] = a;
  }
}
__device__ __forceinline__ void pull_partials(const double (&p)[4], double (&q)[4], int gbase,
                                              int s) {
  const int src = gbase + ((s + 1) & (kLanesPerSignal - 1));
#pragma unroll
  for (int t = 0; t < 4; ++t) q[t] = __shfl(p[t], src, 64);
}
// output i = CNT - 4 + t of the slice: own taps j < 8 - 2t continue the received partial q
template <typename V>
__device__ __forceinline__ double boundary_out(const V& v, int i, int t, double q) {
  double a = q;
#pragma unroll
  for (int j = 0; j < 8 - 2 * t; ++j) a = __builtin_fma(v(2 * i + j), tap_h(j), a);
  return a;
}
template <int CNT>
__device__ __forceinline__ void lowpass_ps(const double* v, double* out, int gbase, int s) {
  static_assert(CNT >= 4, "partial-sum halos need 8 own values");
  double p[4], q[4];
  auto at = [&](int k) { return v[k]; };
  partials_for_left(at, p);
  pull_partials(p, q, gbase, s);
#pragma unroll
  for (int i = 0; i < CNT - 4; ++i) out[i] = fir10<true, false>(v + 2 * i);
#pragma unroll
  for (int t = 0; t < 4; ++t) out[CNT - 4 + t] = boundary_out(at, CNT - 4 + t, t, q[t]);
}
// Level 5 by partial sums: a5[2s + i] = sum_j h[j] a4[4s + 2i + j] takes the lane's own a4 for
// 2i + j < 4, lane s+1's for 4 <= 2i + j < 8 and lane s+2's beyond.  Each lane computes the terms
// it owes lanes s-1 and s-2, and the owner continues lane s+1's partial over its own taps and adds
// lane s+2's: 4 doubles cross lanes instead of 8, for 2 adds and 2 extra multiplies.
__device__ __forceinline__ void level5_ps(const double* a4, double* a5, int gbase, int s) {
  double p1[2], p2[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j1 = 4 - 2 * i;  // as lane s+1 of the consumer: taps j1 .. j1+3 on a4[0..3]
    double a = a4[0] * tap_h(j1);
#pragma unroll
    for (int j = j1 + 1; j < j1 + 4; ++j) a = __builtin_fma(a4[2 * i + j - 4], tap_h(j), a);
    p1[i] = a;
    const int j2 = 8 - 2 * i;  // as lane s+2: taps j2 .. 9 on a4[0 ..]
    double c = a4[0] * tap_h(j2);
#pragma unroll
    for (int j = j2 + 1; j < kTaps; ++j) c = __builtin_fma(a4[2 * i + j - 8], tap_h(j), c);
    p2[i] = c;
  }
  const int src1 = gbase + ((s + 1) & (kLanesPerSignal - 1));
  const int src2 = gbase + ((s + 2) & (kLanesPerSignal - 1));
  double q1[2], q2[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    q1[i] = __shfl(p1[i], src1, 64);
    q2[i] = __shfl(p2[i], src2, 64);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    double a = q1[i];
#pragma unroll
    for (int j = 0; j < 4 - 2 * i; ++j) a = __builtin_fma(a4[2 * i + j], tap_h(j), a);
    a5[i] = a + q2[i];
  }
}
// Levels 2..6 under FMA numerics: partial-sum halos for levels 2-5, value halos for level 6,
// whose taps span 5 lanes.
__device__ __forceinline__ void levels2to6_ps(const double* a1, int gbase, int s, double& a6,
                                              double& d6) {
  double a2[16];
  lowpass_ps<16>(a1, a2, gbase, s);
  double a3[8];
  lowpass_ps<8>(a2, a3, gbase, s);
  double a4[4];
  lowpass_ps<4>(a3, a4, gbase, s);
  double a5[2 + 8];
  level5_ps(a4, a5, gbase, s);
  halo<2, true>(a5, nullptr, gbase, s);
  a6 = fir10<true, false>(a5);
  d6 = fir10<true, true>(a5);
}
// Level 1 under FMA numerics with the decode fused in (as level1_jit): the lane decodes only its
// own 64 samples; the partials its left neighbour needs are formed as soon as the first 10 are
// decoded and leave early.  a1[0..32) receives the lane's level-1 slice.
template <typename Fetch>
__device__ __forceinline__ void level1_ps(Fetch fetch, float r, float b, int gbase, int s,
                                          double (&a1)[40]) {
  const dwt8_f32x2 rr = {r, r}, bb = {b, b};
  double x[kSegLen];
  double p[4], q[4];
#pragma unroll
  for (int i = 0; i < 28; ++i) {  // outputs whose taps x[2i .. 2i+9] are all this lane's
#pragma unroll
    for (int k = (i == 0 ? 0 : 2 * i + 8); k < 2 * i + 10; k += 2) {
      const dwt8_f32x2 v = {fetch(k), fetch(k + 1)};
      const dwt8_f32x2 y = v * rr - bb;
      x[k] = (double)y.x;
      x[k + 1] = (double)y.y;
    }
    if (i == 0) {
      auto at = [&](int k) { return x[k]; };
      partials_for_left(at, p);
      pull_partials(p, q, gbase, s);
    }
    a1[i] = fir10<true, false>(x + 2 * i);
  }
  auto at = [&](int k) { return x[k]; };
#pragma unroll
  for (int t = 0; t < 4; ++t) a1[28 + t] = boundary_out(at, 28 + t, t, q[t]);
}
// The whole cascade under FMA numerics from a fetch of the lane's own 64 samples.
template <typename Fetch>
__device__ __forceinline__ void dwt8_fast_cascade(Fetch fetch, float r, float b, int gbase, int s,
                                                  double& a6, double& d6) {
  double a1[40];
  level1_ps(fetch, r, b, gbase, s, a1);
  levels2to6_ps(a1, gbase, s, a6, d6);
}

// Levels 1-5 collapsed (fma numerics): a5[k] = sum_{m < 280} H5[m] x[32 k + m] (mod 512), the five
// periodic low-pass stages composed into one filter at stride 32 (dwt8_taps.h, generated exactly by
// gen_taps.py).  4,480 multiply-adds per signal for a5 instead of the cascade's 4,960, and the
// cross-lane traffic shrinks to one partial-sum round: lane s owns a5[2s], a5[2s+1]; its sample
// n (and n + 32) meets taps H5[n + 32 j] of the outputs of lanes s, s-1, ..., s-4, so it keeps ten
// partial sums P[j], j = -1..8 (the partial of a5[2(s - d) + i] with j = 2d - i), and receives the
// other four terms of each of its two outputs from lanes s+1..s+4 (8 doubles instead of the
// cascade's 16 halo partials over levels 1-5).  Level 6 (a6, d6 from a5) is unchanged.  The
// samples are taken in pairs (n, n + 32), which meet the same nine taps: one 64-byte scalar load
// per pair plus the ninth from the table's tail, the taps held in SGPRs.  Only the summation order
// differs from the reference's, inside the 1e-9 contract; EXACT keeps the level-by-level cascade.
//
// Each pair's update is a product of polynomials, P(z) += T_n(z) (x1 + z x0) with
// T_n(z) = sum_j H5[n + 32 j] z^j, and runs in a four-point (Toom) form: the nine taps in three
// blocks by j mod 3, T_n(z) = B0(z^3) + z B1(z^3) + z^2 B2(z^3), and the product
// (B0 + w B1 + w^2 B2)(x1 + w x0) = c0 + w c1 + w^2 c2 + w^3 c3 evaluated at w = 0, infinity, 1 and
// -1.  Over all pairs the lane accumulates A0 += B0 x1, Ai += B2 x0, Bp += (B0 + B1 + B2)/2 (x1 + x0)
// and Bm += (B0 - B1 + B2)/2 (x1 - x0), three entries each, and interpolates once:
// c0 = A0, c3 = Ai, c1 = Bp - Bm - c3, c2 = Bp + Bm - c0, P[3q + r] = c_r[q] (+ c3[q - 1] for r = 0).
// That is 12 multiply-adds and two adds (x1 +- x0, nearly always exact) per pair, 11 + 2 once tap 280
// is passed: 440 per lane instead of the direct form's 560.  The constants are exact rational sums
// halved and rounded once (dwt8_taps.h), one 96-byte row per pair.
//   Measured: the two-term Karatsuba form (464 per lane, `git show
//   682923c:eeg_dataanalysispackage_amd/csrc/dwt8.h`, -DEEGFX_TOOM=0) was 2.2 % slower; the direct
//   form (EEGFX_TOOM 0 here, tools/probes/ablations/direct.patch) 4-6 % slower still.
static __constant__ double kH5[kH5Size] = EEGFX_H5_TABLE;
#ifndef EEGFX_TOOM
#define EEGFX_TOOM 1
#endif

// The core takes the samples through two callables: fetch(k) reads raw sample k of the lane's
// slice (k < 64) and decode(v0, v1, x0, x1) turns the raw pair (k, k + 32) into doubles.
// EEGFX_LDS_B64 (A/B builds): the int16 kernels read samples k and k + 1 of a signal with one
// 8-byte LDS read (dwt8_collapsed_core_b64) instead of two 2-byte reads.
#ifndef EEGFX_LDS_B64
#define EEGFX_LDS_B64 0
#endif
typedef const __attribute__((address_space(4))) double* dwt8_const_f64_ptr;

// The four-point update of pair n (x0 = sample n, x1 = sample n + 32) into the 12 accumulators.
__device__ __forceinline__ void toom_pair(dwt8_const_f64_ptr tab, int n, double x0, double x1,
                                          double (&A0)[3], double (&Ai)[3], double (&Bp)[3],
                                          double (&Bm)[3]) {
  // exact when the pair's exponents lie within 29 of each other (the decoded fp32 samples of a
  // window nearly always do); otherwise, and for caller-supplied doubles
  // (features_from_epochs_kernel), one rounding each -- tools/fma_bound.py models both adds as
  // rounded, so the guard's bound covers either case
  const double xp = x1 + x0, xm = x1 - x0;
  const dwt8_const_f64_ptr R = tab + n * kH5Cols;  // this pair's 12 constants (96 bytes)
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    A0[q] = n == 0 ? x1 * R[q] : __builtin_fma(x1, R[q], A0[q]);
    if (n + 32 * (3 * q + 2) < 280)
      Ai[q] = n == 0 ? x0 * R[3 + q] : __builtin_fma(x0, R[3 + q], Ai[q]);
    Bp[q] = n == 0 ? xp * R[6 + q] : __builtin_fma(xp, R[6 + q], Bp[q]);
    Bm[q] = n == 0 ? xm * R[9 + q] : __builtin_fma(xm, R[9 + q], Bm[q]);
  }
  // The pair's updates complete here: without this, the IR ends up ordered chain by chain (all
  // 64 sample reads and 32 constant rows first, every multiply-add after them), which spills.
  asm volatile("" : "+v"(A0[0]), "+v"(A0[1]), "+v"(A0[2]), "+v"(Ai[0]), "+v"(Ai[1]), "+v"(Ai[2]),
               "+v"(Bp[0]), "+v"(Bp[1]), "+v"(Bp[2]), "+v"(Bm[0]), "+v"(Bm[1]), "+v"(Bm[2]));
}

// Interpolation of the four-point accumulators into the ten partial sums, the one partial-sum
// round that completes a5[2s], a5[2s+1], and level 6.
__device__ __forceinline__ void toom_finish(const double (&A0)[3], const double (&Ai)[3],
                                            const double (&Bp)[3], const double (&Bm)[3],
                                            int gbase, int s, double& a6, double& d6) {
  double P[10];  // P[j + 1]
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    P[3 * q] = q > 0 ? A0[q] + Ai[q - 1] : A0[q];
    P[3 * q + 1] = Bp[q] - Bm[q] - Ai[q];
    P[3 * q + 2] = Bp[q] + Bm[q] - A0[q];
  }
  P[9] = Ai[2];
  double a5[2 + 8];
  a5[0] = P[1];
  a5[1] = P[0];
#pragma unroll
  for (int d = 1; d <= 4; ++d) {
    const int src = gbase + ((s + d) & (kLanesPerSignal - 1));
    a5[0] += __shfl(P[2 * d + 1], src, 64);
    a5[1] += __shfl(P[2 * d], src, 64);
  }
  halo<2, true>(a5, nullptr, gbase, s);
  a6 = fir10<true, false>(a5);
  d6 = fir10<true, true>(a5);
}

template <typename Fetch, typename Decode>
__device__ __forceinline__ void dwt8_collapsed_core(Fetch fetch, Decode decode, int gbase, int s,
                                                    double& a6, double& d6) {
  dwt8_const_f64_ptr tab = (dwt8_const_f64_ptr)kH5;
  asm volatile("" : "+s"(tab));  // scalar loads of the table, not per-tap literal moves
#if EEGFX_TOOM
  double A0[3], Ai[3], Bp[3], Bm[3];
  // the samples are fetched two pairs ahead of their use (the per-pair ordering below otherwise
  // leaves each pair's sample reads exposed)
  typedef decltype(+fetch(0)) Raw;  // int for int16 samples (converted at use), float, double
  Raw vq[2][2];
#pragma unroll
  for (int d = 0; d < 2; ++d) { vq[d][0] = fetch(d); vq[d][1] = fetch(d + 32); }
#pragma unroll
  for (int n = 0; n < 32; ++n) {
    const Raw v0 = vq[n % 2][0], v1 = vq[n % 2][1];
    if (n + 2 < 32) { vq[n % 2][0] = fetch(n + 2); vq[n % 2][1] = fetch(n + 2 + 32); }
    double x0, x1;
    decode(v0, v1, x0, x1);
    toom_pair(tab, n, x0, x1, A0, Ai, Bp, Bm);
  }
  toom_finish(A0, Ai, Bp, Bm, gbase, s, a6, d6);
#else
  double P[10];  // P[j + 1]
  // the direct form (A/B builds only): 18 multiply-adds per pair, one scheduling region per pair
  // (without it the c3 kernel hoisted tap rows into SGPRs and spilled them to VGPR lanes)
#pragma unroll
  for (int n = 0; n < 32; ++n) {
    double x0, x1;
    decode(fetch(n), fetch(n + 32), x0, x1);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      if (n + 32 * j >= 280) continue;
      const double t = j < kH5DirectCols ? tab[kH5Direct + n * kH5DirectCols + j] : tab[kH5Tail + n];
      P[j + 1] = n == 0 ? x0 * t : __builtin_fma(x0, t, P[j + 1]);   // sample n -> accumulator j
      if (n == 0 && j == 0) P[0] = x1 * t;                            // sample n + 32 -> j - 1
      else P[j] = __builtin_fma(x1, t, P[j]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  double a5[2 + 8];
  a5[0] = P[1];
  a5[1] = P[0];
#pragma unroll
  for (int d = 1; d <= 4; ++d) {
    const int src = gbase + ((s + d) & (kLanesPerSignal - 1));
    a5[0] += __shfl(P[2 * d + 1], src, 64);
    a5[1] += __shfl(P[2 * d], src, 64);
  }
  halo<2, true>(a5, nullptr, gbase, s);
  a6 = fir10<true, false>(a5);
  d6 = fir10<true, true>(a5);
#endif
}

// The same core for int16 samples in a 3-channel multiplexed window: fetch2(k) reads the 8 bytes
// from sample k of the lane's signal, whose int16 words 0 and 3 are samples k and k + 1 (a frame
// is 3 words), so one LDS read serves two pairs.  Group g = pairs 2g and 2g + 1; the next group's
// two reads are issued before the current group's updates.
template <typename Fetch2, typename Decode>
__device__ __forceinline__ void dwt8_collapsed_core_b64(Fetch2 fetch2, Decode decode, int gbase,
                                                        int s, double& a6, double& d6) {
  dwt8_const_f64_ptr tab = (dwt8_const_f64_ptr)kH5;
  asm volatile("" : "+s"(tab));
  double A0[3], Ai[3], Bp[3], Bm[3];
  uint64_t q0 = fetch2(0), q1 = fetch2(32);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const uint64_t c0 = q0, c1 = q1;
    if (g + 1 < 16) { q0 = fetch2(2 * g + 2); q1 = fetch2(2 * g + 34); }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v0 = h == 0 ? (int)(int16_t)(uint16_t)c0 : (int)(int16_t)(uint16_t)(c0 >> 48);
      const int v1 = h == 0 ? (int)(int16_t)(uint16_t)c1 : (int)(int16_t)(uint16_t)(c1 >> 48);
      double x0, x1;
      decode(v0, v1, x0, x1);
      toom_pair(tab, 2 * g + h, x0, x1, A0, Ai, Bp, Bm);
    }
  }
  toom_finish(A0, Ai, Bp, Bm, gbase, s, a6, d6);
}

// The fused kernels' form: raw samples decoded as (double)((float)v * r - b), two correctly
// rounded fp32 operations (DataProviderUtils.java:49-59, Baseline.java:39-41), a pair at a time
// with packed fp32 math.
// TRACK: also returns in `ymax` the largest |x| of the lane's 64 samples (the guard's measured X
// for float32 recordings, guard.h).
template <bool TRACK = false, typename Fetch>
__device__ __forceinline__ void dwt8_collapsed_cascade(Fetch fetch, float r, float b, int gbase,
                                                       int s, double& a6, double& d6,
                                                       float* ymax = nullptr) {
  const dwt8_f32x2 rr = {r, r}, bb = {b, b};
  float m = 0.0f;
  dwt8_collapsed_core(
      fetch,
      [&](auto v0, auto v1, double& x0, double& x1) {
        const dwt8_f32x2 v = {(float)v0, (float)v1};
        const dwt8_f32x2 y = v * rr - bb;
        if constexpr (TRACK) m = fmaxf(m, fmaxf(fabsf(y.x), fabsf(y.y)));
        x0 = (double)y.x;
        x1 = (double)y.y;
      },
      gbase, s, a6, d6);
  if constexpr (TRACK) *ymax = m;
}

// dwt8_collapsed_cascade over dwt8_collapsed_core_b64 (3-channel int16 windows in LDS).
template <typename Fetch2>
__device__ __forceinline__ void dwt8_collapsed_cascade_b64(Fetch2 fetch2, float r, float b,
                                                           int gbase, int s, double& a6,
                                                           double& d6) {
  const dwt8_f32x2 rr = {r, r}, bb = {b, b};
  dwt8_collapsed_core_b64(
      fetch2,
      [&](int v0, int v1, double& x0, double& x1) {
        const dwt8_f32x2 v = {(float)v0, (float)v1};
        const dwt8_f32x2 y = v * rr - bb;
        x0 = (double)y.x;
        x1 = (double)y.y;
      },
      gbase, s, a6, d6);
}

// The same filter with 4 lanes per signal (fused.hip window4_kernel, an A/B build: 8.9 % fewer VALU
// instructions than the pair form, 2.5 % slower with half the waves per CU; DESIGN_LOG.md §R6):
// lane s owns samples 128 s + k, k < 128, and outputs a5[4 s .. 4 s + 3].  Its samples come in
// groups of four, x_t = sample n + 32 t (t < 4), which meet the same nine taps T_n as a pair does,
// and the group's update is the product T_n(w) X(w) with X(w) = x3 + w x2 + w^2 x1 + w^3 x0: twelve
// partials P[m] (m = j + 3 - t), of which P[0..3] are the lane's own outputs (a5[4 s + 3 - m]),
// P[4..7] lane s-1's and P[8..11] lane s-2's.  In block form, T_n = B0(w^3) + w B1(w^3) +
// w^2 B2(w^3) as in the pair update, (B0 + w B1 + w^2 B2) X(w) = c0 + ... + w^5 c5 is evaluated at
// w = 0, infinity, 1, -1, 2, -2 -- six products of three entries, 18 multiply-adds per group --
// and interpolated once (toom6_finish).  The four evaluations of X cost eight operations (two
// sums, two fma per pair of points), exact whenever the four samples' exponents lie within ~26 of
// each other; tools/fma_bound.py models every one of them as rounded.  Per sample: 6.5 fp64
// operations instead of the pair form's 7, and half as many lanes pay the per-signal finish,
// level 6 and the row epilogue.  The bound is wider (guard.h kGuardK2Toom6, 2.16e-4 against
// 7.02e-5): the interpolation divides by 3 and the +-2 points weigh the samples up to 8x.
static __constant__ double kT6[kT6Rows * kT6Cols] = EEGFX_T6_TABLE;
constexpr int kLanesPerSignal4 = 4;

// The six-point update of group n into the 18 accumulators V[k][q] (k: the points 0, inf, 1, -1,
// 2, -2; the table's constants carry the interpolation's 1/2 and 1/24).
__device__ __forceinline__ void toom6_group(const double (&R)[kT6Cols], int n, double x0,
                                            double x1, double x2, double x3, double (&V)[6][3]) {
  const double E1 = x3 + x1, O1 = x2 + x0;
  const double E2 = __builtin_fma(4.0, x1, x3), O2 = __builtin_fma(4.0, x0, x2);
  const double X[6] = {x3, x0, E1 + O1, E1 - O1, __builtin_fma(2.0, O2, E2),
                       __builtin_fma(-2.0, O2, E2)};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (k == 1 && n + 32 * (3 * q + 2) >= 280) continue;  // B2 past tap 279
      V[k][q] = n == 0 ? X[k] * R[3 * k + q] : __builtin_fma(X[k], R[3 * k + q], V[k][q]);
    }
  }
  // the group's updates complete here (one scheduling region per group, as toom_pair)
  asm volatile("" : "+v"(V[0][0]), "+v"(V[0][1]), "+v"(V[0][2]), "+v"(V[1][0]), "+v"(V[1][1]),
               "+v"(V[1][2]), "+v"(V[2][0]), "+v"(V[2][1]), "+v"(V[2][2]));
  asm volatile("" : "+v"(V[3][0]), "+v"(V[3][1]), "+v"(V[3][2]), "+v"(V[4][0]), "+v"(V[4][1]),
               "+v"(V[4][2]), "+v"(V[5][0]), "+v"(V[5][1]), "+v"(V[5][2]));
}

// Interpolation (per q: c0 = V0, c5 = Vinf, S1 = V1 + Vm1 = c0 + c2 + c4, D1 = V1 - Vm1 =
// c1 + c3 + c5, V2 + Vm2 = (c0 + 4 c2 + 16 c4) / 12, V2 - Vm2 = (c1 + 4 c3 + 16 c5) / 6), the
// twelve partials P[3 q + r] = c_r[q] + c_{r+3}[q-1], the one partial round (lanes s+1, s+2) that
// completes a5[4 s .. 4 s + 3], and level 6: a6[2 s + i], d6[2 s + i], i < 2, from a5[4 s .. 4 s + 11].
__device__ __forceinline__ void toom6_finish(const double (&V)[6][3], int gbase, int s,
                                             double (&a6)[2], double (&d6)[2]) {
  constexpr double kMinusThird = -1.0 / 3.0;
  double c[6][3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double c0 = V[0][q], c5 = V[1][q];
    const double S1 = V[2][q] + V[3][q], D1 = V[2][q] - V[3][q];
    const double T2 = V[4][q] + V[5][q], U2 = V[4][q] - V[5][q];
    const double c4 = __builtin_fma(S1, kMinusThird, __builtin_fma(c0, 0.25, T2));
    const double c2 = (S1 - c0) - c4;
    const double c3 = __builtin_fma(U2, 2.0, __builtin_fma(D1, kMinusThird, c5 * -5.0));
    const double c1 = (D1 - c3) - c5;
    c[0][q] = c0; c[1][q] = c1; c[2][q] = c2; c[3][q] = c3; c[4][q] = c4; c[5][q] = c5;
  }
  double P[12];
#pragma unroll
  for (int m = 0; m < 12; ++m) {
    const int q = m / 3, r = m % 3;
    P[m] = q == 0 ? c[r][0] : q == 3 ? c[r + 3][2] : c[r][q] + c[r + 3][q - 1];
  }
  const int src1 = gbase + ((s + 1) & (kLanesPerSignal4 - 1));
  const int src2 = gbase + ((s + 2) & (kLanesPerSignal4 - 1));
  double a5[12];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a5[i] = (P[3 - i] + __shfl(P[7 - i], src1, 64)) + __shfl(P[11 - i], src2, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a5[4 + i] = __shfl(a5[i], src1, 64);
    a5[8 + i] = __shfl(a5[i], src2, 64);
  }
  a6[0] = fir10<true, false>(a5);
  a6[1] = fir10<true, false>(a5 + 2);
  d6[0] = fir10<true, true>(a5);
  d6[1] = fir10<true, true>(a5 + 2);
}

// fetch(k): raw sample k < 128 of the lane's quarter; decode(v0, v1, x0, x1) as in
// dwt8_collapsed_core.
template <typename Fetch, typename Decode>
__device__ __forceinline__ void dwt8_toom6_core(Fetch fetch, Decode decode, int gbase, int s,
                                                double (&a6)[2], double (&d6)[2]) {
  dwt8_const_f64_ptr tab = (dwt8_const_f64_ptr)kT6;
  asm volatile("" : "+s"(tab));  // scalar loads of the table
  double V[6][3];
  typedef decltype(+fetch(0)) Raw;
  Raw vq[2][4];  // two groups ahead
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int t = 0; t < 4; ++t) vq[d][t] = fetch(d + 32 * t);
#pragma unroll
  for (int n = 0; n < 32; ++n) {
    Raw v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = vq[n % 2][t];
    if (n + 2 < 32) {
#pragma unroll
      for (int t = 0; t < 4; ++t) vq[n % 2][t] = fetch(n + 2 + 32 * t);
    }
    double R[kT6Cols];  // scalar loads (rows held one group ahead measured slower: SGPR spills)
#pragma unroll
    for (int i = 0; i < kT6Cols; ++i) R[i] = tab[n * kT6Cols + i];
    double x0, x1, x2, x3;
    decode(v[0], v[1], x0, x1);
    decode(v[2], v[3], x2, x3);
    toom6_group(R, n, x0, x1, x2, x3, V);
  }
  toom6_finish(V, gbase, s, a6, d6);
}

// dwt8_toom6_core with the fused kernels' decode, (double)((float)v * r - b), a pair at a time.
template <typename Fetch>
__device__ __forceinline__ void dwt8_toom6_cascade(Fetch fetch, float r, float b, int gbase, int s,
                                                   double (&a6)[2], double (&d6)[2]) {
  const dwt8_f32x2 rr = {r, r}, bb = {b, b};
  dwt8_toom6_core(
      fetch,
      [&](auto v0, auto v1, double& x0, double& x1) {
        const dwt8_f32x2 v = {(float)v0, (float)v1};
        const dwt8_f32x2 y = v * rr - bb;
        x0 = (double)y.x;
        x1 = (double)y.y;
      },
      gbase, s, a6, d6);
}

// The largest value of v over the 8 lanes of a signal group.
__device__ __forceinline__ float group8_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  return fmaxf(v, __shfl_xor(v, 4, 64));
}
__device__ __forceinline__ double group8_max(double v) {
  v = fmax(v, __shfl_xor(v, 1, 64));
  v = fmax(v, __shfl_xor(v, 2, 64));
  return fmax(v, __shfl_xor(v, 4, 64));
}

// A double moved across lanes by one DPP control (both halves), e.g. 0xB1 = xor 1, 0x4E = xor 2
// within a quad, 0x141 = row_half_mirror (lane i <- 7 - i within 8): no LDS round trip and no
// lane-address arithmetic, where __shfl_xor costs four VALU and two ds_bpermute per step.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}
// The sum over an aligned group of 8 lanes, identical in all 8 (each step adds a pair of equal
// partial sums in either order).
__device__ __forceinline__ double group8_sum(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  return v + dpp_f64<0x141>(v);
}
// The same over an aligned group of 4 lanes.
__device__ __forceinline__ double group4_sum(double v) {
  v += dpp_f64<0xB1>(v);
  return v + dpp_f64<0x4E>(v);
}

// 1 / sqrt(v) for the fma numerics' row normalisation: v_rsq_f64 refined by two Newton steps
// (relative error ~1e-16, inside the 1e-9 contract); v = 0 gives inf, so an all-zero row still
// normalises to NaN as the reference's 0/0 does.
__device__ __forceinline__ double rsqrt_nr(double v) {
  double r = __builtin_amdgcn_rsq(v);
  r = r * __builtin_fma(-0.5 * v * r, r, 1.5);
  r = r * __builtin_fma(-0.5 * v * r, r, 1.5);
  return r;
}
// The same with one Newton step: relative error ~1e-13 from v_rsq_f64's ~2^-23 start, four orders
// of magnitude inside the 0.5e-9 the guard leaves the normalisation (guard.h); the window kernel's
// three channel waves each compute it (fused.hip), so the step saved is saved three times.
__device__ __forceinline__ double rsqrt_nr1(double v) {
  const double r = __builtin_amdgcn_rsq(v);
  return r * __builtin_fma(-0.5 * v * r, r, 1.5);
}

// One level of the analysis low-pass over a whole wave under EXACT numerics: out[i] =
// fir10(in[2i .. 2i + 9] mod N) for i < N / 2, lane l computing outputs l, l + 64, ...  The ten
// inputs are read as five 16-byte LDS pairs (2i and every pair offset are even, so no pair wraps).
template <int N>
__device__ __forceinline__ void level_wave(const double* in, double* out, int lane) {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  constexpr int H = N / 2;
#pragma unroll
  for (int i0 = 0; i0 < H; i0 += 64) {
    const int i = i0 + lane;
    if (H >= 64 || i < H) {
      double x[kTaps];
#pragma unroll
      for (int t = 0; t < kTaps / 2; ++t) {
        const f64x2 p = *(const f64x2*)(in + ((2 * i + 2 * t) & (N - 1)));
        x[2 * t] = p.x;
        x[2 * t + 1] = p.y;
      }
      out[i] = fir10<false, false>(x);
    }
  }
}

// The six levels of one signal by one wave under EXACT numerics (the per-epoch path, small_epoch):
// each level's outputs spread over the 64 lanes (4, 2, 1 per lane at levels 1-3, then 32 and 16
// lanes), every output the reference's sum in its order (WaveletTransform.java:126-137, the
// eegdsp DWT of SURVEY.md Appendix A: one rounded multiply and one rounded add per tap in j order,
// -ffp-contract=off; fir10 as in the other EXACT paths).
// x: the 512 window doubles in LDS (16-byte aligned); scratch: 384 doubles of this wave's LDS
// (16-byte aligned), levels ping-pong through it.  Returns feature `lane` of the signal: a6[lane]
// on lanes 0-7, d6[lane - 8] on lanes 8-15, 0 elsewhere.  A one-epoch call is latency-bound on one
// workgroup, and this form's per-lane chain is ~190 operations against the 8-lanes-per-signal
// cascade's ~1,200.
__device__ __forceinline__ double dwt8_exact_signal_wave(const double* x, double* scratch,
                                                         int lane) {
  level_wave<512>(x, scratch, lane);
  wave_sync();
  level_wave<256>(scratch, scratch + 256, lane);
  wave_sync();
  level_wave<128>(scratch + 256, scratch, lane);
  wave_sync();
  level_wave<64>(scratch, scratch + 256, lane);
  wave_sync();
  level_wave<32>(scratch + 256, scratch, lane);
  wave_sync();
  double f = 0.0;
  if (lane < 16) {  // level 6 on the 16 values of a5
    const int i = lane & 7;
    double v[kTaps];
#pragma unroll
    for (int j = 0; j < kTaps; ++j) v[j] = scratch[(2 * i + j) & 15];
    f = lane < 8 ? fir10<false, false>(v) : fir10<false, true>(v);
  }
  wave_sync();  // scratch is free for the wave's next signal
  return f;
}

// One feature row under EXACT numerics by one wave, for the rare rows the fma numerics'
// conditioning guard cannot certify (guard.h): for each of the C channels the 512 window samples
// (sample(c, k): the decoded doubles) go to LDS, the six levels run with every output
// sum_j x[(2i + j) mod n] h[j] (g[j] at level 6) in the reference's order -- one rounded multiply
// and one rounded add per tap, the file compiled with -ffp-contract=off -- so the row equals the
// EXACT kernels' value for value; then SignalProcessing.normalize (sequential sum of squares, sqrt,
// divide).  row: C * nfeat doubles of LDS (receives the normalised row); scratch: 768 doubles of
// LDS that no other wave touches.  Few registers: it runs inside the fma kernels' rare path.
static __constant__ double kHG[2 * kTaps] = {
    EEGFX_H0, EEGFX_H1, EEGFX_H2, EEGFX_H3, EEGFX_H4, EEGFX_H5, EEGFX_H6, EEGFX_H7, EEGFX_H8,
    EEGFX_H9, tap_g(0), tap_g(1), tap_g(2), tap_g(3), tap_g(4), tap_g(5), tap_g(6), tap_g(7),
    tap_g(8), tap_g(9)};
// One channel of dwt8_exact_row_wave from its 512 decoded doubles in scratch[0, 512) (LDS, this
// wave's writes synchronised): rowc[k], k < nfeat, receives its unnormalised features; scratch:
// 768 doubles of LDS no other wave touches.
__device__ __forceinline__ void dwt8_exact_channel_lds(int nfeat, double* scratch, double* rowc,
                                                       int lane) {
  double* in = scratch;
  double* out = scratch + kWin;
  int n = kWin;
#pragma unroll 1
  for (int level = 1; level <= 5; ++level) {
#pragma unroll 1
    for (int i = lane; i < n / 2; i += 64) {
      double x[kTaps];
#pragma unroll
      for (int j = 0; j < kTaps; ++j) x[j] = in[(2 * i + j) & (n - 1)];
      double a = x[0] * kHG[0];
#pragma unroll
      for (int j = 1; j < kTaps; ++j) a = a + x[j] * kHG[j];
      out[i] = a;
    }
    wave_sync();
    double* t = in;
    in = out;
    out = t;
    n /= 2;
  }
  if (lane < 16) {  // level 6 on the 16 values of a5: a6[i] (lanes 0-7), d6[i] (lanes 8-15)
    const int i = lane & 7;
    const double* f = kHG + (lane >= 8 ? kTaps : 0);
    double a = in[2 * i] * f[0];
#pragma unroll 1
    for (int j = 1; j < kTaps; ++j) a = a + in[(2 * i + j) & 15] * f[j];
    const int k = lane >= 8 ? 8 + i : i;
    if (k < nfeat) rowc[k] = a;
  }
  wave_sync();
}
// dwt8_exact_channel_lds with the samples from sample(k), k < 512, all of a lane's loads issued
// before the first is used (the path is latency-bound: one window per wave)
template <typename SampleK>
__device__ __forceinline__ void dwt8_exact_channel_wave(SampleK sample, int nfeat, double* scratch,
                                                        double* rowc, int lane) {
  double v[kWin / 64];
#pragma unroll
  for (int q = 0; q < kWin / 64; ++q) v[q] = sample(lane + 64 * q);
#pragma unroll
  for (int q = 0; q < kWin / 64; ++q) scratch[lane + 64 * q] = v[q];
  wave_sync();
  dwt8_exact_channel_lds(nfeat, scratch, rowc, lane);
}
// SignalProcessing.normalize of the F values of `row` (LDS) in place by one wave: sequential sum
// of squares on lane 0, sqrt, divide; scratch: one double of LDS.
__device__ __forceinline__ void dwt8_normalise_row_wave(double* row, int F, double* scratch,
                                                        int lane) {
  if (lane == 0) {
    double acc = 0.0;
#pragma unroll 1
    for (int k = 0; k < F; ++k) acc = acc + row[k] * row[k];
    scratch[0] = sqrt(acc);
  }
  wave_sync();
  const double nv = scratch[0];
#pragma unroll 1
  for (int k = lane; k < F; k += 64) row[k] = row[k] / nv;
  wave_sync();
}
template <typename Sample>
__device__ __forceinline__ void dwt8_exact_row_wave(Sample sample, int C, int nfeat,
                                                    double* scratch, double* row, int lane) {
  // loops kept rolled and the taps read from kHG: the kernels this is inlined into keep their
  // register budget (the unrolled form raised the 3-channel window kernel from 44 to 94 VGPRs)
#pragma unroll 1
  for (int c = 0; c < C; ++c)
    dwt8_exact_channel_wave([&](int k) { return sample(c, k); }, nfeat, scratch, row + c * nfeat,
                            lane);
  dwt8_normalise_row_wave(row, C * nfeat, scratch, lane);
}

// x[0..72): samples [64s, 64s+72) mod 512 of this lane's signal (level-0 slice + halo).
// xch: this wave's exchange area (64 lanes * kSlot doubles); gbase = first lane of the group.
// Returns a6[s] and d6[s].
template <bool FAST, bool SHFL = false>
__device__ __forceinline__ void dwt8_cascade(const double (&x)[kIn], double* xch, int gbase, int s,
                                             double& a6, double& d6) {
  double a1[32 + 8];
  lowpass<32, FAST>(x, a1);
  if constexpr (FAST) {  // x already holds the level-0 halo; levels 2..6 by partial sums
    levels2to6_ps(a1, gbase, s, a6, d6);
    (void)xch;
    return;
  }
  halo<32, SHFL>(a1, xch, gbase, s);
  double a2[16 + 8];
  lowpass<16, FAST>(a1, a2);
  halo<16, SHFL>(a2, xch, gbase, s);
  double a3[8 + 8];
  lowpass<8, FAST>(a2, a3);
  halo<8, SHFL>(a3, xch, gbase, s);
  double a4[4 + 8];
  lowpass<4, FAST>(a3, a4);
  halo<4, SHFL>(a4, xch, gbase, s);
  double a5[2 + 8];
  lowpass<2, FAST>(a4, a5);
  halo<2, SHFL>(a5, xch, gbase, s);
  a6 = fir10<FAST, false>(a5);
  d6 = fir10<FAST, true>(a5);
}

}  // namespace dev
}  // namespace eegfx

#endif  // EEGFX_DWT8_H
