// kernels.hip -- gfx950 kernels of the epoch-to-feature path and their launchers.
//
//   cut_epochs_kernel            a3 + a5..a7: raw multiplexed samples -> baseline-corrected
//                                epochs double[n][C][750]  (OffLineDataProvider.java:216-233)
//   features_from_epochs_kernel  a11..a13: epochs -> L2-normalised dwt-8 features
//                                (WaveletTransform.java:107-141, SignalProcessing.java:38-52)
//   fused kernel                 see fused.hip (raw -> features, the benchmarked hot path)
//   synth_kernel                 deterministic synthetic recordings for tests and bench.py
//
// Compiled with -ffp-contract=off: every fp32/fp64 expression is evaluated as written, one
// correctly rounded IEEE operation at a time, matching the Java (strictfp-equivalent) order.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "dwt8.h"
#include "guard.h"
#include "launch.h"
#include "rows.h"

namespace eegfx {
namespace dev {

// a3 + a5..a7.  One workgroup per epoch.  Lanes 0..C-1 fold the 100 pre-stimulus samples of
// their channel sequentially in fp32 (Baseline.java:29-42 -- order-exact, so no tree reduction),
// then all lanes write the 750 post-stimulus samples, coalesced.
template <typename T>
__global__ __launch_bounds__(256) void cut_epochs_kernel(const T* __restrict__ raw, int64_t n_frames,
                                                         int ct, ChanSel sel, int C,
                                                         const int64_t* __restrict__ pos,
                                                         double* __restrict__ out,
                                                         int* __restrict__ err) {
  __shared__ float base[kMaxChannels];
  const int64_t e = blockIdx.x;
  const int64_t p0 = pos[e];
  // OffLineDataProvider.java:220-225 (see fused.hip position_ok): an invalid position is flagged
  // and cut as pos = 100
  const bool ok = p0 >= kPre && p0 - kPre <= n_frames;
  if (threadIdx.x == 0 && !ok && err)
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int64_t p = ok ? p0 : kPre;
  const int64_t lo = p - kPre;
  if ((int)threadIdx.x < C) {
    const int c = threadIdx.x;
    const int col = sel.col[c];
    const float r = sel.res[c];
    float b = 0.0f;
    for (int i = 0; i < kPre; ++i) {
      const int64_t f = lo + i;
      // Arrays.copyOfRange zero-pads past the end (toFloatArray -> 0.0f).
      const float v = (f >= 0 && f < n_frames) ? (float)raw[f * ct + col] * r : 0.0f;
      b = b + v;
    }
    base[c] = b / (float)kPre;
  }
  __syncthreads();
  double* o = out + e * C * kPost;
  for (int idx = threadIdx.x; idx < C * kPost; idx += blockDim.x) {
    const int c = idx / kPost;
    const int64_t f = p + (idx - c * kPost);
    const float v = (f >= 0 && f < n_frames) ? (float)raw[f * ct + sel.col[c]] * sel.res[c] : 0.0f;
    o[idx] = (double)(v - base[c]);
  }
}

// a5..a7 write pass of the materialised epochs (getData()): the per-(epoch, channel) baselines
// come from the LDS-staged baseline kernels; each lane writes two consecutive samples of one
// channel row as one 16-byte store (750 is even, so a pair never straddles two rows).
template <typename T>
__global__ __launch_bounds__(256) void cut_write_kernel(const T* __restrict__ raw, int64_t n_frames,
                                                        int ct, ChanSel sel, int C,
                                                        const int64_t* __restrict__ pos,
                                                        const float* __restrict__ base,
                                                        double* __restrict__ out) {
  const int64_t e = blockIdx.x;
  const int64_t p0 = pos[e];
  const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : kPre;  // flagged by the baselines
  double* o = out + e * C * kPost;
  for (int idx = 2 * (int)threadIdx.x; idx < C * kPost; idx += 2 * (int)blockDim.x) {
    const int c = idx / kPost;
    const int64_t f = p + (idx - c * kPost);
    const int col = sel.col[c];
    const float r = sel.res[c], b = base[e * C + c];
    // Arrays.copyOfRange zero-pads past the end (toFloatArray -> 0.0f)
    const float v0 = f >= 0 && f < n_frames ? (float)raw[f * ct + col] * r : 0.0f;
    const float v1 = f + 1 >= 0 && f + 1 < n_frames ? (float)raw[(f + 1) * ct + col] * r : 0.0f;
    *(double2*)(o + idx) = make_double2((double)(v0 - b), (double)(v1 - b));
  }
}

// The same write pass for epochs of at most kCutPairs * 256 sample pairs (C <= 3): the channel
// parameters and the epoch's baselines go to LDS first, and each thread issues the raw reads of
// all its pairs before the first store, so a workgroup waits on memory twice instead of twice per
// loop trip (3 channels: 7.3-7.4 -> 6.0-6.7 ms per 1M epochs, profiles/r03as/, r03au/).  Since
// the LDS-staged passes below (4.6 ms there, profiles/r03az/) it serves only the layouts they skip:
// a few channels of a wide montage (ct > 8 C) or a raw buffer that is not dword aligned.
constexpr int kCutPairs = 5;
template <typename T>
__global__ __launch_bounds__(256) void cut_write_small_kernel(
    const T* __restrict__ raw, int64_t n_frames, int ct, ChanSel sel, int C,
    const int64_t* __restrict__ pos, const float* __restrict__ base, double* __restrict__ out) {
  __shared__ int s_col[kMaxChannels];
  __shared__ float s_res[kMaxChannels], s_base[kMaxChannels];
  const int t = threadIdx.x;
  const int64_t e = blockIdx.x;
  if (t < C) {
    s_col[t] = sel.col[t];
    s_res[t] = sel.res[t];
    s_base[t] = base[e * C + t];
  }
  const int64_t p0 = pos[e];
  const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : kPre;  // flagged by the baselines
  __syncthreads();
  double* o = out + e * C * kPost;
  const int npairs = C * (kPost / 2);  // <= 256 * kCutPairs (launcher)
  float v0[kCutPairs], v1[kCutPairs];
#pragma unroll
  for (int u = 0; u < kCutPairs; ++u) {
    const int idx = 256 * u + t;
    v0[u] = v1[u] = 0.0f;
    if (idx < npairs) {
      const int c = idx / (kPost / 2);
      const int64_t f = p + 2 * (idx - c * (kPost / 2));
      const int col = s_col[c];
      const float r = s_res[c];
      // Arrays.copyOfRange zero-pads past the end (toFloatArray -> 0.0f)
      if (f >= 0 && f < n_frames) v0[u] = (float)raw[f * ct + col] * r;
      if (f + 1 >= 0 && f + 1 < n_frames) v1[u] = (float)raw[(f + 1) * ct + col] * r;
    }
  }
#pragma unroll
  for (int u = 0; u < kCutPairs; ++u) {
    const int idx = 256 * u + t;
    if (idx < npairs) {
      const float b = s_base[idx / (kPost / 2)];
      *(double2*)(o + 2 * idx) = make_double2((double)(v0[u] - b), (double)(v1[u] - b));
    }
  }
}

// The one-pass getData + extractFeatures of the staged write passes (FEAT: eegfx_process_recording_
// epochs, OffLineDataProvider.loadData then WaveletTransform.extractFeatures over its epochs,
// OffLineDataProvider.java:216-233 + WaveletTransform.java:107-141): after the workgroup has
// written the epoch's rows, the window frames [175, 687) are still staged in LDS, so the filter
// bank runs on them there -- lane = (channel, segment), 8 lanes per signal, 32 signals per pass
// of the 4 waves (C <= 64: at most two passes) -- instead of a second pass that re-reads the
// 12 KB of window rows from HBM.  smp(f, col): the staged raw sample of post-stimulus frame f;
// gsmp(f, col): the same sample from the recording (both zero past its end).  The decode, filter
// banks, normalisation and the fma guard are those of the fused kernels.  The feature row and the
// guard's rare-path scratch alias the staged frames once every wave is done with them (a barrier),
// so the LDS stays that of the plain write pass: configs[3]'s 51 KB, three workgroups per CU.
template <bool FAST, bool MEASURE, typename Smp, typename GSmp>
__device__ __forceinline__ void staged_features(Smp smp, GSmp gsmp, const int* s_col,
                                                const float* s_res, const float* s_base, int C,
                                                double* stage, double* gx, double* sh,
                                                double* __restrict__ fo, const Guard& guard,
                                                int tid) {
  const int lane = tid & 63, w = tid >> 6, s = lane & 7;
  double a6v[2] = {0.0, 0.0}, d6v[2] = {0.0, 0.0};
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int c0 = 32 * pass + 8 * w;
    if (c0 >= C) break;  // uniform per wave
    const int c = c0 + (lane >> 3);
    const bool valid = c < C;
    const int cc = valid ? c : 0;
    const int col = s_col[cc];
    const float r = s_res[cc], b = s_base[cc];
    auto own = [&](int k) { return smp(175 + kSegLen * s + k, col); };
    if constexpr (FAST) {
      float ym = 0.0f;
      dwt8_collapsed_cascade<MEASURE>(own, r, b, lane & ~7, s, a6v[pass], d6v[pass], &ym);
      double x2;
      if constexpr (MEASURE) {
        const double X = (double)group8_max(ym);
        x2 = X * X;
      } else {
        x2 = guard_x2_int16(r, b);
      }
      if (valid && s == 0) gx[c] = x2;
    } else {
      double a1[40];
      level1_exact(own, r, b, lane & ~7, s, a1);
      halo<32, true>(a1, nullptr, lane & ~7, s);
      dwt8_levels2to6<false, true>(a1, nullptr, lane & ~7, s, a6v[pass], d6v[pass]);
    }
  }
  __syncthreads();  // every wave is done with the staged frames: the row may overwrite them
  double* feat = stage;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int c = 32 * pass + 8 * w + (lane >> 3);
    if (c < C) {
      feat[c * 16 + s] = a6v[pass];
      feat[c * 16 + 8 + s] = d6v[pass];
    }
  }
  __syncthreads();
  const int F = 16 * C;
  if (w == 0) {  // SignalProcessing.normalize (SignalProcessing.java:38-52)
    if constexpr (FAST) {
      double acc = 0.0;
      for (int i = lane; i < F; i += 64) acc = __builtin_fma(feat[i], feat[i], acc);
      double sx = lane < C ? gx[lane] : 0.0;  // C <= 64
      for (int off = 32; off > 0; off >>= 1) {
        acc += __shfl_xor(acc, off, 64);
        sx += __shfl_xor(sx, off, 64);
      }
      bool fails = guard.total && guard_fails(acc, kGuardK2Collapsed, sx);  // wave-uniform
      if (!MEASURE && fails) {  // int16: the second stage, the row's measured max |x|
        if (lane == 0) guard_count_rechecked(guard, 1);
        fails = guard_fails(acc, kGuardK2Collapsed,
                            guard_measured_x2_wave(
                                [&](int c, int k) { return (int)gsmp(175 + k, s_col[c]); },
                                [&](int c, float v) {
                                  float y = v * s_res[c];
                                  y = y - s_base[c];
                                  return (double)y;
                                },
                                C, lane));
      }
      if (lane == 0) {
        sh[0] = rsqrt_nr(acc);
        sh[1] = fails ? 1.0 : 0.0;
      }
    } else if (lane == 0) {
      double acc = 0.0;
      for (int i = 0; i < F; ++i) acc = acc + feat[i] * feat[i];
      sh[0] = sqrt(acc);
    }
  }
  __syncthreads();
  if constexpr (FAST) {
    if (sh[1] != 0.0) {  // the guard's rare path: wave 0 recomputes the row under EXACT from the
                         // recording, the LDS past the row as scratch
      if (w == 0) {
        dwt8_exact_row_wave(
            [&](int c, int k) {
              float y = gsmp(175 + k, s_col[c]) * s_res[c];
              y = y - s_base[c];
              return (double)y;
            },
            C, 16, feat + F, feat, lane);
        if (lane == 0) {
          sh[0] = 1.0;  // the row is normalised
          guard_count_recomputed(guard, 1ull);
        }
      }
      __syncthreads();
    }
  }
  const double nv = sh[0];
  for (int i = tid; i < F; i += 256) fo[i] = FAST ? feat[i] * nv : feat[i] / nv;
}

// LDS of the FEAT variants: the staged frames, or the feature row + the rare path's scratch that
// alias them if larger (16-byte aligned), then the guard's X^2 per channel and two shared words.
__host__ __device__ constexpr size_t staged_features_lds(size_t stage_bytes, int C) {
  return (((stage_bytes > (size_t)(16 * C + 768) * 8 ? stage_bytes : (size_t)(16 * C + 768) * 8)
           + 15) & ~(size_t)15) + 64 * 8 + 16;
}

// The one-pass getData + features for the reference's 3-channel file (6-byte int16 frames, the
// Fz/Cz/Pz selection; configs[0]-[2]): eight epochs per workgroup of four waves, so that the
// filter bank runs with full waves -- wave c = channel c, lane = (epoch, segment), the layout of
// the fused window kernel -- where the per-epoch staged kernel above leaves 232 of 256 lanes idle
// (measured: one pass 8.1 ms against 7.2 ms for the two passes, profiles/r04f).
//  1. stage: each epoch's 750 post-stimulus frames (1,127 dwords from the dword holding its first
//     byte) go to LDS with one skew dword per 96 (every 64 frames), so the 8 segment lanes of a
//     signal, 64 frames apart, read 8 distinct banks; epochs 1,160 dwords apart (8 mod 32).
//  2. rows: every thread decodes sample pairs (float)raw * res - b of (epoch, channel) rows and
//     stores them as 16-byte pairs, consecutive threads on consecutive pairs (the getData()
//     epochs, OffLineDataProvider.java:216-233).
//  3. features: waves 0-2 run the filter bank on the staged window frames [175, 687) (sample k of
//     segment s: half 3 (175 + 64 s + k) + col past the epoch's start half; its skew is
//     2 + s + [k >= 17], or [k >= 16] when the start half is odd and col = 2), then the rows are
//     normalised and stored as in the window kernel, fma rows through the conditioning guard.
constexpr int kCfEpochs = 8;
constexpr int kCfDwords = 1127;  // dwords staged per epoch: (2 + 750 * 6 + 3) / 4, rounded up
constexpr int kCfStride = 1160;  // LDS dwords per epoch: 1,127 + 12 skew dwords, = 8 (mod 32)
__device__ __forceinline__ int cf_lds_dword(int d) { return d + (int)(((uint32_t)d * 683u) >> 16); }
template <bool FAST, bool FEAT = true>
__global__ __launch_bounds__(256) void cut_features_c3_kernel(
    const int16_t* __restrict__ raw, int64_t n_frames, ChanSel sel,
    const int64_t* __restrict__ pos, const float* __restrict__ base, int64_t n,
    double* __restrict__ out, double* __restrict__ fout, Guard guard) {
  constexpr int CT = 3, C = 3, FB = 6, F = 48;
  static_assert(kCfEpochs * F * 8 + 768 * 8 <= kCfEpochs * kCfStride * 4, "rows + scratch alias");
  __shared__ __attribute__((aligned(16))) uint32_t stage[kCfEpochs * kCfStride];
  __shared__ double norm[kCfEpochs];
  __shared__ double gx[kCfEpochs * C];
  __shared__ int64_t sA[kCfEpochs];  // dword index of each epoch's first staged byte
  __shared__ int sH[kCfEpochs];      // 1 when the first frame starts at an odd half
  __shared__ int64_t sP[kCfEpochs];  // the (valid) marker position: frame of the first sample
  __shared__ int s_col[C];
  __shared__ float s_res[C], s_base[kCfEpochs * C];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t e0 = (int64_t)blockIdx.x * kCfEpochs;
  const int ne = n - e0 < kCfEpochs ? (int)(n - e0) : kCfEpochs;
  const int64_t nbytes = n_frames * FB;
  if (tid < kCfEpochs) {
    const int64_t p0 = tid < ne ? pos[e0 + tid] : kPre;
    const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : kPre;  // flagged by the baselines
    sA[tid] = (p * FB) >> 2;
    sH[tid] = (int)((p * FB) & 3) >> 1;
    sP[tid] = p;
  }
  if (tid < C) {
    s_col[tid] = sel.col[tid];
    s_res[tid] = sel.res[tid];
  }
  if (tid < kCfEpochs * C) s_base[tid] = tid < ne * C ? base[e0 * C + tid] : 0.0f;
  __syncthreads();
  {  // 1. stage (8 loads in flight per thread; the dword holding the recording's last two bytes
     //    is read as a half, nothing past the end)
    const uint32_t* src = (const uint32_t*)raw;
    constexpr int TOTAL = kCfEpochs * kCfDwords;
    for (int k0 = 0; k0 < TOTAL; k0 += 8 * 256) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 256 * u + tid;
        const int m = k / kCfDwords, d = k - m * kCfDwords;
        v[u] = 0u;
        if (k < TOTAL && m < ne) {
          const int64_t a = (sA[m] + d) * 4;
          if (a + 4 <= nbytes) v[u] = src[sA[m] + d];
          else if (a + 2 <= nbytes) v[u] = (uint16_t)raw[a >> 1];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 256 * u + tid;
        const int m = k / kCfDwords, d = k - m * kCfDwords;
        if (k < TOTAL) stage[m * kCfStride + cf_lds_dword(d)] = v[u];
      }
    }
  }
  __syncthreads();
  const int16_t* hs = (const int16_t*)stage;
  // staged half h of epoch m (h counted from the epoch's first staged byte)
  auto half = [&](int m, int h) { return hs[2 * m * kCfStride + h + 2 * (int)(((uint32_t)(h >> 1) * 683u) >> 16)]; };
  {  // 2. rows: pair q of (epoch m, channel c) = frames 2q, 2q + 1
    constexpr int HP = kPost / 2, PER_E = C * HP;
    int idx = tid;
    int m = idx / PER_E, rem = idx - m * PER_E;
    int c = rem / HP, q = rem - c * HP;
    for (; idx < ne * PER_E; idx += 256) {
      const int h0 = sH[m] + 6 * q + s_col[c];
      const int64_t g = sP[m] + 2 * q;  // frame of the pair in the file
      const float r = s_res[c], b = s_base[m * C + c];
      // Arrays.copyOfRange zero-pads past the end (toFloatArray -> 0.0f)
      const float v0 = g < n_frames ? (float)half(m, h0) * r : 0.0f;
      const float v1 = g + 1 < n_frames ? (float)half(m, h0 + 3) * r : 0.0f;
      *(double2*)(out + ((e0 + m) * C + c) * kPost + 2 * q) =
          make_double2((double)(v0 - b), (double)(v1 - b));
      q += 256 % HP;
      c += 256 / HP;
      if (q >= HP) { q -= HP; ++c; }
      while (c >= C) { c -= C; ++m; }
    }
  }
  if constexpr (!FEAT) return;  // getData() alone (eegfx_cut_epochs_f64)
  // 3. features: wave c = channel c (waves 0-2), lane = (epoch el, segment s)
  const int el = lane >> 3, s = lane & 7;
  double a6 = 0.0, d6 = 0.0;
  if (w < C) {
    const int c = w, col = s_col[c];
    const int m = el < ne ? el : 0;
    const float r = s_res[c], b = s_base[m * C + c];
    const int hb = sH[m] + col + 3 * (175 + kSegLen * s);  // half of sample 0 of this segment
    const int16_t* own = hs + 2 * m * kCfStride + hb + 2 * (2 + s);
    const bool late16 = sH[m] + col == 3;                 // sample 16 already past the skew
    auto fetch = [&](int k) {
      return (float)own[3 * k + (k >= 17 ? 2 : (k == 16 && late16 ? 2 : 0))];
    };
    if constexpr (FAST) {
      dwt8_collapsed_cascade(fetch, r, b, lane & ~7, s, a6, d6);
      if (s == 0) gx[el * C + c] = guard_x2_int16(r, b);
    } else {
      double a1[40];
      level1_exact(fetch, r, b, lane & ~7, s, a1);
      halo<32, true>(a1, nullptr, lane & ~7, s);
      dwt8_levels2to6<false, true>(a1, nullptr, lane & ~7, s, a6, d6);
    }
  }
  double* fb = (double*)stage;
  __syncthreads();  // every wave is done with the staged frames: the rows may overwrite them
  if (w < C) {
    fb[el * F + w * 16 + s] = a6;
    fb[el * F + w * 16 + 8 + s] = d6;
  }
  __syncthreads();
  if (w == 0) {
    // the guard's rare path: the row recomputed under EXACT from the recording, the LDS past the
    // 8 rows as scratch (the other waves are done)
    auto redo = [&](int e, double* row) {
      const int64_t f0 = sP[e] + 175;
      dwt8_exact_row_wave(
          [&](int cc, int k) {
            const float v = f0 + k < n_frames ? (float)raw[(f0 + k) * CT + s_col[cc]] : 0.0f;
            float y = v * s_res[cc];
            y = y - s_base[e * C + cc];
            return (double)y;
          },
          C, 16, fb + kCfEpochs * F, row, lane);
    };
    // the guard's second stage: the row's measured max |x| per channel, from the recording
    auto recheck = [&](int e) {
      return recheck_c3<FB, 1>((const uint8_t*)raw, n_frames, sel, (sP[e] + 175) * FB,
                            s_base + e * C, nullptr, true, lane);
    };
    normalise_store<F, FAST, C>(fb, norm, fout + e0 * F, ne, lane, gx, guard, redo,
                                per_row_recheck(recheck));
  }
}

// The LDS-staged write pass for frames of a whole number of dwords (e.g. configs[3]'s 32-channel
// montage; used while the staged frames are at most twice the rows written, ct <= 8 C for int16).
// Reading one channel's samples straight from the multiplexed recording puts consecutive lanes a
// whole frame (64 B at 32 int16 channels) apart, so each wave load touches 64 cache lines for 128
// useful bytes (11.9 ms per 50k 32-channel epochs, 1.0 TB/s, profiles/r03at/).  Here workgroup
// (e, chunk) copies frames [f0, f0 + nf) of epoch e's post-stimulus span into LDS with coalesced
// dword loads, one padding dword per frame (frame stride FW + 1 dwords: odd when FW is even, so 64
// lanes reading 64 frames of one channel hit 64 distinct banks), then each lane decodes two
// consecutive samples of one channel row and stores them as one 16-byte pair: 2.3 ms
// (profiles/r03bc/; 16-byte staging loads measured the same as dword loads, profiles/r03az/).  Frames past the recording's end
// read as 0.0f (Arrays.copyOfRange zero padding).
// Chunk size: one chunk per epoch up to 64 KB of LDS (32 int16 channels: 51 KB, 3 workgroups per
// CU) -- each workgroup's rows are then one contiguous 192 KB run.  Chunks of 12 / 16 / 32 KB
// (more workgroups per CU, rows written in pieces) took 3.71 / 3.54 / 3.14 ms against 2.30-2.33 ms
// for 50k 32-channel epochs, C = 3 unchanged (profiles/r03bc/ab.log; -DEEGFX_CUT_LDS_MAX builds).
#ifndef EEGFX_CUT_LDS_MAX
#define EEGFX_CUT_LDS_MAX (64 * 1024)
#endif
constexpr int kCutLdsMax = EEGFX_CUT_LDS_MAX;
template <typename T, bool FEAT = false, bool FAST = false>
__global__ __launch_bounds__(256) void cut_write_lds_kernel(
    const T* __restrict__ raw, int64_t n_frames, int ct, ChanSel sel, int C,
    const int64_t* __restrict__ pos, const float* __restrict__ base, double* __restrict__ out,
    int nfc, double* __restrict__ fout = nullptr, Guard guard = Guard{nullptr, nullptr, nullptr}) {
  extern __shared__ __attribute__((aligned(16))) uint32_t stage[];
  __shared__ int s_col[kMaxChannels];
  __shared__ float s_res[kMaxChannels], s_base[kMaxChannels];
  const int t = threadIdx.x;
  const int64_t e = blockIdx.x;
  const int f0 = (int)blockIdx.y * nfc;
  const int nf = kPost - f0 < nfc ? kPost - f0 : nfc;  // even: nfc and kPost are
  if (t < C) {
    s_col[t] = sel.col[t];
    s_res[t] = sel.res[t];
    s_base[t] = base[e * C + t];
  }
  const int64_t p0 = pos[e];
  const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : kPre;  // flagged by the baselines
  const int FW = ct * (int)sizeof(T) / 4, FS = FW + 1;
  const int64_t g0 = p + f0;  // first frame of this chunk
  const uint32_t* src = (const uint32_t*)raw;
  {  // dword k of the chunk is (frame k / FW, word k % FW); 8 loads in flight per thread
    const int total = nf * FW, sf = 256 / FW, sw = 256 % FW;
    int f = t / FW, w = t - (t / FW) * FW;
    for (int k0 = 0; k0 < total; k0 += 8 * 256) {
      uint32_t v[8];
      int fk[8], wk[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        fk[u] = f;
        wk[u] = w;
        const bool in = k0 + 256 * u + t < total && g0 + f < n_frames;
        v[u] = in ? src[(g0 + f) * FW + w] : 0u;
        f += sf;
        w += sw;
        if (w >= FW) { w -= FW; ++f; }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k0 + 256 * u + t < total) stage[fk[u] * FS + wk[u]] = v[u];
    }
  }
  __syncthreads();
  // rows: pair q of channel c covers frames f0 + 2q, f0 + 2q + 1
  const int hp = nf / 2, npairs = C * hp, sc = 256 / hp, sq = 256 % hp;
  int c = t / hp, q = t - (t / hp) * hp;
  double* o = out + e * C * kPost + f0;
  for (int idx = t; idx < npairs; idx += 256) {
    const int col = s_col[c];
    const float r = s_res[c], b = s_base[c];
    const int f = 2 * q;
    float s0, s1;
    if constexpr (sizeof(T) == 2) {
      const int16_t* h = (const int16_t*)stage;
      s0 = (float)h[2 * f * FS + col];
      s1 = (float)h[2 * (f + 1) * FS + col];
    } else {
      const float* h = (const float*)stage;
      s0 = h[f * FS + col];
      s1 = h[(f + 1) * FS + col];
    }
    // Arrays.copyOfRange zero-pads past the end (toFloatArray -> 0.0f)
    const float v0 = g0 + f < n_frames ? s0 * r : 0.0f;
    const float v1 = g0 + f + 1 < n_frames ? s1 * r : 0.0f;
    *(double2*)(o + (int64_t)c * kPost + f) = make_double2((double)(v0 - b), (double)(v1 - b));
    c += sc;
    q += sq;
    if (q >= hp) { q -= hp; ++c; }
  }
  if constexpr (FEAT) {  // one chunk per epoch (launcher): the window frames are staged
    double* gx = (double*)((uint8_t*)stage + staged_features_lds((size_t)nf * FS * 4, C) - 64 * 8 - 16);
    staged_features<FAST, !std::is_same<T, int16_t>::value>(
        [&](int f, int col) {
          if constexpr (sizeof(T) == 2) return (float)((const int16_t*)stage)[2 * f * FS + col];
          else return ((const float*)stage)[f * FS + col];
        },
        [&](int f, int col) {
          return g0 + f < n_frames ? (float)raw[(g0 + f) * ct + col] : 0.0f;
        },
        s_col, s_res, s_base, C, (double*)stage, gx, gx + 64, fout + e * 16 * C, guard, t);
  }
}

// The same LDS-staged write pass for int16 frames that are not a whole number of dwords (the
// 3-channel path of configs[0]-[2]: 6-byte frames): the chunk's bytes are staged as they lie, from
// the dword that holds its first frame, without per-frame padding; lanes reading the sample pairs
// of one channel are 2 frames apart (3 dwords at 3 channels: an odd stride, no bank conflicts).
// The dword holding the recording's last two bytes is read as a half so no load passes its end.
template <bool FEAT = false, bool FAST = false>
__global__ __launch_bounds__(256) void cut_write_lds_packed_kernel(
    const int16_t* __restrict__ raw, int64_t n_frames, int ct, ChanSel sel, int C,
    const int64_t* __restrict__ pos, const float* __restrict__ base, double* __restrict__ out,
    int nfc, double* __restrict__ fout = nullptr, Guard guard = Guard{nullptr, nullptr, nullptr}) {
  extern __shared__ __attribute__((aligned(16))) uint32_t stage[];
  __shared__ int s_col[kMaxChannels];
  __shared__ float s_res[kMaxChannels], s_base[kMaxChannels];
  const int t = threadIdx.x;
  const int64_t e = blockIdx.x;
  const int f0 = (int)blockIdx.y * nfc;
  const int nf = kPost - f0 < nfc ? kPost - f0 : nfc;
  if (t < C) {
    s_col[t] = sel.col[t];
    s_res[t] = sel.res[t];
    s_base[t] = base[e * C + t];
  }
  const int64_t p0 = pos[e];
  const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : kPre;  // flagged by the baselines
  const int64_t g0 = p + f0;
  const int FB = 2 * ct;
  const int64_t nbytes = n_frames * FB;
  const int64_t b0 = g0 * FB;                 // first byte of the chunk
  const int64_t a0 = b0 >> 2;                 // its dword
  const int delta = (int)(b0 & 3);            // 0 or 2
  const int total = (delta + nf * FB + 3) >> 2;
  const uint32_t* src = (const uint32_t*)raw;
  for (int k0 = 0; k0 < total; k0 += 8 * 256) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + 256 * u + t;
      const int64_t a = (a0 + k) * 4;
      v[u] = 0u;
      if (k < total) {
        if (a + 4 <= nbytes) v[u] = src[a0 + k];
        else if (a + 2 <= nbytes) v[u] = (uint16_t)raw[(a >> 1)];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + 256 * u + t < total) stage[k0 + 256 * u + t] = v[u];
  }
  __syncthreads();
  const int16_t* h = (const int16_t*)((const uint8_t*)stage + delta);
  const int hp = nf / 2, npairs = C * hp, sc = 256 / hp, sq = 256 % hp;
  int c = t / hp, q = t - (t / hp) * hp;
  double* o = out + e * C * kPost + f0;
  for (int idx = t; idx < npairs; idx += 256) {
    const int col = s_col[c];
    const float r = s_res[c], b = s_base[c];
    const int f = 2 * q;
    // Arrays.copyOfRange zero-pads past the end (toFloatArray -> 0.0f)
    const float v0 = g0 + f < n_frames ? (float)h[f * ct + col] * r : 0.0f;
    const float v1 = g0 + f + 1 < n_frames ? (float)h[(f + 1) * ct + col] * r : 0.0f;
    *(double2*)(o + (int64_t)c * kPost + f) = make_double2((double)(v0 - b), (double)(v1 - b));
    c += sc;
    q += sq;
    if (q >= hp) { q -= hp; ++c; }
  }
  if constexpr (FEAT) {  // one chunk per epoch (launcher): the window frames are staged
    double* gx = (double*)((uint8_t*)stage + staged_features_lds((size_t)total * 4, C) - 64 * 8 - 16);
    staged_features<FAST, false>(
        [&](int f, int col) { return (float)h[f * ct + col]; },
        [&](int f, int col) {
          return g0 + f < n_frames ? (float)raw[(g0 + f) * ct + col] : 0.0f;
        },
        s_col, s_res, s_base, C, (double*)stage, gx, gx + 64, fout + e * 16 * C, guard, t);
  }
}

// a11..a13 from materialised epochs.  One wave per workgroup owns 8 epochs and walks their
// channels; lane = 8*epoch + segment (dwt8.h).  For each channel the wave reads the 8 windows
// (512 doubles each, contiguous in the epoch rows) with 16-byte loads, 1 KB of one window per
// load instruction, and writes them to LDS in a bank-skewed layout: segment s of window g at
// g*kFeWin + s*kFeSeg doubles.  kFeSeg = 65 doubles (130 dwords, 2 mod 64) and kFeWin = 520
// (1,040 dwords, 16 mod 64), so the ds_read_b64 of lane (g, s) for any sample index falls on
// banks 16g + 2s (+1) plus a common offset: the 32 lanes of a half-wave use 64 distinct banks.
// (Each lane reading its own 512 contiguous bytes straight from memory touches 64 cache lines
// per load instruction; that pattern moved ~1.9 TB/s.)  The filter bank then runs from LDS: FMA
// the collapsed four-point filter of dwt8_collapsed_core on the doubles as they are, EXACT the
// level-by-level cascade with value halos.  Features collect in LDS, are normalised per epoch
// with the reference's sequential sum of squares and written coalesced.  33 KB of windows per
// workgroup: 4 workgroups per CU.
constexpr int kFeSeg = kSegLen + 1;
constexpr int kFeWin = 8 * kFeSeg;
constexpr size_t kFeWinBytes = sizeof(double) * 8 * kFeWin;
typedef double f64x2_a8 __attribute__((ext_vector_type(2), aligned(8)));

// Under fma numerics each lane also keeps the largest |x| of its samples, and the rows are
// checked against the conditioning guard (guard.h: sum over the channels of the measured X^2); a
// row that fails is recomputed under EXACT by the wave from the epochs in memory, the window LDS
// as scratch (rare).
// ROWS_OUT (wide rows, launcher): the 8 feature rows (8 F doubles: 32 KB at C = 32) do not stay in
// LDS, where they halved the resident workgroups.  After each channel the 8 x nfeat values pass
// through a 1 KB LDS tile, leave as whole 128-byte runs into `out`, and lanes 0-7 add their
// squares to the epoch's sum in index order (the reference's sequential sum,
// SignalProcessing.java:38-52); at the end the wave rescales its rows in place (L2-resident).
template <bool FAST, bool ROWS_OUT>
__global__ __launch_bounds__(64) void features_from_epochs_kernel(const double* __restrict__ ep,
                                                                  int64_t n, int C, int skip,
                                                                  int nfeat, int row_stride,
                                                                  double* __restrict__ out,
                                                                  Guard guard) {
  __shared__ __attribute__((aligned(16))) double win[8 * kFeWin];
  extern __shared__ __attribute__((aligned(16))) double fsmem[];
  const int lane = threadIdx.x;
  const int el = lane >> 3, s = lane & 7;
  const int F = C * nfeat;
  double* feat = fsmem;                             // [8][F], or the [8][16] tile (ROWS_OUT)
  double* norm = feat + (ROWS_OUT ? 8 * 16 : 8 * F);  // [8]
  const int64_t e0 = (int64_t)blockIdx.x * 8;
  const int64_t ne = (n - e0) < 8 ? (n - e0) : 8;
  double* o = out + e0 * F;
  // quad q = 64 (j % 4) + lane of window j / 4: doubles 2q, 2q + 1 of segment q / 32.  Epochs
  // past n read the last epoch's window (the loads stay unconditional; the result is dropped).
  // Channel c + 1's windows are in flight while channel c runs the filter bank.
  f64x2_a8 v[32];
  auto load = [&](int c) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int g = j >> 2;
      const int64_t e = e0 + (g < ne ? g : ne - 1);
      const int q = ((j & 3) << 6) | lane;
      v[j] = __builtin_nontemporal_load((const f64x2_a8*)(ep + (e * C + c) * row_stride + skip + 2 * q));
    }
  };
  load(0);
  double sx = 0.0;   // fma: sum over the channels of this lane's signal's X^2
  double acc = 0.0;  // ROWS_OUT, lanes < ne: epoch `lane`'s sum of squares so far
  for (int c = 0; c < C; ++c) {
    wave_sync();  // the previous channel's LDS reads precede these writes
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int q = ((j & 3) << 6) | lane;
      double* d = win + (j >> 2) * kFeWin + (q >> 5) * kFeSeg + 2 * (q & 31);
      d[0] = v[j].x;
      d[1] = v[j].y;
    }
    wave_sync();
    if (c + 1 < C) load(c + 1);
    const double* own = win + el * kFeWin + s * kFeSeg;
    double a6, d6;
    if constexpr (FAST) {
      double xm = 0.0;
      dwt8_collapsed_core([&](int k) { return own[k]; },
                          [&](double v0, double v1, double& x0, double& x1) {
                            xm = fmax(xm, fmax(fabs(v0), fabs(v1)));
                            x0 = v0;
                            x1 = v1;
                          },
                          lane & ~7, s, a6, d6);
      xm = group8_max(xm);
      sx += xm * xm;
    } else {
      const double* sig = win + el * kFeWin;
      double x[kIn];
#pragma unroll
      for (int k = 0; k < kIn; ++k) x[k] = k < kSegLen ? own[k] : sig[((s + 1) & 7) * kFeSeg + k - kSegLen];
      dwt8_cascade<false, true>(x, nullptr, lane & ~7, s, a6, d6);
    }
    if constexpr (ROWS_OUT) {
      feat[el * 16 + s] = a6;  // the tile's previous reads finished before the window writes
      feat[el * 16 + 8 + s] = d6;
      wave_sync();
      for (int idx = lane; idx < ne * nfeat; idx += 64) {
        const int e = idx / nfeat, j = idx - e * nfeat;
        o[(int64_t)e * F + c * nfeat + j] = feat[e * 16 + j];
      }
      if (lane < ne)
        for (int j = 0; j < nfeat; ++j) {
          const double f = feat[lane * 16 + j];
          acc = acc + f * f;  // Math.pow(f, 2) summed in index order
        }
    } else if (el < ne) {
      if (s < nfeat) feat[el * F + c * nfeat + s] = a6;
      if (8 + s < nfeat) feat[el * F + c * nfeat + 8 + s] = d6;
    }
  }
  wave_sync();
  const double sx_row = __shfl(sx, (lane & 7) * 8, 64);  // epoch `lane`'s X^2 sum (lanes < 8)
  bool fails = false;
  if (lane < ne) {
    if constexpr (!ROWS_OUT) {
      for (int i = 0; i < F; ++i) {
        const double f = feat[lane * F + i];
        acc = acc + f * f;  // Math.pow(f, 2) summed in index order
      }
    }
    norm[lane] = sqrt(acc);
    fails = FAST && guard.total && guard_fails(acc, kGuardK2Collapsed, sx_row);
  }
  if constexpr (FAST) {  // the guard's rare path: flagged rows recomputed under EXACT in place
    uint64_t flagged = __ballot(fails);
    if (flagged) {
      wave_sync();
      if (lane == 0) guard_count_recomputed(guard, (unsigned long long)__popcll(flagged));
      do {
        const int e = __ffsll((unsigned long long)flagged) - 1;
        const double* row = ep + (e0 + e) * C * (int64_t)row_stride + skip;
        static_assert(768 + kMaxChannels * 16 <= 8 * kFeWin, "the recomputed row fits the windows");
        double* dst = ROWS_OUT ? win + 768 : feat + e * F;  // past the 768-double scratch
        dwt8_exact_row_wave([&](int c, int k) { return row[(int64_t)c * row_stride + k]; }, C,
                            nfeat, win, dst, lane);
        if constexpr (ROWS_OUT) {
          wave_sync();
          for (int i = lane; i < F; i += 64) o[(int64_t)e * F + i] = dst[i];
          wave_sync();
        }
        if (lane == 0) norm[e] = 1.0;  // the row is normalised
        flagged &= flagged - 1;
      } while (flagged);
    }
  }
  wave_sync();
  if constexpr (ROWS_OUT) {
    __threadfence_block();  // this wave's raw rows are complete before it reads them back
    for (int e = 0; e < ne; ++e) {  // eight loads in flight per batch (L2 round trips)
      double* r = o + (int64_t)e * F;
      const double nv = norm[e];
      for (int i0 = 0; i0 < F; i0 += 8 * 64) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + 64 * u + lane;
          t[u] = i < F ? r[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + 64 * u + lane;
          if (i < F) r[i] = t[u] / nv;
        }
      }
    }
  } else {
    for (int idx = lane; idx < ne * F; idx += 64) o[idx] = feat[idx] / norm[idx / F];
  }
}

// a11..a13 for small host batches (the per-epoch IFeatureExtraction drop-in): one workgroup per
// epoch reads the epoch's packed window rows (C x 512 doubles, pinned host memory mapped into the
// device) with 16-byte loads, all issued before the first wait -- one host-link round trip instead
// of the 72 dependent-free but scattered 8-byte loads per lane of features_from_epochs_kernel --
// stages them in LDS, runs each channel's six levels on a whole wave (dwt8_exact_signal_wave,
// channels dealt over the four waves), normalises, and writes the row back across the link.
// C <= kSmallMaxC.
//
// One epoch on one workgroup is a latency problem, not a throughput one, so this path computes
// EXACT numerics under both settings: the whole-wave levels keep each lane's dependent chain short
// (~190 operations) where the batch kernels' 8-lanes-per-signal fma cascade runs ~1,200 per lane,
// and an EXACT row needs no conditioning guard.  Under fma numerics the rows are therefore the
// EXACT ones (inside the 1e-9 contract by definition); the guard's counters do not count them.
constexpr int kSmallMaxC = 16;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "features_small_kernel stages 80 KB of LDS per workgroup: gfx950 (160 KB per CU) only"
#endif
struct SmallLds {
  double xs[kSmallMaxC * kWin];
  double scr[4][384];  // per-wave level scratch (dwt8_exact_signal_wave)
  double feat[kSmallMaxC * 16];
  double norm;
};
static_assert(sizeof(SmallLds) <= 160 * 1024, "features_small_kernel's LDS exceeds one gfx950 CU");

// One epoch (its C x 512 window doubles at `src`, 16-byte aligned) -> its row at `dst`, by a
// workgroup of 256 threads (uniform control flow; ends with a barrier).
__device__ __forceinline__ void small_epoch(const double* __restrict__ src_rows, int C, int nfeat,
                                            double* __restrict__ dst, SmallLds& sh) {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const f64x2* src = (const f64x2*)src_rows;
  const int npairs = C * kWin / 2;  // <= 4096: at most 16 per thread
  f64x2 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int i = tid + 256 * k;
    if (i < npairs) v[k] = src[i];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int i = tid + 256 * k;
    if (i < npairs) *(f64x2*)(sh.xs + 2 * i) = v[k];
  }
  __syncthreads();
  const int F = C * nfeat;
  for (int c = w; c < C; c += 4) {  // uniform per wave
    const double f = dwt8_exact_signal_wave(sh.xs + c * kWin, sh.scr[w], lane);
    if (lane < nfeat) sh.feat[c * nfeat + lane] = f;
  }
  __syncthreads();
  // SignalProcessing.normalize: Math.pow(f, 2) summed in index order.  Wave 0 squares 64
  // features at a time, one per lane, and the running sum walks the lanes in order (readlane),
  // so the additions are the reference's, in its order, without a serial LDS round trip each.
  if (w == 0) {
    double acc = 0.0;
    for (int base = 0; base < F; base += 64) {
      const int i = base + lane;
      const double sq = i < F ? sh.feat[i] * sh.feat[i] : 0.0;
      const int m = F - base < 64 ? F - base : 64;
      for (int j = 0; j < m; ++j) acc = acc + lane_value(sq, j);
    }
    if (lane == 0) sh.norm = sqrt(acc);
  }
  __syncthreads();
  for (int i = tid; i < F; i += 256) dst[i] = sh.feat[i] / sh.norm;
  __syncthreads();  // sh is reused by the next epoch
}

__global__ __launch_bounds__(256) void features_small_kernel(const double* __restrict__ rows,
                                                             int C, int nfeat,
                                                             double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) SmallLds sh;
  const int64_t e = blockIdx.x;
  small_epoch(rows + e * C * kWin, C, nfeat, out + e * C * nfeat, sh);
}

// The opt-in resident form of the same path (eegfx_ctx_set_mailbox): one workgroup that stays on
// the device and serves the context's small host batches without a launch each.  Wave 0 polls
// the 64-bit request word of a host-mapped MailboxCmd (system-scope atomic loads, a short s_sleep
// between polls; the word carries the sequence number and the whole request); a new request's
// epochs are read from its pinned rows, computed by small_epoch exactly as
// features_small_kernel does, and written to its pinned output, then the completed sequence
// number is published (system-scope release after every wave's stores).  The kernel returns when
// the host sets `stop`, or after idle_ticks (s_memrealtime, 100 MHz) without a request -- every
// wave reaches that exit; the host relaunches it on the next request.  At entry it publishes its
// launch generation in `alive`: the host posts a request only to a server that has started (a
// kernel still queued behind other work is never handed a request the launch path might also
// serve).
__global__ __launch_bounds__(256) void features_mailbox_kernel(MailboxCmd* mb, uint64_t idle_ticks,
                                                               uint32_t gen) {
  __shared__ __attribute__((aligned(16))) SmallLds sh;
  __shared__ uint32_t cmd[2];  // request to serve, 0 = return
  const int tid = threadIdx.x;
  // Control flow stays wave-uniform throughout: wave 0 polls with all 64 lanes (one request per
  // poll, the loaded word made uniform with readfirstlane).  A lane-divergent `if (tid == 0)`
  // poll at the loop top let the compiler structurise the loop so that lanes other than 0 went
  // round the served request again instead of waiting at the barrier -- the server then never
  // answered.
  const bool wave0 = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
  uint32_t last = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)__hip_atomic_load(&mb->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
  const double* rows = mb->rows;
  double* out = mb->out;
  if (tid == 0) __hip_atomic_store(&mb->alive, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (wave0) {
      uint64_t go = 0;
      const uint64_t t0 = wall_clock64();
      for (;;) {
        // both words in one round trip across the link: relaxed loads issued back to back (an
        // acquire load would wait for its value before the second load); the acquire is the
        // system-scope fence every wave runs once a request is seen
        const uint64_t r = __hip_atomic_load(&mb->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t st = __hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)r);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(r >> 32));
        if (hi != last) {
          go = (uint64_t)hi << 32 | lo;
          break;
        }
        if (__builtin_amdgcn_readfirstlane((int)st)) break;
        if (wall_clock64() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (tid == 0) {
        cmd[0] = (uint32_t)(go >> 32);
        cmd[1] = (uint32_t)go;
      }
    }
    __syncthreads();
    const uint32_t seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)cmd[0]);
    if (seq == 0) break;  // stop or idle
    const uint32_t word = (uint32_t)__builtin_amdgcn_readfirstlane((int)cmd[1]);
    const int C = (int)((word >> 26) & 31) + 1, nfeat = (int)((word >> 21) & 31) + 1;
    const int64_t n = (int64_t)(word & ((1u << 21) - 1));
    // every wave: no stale line of the (reused) pinned rows from an earlier request
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    for (int64_t e = 0; e < n; ++e)
      small_epoch(rows + e * C * kWin, C, nfeat, out + e * C * nfeat, sh);
    __threadfence_system();  // this thread's rows reach the host before the flag below
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&mb->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    last = seq;
  }
}

// ---- synthetic recordings ------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float unit_noise(uint64_t seed, uint64_t key) {  // [-1, 1)
  return (float)(splitmix64(seed ^ splitmix64(key)) >> 40) * (2.0f / 16777216.0f) - 1.0f;
}

// DC -25000 counts, a bounded random walk (piecewise-linear between random knots every 64 and
// 1024 frames), a 10 Hz sinusoid of 200 counts and white noise, clipped to int16; about one
// sample in 65536 is a -32768 saturation.
__global__ __launch_bounds__(256) void synth_kernel(int16_t* __restrict__ dst, int64_t n_frames,
                                                    int ct, uint64_t seed) {
  const int64_t total = n_frames * ct;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = idx / ct;
    const int c = (int)(idx - t * ct);
    const uint64_t ck = (uint64_t)c << 48;
    const int64_t k1 = t >> 6, k2 = t >> 10;
    const float f1 = (float)(t & 63) * (1.0f / 64.0f), f2 = (float)(t & 1023) * (1.0f / 1024.0f);
    const float w1 = unit_noise(seed, ck | (uint64_t)(2 * k1)) * (1.0f - f1) +
                     unit_noise(seed, ck | (uint64_t)(2 * k1 + 2)) * f1;
    const float w2 = unit_noise(seed + 1, ck | (uint64_t)k2) * (1.0f - f2) +
                     unit_noise(seed + 1, ck | (uint64_t)(k2 + 1)) * f2;
    const float sine = 200.0f * __sinf(6.2831853f * 10.0f * (float)(t % 1000) / 1000.0f + (float)c);
    const float noise = 40.0f * unit_noise(seed + 2, (uint64_t)idx);
    float v = -25000.0f + 1500.0f * w1 + 4000.0f * w2 + sine + noise;
    if (unit_noise(seed + 3, (uint64_t)idx) < -0.99997f) v = -40000.0f;
    v = fminf(fmaxf(v, -32768.0f), 32767.0f);
    dst[idx] = (int16_t)__float2int_rn(v);
  }
}

}  // namespace dev

// ---- launchers ---------------------------------------------------------------------------------
// Frames per LDS chunk of the staged getData passes: an even count, the 750 frames split into as
// few chunks as keep each chunk's LDS (frame_bytes per frame + slack) within kCutLdsMax.
static int cut_chunk_frames(int frame_bytes, int slack) {
  for (int nch = 1;; ++nch) {
    const int nfc = ((dev::kPost + nch - 1) / nch + 1) & ~1;
    if ((int64_t)nfc * frame_bytes + slack <= dev::kCutLdsMax || nfc <= 2) return nfc;
  }
}
hipError_t launch_cut_epochs(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                             const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                             double* out, void* scratch, int* err) {
  if (n == 0) return hipSuccess;
  dim3 grid((unsigned)n), block(256);
  // baselines by the staged kernels when a layout fits them, then the coalesced write pass
  hipError_t be = hipErrorNotSupported;
  const bool aligned = ((uintptr_t)out & 15) == 0;  // the write pass stores 16-byte pairs
  if (!aligned) scratch = nullptr;
  if (scratch && fmt == 0 && ct == 3 && C == 3)
    be = launch_fused_baseline(st, raw, n_frames, ct, sel, C, pos, n, scratch, err, nullptr);
  else if (scratch && baseline_any_supported(fmt, ct, C))
    be = launch_baseline_any(st, raw, fmt, n_frames, ct, sel, C, pos, n, scratch, err, nullptr);
  if (be == hipSuccess && fmt == 0 && ct == 3 && C == 3 && ((uintptr_t)raw & 3) == 0) {
    // the reference's 3-channel file: the eight-epoch staged kernel without its feature phase
    // (4.8 -> 4.4 ms per 1M epochs against the per-epoch staged kernel, profiles/r04g)
    const dim3 g8((unsigned)((n + dev::kCfEpochs - 1) / dev::kCfEpochs));
    hipLaunchKernelGGL((dev::cut_features_c3_kernel<false, false>), g8, block, 0, st,
                       (const int16_t*)raw, n_frames, sel, pos, (const float*)scratch, n, out,
                       nullptr, Guard{nullptr, nullptr, nullptr});
    return hipGetLastError();
  }
  if (be == hipSuccess) {
    const bool small = C * (dev::kPost / 2) <= 256 * dev::kCutPairs;
    const int fbytes = ct * (fmt == 0 ? 2 : 4);
    // LDS staging reads every byte of the epoch's frames: used while they are at most twice the
    // rows written (ct <= 8 C int16), so a few channels of a wide montage keep the direct reads
    const bool stage = ((uintptr_t)raw & 3) == 0 && (int64_t)dev::kPost * fbytes <= 2 * 6000LL * C;
    if (stage && fbytes % 4 != 0 && fmt == 0) {
      const int nfc = cut_chunk_frames(fbytes, 8);
      const int nchunks = (dev::kPost + nfc - 1) / nfc;
      dim3 g2((unsigned)n, (unsigned)nchunks);
      hipLaunchKernelGGL(dev::cut_write_lds_packed_kernel<>, g2, block, (size_t)nfc * fbytes + 8, st,
                         (const int16_t*)raw, n_frames, ct, sel, C, pos, (const float*)scratch,
                         out, nfc);
    } else if (stage && fbytes % 4 == 0) {
      // wide layouts: LDS-staged chunks of the epoch, an even number of frames each
      const int fs_bytes = (fbytes / 4 + 1) * 4;
      const int nfc = cut_chunk_frames(fs_bytes, 0);
      const int nchunks = (dev::kPost + nfc - 1) / nfc;
      dim3 g2((unsigned)n, (unsigned)nchunks);
      const size_t lds = (size_t)nfc * fs_bytes;
      if (fmt == 0)
        hipLaunchKernelGGL(dev::cut_write_lds_kernel<int16_t>, g2, block, lds, st,
                           (const int16_t*)raw, n_frames, ct, sel, C, pos, (const float*)scratch,
                           out, nfc);
      else
        hipLaunchKernelGGL(dev::cut_write_lds_kernel<float>, g2, block, lds, st, (const float*)raw,
                           n_frames, ct, sel, C, pos, (const float*)scratch, out, nfc);
    } else if (fmt == 0 && small)
      hipLaunchKernelGGL(dev::cut_write_small_kernel<int16_t>, grid, block, 0, st,
                         (const int16_t*)raw, n_frames, ct, sel, C, pos, (const float*)scratch, out);
    else if (fmt == 0)
      hipLaunchKernelGGL(dev::cut_write_kernel<int16_t>, grid, block, 0, st, (const int16_t*)raw,
                         n_frames, ct, sel, C, pos, (const float*)scratch, out);
    else if (small)
      hipLaunchKernelGGL(dev::cut_write_small_kernel<float>, grid, block, 0, st,
                         (const float*)raw, n_frames, ct, sel, C, pos, (const float*)scratch, out);
    else
      hipLaunchKernelGGL(dev::cut_write_kernel<float>, grid, block, 0, st, (const float*)raw,
                         n_frames, ct, sel, C, pos, (const float*)scratch, out);
    return hipGetLastError();
  }
  if (fmt == 0)
    hipLaunchKernelGGL(dev::cut_epochs_kernel<int16_t>, grid, block, 0, st,
                       (const int16_t*)raw, n_frames, ct, sel, C, pos, out, err);
  else
    hipLaunchKernelGGL(dev::cut_epochs_kernel<float>, grid, block, 0, st, (const float*)raw,
                       n_frames, ct, sel, C, pos, out, err);
  return hipGetLastError();
}

hipError_t launch_cut_features(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                               double* out, double* feat, bool fast, void* scratch, int* err,
                               const Guard& guard) {
  if (!cut_features_supported(fmt, ct, C, raw, out, feat)) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  hipError_t be = fmt == 0 && ct == 3 && C == 3
                      ? launch_fused_baseline(st, raw, n_frames, ct, sel, C, pos, n, scratch, err,
                                              nullptr)
                      : launch_baseline_any(st, raw, fmt, n_frames, ct, sel, C, pos, n, scratch, err,
                                            nullptr);
  if (be != hipSuccess) return be;
  const dim3 grid((unsigned)n), block(256);
  const int fbytes = ct * (fmt == 0 ? 2 : 4);
  const float* bs = (const float*)scratch;
  const Guard g = fast ? guard : Guard{nullptr, nullptr, nullptr};
  if (fmt == 0 && ct == 3 && C == 3) {  // the reference's file: eight epochs per workgroup
    const dim3 g8((unsigned)((n + dev::kCfEpochs - 1) / dev::kCfEpochs));
    if (fast)
      hipLaunchKernelGGL(dev::cut_features_c3_kernel<true>, g8, block, 0, st, (const int16_t*)raw,
                         n_frames, sel, pos, bs, n, out, feat, g);
    else
      hipLaunchKernelGGL(dev::cut_features_c3_kernel<false>, g8, block, 0, st, (const int16_t*)raw,
                         n_frames, sel, pos, bs, n, out, feat, g);
  } else if (fbytes % 4 != 0) {  // int16, packed frames
    const size_t lds = dev::staged_features_lds((size_t)dev::kPost * fbytes + 8, C);
    if (fast)
      hipLaunchKernelGGL((dev::cut_write_lds_packed_kernel<true, true>), grid, block, lds, st,
                         (const int16_t*)raw, n_frames, ct, sel, C, pos, bs, out, dev::kPost, feat, g);
    else
      hipLaunchKernelGGL((dev::cut_write_lds_packed_kernel<true, false>), grid, block, lds, st,
                         (const int16_t*)raw, n_frames, ct, sel, C, pos, bs, out, dev::kPost, feat, g);
  } else {
    const int fs_bytes = (fbytes / 4 + 1) * 4;
    const size_t lds = dev::staged_features_lds((size_t)dev::kPost * fs_bytes, C);
#define EEGFX_CF(T, FA)                                                                           \
    hipLaunchKernelGGL((dev::cut_write_lds_kernel<T, true, FA>), grid, block, lds, st, (const T*)raw, \
                       n_frames, ct, sel, C, pos, bs, out, dev::kPost, feat, g)
    if (fmt == 0) { if (fast) EEGFX_CF(int16_t, true); else EEGFX_CF(int16_t, false); }
    else { if (fast) EEGFX_CF(float, true); else EEGFX_CF(float, false); }
#undef EEGFX_CF
  }
  return hipGetLastError();
}

// The one-pass kernels stage the whole post-stimulus span of an epoch (one chunk) plus the
// feature row and scratch in at most 64 KB of LDS: int16 files up to ~40 channels, float32 ~20.
bool cut_features_supported(int fmt, int ct, int C, const void* raw, const double* out,
                            const double* feat) {
  if (!(fmt == 0 || fmt == 1) || C < 1 || C > kMaxChannels || ct < 1) return false;
  if (((uintptr_t)raw & 3) || ((uintptr_t)out & 15) || !feat) return false;
  // the 3-channel kernel stores its rows as 16-byte pairs (normalise_store); the staged kernels
  // store doubles
  if (fmt == 0 && ct == 3 && C == 3 && ((uintptr_t)feat & 15)) return false;
  const int fbytes = ct * (fmt == 0 ? 2 : 4);
  const size_t stage = fbytes % 4 != 0 ? (size_t)dev::kPost * fbytes + 8
                                       : (size_t)dev::kPost * ((fbytes / 4 + 1) * 4);
  if (fbytes % 4 != 0 && fmt != 0) return false;
  if (!(fmt == 0 && ct == 3 && C == 3) && !baseline_any_supported(fmt, ct, C)) return false;
  return dev::staged_features_lds(stage, C) <= 64 * 1024;
}

hipError_t launch_features_from_epochs(hipStream_t st, const double* ep, int64_t n, int C, int skip,
                                       int nfeat, bool fast, double* out, int row_stride,
                                       const Guard& guard) {
  if (n == 0) return hipSuccess;
  // The rows stay in LDS while the workgroup (33 KB of windows + 8 rows) still fits three times
  // per CU (C <= 20 at 16 features); wider rows go through `out`, which keeps four per CU.
  // Measured (profiles/r04q/, fma / EXACT): C = 24 rows in LDS 2.86 / 3.52 ms, through `out`
  // 2.61 / 2.77 ms; C = 32 2.88 / 3.53 vs 2.82 / 2.96 ms; C = 16 2.40 / 2.54 vs 2.57 / 2.72 ms.
  const size_t lds_rows = dev::kFeWinBytes + sizeof(double) * (8 * (size_t)C * nfeat + 8);
  const bool rows_out = 3 * lds_rows > 160 * 1024;
  const size_t smem = sizeof(double) * (rows_out ? 8 * 16 + 8 : 8 * (size_t)C * nfeat + 8);
  dim3 grid((unsigned)((n + 7) / 8)), block(64);
  const Guard none{nullptr, nullptr, nullptr};
#define EEGFX_FFE(FA, RO)                                                                         \
  hipLaunchKernelGGL((dev::features_from_epochs_kernel<FA, RO>), grid, block, smem, st, ep, n, C,  \
                     skip, nfeat, row_stride, out, FA ? guard : none)
  if (fast) { if (rows_out) EEGFX_FFE(true, true); else EEGFX_FFE(true, false); }
  else { if (rows_out) EEGFX_FFE(false, true); else EEGFX_FFE(false, false); }
#undef EEGFX_FFE
  return hipGetLastError();
}

bool features_small_supported(int C) { return C >= 1 && C <= dev::kSmallMaxC; }

hipError_t launch_features_mailbox(hipStream_t st, MailboxCmd* mb, uint64_t idle_ticks,
                                   uint32_t gen) {
  hipLaunchKernelGGL(dev::features_mailbox_kernel, dim3(1), dim3(256), 0, st, mb, idle_ticks, gen);
  return hipGetLastError();
}

hipError_t launch_features_small(hipStream_t st, const double* rows, int64_t n, int C, int nfeat,
                                 double* out) {
  if (n == 0) return hipSuccess;
  if (!features_small_supported(C)) return hipErrorNotSupported;
  hipLaunchKernelGGL(dev::features_small_kernel, dim3((unsigned)n), dim3(256), 0, st, rows, C,
                     nfeat, out);
  return hipGetLastError();
}

hipError_t launch_synth(hipStream_t st, int16_t* dst, int64_t n_frames, int ct, uint64_t seed) {
  const int64_t total = n_frames * ct;
  if (total == 0) return hipSuccess;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(dev::synth_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dst, n_frames,
                     ct, seed);
  return hipGetLastError();
}

}  // namespace eegfx
