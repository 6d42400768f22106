// wide.hip -- fused raw -> features for any multiplexed layout (any channel count, any selected
// channels, int16 or float32 samples): BASELINE.json configs[3], the 32-channel montage with all
// channels through the DWT (512-dim features), and every layout the 3-channel kernels of fused.hip
// do not cover.
//
//   baseline_any_kernel   a5 + a6 prefix: lane = (epoch, selected channel) folds its 100
//                         pre-stimulus samples sequentially in fp32 (Baseline.java:29-42); for a
//                         multiplexed file the lanes of one epoch read adjacent samples of a frame.
//   window_wide_kernel    a3 + a7 + a11..a13 for EPW epochs per workgroup: the 512-frame windows
//                         are staged in LDS as 8 segment blocks of 64 frames (block s = global
//                         quads floor16(B) + 64*FB*s + 16*i, i <= 4*FB: the +1 quad absorbs the
//                         window's misalignment, and the block stride is 4 (mod 32) dwords so the
//                         8 segments of a half-wave sit on distinct banks), then the dwt8.h
//                         filter bank runs with wave lanes = 8 signals x 8 segments, signals =
//                         (epoch, channel) pairs, and the rows are normalised with the
//                         reference's sequential sum of squares (EXACT) or a lane-parallel one
//                         (FMA) before one coalesced store.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "dwt8.h"
#include "guard.h"
#include "launch.h"
#include "lds_dma.h"

namespace eegfx {
namespace dev {

typedef uint32_t wq_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t wq_a16 __attribute__((ext_vector_type(4), aligned(16)));

// The pre-stimulus frames [pos-100, pos) of EB epochs are staged in LDS by LDS-DMA (block m at
// m*BSTQ quads: the block's quads are contiguous in the recording, and the +1 quad of stride skews
// consecutive blocks by 4 banks), then lane (epoch, selected channel) folds its 100 samples from
// LDS.  Quads outside the recording are staged as zeros, which is the reference's zero padding
// for the fold (a padded +0.0f adds nothing, and the running sum is never -0.0f).
template <typename T, bool STREAM = false>
__global__ __launch_bounds__(256) void baseline_any_kernel(const uint8_t* __restrict__ raw,
                                                           int64_t n_frames, int ct, ChanSel sel,
                                                           int C, const int64_t* __restrict__ pos,
                                                           int64_t n, int EB, int BSTQ,
                                                           float* __restrict__ bout,
                                                           int* __restrict__ err,
                                                           int* __restrict__ guard_count,
                                                           const unsigned long long* rechecked,
                                                           unsigned long long* adapt,
                                                           unsigned int* track_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ int64_t sB[256];
  const int FB = ct * (int)sizeof(T);
  const int64_t nbytes = n_frames * FB;
  const int64_t e0 = (int64_t)blockIdx.x * EB;
  const int ne = (n - e0) < EB ? (int)(n - e0) : EB;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nw = blockDim.x / 64;
  const int NQ = BSTQ - 1;  // quads staged per epoch
  // the window kernel that follows appends to the guard list (fma numerics)
  if (guard_count && blockIdx.x == 0 && tid == 0) *guard_count = 0;
  // the 32-channel window kernel's guard strategy for this launch (guard.h guard_adapt_update)
  if (adapt && rechecked && blockIdx.x == 0 && tid < 64)
    guard_adapt_update(rechecked, adapt, track_out, n, tid);
  const int rows = (NQ + 63) / 64;
  if (tid < ne) {
    const int64_t p = pos[e0 + tid];
    // OffLineDataProvider.java:220-225 (see fused.hip position_ok)
    const bool ok = p >= kPre && p - kPre <= n_frames;
    if (!ok && err) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    sB[tid] = ((ok ? p : kPre) - kPre) * FB;  // an invalid position is cut as pos = 100
  }
  __syncthreads();
  int m = 0, j = w;
  while (j >= rows) { j -= rows; ++m; }
  int mc = -1;
  int64_t Bq = 0;
  bool full = true;
  for (; m < ne;) {
    if (m != mc) {  // uniform
      mc = m;
      const int64_t v = sB[m] & ~(int64_t)15;  // same address in every lane: make it an SGPR pair
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
      Bq = (int64_t)(((uint64_t)hi << 32) | lo);
      full = Bq >= 0 && Bq + 16 * NQ <= nbytes;
    }
    const int q = 64 * j + lane;
    uint8_t* dst = smem + ((size_t)m * BSTQ + 64 * j) * 16;
    if (q < NQ) {
      const int64_t A = Bq + 16 * q;
      if (full || (A >= 0 && A + 16 <= nbytes)) {
        dma16_s<STREAM>(raw + Bq, (uint32_t)(16 * q), dst);
      } else {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (A + 16 > 0 && A < nbytes) {  // the recording starts or ends inside this quad
          uint32_t t[4] = {0u, 0u, 0u, 0u};
          for (int k = 0; k < 4; ++k) {
            const int64_t a = A + 4 * k;
            if (a >= 0 && a + 4 <= nbytes) t[k] = *(const uint32_t*)(raw + a);
            else if (a >= 0 && a + 2 <= nbytes) t[k] = *(const uint16_t*)(raw + a);
          }
          v = make_uint4(t[0], t[1], t[2], t[3]);
        }
        *(uint4*)(dst + 16 * lane) = v;
      }
    }
    j += nw;
    while (j >= rows) { j -= rows; ++m; }
  }
  dma_drain();
  __syncthreads();
  if (tid >= ne * C) return;
  const int me = tid / C, c = tid - me * C;
  const uint8_t* blk = smem + (size_t)me * BSTQ * 16 + (int)(sB[me] & 15) + sel.col[c] * (int)sizeof(T);
  const float r = sel.res[c];
  float b = 0.0f;
#pragma unroll 10
  for (int i = 0; i < kPre; ++i) b = b + (float)*(const T*)(blk + i * FB) * r;
  bout[(e0 + me) * C + c] = b / (float)kPre;
}

// One 16-byte quad of the recording at byte offset A (16-aligned), zero outside it.
__device__ __forceinline__ wq_a4 wide_load16(const uint8_t* __restrict__ raw, int64_t nbytes,
                                             int64_t A) {
  if (A >= 0 && A + 16 <= nbytes) return *(const wq_a16*)(raw + A);
  wq_a4 v = {0u, 0u, 0u, 0u};
  if (A >= 0 && A < nbytes) {
    uint32_t t[4] = {0u, 0u, 0u, 0u};
    for (int i = 0; i < 4; ++i) {
      const int64_t a = A + 4 * i;
      if (a + 4 <= nbytes) t[i] = *(const uint32_t*)(raw + a);
      else if (a + 2 <= nbytes) t[i] = *(const uint16_t*)(raw + a);
    }
    v.x = t[0]; v.y = t[1]; v.z = t[2]; v.w = t[3];
  }
  return v;
}

template <typename T>
__device__ __forceinline__ float sample_at(const uint8_t* p) {
  return (float)*(const T*)p;
}

// Per-workgroup LDS: EPW epochs x 8 segment blocks of SEGQ quads, then EPW x F features, then
// EPW norms, then (fma) the guard's EPW x C per-signal X^2 (guard.h: int16 from r and b, float32
// the measured max |x|).  SEGQ = 4*FB + 1, FB = ct*sizeof(T) bytes per frame; FBC != 0 fixes FB at compile
// time (configs[3]'s 32-channel int16 montage: 64), so every sample read of the decode is an
// immediate LDS offset instead of an address computed per sample.
template <typename T, bool FAST, int EPW, int FBC = 0, bool STREAM = false>
__global__ __launch_bounds__(256) void window_wide_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, int ct, ChanSel sel, int C,
    const int64_t* __restrict__ pos, const float* __restrict__ base, int64_t n,
    double* __restrict__ out, Guard guard) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int FB = FBC ? FBC : ct * (int)sizeof(T);
  const int SEGQ = 4 * FB + 1;
  const int EQ = 8 * SEGQ;
  const int F = 16 * C;
  uint8_t* win = smem;
  double* feat = (double*)(smem + (size_t)EPW * EQ * 16);
  double* norm = feat + EPW * F;
  double* gx = norm + EPW;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t e0 = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * EPW;
  const int ne = (n - e0) < EPW ? (int)(n - e0) : EPW;
  const int64_t nbytes = n_frames * FB;

  // stage the windows: quad i of epoch m = global quad floor16(B_m) + 64*FB*(i/SEGQ) + 16*(i%SEGQ),
  // by LDS-DMA rows of 64 quads (wave w takes rows w, w+4, ...): one SGPR base per epoch, the
  // lane's quad offset from a float reciprocal (exact: i < 2^16, SEGQ < 2^12).  Quads the recording
  // ends inside are filled directly.
  const int nw = blockDim.x / 64;
  const int nrows = (EQ + 63) / 64;
  const float inv_segq = 1.0f / (float)SEGQ;
  // invalid positions (flagged by baseline_any_kernel) are cut as pos = 100, before any offset
  // is formed from them
  auto wpos = [&](int m) {
    const int64_t p = pos[e0 + m];
    return p >= kPre && p - kPre <= n_frames ? p : (int64_t)kPre;
  };
  int64_t Bq[EPW];
#pragma unroll
  for (int m = 0; m < EPW; ++m) Bq[m] = (((wpos(m < ne ? m : 0) + 175) * FB) & ~(int64_t)15);
  const int64_t span = (int64_t)64 * FB * 7 + 16 * SEGQ;
#pragma unroll
  for (int m = 0; m < EPW; ++m) {
    if (m >= ne) break;  // uniform
    const uint8_t* sb = raw + Bq[m];
    const bool full = Bq[m] >= 0 && Bq[m] + span <= nbytes;
    for (int j = w; j < nrows; j += nw) {
      const int i = 64 * j + lane;
      const int sg = (int)(((float)i + 0.5f) * inv_segq);
      const uint32_t off = (uint32_t)(64 * FB * sg + 16 * (i - sg * SEGQ));
      uint8_t* dst = win + ((size_t)m * EQ + 64 * j) * 16;
      if (i < EQ) {
        if (full || (Bq[m] + off >= 0 && Bq[m] + off + 16 <= nbytes)) {
          dma16_s<STREAM>(sb, off, dst);
        } else {
          const wq_a4 v = wide_load16(raw, nbytes, Bq[m] + off);
          uint32_t* d = (uint32_t*)(dst + 16 * lane);
          d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
      }
    }
  }
  dma_drain();
  __syncthreads();

  // filter bank: signal = (epoch m, channel c), 8 per wave per pass
  const int sig_lane = lane >> 3, s = lane & 7;
  const int nsig = ne * C;
  for (int sig0 = w * 8; sig0 < nsig; sig0 += 32) {  // uniform per wave
    const int sig = sig0 + sig_lane;
    const bool valid = sig < nsig;
    const int m = valid ? sig / C : 0, c = valid ? sig - m * C : 0;
    const int64_t B = (wpos(m) + 175) * FB;
    const uint8_t* eb = win + (size_t)m * EQ * 16 + (int)(B & 15) + sel.col[c] * (int)sizeof(T);
    const uint8_t* own = eb + 16 * SEGQ * s;
    const uint8_t* nxt = eb + 16 * SEGQ * ((s + 1) & 7);
    const float r = sel.res[c];
    const float b = valid ? base[(e0 + m) * C + c] : 0.0f;
    double a6, d6;
    if constexpr (FAST) {  // the 8 lanes of a group share the signal: partial-sum halos
      constexpr bool MEASURE = !std::is_same<T, int16_t>::value;  // no a-priori bound for float32
      float ym = 0.0f;
      dwt8_collapsed_cascade<MEASURE>([&](int k) { return sample_at<T>(own + k * FB); }, r, b,
                                      lane & ~7, s, a6, d6, &ym);
      double x2;
      if constexpr (MEASURE) {
        const double X = (double)group8_max(ym);
        x2 = X * X;
      } else {
        x2 = guard_x2_int16(r, b);
      }
      if (valid && s == 0) gx[m * C + c] = x2;
    } else {
      double a1[40];
      (void)nxt;
      level1_exact([&](int k) { return sample_at<T>(own + k * FB); }, r, b, lane & ~7, s, a1);
      halo<32, true>(a1, nullptr, lane & ~7, s);
      dwt8_levels2to6<FAST, true>(a1, nullptr, lane & ~7, s, a6, d6);
    }
    if (valid) {
      feat[m * F + c * 16 + s] = a6;
      feat[m * F + c * 16 + 8 + s] = d6;
    }
  }
  __syncthreads();

  // SignalProcessing.normalize (SignalProcessing.java:38-52)
  if constexpr (FAST) {
    // lane-parallel sum of squares per epoch (order-free: the FMA contract is 1e-9)
    for (int m = w; m < ne; m += blockDim.x / 64) {
      double acc = 0.0;
      for (int i = lane; i < F; i += 64) acc = __builtin_fma(feat[m * F + i], feat[m * F + i], acc);
      double sx = lane < C ? gx[m * C + lane] : 0.0;  // C <= 64
      for (int off = 32; off > 0; off >>= 1) {
        acc += __shfl_xor(acc, off, 64);
        sx += __shfl_xor(sx, off, 64);
      }
      bool fails = guard.count && guard_fails(acc, kGuardK2Collapsed, sx);  // wave-uniform
      if (std::is_same<T, int16_t>::value && fails) {  // the second stage on the staged window
        if (lane == 0) guard_count_rechecked(guard, 1);
        const int64_t B = (wpos(m) + 175) * FB;
        const uint8_t* eb = win + (size_t)m * EQ * 16 + (int)(B & 15);
        fails = guard_fails(
            acc, kGuardK2Collapsed,
            guard_measured_x2_wave(
                [&](int c, int k) -> int {
                  return (int)sample_at<T>(eb + sel.col[c] * (int)sizeof(T) + 16 * SEGQ * (k >> 6) +
                                           FB * (k & 63));
                },
                [&](int c, float v) {
                  float y = v * sel.res[c];
                  y = y - base[(e0 + m) * C + c];
                  return (double)y;
                },
                C, lane));
      }
      if (lane == 0) {
        norm[m] = rsqrt_nr(acc);  // the reciprocal norm (multiplied below)
        if (fails) guard_flag(guard, e0 + m);
      }
    }
  } else {
    // the reference's sequential fold, index order, one lane per epoch
    if (tid < ne) {
      double acc = 0.0;
      for (int i = 0; i < F; ++i) {
        const double f = feat[tid * F + i];
        acc = acc + f * f;
      }
      norm[tid] = sqrt(acc);
    }
  }
  __syncthreads();
  double* o = out + e0 * F;
  for (int i = tid; i < ne * F; i += blockDim.x) {
    const double v = FAST ? feat[i] * norm[i / F] : feat[i] / norm[i / F];
    if constexpr (STREAM) __builtin_nontemporal_store(v, o + i);
    else o[i] = v;
  }
}

// configs[3]: the full 32-channel int16 montage with every channel through the DWT (512-dim rows),
// one epoch at a time per workgroup of 4 waves (wave w = channels 8w..8w+7, lane = (channel,
// segment)).  Everything the generic kernel computes from runtime sizes is constexpr here: the
// staging rows (wave w issues rows w, w+4, ...; scalar row bases, two VALU instructions of lane
// offset per row, no per-lane bounds test when the window lies inside the recording), the signal
// -> channel map (shifts) and the row normalisation (FMA: rsqrt_nr, one multiply per feature;
// EXACT keeps the reference's sequential sum and division).  Measured against the generic kernel
// at FB = 64 (tools/probes, 666 launches of 250k epochs): 2.58 -> 2.46 ms, 1,114 -> 1,040 VALU
// instructions per wave.
struct C32 {
  static constexpr int C = 32, FB = 64, SEGQ = 4 * FB + 1, EQ = 8 * SEGQ, F = 16 * C;
  static constexpr int NROWS = (EQ + 63) / 64;  // 33
  static constexpr int64_t SPAN = (int64_t)64 * FB * 7 + 16 * SEGQ;
};

// Byte offset of epoch e's window (an invalid position, flagged by the baselines, is cut as 100).
__device__ __forceinline__ int64_t c32_window(const int64_t* __restrict__ pos, int64_t e,
                                              int64_t n_frames) {
  const int64_t p0 = pos[e];
  const int64_t p = p0 >= kPre && p0 - kPre <= n_frames ? p0 : (int64_t)kPre;
  return (p + 175) * C32::FB;
}

// Stages the window at byte B into `win` (this wave's rows).  Row j = w + 4t holds LDS quads
// i = 64 j + lane; quad i = SEGQ sg + rem lands from byte 4096 sg + 16 rem = 16 i - 16 sg of the
// window.  A row spans 64 < SEGQ quads, so it crosses at most one segment boundary: sg = s0 +
// [lane >= t_j] with s0 = floor(64 j / SEGQ), and the offset splits into a scalar row base
// (1024 j - 16 s0) and a per-lane 16 lane - 16 [lane >= t_j] (two VALU instructions per row).
// Returns whether the whole window lay inside the recording (every row one LDS-DMA, 9 for wave 0
// and 8 for the others, tracked by vmcnt); otherwise the quads past either end were filled
// directly.
template <bool STREAM>
__device__ __forceinline__ bool c32_issue(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          int64_t B, uint8_t* win, int w, int lane) {
  using K = C32;
  const int64_t Bq = B & ~(int64_t)15;
  const bool full = Bq >= 0 && Bq + K::SPAN <= nbytes;
  const uint32_t lane16 = 16u * (uint32_t)lane;
#pragma unroll
  for (int t = 0; t < (K::NROWS + 3) / 4; ++t) {
    const int j = w + 4 * t;
    if (j < K::NROWS) {  // uniform
      const int s0 = (64 * j) / K::SEGQ;
      const int tj = K::SEGQ * (s0 + 1) - 64 * j;
      const uint32_t voff = lane16 - (lane >= tj ? 16u : 0u);
      const int64_t rowb = 1024 * (int64_t)j - 16 * (int64_t)s0;
      uint8_t* dst = win + (size_t)(64 * j) * 16;
      const bool lane_in = 64 * j + 64 <= K::EQ || 64 * j + lane < K::EQ;
      if (full) {  // uniform: the whole window lies inside the recording
        if (lane_in) dma16_s<STREAM>(raw + Bq + rowb, voff, dst);
      } else if (lane_in) {
        const int64_t A = Bq + rowb + voff;
        if (A >= 0 && A + 16 <= nbytes) {
          dma16_s<STREAM>(raw + Bq + rowb, voff, dst);
        } else {
          const wq_a4 v = wide_load16(raw, nbytes, A);
          uint32_t* d = (uint32_t*)(dst + 16 * lane);
          d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
      }
    }
  }
  return full;
}

// LDS of a 32-channel workgroup beside its window buffer(s).
struct C32Shared {
  double feat[C32::F];
  double norm1;
  double gx[C32::C];  // the guard's X^2 per channel (fma numerics)
  int redo;
  double part[4];     // per-wave sums of squares (EEGFX_C32_REG)
  double gxw[4];      // per-wave sums of the guard's X^2 (EEGFX_C32_REG)
  double gxm[C32::C];  // measured X_c^2 per channel (the tracking variant, EEGFX_TRACK_X)
};

// fma numerics, A/B builds: 1 = every lane normalises and stores its own a6, d6 from registers (the row's sum
// of squares from per-wave DPP / cross-lane sums combined through LDS, one barrier), the
// features through LDS only for a row the guard flags; 0 = the features through LDS, wave 0 sums
// and tests the row and every thread stores 16 bytes of it (the product: the register form measured
// 2.0 % slower, 2.044 vs 2.000 ms per launch, profiles/r06/c32_reg_ab.log -- the cross-lane sums
// cost more than wave 0's pass over the row).
#ifndef EEGFX_C32_REG
#define EEGFX_C32_REG 0
#endif

// The sum over the wave's 64 lanes (the same value in all of them).
__device__ __forceinline__ double wave_sum64(double v) {
  v = group8_sum(v);
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// Filter bank, normalisation and store of epoch e from its staged window (published by a
// barrier); this lane's channel c = 8 w + lane / 8 has column col_c, resolution r and baseline b
// (loaded by the caller, so no memory access of the common path follows a DMA it must not wait
// for).  Ends with every wave done reading `win` and sh.feat.
template <bool FAST, bool STREAM, bool TRK = false>
__device__ __forceinline__ void c32_compute(const uint8_t* __restrict__ raw, int64_t n_frames,
                                            const ChanSel& sel, const float* __restrict__ base,
                                            int64_t e, int64_t B, float b, int col_c, float r,
                                            uint8_t* win, C32Shared& sh, double* __restrict__ out,
                                            const Guard& guard, int tid) {
  using K = C32;
  constexpr int C = K::C, FB = K::FB, SEGQ = K::SEGQ, F = K::F;
  const int lane = tid & 63, w = tid >> 6;
  const int c = w * 8 + (lane >> 3), s = lane & 7;
  const uint8_t* eb = win + (int)(B & 15) + col_c * 2;
  const uint8_t* own = eb + 16 * SEGQ * s;
  const uint8_t* nxt = eb + 16 * SEGQ * ((s + 1) & 7);
  double a6, d6;
  constexpr bool TRACK = FAST && TRK && EEGFX_GUARD;
  if constexpr (FAST) {
#if EEGFX_COLLAPSED
    float ymax = 0.0f;
    dwt8_collapsed_cascade<TRACK>([&](int k) { return sample_at<int16_t>(own + k * FB); }, r, b,
                                  lane & ~7, s, a6, d6, &ymax);
    if constexpr (TRACK) {  // the tracking variant: this channel's measured X_c over its 8 lanes
      uint32_t u = __float_as_uint(ymax);
      u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0xB1, 0xF, 0xF, true));
      u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x4E, 0xF, 0xF, true));
      u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x141, 0xF, 0xF, true));
      const double X = (double)__uint_as_float(u);
      if (s == 0) sh.gxm[c] = X * X;
    }
#else
    dwt8_fast_cascade([&](int k) { return sample_at<int16_t>(own + k * FB); }, r, b, lane & ~7, s,
                      a6, d6);
#endif
  } else {
    double a1[40];
    (void)nxt;
    level1_exact([&](int k) { return sample_at<int16_t>(own + k * FB); }, r, b, lane & ~7, s, a1);
    halo<32, true>(a1, nullptr, lane & ~7, s);
    dwt8_levels2to6<FAST, true>(a1, nullptr, lane & ~7, s, a6, d6);
  }
  double* feat = sh.feat;
  double* o = out + e * F;
  if constexpr (FAST && EEGFX_C32_REG) {
    const double q = wave_sum64(__builtin_fma(a6, a6, d6 * d6));
    const double gq = wave_sum64(EEGFX_GUARD && s == 0 ? guard_x2_int16(r, b) : 0.0);
    if (lane == 0) {
      sh.part[w] = q;
      sh.gxw[w] = gq;
    }
    if (EEGFX_GUARD && s == 0) sh.gx[c] = guard_x2_int16(r, b);  // for the rare path below
    __syncthreads();
    const double acc = ((sh.part[0] + sh.part[1]) + sh.part[2]) + sh.part[3];
    const double sx = ((sh.gxw[0] + sh.gxw[1]) + sh.gxw[2]) + sh.gxw[3];
    const bool fails = EEGFX_GUARD && guard.total && guard_fails(acc, kGuardK2Collapsed, sx);
    if (!fails) {  // uniform: every lane stores its two features
      const double inv = rsqrt_nr1(acc);
      if constexpr (STREAM) {
        __builtin_nontemporal_store(a6 * inv, o + c * 16 + s);
        __builtin_nontemporal_store(d6 * inv, o + c * 16 + 8 + s);
      } else {
        o[c * 16 + s] = a6 * inv;
        o[c * 16 + 8 + s] = d6 * inv;
      }
      return;
    }
    // the guard's second stage and rare recompute, as below, from the features in LDS
    feat[c * 16 + s] = a6;
    feat[c * 16 + 8 + s] = d6;
    __syncthreads();
  } else {
    feat[c * 16 + s] = a6;
    feat[c * 16 + 8 + s] = d6;
    if (FAST && EEGFX_GUARD && s == 0) sh.gx[c] = guard_x2_int16(r, b);
    __syncthreads();
  }
  if constexpr (FAST) {
    if (w == 0) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < F / 64; ++k) acc = __builtin_fma(feat[lane + 64 * k], feat[lane + 64 * k], acc);
      double sx = lane < C ? sh.gx[lane] : 0.0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        acc += __shfl_xor(acc, off, 64);
        sx += __shfl_xor(sx, off, 64);
      }
      bool fails = EEGFX_GUARD && guard.total && guard_fails(acc, kGuardK2Collapsed, sx);
      if (TRACK && fails) {  // the second stage from the measured X_c of every channel
        if (lane == 0) guard_count_rechecked(guard, 1);
        double sm = lane < C ? sh.gxm[lane] : 0.0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sm += __shfl_xor(sm, off, 64);
        fails = guard_fails(acc, kGuardK2Collapsed, sm * (1.0 + 0x1p-20));
      } else if (fails) {  // wave-uniform, rare: the second stage on the staged window (intact)
        if (lane == 0) guard_count_rechecked(guard, 1);
        fails = guard_fails(
            acc, kGuardK2Collapsed,
            guard_measured_x2_wave(
                [&](int cc, int k) -> int {
                  return *(const int16_t*)(win + (int)(B & 15) + sel.col[cc] * 2 +
                                           16 * SEGQ * (k >> 6) + FB * (k & 63));
                },
                [&](int cc, float v) {
                  float y = v * sel.res[cc];
                  y = y - base[e * C + cc];
                  return (double)y;
                },
                C, lane));
      }
      if (lane == 0) {
        sh.norm1 = rsqrt_nr(acc);
        sh.redo = fails;
      }
    }
    __syncthreads();
    if (sh.redo) {
      // the guard's rare path: the row recomputed under EXACT, channels w, w+4, ... by wave w (the
      // window LDS free: 768 doubles of scratch per wave), then normalised by wave 0
      constexpr int NW = 256 / 64;
      static_assert(NW * 768 * 8 <= K::EQ * 16, "EXACT scratch fits the window buffer");
      const int64_t f0 = B / FB;
      double* scratch = (double*)win + w * 768;
#pragma unroll 1
      for (int cc = w; cc < C; cc += NW) {
        const int col = sel.col[cc];
        const float rc = sel.res[cc], bc = base[e * C + cc];
        dwt8_exact_channel_wave(
            [&](int k) {
              const float x = f0 + k < n_frames
                                  ? (float)*(const int16_t*)(raw + B + (int64_t)k * FB + 2 * col)
                                  : 0.0f;
              float y = x * rc;
              y = y - bc;
              return (double)y;
            },
            16, scratch, feat + cc * 16, lane);
      }
      __syncthreads();
      if (w == 0) {
        dwt8_normalise_row_wave(feat, F, scratch, lane);
        if (lane == 0) {
          sh.norm1 = 1.0;  // the row is normalised
          guard_count_recomputed(guard, 1ull);
        }
      }
      __syncthreads();
    }
    const double inv = sh.norm1;
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const f64x2 v = *(const f64x2*)(feat + 2 * tid);
    const f64x2 q = {v.x * inv, v.y * inv};
    if constexpr (STREAM) __builtin_nontemporal_store(q, (f64x2*)(o + 2 * tid));
    else *(f64x2*)(o + 2 * tid) = q;
  } else {
    if (tid == 0) {
      double acc = 0.0;
      for (int k = 0; k < F; ++k) acc = acc + feat[k] * feat[k];
      sh.norm1 = sqrt(acc);
    }
    __syncthreads();
    const double nv = sh.norm1;
    for (int k = tid; k < F; k += 256) {
      const double v = feat[k] / nv;
      if constexpr (STREAM) __builtin_nontemporal_store(v, o + k);
      else o[k] = v;
    }
  }
}

template <bool FAST, bool STREAM, bool TRK = false>
__global__ __launch_bounds__(256) void window_c32_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel,
    const int64_t* __restrict__ pos, const float* __restrict__ base, int64_t n,
    double* __restrict__ out, Guard guard) {
  __shared__ __attribute__((aligned(16))) uint8_t win[C32::EQ * 16];
  __shared__ C32Shared sh;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t e = (int64_t)xcd_tile(blockIdx.x, gridDim.x);
  const int64_t B = c32_window(pos, e, n_frames);
  (void)c32_issue<STREAM>(raw, n_frames * C32::FB, B, win, w, lane);
  const int c = w * 8 + (lane >> 3);
  const float b = base[e * C32::C + c];
  dma_drain();
  __syncthreads();
  c32_compute<FAST, STREAM, TRK>(raw, n_frames, sel, base, e, B, b, sel.col[c], sel.res[c], win,
                                 sh, out, guard, tid);
}

}  // namespace dev

namespace {
template <typename T, bool FAST, int EPW, int FBC = 0, bool STREAM = false>
hipError_t launch_wide_t(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                         const ChanSel& sel, int C, const int64_t* pos, const float* base,
                         int64_t n, double* out, const Guard& guard) {
  const int FB = ct * (int)sizeof(T);
  const size_t lds = (size_t)EPW * 8 * (4 * FB + 1) * 16 + (size_t)EPW * 16 * C * 8 + EPW * 8 +
                     (FAST ? (size_t)EPW * C * 8 : 0);
  const dim3 grid((unsigned)((n + EPW - 1) / EPW));
  hipLaunchKernelGGL((dev::window_wide_kernel<T, FAST, EPW, FBC, STREAM>), grid, dim3(256), lds, st,
                     (const uint8_t*)raw, n_frames, ct, sel, C, pos, base, n, out, guard);
  return hipGetLastError();
}
}  // namespace

// LDS of one epoch's staged window + features; the wide kernel runs two epochs per workgroup
// while that fits comfortably (two or more workgroups per CU), one otherwise.
static size_t wide_lds_per_epoch(int fmt, int ct, int C) {
  const int FB = ct * (fmt == 0 ? 2 : 4);
  return (size_t)8 * (4 * FB + 1) * 16 + (size_t)16 * C * 8 + 8 + (size_t)C * 8;
}

bool wide_supported(int fmt, int ct, int C) {
  return (fmt == 0 || fmt == 1) && C >= 1 && C <= kMaxChannels && ct >= 1 &&
         wide_lds_per_epoch(fmt, ct, C) <= 64 * 1024;
}

static int baseline_any_tile(int fmt, int ct, int C, int* bstq) {
  const int FB = ct * (fmt == 0 ? 2 : 4);
  const int BSTQ = (dev::kPre * FB + 15) / 16 + 2;  // staged quads + 1 quad of bank skew
  int EB = 256 / C;  // lanes = (epoch, channel) pairs (<= 256 epochs: the sB table)
  while (EB > 1 && (size_t)EB * BSTQ * 16 > 56 * 1024) --EB;
  if (bstq) *bstq = BSTQ;
  return EB;
}

bool baseline_any_supported(int fmt, int ct, int C) {
  if (!(fmt == 0 || fmt == 1) || C < 1 || C > 256 || ct < 1) return false;
  int bstq = 0;
  const int EB = baseline_any_tile(fmt, ct, C, &bstq);
  return (size_t)EB * bstq * 16 <= 64 * 1024;
}

hipError_t launch_baseline_any(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                               void* scratch, int* err, int* guard_count, const Guard* guard) {
  const unsigned long long* rechecked = guard ? guard->rechecked : nullptr;
  unsigned long long* adapt = guard && guard->total ? guard->adapt : nullptr;
  unsigned int* track_out = adapt ? guard->track_out : nullptr;
  if (n == 0) return hipSuccess;
  int BSTQ = 0;
  const int EB = baseline_any_tile(fmt, ct, C, &BSTQ);
  const size_t lds = (size_t)EB * BSTQ * 16;
  const dim3 grid((unsigned)((n + EB - 1) / EB));
  if (fmt == 0 && streaming_reads(n_frames, n, dev::kPre + 687))  // pre-stimulus frames unshared
    hipLaunchKernelGGL((dev::baseline_any_kernel<int16_t, true>), grid, dim3(256), lds, st,
                       (const uint8_t*)raw, n_frames, ct, sel, C, pos, n, EB, BSTQ, (float*)scratch, err,
                       guard_count, rechecked, adapt, track_out);
  else if (fmt == 0)
    hipLaunchKernelGGL(dev::baseline_any_kernel<int16_t>, grid, dim3(256), lds, st,
                       (const uint8_t*)raw, n_frames, ct, sel, C, pos, n, EB, BSTQ, (float*)scratch, err,
                       guard_count, rechecked, adapt, track_out);
  else
    hipLaunchKernelGGL(dev::baseline_any_kernel<float>, grid, dim3(256), lds, st,
                       (const uint8_t*)raw, n_frames, ct, sel, C, pos, n, EB, BSTQ, (float*)scratch, err,
                       guard_count, rechecked, adapt, track_out);
  return hipGetLastError();
}

static hipError_t launch_window_wide_kernels(hipStream_t st, const void* raw, int fmt,
                                             int64_t n_frames, int ct, const ChanSel& sel, int C,
                                             const int64_t* pos, int64_t n, bool fast,
                                             const void* scratch, double* out, const Guard& guard,
                                             bool track);

// The generic kernels append the rows that fail the fma guard to the list (their LDS has no room
// for the recomputation) and the follow-up launch recomputes them (guard.hip); the 32-channel
// kernel recomputes its own (guard.total only).
hipError_t launch_window_wide(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                              const ChanSel& sel, int C, const int64_t* pos, int64_t n, bool fast,
                              const void* scratch, double* out, const Guard& guard, bool track) {
  if (n == 0) return hipSuccess;
  const hipError_t e = launch_window_wide_kernels(st, raw, fmt, n_frames, ct, sel, C, pos, n, fast,
                                                  scratch, out, guard, track);
  if (e != hipSuccess || !fast || !guard.count) return e;
  if (fmt == 0 && ct == 32 && C == 32 && ((uintptr_t)out & 15) == 0) return hipSuccess;
  return launch_guard_fixup_raw(st, raw, fmt, n_frames, ct, sel, C, pos, scratch, guard, out);
}

static hipError_t launch_window_wide_kernels(hipStream_t st, const void* raw, int fmt,
                                             int64_t n_frames, int ct, const ChanSel& sel, int C,
                                             const int64_t* pos, int64_t n, bool fast,
                                             const void* scratch, double* out, const Guard& guard,
                                             bool track) {
  const float* base = (const float*)scratch;
  const bool two = wide_lds_per_epoch(fmt, ct, C) <= 32 * 1024;  // dynamic LDS stays <= 64 KB
#define EEGFX_W(T, FA)                                                                        \
  return two ? launch_wide_t<T, FA, 2>(st, raw, n_frames, ct, sel, C, pos, base, n, out, guard)       \
             : launch_wide_t<T, FA, 1>(st, raw, n_frames, ct, sel, C, pos, base, n, out, guard);
  if (fmt == 0 && ct == 32 && C == 32 && ((uintptr_t)out & 15) == 0) {  // configs[3]
    const bool nt = streaming_reads(n_frames, n, dev::kWin + 8);
    const dim3 g((unsigned)n);
#define EEGFX_C32(FA, NTV, TK)                                                              \
    hipLaunchKernelGGL((dev::window_c32_kernel<FA, NTV, TK>), g, dim3(256), 0, st,           \
                       (const uint8_t*)raw, n_frames, sel, pos, base, n, out, guard)
    // the guard's second stage by tracking max |x| (guard.h EEGFX_TRACK_X)
    const bool trk = EEGFX_TRACK_X != 0 && (EEGFX_TRACK_X == 2 || track) && guard.total;
    if (fast && trk) { if (nt) EEGFX_C32(true, true, true); else EEGFX_C32(true, false, true); }
    else if (fast) { if (nt) EEGFX_C32(true, true, false); else EEGFX_C32(true, false, false); }
    else { if (nt) EEGFX_C32(false, true, false); else EEGFX_C32(false, false, false); }
#undef EEGFX_C32
    return hipGetLastError();
  }
  if (fmt == 0 && ct == 32 && !two) {  // the frame size as a compile-time constant
    // streaming (non-temporal) window reads and row stores when the windows are disjoint
    if (streaming_reads(n_frames, n, dev::kWin + 8))
      return fast ? launch_wide_t<int16_t, true, 1, 64, true>(st, raw, n_frames, ct, sel, C, pos, base, n, out, guard)
                  : launch_wide_t<int16_t, false, 1, 64, true>(st, raw, n_frames, ct, sel, C, pos, base, n, out, guard);
    return fast ? launch_wide_t<int16_t, true, 1, 64>(st, raw, n_frames, ct, sel, C, pos, base, n, out, guard)
                : launch_wide_t<int16_t, false, 1, 64>(st, raw, n_frames, ct, sel, C, pos, base, n, out, guard);
  }
  if (fmt == 0) {
    if (fast) { EEGFX_W(int16_t, true) } else { EEGFX_W(int16_t, false) }
  } else {
    if (fast) { EEGFX_W(float, true) } else { EEGFX_W(float, false) }
  }
#undef EEGFX_W
}

}  // namespace eegfx
