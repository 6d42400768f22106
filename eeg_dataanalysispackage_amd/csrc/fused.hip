// fused.hip -- the benchmarked hot path: multiplexed int16 recording -> dwt-8 feature matrix.
//
// Replaces the reference's per-epoch chain
//   OffLineDataProvider.java:185-233  readBinaryData x3, copyOfRange, toFloatArray,
//                                      Baseline.correct, EpochHolder.setXZ
//   WaveletTransform.java:107-141      copy 512, eegdsp DWT, keep 16, normalize
// without materialising the 18 KB double[3][750] epoch: only the 612 frames that reach the
// features (100 baseline + 512 window) are read from HBM, and only the 384 B feature row is
// written back (4,064 algorithmic bytes per epoch).
//
// Two launches on one stream:
//
//  baseline_kernel  100 pre-stimulus frames of 64 epochs staged in LDS (16-byte loads,
//                   realigned); lane e of wave c folds (epoch e, channel c) sequentially in fp32
//                   (Baseline.java:29-42 is order-exact, so deliberately not a tree reduction);
//                   writes b[n][C] (12 B per epoch).  Every lane of the workgroup is busy.
//
//  window_kernel    persistent, one workgroup = C waves (wave c = channel c), one sub-tile = 8
//                   epochs.  Software pipeline per sub-tile t:
//                     write the raw window of t (held in VGPRs) into LDS, realigned, in a
//                     bank-conflict-free layout  ->  barrier  ->  issue the global loads of the
//                     next sub-tile (they land in VGPRs while the filter bank runs)  ->  decode
//                     ((float)raw*res - b, widened) and run the dwt8.h cascade  ->  barrier  ->
//                     one wave (rotating) normalises the 8 x 48 features (sequential sum of
//                     squares, as SignalProcessing.java:38-52) and stores them coalesced.
//                   HBM latency is hidden behind the filter bank of the previous sub-tile; two
//                   barriers per sub-tile, no load is ever waited for at a barrier.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "dwt8.h"
#include "launch.h"

namespace eegfx {
namespace dev {

// 16-byte vector with 4-byte alignment: the staged streams start at arbitrary even byte offsets;
// gfx950 global_load_dwordx4 only needs dword alignment.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4_a16 __attribute__((ext_vector_type(4), aligned(16)));

constexpr int kTile = 64;  // epochs per baseline workgroup (one per lane)

constexpr int round_up_res(int v, int mod, int res) {  // smallest x >= v with x % mod == res
  return v + (((res - v % mod) % mod) + mod) % mod;
}
constexpr int kSub = 8;    // epochs per window sub-tile (8 epochs x 8 segments = 64 lanes)

template <int CT>
struct Geometry {
  static constexpr int FB = 2 * CT;                     // bytes per int16 frame
  static constexpr int BASE_QUADS = (kPre * FB + 15) / 16;
  static constexpr int BASE_BLKS = (BASE_QUADS + 7) / 8;
  static constexpr int BSTR = (BASE_QUADS * 4) | 1;      // odd dword stride: conflict-free folds
  static constexpr int SEG_QUADS = kSegLen * FB / 16;   // 24 for CT = 3
  static constexpr int WIN_QUADS = 8 * SEG_QUADS;       // 192
  static constexpr int WIN_BLKS = WIN_QUADS / 8;        // 24 blocks of 8 quads
  // Window LDS layout, dwords: epoch e, segment s at e*ESTR + s*SSTR.  SSTR = 4, ESTR = 1
  // (mod 32) puts the 32 lanes (4 epochs x 8 segments) of each half-wave on 32 distinct banks for
  // the ds_read_u16 sample reads, and a half-wave of writers (4 epochs x 8 consecutive quads of
  // one segment) on 32 distinct banks for the ds_write_b32 stores.
  static constexpr int SSTR = SEG_QUADS * 4 + ((4 - (SEG_QUADS * 4) % 32) + 32) % 32;
  static constexpr int ESTR = 8 * SSTR + ((1 - (8 * SSTR) % 32) + 32) % 32;
  static constexpr int WIN_DW = kSub * ESTR;
  static_assert((kSegLen * FB) % 16 == 0, "segment must be whole quads");
  static_assert(SEG_QUADS % 8 == 0, "segment must be whole 8-quad blocks");
  static_assert(SSTR % 32 == 4 && ESTR % 32 == 1, "bank-spreading strides");
};

// The 5 aligned dwords covering 16 stream bytes starting at byte B + 16q (B even, may be
// unaligned).  Bytes outside [0, nbytes) read as zero (copyOfRange zero padding).
struct Quad {
  uint32_t w[5];
};

__device__ __forceinline__ void load_quad(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          int64_t A, Quad& d) {
  if (A >= 0 && A + 20 <= nbytes) {
    const u32x4_a4 v = *(const u32x4_a4*)(raw + A);
    d.w[0] = v.x; d.w[1] = v.y; d.w[2] = v.z; d.w[3] = v.w;
    d.w[4] = *(const uint32_t*)(raw + A + 16);
  } else {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int64_t a = A + 4 * i;
      uint32_t x = 0;
      if (a >= 0 && a + 4 <= nbytes) x = *(const uint32_t*)(raw + a);
      else if (a >= 0 && a + 2 <= nbytes) x = *(const uint16_t*)(raw + a);
      d.w[i] = x;
    }
  }
}

__device__ __forceinline__ void store_quad(const Quad& d, uint32_t sh, uint32_t* dst) {
#pragma unroll
  for (int i = 0; i < 4; ++i) dst[i] = __builtin_amdgcn_alignbit(d.w[i + 1], d.w[i], sh);
}

// ---- baseline_kernel -------------------------------------------------------------------------
template <int CT, int C>
__global__ __launch_bounds__(64 * C) void baseline_kernel(const uint8_t* __restrict__ raw,
                                                          int64_t n_frames, ChanSel sel,
                                                          const int64_t* __restrict__ pos,
                                                          int64_t n, float* __restrict__ bout) {
  using Gm = Geometry<CT>;
  constexpr int NHALF = 2 * C;  // half-waves per workgroup
  __shared__ __attribute__((aligned(16))) uint32_t stage[kTile * Gm::BSTR];
  __shared__ int64_t tpos[kTile];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t nbytes = n_frames * Gm::FB;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  const int nt = (n - t0) < kTile ? (int)(n - t0) : kTile;
  if (tid < kTile) tpos[tid] = tid < nt ? pos[t0 + tid] : 0;
  __syncthreads();
  // half-wave task = 4 epochs x 8 consecutive quads of one 8-quad block
  const int hw = w * 2 + (lane >> 5), e4 = (lane >> 3) & 3, q8 = lane & 7;
  for (int task = hw; task < (kTile / 4) * Gm::BASE_BLKS; task += NHALF) {
    const int eg = task / Gm::BASE_BLKS, blk = task - eg * Gm::BASE_BLKS;
    const int e = eg * 4 + e4, q = blk * 8 + q8;
    if (q < Gm::BASE_QUADS) {
      uint32_t* dst = stage + e * Gm::BSTR + 4 * q;
      if (e < nt) {
        const int64_t B = (tpos[e] - kPre) * Gm::FB;
        Quad d;
        load_quad(raw, nbytes, (B & ~(int64_t)3) + 16 * q, d);
        store_quad(d, (uint32_t)(B & 3) * 8u, dst);
      } else {
        dst[0] = dst[1] = dst[2] = dst[3] = 0;
      }
    }
  }
  __syncthreads();
  const int c = w, e = lane;
  const float r = sel.res[c];
  const int16_t* src = (const int16_t*)(stage + e * Gm::BSTR) + sel.col[c];
  float b = 0.0f;
#pragma unroll 20
  for (int i = 0; i < kPre; ++i) b = b + (float)src[i * CT] * r;
  if (e < nt) bout[(t0 + e) * C + c] = b / (float)kPre;
}

// ---- window_kernel ---------------------------------------------------------------------------
// Prefetched state of one sub-tile held by one thread: 8 quads (one per epoch), its shift amounts,
// and the baseline of the (epoch, channel) signal this lane owns.
struct Prefetch {
  Quad q[kSub];
  uint32_t sh[kSub];
  float b;
};

template <int CT, int C, bool FAST, int MINW = 2, bool SHFL = false>
__global__ __launch_bounds__(64 * C, MINW) void window_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using Gm = Geometry<CT>;
  constexpr int F = C * 16;
  static_assert(C * 2 * 4 == Gm::WIN_BLKS, "quad mapping assumes C = 3 (24 blocks per window)");
  __shared__ __attribute__((aligned(16))) uint32_t win[Gm::WIN_DW];
  __shared__ __attribute__((aligned(16))) double xch[SHFL ? 2 : C * 64 * kSlot];
  __shared__ __attribute__((aligned(16))) double feat[2][kSub * F];
  __shared__ double norm[kSub];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int el = lane >> 3, s = lane & 7;  // compute mapping: epoch, segment
  // load mapping: half-wave = 4 epochs x 8 consecutive quads of one block
  const int h = lane >> 5, e4 = (lane >> 3) & 3, q8 = lane & 7;
  const int64_t nbytes = n_frames * Gm::FB;
  const int64_t nsub = (n + kSub - 1) / kSub;
  const int col = sel.col[w];
  const float r = sel.res[w];

  // thread's quad for epoch m (m = 0..7): epoch (m&1)*4 + e4, block (m>>1)*6 + 2w + h
  auto prefetch = [&](int64_t t, Prefetch& p) {
    const int64_t e0 = t * kSub;
#pragma unroll
    for (int m = 0; m < kSub; ++m) {
      const int e = (m & 1) * 4 + e4;
      const int blk = (m >> 1) * 6 + 2 * w + h;
      const int sg = blk / 3, q = (blk - sg * 3) * 8 + q8;
      if (e0 + e < n) {
        const int64_t B = (pos[e0 + e] + (175 + kSegLen * sg)) * Gm::FB;
        p.sh[m] = (uint32_t)(B & 3) * 8u;
        load_quad(raw, nbytes, (B & ~(int64_t)3) + 16 * q, p.q[m]);
      } else {
        p.sh[m] = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) p.q[m].w[i] = 0;
      }
    }
    p.b = (e0 + el < n) ? base[(e0 + el) * C + w] : 0.0f;
  };

  Prefetch pf;
  int64_t t = blockIdx.x;
  if (t < nsub) prefetch(t, pf);
  int it = 0;
  for (; t < nsub; t += gridDim.x, ++it) {
    // 1. the prefetched raw window of sub-tile t -> LDS
#pragma unroll
    for (int m = 0; m < kSub; ++m) {
      const int e = (m & 1) * 4 + e4;
      const int blk = (m >> 1) * 6 + 2 * w + h;
      const int sg = blk / 3, q = (blk - sg * 3) * 8 + q8;
      store_quad(pf.q[m], pf.sh[m], win + e * Gm::ESTR + sg * Gm::SSTR + 4 * q);
    }
    const float b = pf.b;
    __syncthreads();  // (A) window(t) complete
    // 2. loads of the next sub-tile fly while the filter bank runs
    const int64_t tn = t + gridDim.x;
    if (tn < nsub) prefetch(tn, pf);
    // 3. decode + cascade
    const int16_t* own = (const int16_t*)(win + el * Gm::ESTR + s * Gm::SSTR) + col;
    const int16_t* nxt = (const int16_t*)(win + el * Gm::ESTR + ((s + 1) & 7) * Gm::SSTR) + col;
    double x[kIn];
#pragma unroll
    for (int k = 0; k < kSegLen; ++k) x[k] = (double)((float)own[k * CT] * r - b);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[kSegLen + k] = (double)((float)nxt[k * CT] * r - b);
    double a6, d6;
    dwt8_cascade<FAST, SHFL>(x, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
    double* fb = feat[it & 1];
    fb[el * F + w * 16 + s] = a6;
    fb[el * F + w * 16 + 8 + s] = d6;
    __syncthreads();  // (B) features(t) complete; every wave is done reading window(t)
    // 4. one wave (rotating) normalises and stores; the others move on to sub-tile t+1
    if (w == it % C) {
      if (lane < kSub) {
        double acc = 0.0;
#pragma unroll 8
        for (int i = 0; i < F; ++i) {
          const double f = fb[lane * F + i];
          acc = acc + f * f;  // Math.pow(f, 2) summed in index order
        }
        norm[lane] = sqrt(acc);
      }
      wave_sync();
      const int64_t e0 = t * kSub;
      const int ne = (n - e0) < kSub ? (int)(n - e0) : kSub;
      double* o = out + e0 * F;
      for (int i = 2 * lane; i < ne * F; i += 128) {
        const double v0 = fb[i] / norm[i / F];
        const double v1 = fb[i + 1] / norm[(i + 1) / F];
        *(double2*)(o + i) = make_double2(v0, v1);
      }
    }
  }
}

// Non-persistent variant: one workgroup per sub-tile, stage -> barrier -> cascade -> barrier ->
// normalise; latency is hidden by running more workgroups per CU instead of prefetching.
// ABL: perf ablations (EEGFX_PERF_ABLATION, experiments only): 1 no filter bank, 2 no HBM reads,
// 3 no LDS sample reads/decode, 4 no normalisation (raw coefficients stored).
template <int CT, int C, bool FAST, int MINW, bool SHFL, int ABL = 0>
__global__ __launch_bounds__(64 * C, MINW) void window_simple_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using Gm = Geometry<CT>;
  constexpr int F = C * 16;
  __shared__ __attribute__((aligned(16))) uint32_t win[Gm::WIN_DW];
  __shared__ __attribute__((aligned(16))) double xch[SHFL ? 2 : C * 64 * kSlot];
  __shared__ __attribute__((aligned(16))) double feat[kSub * F];
  __shared__ double norm[kSub];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int el = lane >> 3, s = lane & 7;
  const int h = lane >> 5, e4 = (lane >> 3) & 3, q8 = lane & 7;
  const int64_t nbytes = n_frames * Gm::FB;
  const int64_t e0 = (int64_t)blockIdx.x * kSub;
#pragma unroll
  for (int m = 0; m < kSub; ++m) {
    const int e = (m & 1) * 4 + e4;
    const int blk = (m >> 1) * 6 + 2 * w + h;
    const int sg = blk / 3, q = (blk - sg * 3) * 8 + q8;
    uint32_t* dst = win + e * Gm::ESTR + sg * Gm::SSTR + 4 * q;
    if (e0 + e < n && ABL != 2) {
      const int64_t B = (pos[e0 + e] + (175 + kSegLen * sg)) * Gm::FB;
      Quad d;
      load_quad(raw, nbytes, (B & ~(int64_t)3) + 16 * q, d);
      store_quad(d, (uint32_t)(B & 3) * 8u, dst);
    } else {
      dst[0] = dst[1] = dst[2] = dst[3] = 0;
    }
  }
  const float b = (e0 + el < n) ? base[(e0 + el) * C + w] : 0.0f;
  const int col = sel.col[w];
  const float r = sel.res[w];
  __syncthreads();
  const int16_t* own = (const int16_t*)(win + el * Gm::ESTR + s * Gm::SSTR) + col;
  const int16_t* nxt = (const int16_t*)(win + el * Gm::ESTR + ((s + 1) & 7) * Gm::SSTR) + col;
  double x[kIn];
  if constexpr (ABL == 3) {
#pragma unroll
    for (int k = 0; k < kIn; ++k) x[k] = (double)((float)(k + s) * r - b);
  } else {
#pragma unroll
    for (int k = 0; k < kSegLen; ++k) x[k] = (double)((float)own[k * CT] * r - b);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[kSegLen + k] = (double)((float)nxt[k * CT] * r - b);
  }
  double a6, d6;
  if constexpr (ABL == 1) {
    a6 = x[0]; d6 = x[1];
#pragma unroll
    for (int k = 2; k < kIn; ++k) a6 += x[k];
  } else {
    dwt8_cascade<FAST, SHFL>(x, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
  }
  if constexpr (ABL == 4) {
    if (e0 + el < n) {
      out[(e0 + el) * F + w * 16 + s] = a6;
      out[(e0 + el) * F + w * 16 + 8 + s] = d6;
    }
    return;
  }
  feat[el * F + w * 16 + s] = a6;
  feat[el * F + w * 16 + 8 + s] = d6;
  __syncthreads();
  if (w == 0) {
    if (lane < kSub) {
      double acc = 0.0;
#pragma unroll 8
      for (int i = 0; i < F; ++i) {
        const double f = feat[lane * F + i];
        acc = acc + f * f;
      }
      norm[lane] = sqrt(acc);
    }
    wave_sync();
    const int ne = (n - e0) < kSub ? (int)(n - e0) : kSub;
    double* o = out + e0 * F;
    for (int i = 2 * lane; i < ne * F; i += 128) {
      const double v0 = feat[i] / norm[i / F];
      const double v1 = feat[i + 1] / norm[(i + 1) / F];
      *(double2*)(o + i) = make_double2(v0, v1);
    }
  }
}

// ---- aligned-load variant ----------------------------------------------------------------------
// Every HBM read is an aligned 16-byte load.  Epoch e's window is copied unshifted: LDS quad i of
// the epoch holds global quad floor16(B) + 384*(i/25) + 16*(i%25) (segment s = quads 25s..25s+24,
// i.e. 100 dwords = 4 (mod 32) apart, the 25th quad covering the sub-16-byte misalignment), and
// each lane folds the misalignment (B & 15) into its read base.  ESTR = 1 (mod 32) keeps the
// half-wave writers (4 epochs x 8 consecutive quads) and readers (4 epochs x 8 segments) on
// distinct banks up to the per-epoch misalignment shift.
template <int CT>
struct AGeom {
  static constexpr int FB = 2 * CT;
  static constexpr int SEGQ = kSegLen * FB / 16 + 1;     // 25
  static constexpr int EPQ = 8 * SEGQ;                    // 200 quads per epoch
  static constexpr int ESTR = round_up_res(EPQ * 4, 32, 1);  // 801 dwords
  static constexpr int BASEQ = (kPre * FB + 15) / 16 + 1;    // 39 quads (600 B + misalignment)
  static constexpr int BSTR = round_up_res(BASEQ * 4, 32, 29);  // odd, 29 (mod 32)
};

__device__ __forceinline__ void lds_store4(uint32_t* dst, const u32x4_a4& v) {
  dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
}

__device__ __forceinline__ u32x4_a4 load16(const uint8_t* __restrict__ raw, int64_t nbytes,
                                           int64_t A) {  // A 16-byte aligned
  if (A >= 0 && A + 16 <= nbytes) return *(const u32x4_a16*)(raw + A);
  u32x4_a4 v = {0u, 0u, 0u, 0u};
  if (A >= 0 && A < nbytes) {  // the recording ends inside this quad (even byte count)
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

template <int CT, int C>
__global__ __launch_bounds__(64 * C) void baseline_aligned_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    int64_t n, float* __restrict__ bout) {
  using G = AGeom<CT>;
  constexpr int NT = 64 * C;
  __shared__ __attribute__((aligned(16))) uint32_t stage[kTile * G::BSTR];
  __shared__ int64_t tB[kTile];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t nbytes = n_frames * G::FB;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  const int nt = (n - t0) < kTile ? (int)(n - t0) : kTile;
  if (tid < kTile) tB[tid] = tid < nt ? (pos[t0 + tid] - kPre) * G::FB : 0;
  __syncthreads();
  for (int i = tid; i < kTile * G::BASEQ; i += NT) {
    const int e = i / G::BASEQ, q = i - e * G::BASEQ;
    const u32x4_a4 v = e < nt ? load16(raw, nbytes, (tB[e] & ~(int64_t)15) + 16 * q)
                              : u32x4_a4{0u, 0u, 0u, 0u};
    lds_store4(stage + e * G::BSTR + 4 * q, v);
  }
  __syncthreads();
  const int c = w, e = lane;
  const float r = sel.res[c];
  const int16_t* src = (const int16_t*)((const uint8_t*)(stage + e * G::BSTR) + (tB[e] & 15)) +
                       sel.col[c];
  float b = 0.0f;
#pragma unroll 20
  for (int i = 0; i < kPre; ++i) b = b + (float)src[i * CT] * r;
  if (e < nt) bout[(t0 + e) * C + c] = b / (float)kPre;
}

template <int CT, int C, bool FAST, int MINW, bool SHFL>
__global__ __launch_bounds__(64 * C, MINW) void window_aligned_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using G = AGeom<CT>;
  constexpr int F = C * 16;
  constexpr int NHALF = 2 * C;
  __shared__ __attribute__((aligned(16))) uint32_t win[kSub * G::ESTR];
  __shared__ __attribute__((aligned(16))) double xch[SHFL ? 2 : C * 64 * kSlot];
  __shared__ __attribute__((aligned(16))) double feat[kSub * F];
  __shared__ double norm[kSub];
  __shared__ int64_t tB[kSub];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int el = lane >> 3, s = lane & 7;
  const int64_t nbytes = n_frames * G::FB;
  const int64_t e0 = (int64_t)blockIdx.x * kSub;
  const int ne = (n - e0) < kSub ? (int)(n - e0) : kSub;
  if (tid < kSub) tB[tid] = tid < ne ? (pos[e0 + tid] + 175) * G::FB : 0;
  const float b = el < ne ? base[(e0 + el) * C + w] : 0.0f;
  __syncthreads();
  // half-wave task: 4 epochs x 8 consecutive quads; 2 epoch groups x 25 blocks = 50 tasks
  {
    const int hw = w * 2 + (lane >> 5), e4 = (lane >> 3) & 3, q8 = lane & 7;
    for (int task = hw; task < 2 * (G::EPQ / 8); task += NHALF) {
      const int eg = task / (G::EPQ / 8), blk = task - eg * (G::EPQ / 8);
      const int e = eg * 4 + e4, i = blk * 8 + q8;
      const int sg = i / G::SEGQ, j = i - sg * G::SEGQ;
      const u32x4_a4 v =
          e < ne ? load16(raw, nbytes, (tB[e] & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * j)
                 : u32x4_a4{0u, 0u, 0u, 0u};
      lds_store4(win + e * G::ESTR + 4 * i, v);
    }
  }
  __syncthreads();
  const int col = sel.col[w];
  const float r = sel.res[w];
  const uint8_t* eb = (const uint8_t*)(win + el * G::ESTR) + (tB[el] & 15) + 2 * col;
  const int16_t* own = (const int16_t*)(eb + 16 * G::SEGQ * s);
  const int16_t* nxt = (const int16_t*)(eb + 16 * G::SEGQ * ((s + 1) & 7));
  double x[kIn];
#pragma unroll
  for (int k = 0; k < kSegLen; ++k) x[k] = (double)((float)own[k * CT] * r - b);
#pragma unroll
  for (int k = 0; k < 8; ++k) x[kSegLen + k] = (double)((float)nxt[k * CT] * r - b);
  double a6, d6;
  dwt8_cascade<FAST, SHFL>(x, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
  feat[el * F + w * 16 + s] = a6;
  feat[el * F + w * 16 + 8 + s] = d6;
  __syncthreads();
  // normalisation spread over the waves: wave w owns epochs w, w+C, ...
  for (int e = w; e < ne; e += C) {
    double acc = 0.0;
    if (lane == 0) {
#pragma unroll 8
      for (int i = 0; i < F; ++i) {
        const double f = feat[e * F + i];
        acc = acc + f * f;  // Math.pow(f, 2) summed in index order
      }
    }
    const double nrm = sqrt(__shfl(acc, 0, 64));
    double* o = out + (e0 + e) * F;
    for (int i = lane; i < F; i += 64) o[i] = feat[e * F + i] / nrm;
  }
}

}  // namespace dev

namespace {
// Implementation choice (perf experiments): EEGFX_FUSED_IMPL = "<p|s><minw><shfl>", e.g. "s31".
struct Impl {
  bool persistent;
  int minw;
  bool shfl;
  bool aligned;
};
Impl impl_choice() {
  static const Impl v = [] {
    Impl d{false, 4, true, true};
    const char* e = getenv("EEGFX_FUSED_IMPL");
    if (e && strlen(e) == 3) {
      d.persistent = e[0] == 'p';
      d.aligned = e[0] == 'a';
      d.minw = e[1] - '0';
      d.shfl = e[2] == '1';
    }
    return d;
  }();
  return v;
}

template <typename K>
int resident_blocks(K kernel, int threads) {
  int dev_id = 0, per_cu = 0, cus = 0;
  (void)hipGetDevice(&dev_id);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_id);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kernel),
                                                     threads, 0);
  return (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 256);
}

int ablation() {
  static const int v = [] {
    const char* e = getenv("EEGFX_PERF_ABLATION");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <bool FAST, int ABL>
void launch_ablation(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                     const int64_t* pos, const float* base, int64_t n, double* out) {
  const int64_t nsub = (n + dev::kSub - 1) / dev::kSub;
  hipLaunchKernelGGL((dev::window_simple_kernel<3, 3, FAST, 4, true, ABL>), dim3((unsigned)nsub),
                     dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel, pos, base, n, out);
}

template <bool FAST, bool PERS, int MINW, bool SHFL>
void launch_window(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                   const int64_t* pos, const float* base, int64_t n, double* out) {
  const int64_t nsub = (n + dev::kSub - 1) / dev::kSub;
  if constexpr (PERS) {
    static int res = resident_blocks(dev::window_kernel<3, 3, FAST, MINW, SHFL>, 192);
    const unsigned g = (unsigned)(nsub < res ? nsub : res);
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, MINW, SHFL>), dim3(g), dim3(192), 0, st,
                       (const uint8_t*)raw, n_frames, sel, pos, base, n, out);
  } else {
    hipLaunchKernelGGL((dev::window_simple_kernel<3, 3, FAST, MINW, SHFL>), dim3((unsigned)nsub),
                       dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel, pos, base, n, out);
  }
}

template <bool FAST, int MINW, bool SHFL>
void launch_aligned(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                    const int64_t* pos, float* base, int64_t n, double* out) {
  const dim3 bgrid((unsigned)((n + dev::kTile - 1) / dev::kTile));
  hipLaunchKernelGGL((dev::baseline_aligned_kernel<3, 3>), bgrid, dim3(192), 0, st,
                     (const uint8_t*)raw, n_frames, sel, pos, n, base);
  const int64_t nsub = (n + dev::kSub - 1) / dev::kSub;
  hipLaunchKernelGGL((dev::window_aligned_kernel<3, 3, FAST, MINW, SHFL>), dim3((unsigned)nsub),
                     dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel, pos, base, n, out);
}

template <bool FAST>
hipError_t launch3(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                   const int64_t* pos, float* base, int64_t n, double* out) {
  {
    const Impl im = impl_choice();
    if (!im.persistent && im.aligned) {
      if (im.minw == 4) launch_aligned<FAST, 4, true>(st, raw, n_frames, sel, pos, base, n, out);
      else if (im.minw == 3) launch_aligned<FAST, 3, true>(st, raw, n_frames, sel, pos, base, n, out);
      else launch_aligned<FAST, 2, true>(st, raw, n_frames, sel, pos, base, n, out);
      return hipGetLastError();
    }
  }
  const dim3 bgrid((unsigned)((n + dev::kTile - 1) / dev::kTile));
  hipLaunchKernelGGL((dev::baseline_kernel<3, 3>), bgrid, dim3(192), 0, st, (const uint8_t*)raw,
                     n_frames, sel, pos, n, base);
  switch (ablation()) {
    case 1: launch_ablation<FAST, 1>(st, raw, n_frames, sel, pos, base, n, out); return hipGetLastError();
    case 2: launch_ablation<FAST, 2>(st, raw, n_frames, sel, pos, base, n, out); return hipGetLastError();
    case 3: launch_ablation<FAST, 3>(st, raw, n_frames, sel, pos, base, n, out); return hipGetLastError();
    case 4: launch_ablation<FAST, 4>(st, raw, n_frames, sel, pos, base, n, out); return hipGetLastError();
    default: break;
  }
  const Impl im = impl_choice();
  const int key = (im.persistent ? 100 : 0) + im.minw * 10 + (im.shfl ? 1 : 0);
  switch (key) {
    case 20: launch_window<FAST, false, 2, false>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 21: launch_window<FAST, false, 2, true>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 30: launch_window<FAST, false, 3, false>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 40: launch_window<FAST, false, 4, false>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 41: launch_window<FAST, false, 4, true>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 120: launch_window<FAST, true, 2, false>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 121: launch_window<FAST, true, 2, true>(st, raw, n_frames, sel, pos, base, n, out); break;
    case 131: launch_window<FAST, true, 3, true>(st, raw, n_frames, sel, pos, base, n, out); break;
    default: launch_window<FAST, false, 3, true>(st, raw, n_frames, sel, pos, base, n, out); break;
  }
  return hipGetLastError();
}
}  // namespace

size_t fused_scratch_bytes(int64_t n, int C) { return sizeof(float) * (size_t)n * (size_t)C; }

hipError_t launch_fused_features(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 bool fast, void* scratch, double* out) {
  if (fmt != 0 || ct != 3 || C != 3 || ((uintptr_t)out & 15) != 0) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  float* base = (float*)scratch;
  return fast ? launch3<true>(st, raw, n_frames, sel, pos, base, n, out)
              : launch3<false>(st, raw, n_frames, sel, pos, base, n, out);
}

}  // namespace eegfx
