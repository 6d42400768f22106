// fused.hip -- the benchmarked hot path: multiplexed int16 recording -> dwt-8 feature matrix.
//
// One launch replaces the reference's whole per-epoch chain
//   OffLineDataProvider.java:185-233  readBinaryData x3, copyOfRange, toFloatArray,
//                                      Baseline.correct, EpochHolder.setXZ
//   WaveletTransform.java:107-141      copy 512, eegdsp DWT, keep 16, normalize
// without materialising the 18 KB double[3][750] epoch: only the 612 frames that reach the
// features (100 baseline + 512 window) are read from HBM, and only the 384 B feature row is
// written back (4,064 algorithmic bytes per epoch).
//
// Workgroup = NW = C waves (wave w = channel w), tile = 64 epochs.
//  Phase A  the 100 pre-stimulus frames of all 64 epochs are staged in LDS (coalesced 16-byte
//           loads, realigned to each epoch's first byte); lane e of wave c folds the 100 samples
//           of (epoch e, channel c) sequentially in fp32 (Baseline.java:29-42 is order-exact,
//           so this is deliberately not a tree reduction) -> 64*C baselines in one pass with
//           every lane busy.
//  Phase B  8 sub-tiles of 8 epochs: the 512-frame windows are staged in LDS in 8 segments of
//           64 frames with bank-spreading strides; lane (e, s) of wave c decodes its 72 samples
//           ((float)raw*res - b, widened) straight from the staged int16 and runs the dwt8.h
//           cascade; the 8 x C*16 features are normalised (sequential sum of squares) and
//           stored as one coalesced 16-byte store per thread.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dwt8.h"
#include "launch.h"

namespace eegfx {
namespace dev {

// 16-byte vector with 4-byte alignment: the staged streams start at arbitrary even byte offsets;
// gfx950 global_load_dwordx4 only needs dword alignment.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

constexpr int round_to_residue(int v, int mod, int res) {  // smallest x >= v with x % mod == res
  return v + (((res - v % mod) % mod) + mod) % mod;
}

constexpr int kTile = 64;  // epochs per workgroup (one per lane in phase A)
constexpr int kSub = 8;    // epochs per phase-B sub-tile (8 epochs x 8 segments = 64 lanes)

template <int CT>
struct Geometry {
  static constexpr int FB = 2 * CT;                       // bytes per int16 frame
  static constexpr int BASE_BYTES = kPre * FB;            // 600 for CT=3
  static constexpr int BASE_QUADS = (BASE_BYTES + 15) / 16;
  static constexpr int BSTR = ((BASE_QUADS * 4) | 1);      // odd dword stride: conflict-free
  static constexpr int SEG_BYTES = kSegLen * FB;          // 384
  static constexpr int SEG_QUADS = SEG_BYTES / 16;        // 24
  static constexpr int SEG_DW = SEG_BYTES / 4;            // 96
  // Lane (e, s) of a wave reads dword e*ESTR + s*SSTR + k(sample): SSTR = 4, ESTR = 1 (mod 32)
  // puts the 32 lanes of each half-wave on 32 distinct banks (ds_read_u16 banks = dword mod 32).
  static constexpr int SSTR = round_to_residue(SEG_DW, 32, 4);       // 100
  static constexpr int ESTR = round_to_residue(8 * SSTR, 32, 1);     // 801
  static constexpr int WIN_DW = kSub * ESTR;
  static constexpr int XCH_OFF_DW = (WIN_DW + 3) & ~3;              // 16-byte aligned
  static_assert(SEG_BYTES % 16 == 0, "segment must be a whole number of quads");
  static_assert(SSTR % 32 == 4 && SSTR >= SEG_DW, "segment stride");
};

// Copies quad q (16 bytes) of the byte stream that starts at global byte B into LDS dwords
// dst[0..4), realigned so that dst byte 0 is stream byte 16q.  Bytes outside [0, nbytes) read as
// zero (Arrays.copyOfRange zero padding past the end of the recording).
__device__ __forceinline__ void stage_quad(const uint8_t* __restrict__ raw, int64_t nbytes,
                                           int64_t B, int q, uint32_t* dst) {
  const int64_t A = (B & ~(int64_t)3) + 16 * (int64_t)q;
  const uint32_t sh = (uint32_t)(B & 3) * 8u;
  uint32_t w[5];
  if (A >= 0 && A + 20 <= nbytes) {
    const u32x4_a4 v = *(const u32x4_a4*)(raw + A);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    w[4] = *(const uint32_t*)(raw + A + 16);
  } else {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int64_t a = A + 4 * i;
      uint32_t x = 0;
      if (a >= 0 && a + 4 <= nbytes) x = *(const uint32_t*)(raw + a);
      else if (a >= 0 && a + 2 <= nbytes) x = *(const uint16_t*)(raw + a);
      w[i] = x;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) dst[i] = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
}

template <int CT, int C, bool FAST>
__global__ __launch_bounds__(64 * C) void fused_features_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel,
    const int64_t* __restrict__ pos, int64_t n, double* __restrict__ out) {
  using Gm = Geometry<CT>;
  constexpr int NT = 64 * C;
  constexpr int F = C * 16;
  constexpr int XCH_DW = C * 64 * kSlot * 2;  // exchange area (doubles -> dwords)
  constexpr int REGION_DW = (kTile * Gm::BSTR) > (Gm::XCH_OFF_DW + XCH_DW)
                                ? (kTile * Gm::BSTR) : (Gm::XCH_OFF_DW + XCH_DW);
  __shared__ __attribute__((aligned(16))) uint32_t region[REGION_DW];
  __shared__ __attribute__((aligned(16))) double feat[kSub * F];
  __shared__ double norm[kSub];
  __shared__ float bvals[C][kTile];
  __shared__ int64_t tpos[kTile];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int64_t nbytes = n_frames * Gm::FB;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  const int nt = (n - t0) < kTile ? (int)(n - t0) : kTile;

  if (tid < kTile) tpos[tid] = tid < nt ? pos[t0 + tid] : 0;
  __syncthreads();

  // ---- phase A: baselines --------------------------------------------------------------------
  for (int i = tid; i < kTile * Gm::BASE_QUADS; i += NT) {
    const int e = i / Gm::BASE_QUADS, q = i - e * Gm::BASE_QUADS;
    uint32_t* dst = region + e * Gm::BSTR + 4 * q;
    if (e < nt) {
      stage_quad(raw, nbytes, (tpos[e] - kPre) * Gm::FB, q, dst);
    } else {
      dst[0] = dst[1] = dst[2] = dst[3] = 0;
    }
  }
  __syncthreads();
  {
    const int c = w, e = lane;
    const float r = sel.res[c];
    const int16_t* src = (const int16_t*)(region + e * Gm::BSTR) + sel.col[c];
    float b = 0.0f;
#pragma unroll 10
    for (int i = 0; i < kPre; ++i) b = b + (float)src[i * CT] * r;
    bvals[c][e] = b / (float)kPre;
  }
  __syncthreads();

  // ---- phase B: windows + cascade ------------------------------------------------------------
  uint32_t* win = region;
  double* xch = (double*)(region + Gm::XCH_OFF_DW);
  const int c = w;
  const int el = lane >> 3, s = lane & 7;
  const int col = sel.col[c];
  const float r = sel.res[c];
  for (int j = 0; j < kTile / kSub; ++j) {
    const int eb = j * kSub;
    if (eb >= nt) break;  // uniform across the workgroup
    for (int i = tid; i < kSub * 8 * Gm::SEG_QUADS; i += NT) {
      const int e = i / (8 * Gm::SEG_QUADS);
      const int rem = i - e * (8 * Gm::SEG_QUADS);
      const int sg = rem / Gm::SEG_QUADS, q = rem - sg * Gm::SEG_QUADS;
      uint32_t* dst = win + e * Gm::ESTR + sg * Gm::SSTR + 4 * q;
      if (eb + e < nt) {
        const int64_t B = (tpos[eb + e] + (175 + kSegLen * sg)) * Gm::FB;
        stage_quad(raw, nbytes, B, q, dst);
      } else {
        dst[0] = dst[1] = dst[2] = dst[3] = 0;
      }
    }
    __syncthreads();

    const float b = bvals[c][eb + el];
    const int16_t* own = (const int16_t*)(win + el * Gm::ESTR + s * Gm::SSTR) + col;
    const int16_t* nxt = (const int16_t*)(win + el * Gm::ESTR + ((s + 1) & 7) * Gm::SSTR) + col;
    double x[kIn];
#pragma unroll
    for (int k = 0; k < kSegLen; ++k) x[k] = (double)((float)own[k * CT] * r - b);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[kSegLen + k] = (double)((float)nxt[k * CT] * r - b);
    double a6, d6;
    dwt8_cascade<FAST>(x, xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
    feat[el * F + c * 16 + s] = a6;
    feat[el * F + c * 16 + 8 + s] = d6;
    __syncthreads();
    if (tid < kSub) {
      double acc = 0.0;
#pragma unroll 8
      for (int i = 0; i < F; ++i) {
        const double f = feat[tid * F + i];
        acc = acc + f * f;
      }
      norm[tid] = sqrt(acc);
    }
    __syncthreads();
    const int ne = (nt - eb) < kSub ? (nt - eb) : kSub;
    double* o = out + (t0 + eb) * F;
    for (int i = 2 * tid; i < ne * F; i += 2 * NT) {
      const double v0 = feat[i] / norm[i / F];
      const double v1 = feat[i + 1] / norm[(i + 1) / F];
      if (i + 1 < ne * F) {
        *(double2*)(o + i) = make_double2(v0, v1);
      } else {
        o[i] = v0;
      }
    }
  }
}

}  // namespace dev

hipError_t launch_fused_features(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 bool fast, double* out) {
  if (fmt != 0 || ct != 3 || C != 3 || ((uintptr_t)out & 15) != 0) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  dim3 grid((unsigned)((n + dev::kTile - 1) / dev::kTile)), block(64 * 3);
  if (fast)
    hipLaunchKernelGGL((dev::fused_features_kernel<3, 3, true>), grid, block, 0, st,
                       (const uint8_t*)raw, n_frames, sel, pos, n, out);
  else
    hipLaunchKernelGGL((dev::fused_features_kernel<3, 3, false>), grid, block, 0, st,
                       (const uint8_t*)raw, n_frames, sel, pos, n, out);
  return hipGetLastError();
}

}  // namespace eegfx
