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
// Two launches on one stream (DESIGN.md "Kernels"):
//
//  baseline_kernel  the 100 pre-stimulus frames of 64 epochs are staged in LDS with aligned
//                   16-byte loads (all issued before the first wait); lane e of wave c folds
//                   (epoch e, channel c) sequentially in fp32 -- Baseline.java:29-42 is
//                   order-exact, so this is deliberately not a tree reduction -- and writes
//                   b[n][C] (12 B per epoch).  Every lane of the workgroup folds one signal.
//
//  window_kernel    workgroup = C waves (wave c = channel c), sub-tile = 8 epochs x 8 lanes per
//                   signal (dwt8.h).  The 512-frame windows arrive by LDS-DMA
//                   (global_load_lds_dwordx4: 16-byte aligned per-lane sources, no VGPRs) into a
//                   per-epoch LDS layout whose strides keep every half-wave of ds_read_u16 on
//                   distinct banks; each lane folds the window's sub-16-byte misalignment into
//                   its read base.  Lanes copy their 72 raw samples to VGPRs, a barrier frees
//                   the window (the DMA of the next sub-tile, when the workgroup has one, then
//                   overlaps the filter bank), decode (float)raw*res - b two samples at a time,
//                   run the cascade, and one wave normalises the 8 x 48 features (sequential
//                   sum of squares, SignalProcessing.java:38-52) and stores them coalesced.
//
// The variant selector at the bottom exists for the perf study recorded in DESIGN.md (register
// budget x halo transport x sub-tiles per workgroup); the default is the measured best.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "dwt8.h"
#include "launch.h"

namespace eegfx {
namespace dev {

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4_a16 __attribute__((ext_vector_type(4), aligned(16)));

constexpr int kTile = 64;  // epochs per baseline workgroup (one per lane)
constexpr int kSub = 8;    // epochs per window sub-tile (8 epochs x 8 segments = 64 lanes)

constexpr int round_up_res(int v, int mod, int res) {  // smallest x >= v with x % mod == res
  return v + (((res - v % mod) % mod) + mod) % mod;
}

// LDS geometry for a CT-channel int16 recording.  Epoch e's window occupies EPQ contiguous quads
// from dword e*ESTR: quad i holds global quad floor16(B_e) + 384*(i/25) + 16*(i%25), i.e. segment
// s (64 frames, 384 B for CT = 3) is 25 quads = 100 dwords = 4 (mod 32) after segment s-1, the
// 25th quad covering the misalignment.  ESTR = 1 (mod 32), so the 32 lanes of a half-wave
// (4 epochs x 8 segments) read 32 distinct banks up to each epoch's misalignment shift.
template <int CT>
struct Geometry {
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

// Issue-then-consume staging: the bulk load of an in-range quad is unconditional (an out-of-range
// lane reads the first quad of the recording and discards it), so the compiler batches every
// load of a thread before the first wait; the rare quad that straddles the end of the recording
// is patched afterwards by load16.
__device__ __forceinline__ u32x4_a4 load16_bulk(const uint8_t* __restrict__ raw, int64_t nbytes,
                                                int64_t A, bool want) {
  const bool full = want && A >= 0 && A + 16 <= nbytes;
  const u32x4_a4 v = *(const u32x4_a16*)(raw + (full ? A : 0));
  const u32x4_a4 z = {0u, 0u, 0u, 0u};
  return full ? v : z;
}
__device__ __forceinline__ bool straddles_end(int64_t A, int64_t nbytes, bool want) {
  return want && A >= 0 && A < nbytes && A + 16 > nbytes;
}

template <int CT, int C>
__global__ __launch_bounds__(64 * C) void baseline_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    int64_t n, float* __restrict__ bout) {
  using G = Geometry<CT>;
  constexpr int NT = 64 * C;
  __shared__ __attribute__((aligned(16))) uint32_t stage[kTile * G::BSTR];
  __shared__ int64_t tB[kTile];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t nbytes = n_frames * G::FB;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  const int nt = (n - t0) < kTile ? (int)(n - t0) : kTile;
  if (tid < kTile) tB[tid] = tid < nt ? (pos[t0 + tid] - kPre) * G::FB : 0;
  __syncthreads();
  constexpr int ITERS = (kTile * G::BASEQ + NT - 1) / NT;  // 13
  u32x4_a4 v[ITERS];
  int64_t A[ITERS];
  bool want[ITERS];
  const bool tiny = nbytes < 16;
#pragma unroll
  for (int k = 0; k < ITERS; ++k) {
    const int i = tid + k * NT;
    const int e = i / G::BASEQ, q = i - e * G::BASEQ;
    want[k] = i < kTile * G::BASEQ && e < nt;
    A[k] = want[k] ? (tB[e] & ~(int64_t)15) + 16 * q : 0;
    v[k] = load16_bulk(raw, nbytes, A[k], want[k] && !tiny);
  }
#pragma unroll
  for (int k = 0; k < ITERS; ++k)
    if (straddles_end(A[k], nbytes, want[k]) || (tiny && want[k])) v[k] = load16(raw, nbytes, A[k]);
#pragma unroll
  for (int k = 0; k < ITERS; ++k) {
    const int i = tid + k * NT;
    if (i < kTile * G::BASEQ) {
      const int e = i / G::BASEQ, q = i - e * G::BASEQ;
      lds_store4(stage + e * G::BSTR + 4 * q, v[k]);
    }
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

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Byte offset of sub-tile epoch e's window: B_e = (pos + 175) * FB; quads are fetched from
// floor16(B_e) and the lanes fold (B_e & 15) into their read base.  e0 and e are wave-uniform,
// so these are scalar loads (lgkmcnt), which keeps every vector-memory counter slot for the DMAs.
template <int CT>
__device__ __forceinline__ int64_t window_byte(const int64_t* __restrict__ pos, int64_t e) {
  return (pos[e] + 175) * (2 * CT);
}

// a3 + a6 + a7 on 72 raw samples: (double)((float)raw * res - b), the multiply and the subtraction
// each one correctly rounded fp32 operation (DataProviderUtils.java:49-59, Baseline.java:39-41),
// evaluated two samples at a time with packed fp32 math (v_pk_mul_f32 / v_pk_add_f32).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void decode_pairs(const int16_t (&xr)[kIn], float r, float b,
                                             double (&x)[kIn]) {
  const f32x2 rr = {r, r}, bb = {b, b};
#pragma unroll
  for (int k = 0; k < kIn; k += 2) {
    const f32x2 v = {(float)xr[k], (float)xr[k + 1]};
    const f32x2 y = v * rr - bb;
    x[k] = (double)y.x;
    x[k + 1] = (double)y.y;
  }
}

// SignalProcessing.normalize (SignalProcessing.java:38-52) for the <= 8 feature rows of a
// sub-tile, executed by one wave: lane e < ne folds Math.pow(f, 2) over row e in index order
// (the 8 dependent chains run side by side), then the 64 lanes divide and store the rows
// (coalesced 16-byte stores).  `norm` is an 8-double LDS scratch owned by the calling wave.
template <int F>
__device__ __forceinline__ void normalise_store(const double* fb, double* norm, double* o, int ne,
                                                int lane) {
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

// One global_load_lds_dwordx4: lane l's 16 bytes at `src` land at LDS byte address
// lds_base + 16*l.  Issued through inline asm so that the compiler's waitcnt pass neither
// serialises consecutive DMAs nor waits on them; the kernel drains them itself with an explicit
// `s_waitcnt vmcnt(0)` before the barrier that publishes the window (vmcnt retires in order, so
// any wait the compiler places for its own loads can only over-wait, never under-wait).
__device__ __forceinline__ void dma16(const uint8_t* src, uint32_t* lds_dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(lds_ptr_t)lds_dst;
  uint32_t saved;  // m0 is compiler-reserved: restore it inside the same statement
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, off\n\t"
      "s_nop 0\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "s"(lds), "v"(src)
      : "memory");
}

// Issues the LDS-DMA of one sub-tile's windows (wave w takes DMA instructions w, w+C, ...; every
// guard is wave-uniform, so no VMEM op other than the DMAs is issued and nothing waits on them).
// Returns whether some in-range quad of this wave could not be DMA'd (past the recording end).
template <int CT, int C>
__device__ __forceinline__ bool dma_issue(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const int64_t* __restrict__ pos, int64_t n, int64_t e0,
                                          uint32_t* win, int w, int lane) {
  using G = Geometry<CT>;
  constexpr int PER_E = (G::EPQ + 63) / 64;
  constexpr int NI = kSub * PER_E;
  bool need_fix = false;
#pragma unroll
  for (int it = 0; it < (NI + C - 1) / C; ++it) {
    const int m = w + it * C;
    if (m < NI) {
      const int e = m / PER_E, j = m - e * PER_E;
      if (e0 + e < n) {
        const int64_t B = window_byte<CT>(pos, e0 + e);
        const int i = 64 * j + lane;
        const int sg = i / G::SEGQ, q = i - sg * G::SEGQ;
        const int64_t A = (B & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * q;
        if (i < G::EPQ) {
          if (A + 16 <= nbytes) dma16(raw + A, win + e * G::ESTR + 256 * j);
          else need_fix = true;
        }
      }
    }
  }
  return need_fix;
}

// Direct (non-DMA) fill of the quads dma_issue skipped: zero or partial quads at the recording end.
template <int CT, int C>
__device__ __forceinline__ void dma_fixup(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const int64_t* __restrict__ pos, int64_t n, int64_t e0,
                                          uint32_t* win, int w, int lane) {
  using G = Geometry<CT>;
  constexpr int PER_E = (G::EPQ + 63) / 64;
  constexpr int NI = kSub * PER_E;
  for (int m = w; m < NI; m += C) {
    const int e = m / PER_E, j = m - e * PER_E;
    const int i = 64 * j + lane;
    if (e0 + e >= n || i >= G::EPQ) continue;
    const int sg = i / G::SEGQ, q = i - sg * G::SEGQ;
    const int64_t A = (window_byte<CT>(pos, e0 + e) & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * q;
    if (A + 16 > nbytes) lds_store4(win + e * G::ESTR + 256 * j + 4 * lane, load16(raw, nbytes, A));
  }
}

// LDS-DMA pipeline: the window of sub-tile k+1 is fetched by global_load_lds_dwordx4 (16-byte
// aligned per-lane sources, dword-aligned contiguous LDS destinations, no VGPRs) into the single
// window buffer as soon as every lane has copied its raw samples of sub-tile k into registers;
// the transfer overlaps the whole filter bank.  K sub-tiles per workgroup, unrolled; the barrier
// that publishes the features of sub-tile k also publishes the window of k+1.
template <int CT, int C, bool FAST, int MINW, int K, bool SHFL = true>
__global__ __launch_bounds__(64 * C, MINW) void window_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using G = Geometry<CT>;
  constexpr int F = C * 16;
  __shared__ __attribute__((aligned(16))) uint32_t win[kSub * G::ESTR];
  __shared__ __attribute__((aligned(16))) double feat[2][kSub * F];
  __shared__ int tdelta[2][kSub];
  __shared__ double norm[kSub];
  __shared__ __attribute__((aligned(16))) double xch[SHFL ? 2 : C * 64 * kSlot];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int el = lane >> 3, s = lane & 7;
  const int64_t nbytes = n_frames * G::FB;
  const int col = sel.col[w];
  const float r = sel.res[w];
  const int64_t first = (int64_t)blockIdx.x * K * kSub;

  if (w == 0 && lane < kSub)
    tdelta[0][lane] = first + lane < n ? (int)(window_byte<CT>(pos, first + lane) & 15) : 0;
  float bcur = (first + el < n) ? base[(first + el) * C + w] : 0.0f;
  if (dma_issue<CT, C>(raw, nbytes, pos, n, first, win, w, lane))
    dma_fixup<CT, C>(raw, nbytes, pos, n, first, win, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < K; ++kk) {
    const int64_t e0 = first + (int64_t)kk * kSub;
    if (e0 >= n) break;  // uniform
    // 1. this lane's 72 raw samples -> registers
    const uint8_t* eb = (const uint8_t*)(win + el * G::ESTR) + tdelta[kk & 1][el] + 2 * col;
    const int16_t* own = (const int16_t*)(eb + 16 * G::SEGQ * s);
    const int16_t* nxt = (const int16_t*)(eb + 16 * G::SEGQ * ((s + 1) & 7));
    int16_t xr[kIn];
#pragma unroll
    for (int k = 0; k < kSegLen; ++k) xr[k] = own[k * CT];
#pragma unroll
    for (int k = 0; k < 8; ++k) xr[kSegLen + k] = nxt[k * CT];
    const float b = bcur;
    __syncthreads();  // (A) every lane holds its samples: the window is free
    // 2. the next sub-tile streams into the window while the filter bank runs
    const int64_t e1 = e0 + kSub;
    const bool more = kk + 1 < K && e1 < n;
    bool need_fix = false;
    if (more) {
      if (w == 0 && lane < kSub)
        tdelta[(kk + 1) & 1][lane] = e1 + lane < n ? (int)(window_byte<CT>(pos, e1 + lane) & 15) : 0;
      bcur = (e1 + el < n) ? base[(e1 + el) * C + w] : 0.0f;
      need_fix = dma_issue<CT, C>(raw, nbytes, pos, n, e1, win, w, lane);
    }
    double x[kIn];
    decode_pairs(xr, r, b, x);
    double a6, d6;
    dwt8_cascade<FAST, SHFL>(x, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
    double* fb = feat[kk & 1];
    fb[el * F + w * 16 + s] = a6;
    fb[el * F + w * 16 + 8 + s] = d6;
    if (need_fix) dma_fixup<CT, C>(raw, nbytes, pos, n, e1, win, w, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (B) features(kk) and window(kk+1) complete
    // normalisation: one wave (rotating over the sub-tiles of the workgroup); lanes 0..7 run the
    // 8 sequential sums of squares side by side, then all 64 lanes divide and store.
    if (w == kk % C) normalise_store<F>(fb, norm, out + e0 * F, (n - e0) < kSub ? (int)(n - e0) : kSub, lane);
  }
}

}  // namespace dev

namespace {
// Variant selector (perf study): EEGFX_FUSED_IMPL = "<d|l><minw><K>": d = cross-lane
// (ds_bpermute) halos, l = LDS-slot halos; minw = launch-bounds waves per EU; K = sub-tiles per
// workgroup.  Default "d41".
struct Impl {
  bool shfl = true;
  int minw = 4;
  int k = 1;
};
Impl impl_choice() {
  static const Impl v = [] {
    Impl d;
    const char* e = getenv("EEGFX_FUSED_IMPL");
    if (e && strlen(e) == 3 && (e[0] == 'd' || e[0] == 'l')) {
      d.shfl = e[0] == 'd';
      d.minw = e[1] - '0';
      d.k = e[2] - '0';
    }
    return d;
  }();
  return v;
}

template <bool FAST>
void launch_window3(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                    const int64_t* pos, const float* base, int64_t n, double* out) {
  const Impl im = impl_choice();
  const int64_t nsub = (n + dev::kSub - 1) / dev::kSub;
  const dim3 g((unsigned)((nsub + im.k - 1) / im.k));
  bool launched = false;
#define EEGFX_D(MW, KK, SH)                                                                       \
  if (!launched && im.minw == MW && im.k == KK && im.shfl == SH) {                                \
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, MW, KK, SH>), g, dim3(192), 0, st,          \
                       (const uint8_t*)raw, n_frames, sel, pos, base, n, out);                    \
    launched = true;                                                                              \
  }
  EEGFX_D(4, 1, true) EEGFX_D(3, 1, true) EEGFX_D(2, 2, true) EEGFX_D(3, 2, true)
  EEGFX_D(3, 1, false) EEGFX_D(3, 2, false)
#undef EEGFX_D
  if (!launched)
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, 4, 1, true>), dim3((unsigned)nsub),
                       dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel, pos, base, n, out);
}
}  // namespace

bool fused_supported(int fmt, int ct, int C, const double* out) {
  return fmt == 0 && ct == 3 && C == 3 && ((uintptr_t)out & 15) == 0;
}

size_t fused_scratch_bytes(int64_t n, int C) { return sizeof(float) * (size_t)n * (size_t)C; }

int64_t fused_window_bytes_per_epoch(int ct, int C) {
  return (int64_t)dev::kWin * ct * 2 + (int64_t)C * 4 + 8 + (int64_t)C * 16 * 8;
}

hipError_t launch_fused_baseline(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 void* scratch) {
  if (ct != 3 || C != 3) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  const dim3 bgrid((unsigned)((n + dev::kTile - 1) / dev::kTile));
  hipLaunchKernelGGL((dev::baseline_kernel<3, 3>), bgrid, dim3(192), 0, st, (const uint8_t*)raw,
                     n_frames, sel, pos, n, (float*)scratch);
  return hipGetLastError();
}

hipError_t launch_fused_window(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n, bool fast,
                               const void* scratch, double* out) {
  if (ct != 3 || C != 3) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  if (fast) launch_window3<true>(st, raw, n_frames, sel, pos, (const float*)scratch, n, out);
  else launch_window3<false>(st, raw, n_frames, sel, pos, (const float*)scratch, n, out);
  return hipGetLastError();
}

}  // namespace eegfx
