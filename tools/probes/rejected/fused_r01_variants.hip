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
#include "lds_dma.h"

// Perf-study builds only (tools/probes/window_probe.hip): bit 0 drops the window DMA (and its
// waits), bit 1 the LDS reads + decode, bit 2 the filter bank; the library is built with 0.
#ifndef EEGFX_FUSED_ABLATION
#define EEGFX_FUSED_ABLATION 0
#endif
// FMA-mode row store: 0 = each lane stores its own 6 normalised features (16-byte pieces 48 bytes
// apart), 1 = rows staged back into LDS and stored as contiguous 1 KB wave stores, 2 = as 1 with
// non-temporal stores (0.928 -> 0.924 ms in tools/probes, twice; the default).
#ifndef EEGFX_STORE_MODE
#define EEGFX_STORE_MODE 2
#endif
// Level-0 halo: 0 = every lane decodes its 8 halo samples from LDS, 1 = lanes decode only their
// 64 own samples and take the halo (8 doubles) from lane s+1 through ds_bpermute.
#ifndef EEGFX_HALO0_SHFL
#define EEGFX_HALO0_SHFL 0
#endif
// Decode of the K == 1 kernel: 0 = the whole 72-sample slice decoded up front, two samples per
// packed fp32 op (116 VGPRs: 4 waves/SIMD); 1 = the same one sample per op (72 more VALU ops per
// wave, 96 VGPRs: 5 waves/SIMD, 2 % faster than 0); 2 = packed pairs decoded just in time inside
// level 1 (level1_lds: 94 VGPRs, 5 waves/SIMD, and the 72 VALU ops of 1 saved).
#ifndef EEGFX_DECODE_SCALAR
#define EEGFX_DECODE_SCALAR 2
#endif

namespace eegfx {
namespace dev {

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4_a16 __attribute__((ext_vector_type(4), aligned(16)));

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
// NT: non-temporal read, for pre-stimulus frames no other epoch's window or baseline shares
// (baseline_kernel 0.136 -> 0.124 ms with markers 1,000 frames apart, tools/probes).
template <bool NT = false>
__device__ __forceinline__ u32x4_a4 load16_bulk(const uint8_t* __restrict__ raw, int64_t nbytes,
                                                int64_t A, bool want) {
  const bool full = want && A >= 0 && A + 16 <= nbytes;
  const u32x4_a16* src = (const u32x4_a16*)(full ? raw + A : safe_quad(raw, nbytes));
  u32x4_a4 v;
  if constexpr (NT) v = __builtin_nontemporal_load(src);
  else v = *src;
  const u32x4_a4 z = {0u, 0u, 0u, 0u};
  return full ? v : z;
}
__device__ __forceinline__ bool straddles_end(int64_t A, int64_t nbytes, bool want) {
  return want && A >= 0 && A < nbytes && A + 16 > nbytes;
}

template <int CT, int C, int TILE, bool STREAM = false>
__global__ __launch_bounds__((TILE * C + 63) / 64 * 64) void baseline_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    int64_t n, float* __restrict__ bout) {
  using G = Geometry<CT>;
  constexpr int NT = (TILE * C + 63) / 64 * 64;
  __shared__ __attribute__((aligned(16))) uint32_t stage[TILE * G::BSTR];
  __shared__ int64_t tB[TILE];
  const int tid = threadIdx.x;
  const int64_t nbytes = n_frames * G::FB;
  const int64_t t0 = (int64_t)blockIdx.x * TILE;
  const int nt = (n - t0) < TILE ? (int)(n - t0) : TILE;
  if (tid < TILE) tB[tid] = tid < nt ? (pos[t0 + tid] - kPre) * G::FB : 0;
  __syncthreads();
  constexpr int ITERS = (TILE * G::BASEQ + NT - 1) / NT;
  u32x4_a4 v[ITERS];
  int64_t A[ITERS];
  bool want[ITERS];
  const bool tiny = nbytes < 16;
#pragma unroll
  for (int k = 0; k < ITERS; ++k) {
    const int i = tid + k * NT;
    const int e = i / G::BASEQ, q = i - e * G::BASEQ;
    want[k] = i < TILE * G::BASEQ && e < nt;
    A[k] = want[k] ? (tB[e] & ~(int64_t)15) + 16 * q : 0;
    v[k] = load16_bulk<STREAM>(raw, nbytes, A[k], want[k] && !tiny);
  }
#pragma unroll
  for (int k = 0; k < ITERS; ++k)
    if (straddles_end(A[k], nbytes, want[k]) || (tiny && want[k])) v[k] = load16(raw, nbytes, A[k]);
#pragma unroll
  for (int k = 0; k < ITERS; ++k) {
    const int i = tid + k * NT;
    if (i < TILE * G::BASEQ) {
      const int e = i / G::BASEQ, q = i - e * G::BASEQ;
      lds_store4(stage + e * G::BSTR + 4 * q, v[k]);
    }
  }
  __syncthreads();
  if (tid >= TILE * C) return;
  const int c = tid / TILE, e = tid - c * TILE;
  const float r = sel.res[c];
  const int16_t* src = (const int16_t*)((const uint8_t*)(stage + e * G::BSTR) + (tB[e] & 15)) +
                       sel.col[c];
  float b = 0.0f;
  if constexpr (EEGFX_FUSED_ABLATION & 64) {  // perf study: staging only, no fold
    b = (float)src[0] * r;
  } else {
#pragma unroll 20
    for (int i = 0; i < kPre; ++i) b = b + (float)src[i * CT] * r;
  }
  if (e < nt) bout[(t0 + e) * C + c] = b / (float)kPre;
}

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
template <int N = kIn>
__device__ __forceinline__ void decode_pairs(const int16_t (&xr)[kIn], float r, float b,
                                             double (&x)[kIn]) {
  const f32x2 rr = {r, r}, bb = {b, b};
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    const f32x2 v = {(float)xr[k], (float)xr[k + 1]};
    const f32x2 y = v * rr - bb;
    x[k] = (double)y.x;
    x[k + 1] = (double)y.y;
  }
}

// decode_pairs reading the samples straight from the staged window: own[k*CT] for k < 64, then
// the 8 halo samples nxt[k*CT] of the next segment.
template <int CT, int N = kIn>
__device__ __forceinline__ void decode_lds(const int16_t* own, const int16_t* nxt, float r, float b,
                                           double (&x)[kIn]) {
#if EEGFX_DECODE_SCALAR
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int16_t v0 = k < kSegLen ? own[k * CT] : nxt[(k - kSegLen) * CT];
    x[k] = (double)((float)v0 * r - b);
  }
  return;
#endif
  const f32x2 rr = {r, r}, bb = {b, b};
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    const int16_t v0 = k < kSegLen ? own[k * CT] : nxt[(k - kSegLen) * CT];
    const int16_t v1 = k + 1 < kSegLen ? own[(k + 1) * CT] : nxt[(k + 1 - kSegLen) * CT];
    const f32x2 v = {(float)v0, (float)v1};
    const f32x2 y = v * rr - bb;
    x[k] = (double)y.x;
    x[k + 1] = (double)y.y;
  }
}

// Decode fused into level 1 (EEGFX_DECODE_SCALAR == 2): the samples are decoded two at a time
// (packed fp32 multiply and subtract: the same two correctly rounded fp32 operations per sample)
// just before the first level-1 output that needs them, so only the 10-sample sliding window
// and the level-1 outputs are live -- the packed decode at the register budget of the scalar one.
template <int CT, bool FAST>
__device__ __forceinline__ void level1_lds(const int16_t* own, const int16_t* nxt, float r, float b,
                                           double (&a1)[40]) {
  level1_jit<FAST>(
      [&](int k) { return (float)(k < kSegLen ? own[k * CT] : nxt[(k - kSegLen) * CT]); }, r, b,
      a1);
}

// SignalProcessing.normalize (SignalProcessing.java:38-52) for the <= 8 feature rows of a
// sub-tile, executed by one wave: lane e < ne folds Math.pow(f, 2) over row e in index order
// (the 8 dependent chains run side by side), then the 64 lanes divide and store the rows
// (coalesced 16-byte stores).  `norm` is an 8-double LDS scratch owned by the calling wave.
template <int F, bool FAST = false>
__device__ __forceinline__ void normalise_store(const double* fb, double* norm, double* o, int ne,
                                                int lane) {
  if constexpr (FAST && F % 16 == 0) {
    // FMA contract (1e-9): the 8 lanes of an epoch each square-sum F/8 features, a 3-step
    // butterfly completes the row sum, and the row is scaled by one reciprocal (x * (1/s) is
    // within 1 ulp of x / s; an all-zero row still gives NaN = 0 * inf).
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
    const double inv = 1.0 / sqrt(acc);
    if constexpr (EEGFX_STORE_MODE == 0) {
      if (e < ne) {
#pragma unroll
        for (int i = 0; i < P; i += 2)
          *(double2*)(o + e * F + p * P + i) = make_double2(v[i] * inv, v[i + 1] * inv);
      }
    } else {
      double* fw = const_cast<double*>(fb);
      if (e < ne) {
#pragma unroll
        for (int i = 0; i < P; i += 2)
          *(double2*)(fw + e * F + p * P + i) = make_double2(v[i] * inv, v[i + 1] * inv);
      }
      wave_sync();
      for (int i = 2 * lane; i < ne * F; i += 128) {
        typedef double f64x2 __attribute__((ext_vector_type(2)));
        const f64x2 q = *(const f64x2*)(fw + i);
        if constexpr (EEGFX_STORE_MODE == 2) __builtin_nontemporal_store(q, (f64x2*)(o + i));
        else *(f64x2*)(o + i) = q;
      }
      wave_sync();
    }
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

// Byte offset, from floor16(B_e), of the global quad that lands in LDS quad i of an epoch window
// (segment i / SEGQ, quad i % SEGQ of that segment).  Depends on the lane only, so a kernel
// computes it once per DMA row j (i = 64*j + lane) and every DMA of every epoch reuses it.
template <int CT>
__device__ __forceinline__ uint32_t quad_offset(int i) {
  using G = Geometry<CT>;
  const int sg = i / G::SEGQ;
  return (uint32_t)(kSegLen * G::FB * sg + 16 * (i - G::SEGQ * sg));
}

template <int CT>
struct DmaRows {
  static constexpr int PER_E = (Geometry<CT>::EPQ + 63) / 64;  // 4 DMA rows per epoch window
  uint32_t off[PER_E];
  __device__ __forceinline__ explicit DmaRows(int lane) {
#pragma unroll
    for (int j = 0; j < PER_E; ++j) off[j] = quad_offset<CT>(64 * j + lane);
  }
};

// Issues the LDS-DMA of one sub-tile's windows: wave w stages epochs w, w+C, w+2C, ... (every
// DMA row of each).  The marker positions of those epochs are loaded (scalar) before the first
// DMA, so the DMAs leave back to back; an epoch whose whole window lies inside the recording (a
// scalar test) takes the unguarded path.  Returns whether some in-range quad of this lane could
// not be DMA'd (the recording ends inside the window).
template <int CT, int C, bool NT = false>
__device__ __forceinline__ bool dma_issue(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const int64_t* __restrict__ pos, int64_t n, int64_t e0,
                                          uint32_t* win, int w, int lane, const DmaRows<CT>& rows) {
  using G = Geometry<CT>;
  constexpr int PER_E = DmaRows<CT>::PER_E;
  constexpr int NE = (kSub + C - 1) / C;
  constexpr int64_t kSpanB = kSegLen * G::FB * 7 + 16 * (G::SEGQ - 1) + 16;
  int64_t Bq[NE];
#pragma unroll
  for (int t = 0; t < NE; ++t) {  // unconditional (clamped) loads: one scalar round trip
    const int64_t ei = e0 + (w + t * C < kSub ? w + t * C : kSub - 1);
    Bq[t] = window_byte<CT>(pos, ei < n ? ei : n - 1) & ~(int64_t)15;
  }
  bool need_fix = false;
#pragma unroll
  for (int t = 0; t < NE; ++t) {
    const int e = w + t * C;
    if (e >= kSub || e0 + e >= n) continue;  // uniform
    const uint8_t* sb = raw + Bq[t];
    uint32_t* dst = win + e * G::ESTR;
    if (Bq[t] + kSpanB <= nbytes) {
#pragma unroll
      for (int j = 0; j < PER_E; ++j)
        if (64 * (j + 1) <= G::EPQ || 64 * j + lane < G::EPQ) dma16_s<NT>(sb, rows.off[j], dst + 256 * j);
    } else {
#pragma unroll
      for (int j = 0; j < PER_E; ++j) {
        if (64 * j + lane >= G::EPQ) continue;
        if (Bq[t] + rows.off[j] + 16 <= nbytes) dma16_s<NT>(sb, rows.off[j], dst + 256 * j);
        else need_fix = true;
      }
    }
  }
  return need_fix;
}

// Direct (non-DMA) fill of the quads dma_issue skipped (same wave -> epoch mapping): zero or
// partial quads at the recording end.
template <int CT, int C>
__device__ __forceinline__ void dma_fixup(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const int64_t* __restrict__ pos, int64_t n, int64_t e0,
                                          uint32_t* win, int w, int lane, const DmaRows<CT>& rows) {
  using G = Geometry<CT>;
  constexpr int PER_E = DmaRows<CT>::PER_E;
  for (int e = w; e < kSub; e += C) {
    if (e0 + e >= n) break;
    const int64_t Bq = window_byte<CT>(pos, e0 + e) & ~(int64_t)15;
#pragma unroll
    for (int j = 0; j < PER_E; ++j) {
      const int64_t A = Bq + rows.off[j];
      if (64 * j + lane < G::EPQ && A + 16 > nbytes)
        lds_store4(win + e * G::ESTR + 256 * j + 4 * lane, load16(raw, nbytes, A));
    }
  }
}

// The baseline of (epoch first+el, channel col) inside the window kernel (FUSEB): a3 + a5 + a6's
// prefix, Baseline.java:29-42, without the separate baseline_kernel pass.  The 8 lanes of an
// epoch group (s = 0..7) each load and scale a 13-sample chunk of the 100 pre-stimulus frames
// ((float)raw * res, one rounded fp32 multiply; frames outside the recording are the reference's
// +0.0f padding), then fold them in sample order as ONE sequential chain: stage k adds lane k's
// chunk to the running sum and hands it to lane k+1 -- the exact operation sequence of the
// reference's loop.  Returns b / 100 in every lane of the group.  The loads are issued before the
// window DMAs, so the chain waits only as long as the window does.
template <int CT>
__device__ __forceinline__ void fused_baseline_load(const uint8_t* __restrict__ raw, int64_t n_frames,
                                                    const int64_t* __restrict__ pos, int64_t n,
                                                    int64_t first, int el, int s, int col, float r,
                                                    float (&p)[13]) {
  constexpr int CH = 13;
  const int64_t nbytes = n_frames * 2 * CT;
  const int64_t e = first + el < n ? first + el : n - 1;
  const int64_t f0 = pos[e] - kPre + CH * s;
  const int16_t* placeholder = (const int16_t*)safe_quad(raw, nbytes);
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int64_t f = f0 + j;
    const bool in = CH * s + j < kPre && f >= 0 && f < n_frames;
    const int16_t v = *(in ? (const int16_t*)raw + f * CT + col : placeholder);
    p[j] = in ? (float)v * r : 0.0f;
  }
}
__device__ __forceinline__ float fused_baseline_fold(const float (&p)[13], int lane, int s) {
  constexpr int CH = 13;
  float acc = 0.0f;
#pragma unroll
  for (int stage = 0; stage < 8; ++stage) {
    if (s == stage) {
#pragma unroll
      for (int j = 0; j < (stage < 7 ? CH : kPre - 7 * CH); ++j) acc = acc + p[j];
    }
    if (stage < 7) {
      const float prev = __shfl(acc, (lane & ~7) | stage, 64);
      if (s == stage + 1) acc = prev;
    }
  }
  const float b = __shfl(acc, lane | 7, 64);
  return b / (float)kPre;
}

// LDS-DMA pipeline: the window of sub-tile k+1 is fetched by global_load_lds_dwordx4 (16-byte
// aligned per-lane sources, dword-aligned contiguous LDS destinations, no VGPRs) into the single
// window buffer as soon as every lane has copied its raw samples of sub-tile k into registers;
// the transfer overlaps the whole filter bank.  K sub-tiles per workgroup, unrolled; the barrier
// that publishes the features of sub-tile k also publishes the window of k+1.
template <int CT, int C, bool FAST, int MINW, int K, bool SHFL = true, bool FUSEB = false,
          bool NT = false>
__global__ __launch_bounds__(64 * C, MINW) void window_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using G = Geometry<CT>;
  constexpr int F = C * 16;
  __shared__ __attribute__((aligned(16))) uint32_t win[kSub * G::ESTR];
  // K > 1: double-buffered feature rows; K == 1: the rows reuse the start of the window buffer
  // once every wave has decoded its samples (26 KB of LDS per workgroup instead of 32)
  __shared__ __attribute__((aligned(16))) double feat[K > 1 ? 2 : 1][K > 1 ? kSub * F : 2];
  __shared__ int tdelta[2][kSub];
  __shared__ double norm[kSub];
  __shared__ __attribute__((aligned(16))) double xch[SHFL ? 2 : C * 64 * kSlot];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int el = lane >> 3, s = lane & 7;
  const int64_t nbytes = n_frames * G::FB;
  const int col = sel.col[w];
  const float r = sel.res[w];
  const int64_t first = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * K * kSub;

  if (w == 0 && lane < kSub)
    tdelta[0][lane] = first + lane < n ? (int)(window_byte<CT>(pos, first + lane) & 15) : 0;
  static_assert(!FUSEB || K == 1, "in-kernel baselines: one sub-tile per workgroup");
  float bp[13];
  if constexpr (FUSEB) fused_baseline_load<CT>(raw, n_frames, pos, n, first, el, s, col, r, bp);
  float bcur = FUSEB ? 0.0f : ((first + el < n) ? base[(first + el) * C + w] : 0.0f);
  const DmaRows<CT> rows(lane);
  if (!(EEGFX_FUSED_ABLATION & 1) && dma_issue<CT, C, NT>(raw, nbytes, pos, n, first, win, w, lane, rows))
    dma_fixup<CT, C>(raw, nbytes, pos, n, first, win, w, lane, rows);
  if constexpr (FUSEB) bcur = fused_baseline_fold(bp, lane, s);
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
    // With one sub-tile per workgroup nothing refills the window, so the samples are decoded
    // straight from LDS (no int16 staging array: 72 fewer live VGPRs, no spill); with K > 1
    // they are copied to registers first and barrier A frees the window for the next DMA.
    int16_t xr[kIn];
    if constexpr (K > 1) {
#pragma unroll
      for (int k = 0; k < kSegLen; ++k) xr[k] = own[k * CT];
      if constexpr (!EEGFX_HALO0_SHFL) {
#pragma unroll
        for (int k = 0; k < 8; ++k) xr[kSegLen + k] = nxt[k * CT];
      }
    }
    const float b = bcur;
    if constexpr (K > 1) __syncthreads();  // (A) every lane holds its samples: the window is free
    // 2. the next sub-tile streams into the window while the filter bank runs
    const int64_t e1 = e0 + kSub;
    const bool more = kk + 1 < K && e1 < n;
    bool need_fix = false;
    if (more) {
      if (w == 0 && lane < kSub)
        tdelta[(kk + 1) & 1][lane] = e1 + lane < n ? (int)(window_byte<CT>(pos, e1 + lane) & 15) : 0;
      bcur = (e1 + el < n) ? base[(e1 + el) * C + w] : 0.0f;
      if (!(EEGFX_FUSED_ABLATION & 1)) need_fix = dma_issue<CT, C, NT>(raw, nbytes, pos, n, e1, win, w, lane, rows);
    }
    double a6, d6;
    if constexpr (K == 1 && EEGFX_DECODE_SCALAR == 2 && !(EEGFX_FUSED_ABLATION & 6) &&
                  !EEGFX_HALO0_SHFL) {
      double a1[40];
      level1_lds<CT, FAST>(own, nxt, r, b, a1);
      halo<32, SHFL>(a1, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s);
      dwt8_levels2to6<FAST, SHFL>(a1, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
    } else {
    double x[kIn];
    if constexpr (EEGFX_FUSED_ABLATION & 2) {
#pragma unroll
      for (int k = 0; k < kIn; ++k) x[k] = (double)b + k;
    } else if constexpr (K == 1) {
      decode_lds<CT, EEGFX_HALO0_SHFL ? kSegLen : kIn>(own, nxt, r, b, x);
      if constexpr (EEGFX_HALO0_SHFL) halo_shuffle<kSegLen>(x, lane & ~7, s);
    } else if constexpr (EEGFX_HALO0_SHFL) {
      decode_pairs<kSegLen>(xr, r, b, x);
      halo_shuffle<kSegLen>(x, lane & ~7, s);
    } else {
      decode_pairs(xr, r, b, x);
    }
    if constexpr (EEGFX_FUSED_ABLATION & 4) {
      a6 = 0.0;
#pragma unroll
      for (int k = 0; k < kIn; ++k) a6 += x[k];
      d6 = a6;
    } else {
      dwt8_cascade<FAST, SHFL>(x, SHFL ? xch : xch + w * 64 * kSlot, lane & ~7, s, a6, d6);
    }
    }
    double* fb = K > 1 ? feat[kk & 1] : (double*)win;
    if constexpr (K == 1) __syncthreads();  // every wave has read its samples: rows may overwrite
    // the row slot is recomputed here from an opaque copy of the lane id, so its address is not
    // kept live across the filter bank (it was the one spilled VGPR)
    int l2 = lane;
    asm volatile("" : "+v"(l2));
    const int slot = (l2 >> 3) * F + w * 16 + (l2 & 7);
    fb[slot] = a6;
    fb[slot + 8] = d6;
    if (need_fix) dma_fixup<CT, C>(raw, nbytes, pos, n, e1, win, w, lane, rows);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (B) features(kk) and window(kk+1) complete
    // normalisation: one wave (rotating over the sub-tiles of the workgroup); lanes 0..7 run the
    // 8 sequential sums of squares side by side, then all 64 lanes divide and store.
    if (w == kk % C) normalise_store<F, FAST>(fb, norm, out + e0 * F, (n - e0) < kSub ? (int)(n - e0) : kSub, lane);
  }
}


// ================================================================================================
// window_p_kernel -- window_kernel's sub-tile computation in a persistent workgroup with the next
// sub-tile's window in flight during the filter bank.  window_kernel's one-shot workgroups pay two
// dependent memory round trips before any arithmetic (marker positions, then the window DMA);
// here the positions of sub-tile i+1 are in LDS before sub-tile i starts (loaded two iterations
// ahead into a register) and its LDS-DMA is issued right after the current window has been copied
// to registers (barrier A), into the same single window buffer -- the same LDS (32 KB) and VGPR
// budget as window_kernel, so the same 5 workgroups per CU stay resident.
template <int CT, int C>
__device__ __forceinline__ bool dma_issue_b(const uint8_t* __restrict__ raw, int64_t nbytes,
                                            const int64_t* wbB, uint32_t* win, int w, int lane) {
  using G = Geometry<CT>;
  constexpr int PER_E = (G::EPQ + 63) / 64;
  constexpr int NI = kSub * PER_E;
  bool need_fix = false;
#pragma unroll
  for (int it = 0; it < (NI + C - 1) / C; ++it) {
    const int m = w + it * C;
    if (m < NI) {
      const int e = m / PER_E, j = m - e * PER_E;
      const int64_t B = wbB[e];
      if (B >= 0) {
        const int i = 64 * j + lane;
        const int sg = i / G::SEGQ, q = i - sg * G::SEGQ;
        const int64_t A = (B & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * q;
        if (i < G::EPQ) {
          // perf-study bit 8: every DMA reads one L2-resident quad (LDS-write + issue cost only)
          const int64_t src = (EEGFX_FUSED_ABLATION & 8) ? ((int64_t)(lane & 15) << 4) : A;
          if (A + 16 <= nbytes) dma16(raw + src, win + e * G::ESTR + 256 * j);
          else need_fix = true;
        }
      }
    }
  }
  return need_fix;
}

template <int CT, int C>
__device__ __forceinline__ void dma_fixup_b(const uint8_t* __restrict__ raw, int64_t nbytes,
                                            const int64_t* wbB, uint32_t* win, int w, int lane) {
  using G = Geometry<CT>;
  constexpr int PER_E = (G::EPQ + 63) / 64;
  constexpr int NI = kSub * PER_E;
  for (int m = w; m < NI; m += C) {
    const int e = m / PER_E, j = m - e * PER_E;
    const int i = 64 * j + lane;
    const int64_t B = wbB[e];
    if (B < 0 || i >= G::EPQ) continue;
    const int sg = i / G::SEGQ, q = i - sg * G::SEGQ;
    const int64_t A = (B & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * q;
    if (A + 16 > nbytes) lds_store4(win + e * G::ESTR + 256 * j + 4 * lane, load16(raw, nbytes, A));
  }
}

template <int CT, int C, bool FAST, int MINW>
__global__ __launch_bounds__(64 * C, MINW) void window_p_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using G = Geometry<CT>;
  constexpr int F = C * 16;
  __shared__ __attribute__((aligned(16))) uint32_t win[kSub * G::ESTR];
  __shared__ __attribute__((aligned(16))) double feat[kSub * F];
  __shared__ double norm[kSub];
  __shared__ int64_t wbB[3][kSub];  // window byte offsets (-1: no epoch), ring over iterations
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int el = lane >> 3, s = lane & 7;
  const int64_t nbytes = n_frames * G::FB;
  const int col = sel.col[w];
  const float r = sel.res[w];
  const int64_t nsub = (n + kSub - 1) / kSub;
  const int64_t stride = gridDim.x;
  int64_t sub = blockIdx.x;
  if (sub >= nsub) return;
  auto wbyte = [&](int64_t sb) -> int64_t {  // wave 0 lanes 0..7: window byte offset of epoch lane
    const int64_t e = sb * kSub + lane;
    return sb < nsub && lane < kSub && e < n ? (pos[e] + 175) * G::FB : -1;
  };
  int64_t pq = 0;
  if (w == 0) {
    const int64_t b0 = wbyte(sub), b1 = wbyte(sub + stride);
    if (lane < kSub) {
      wbB[0][lane] = b0;
      wbB[1][lane] = b1;
    }
    pq = wbyte(sub + 2 * stride);
  }
  float bcur = (sub * kSub + el < n) ? base[(sub * kSub + el) * C + w] : 0.0f;
  __syncthreads();
  if (!(EEGFX_FUSED_ABLATION & 1) && dma_issue_b<CT, C>(raw, nbytes, wbB[0], win, w, lane))
    dma_fixup_b<CT, C>(raw, nbytes, wbB[0], win, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t it = 0; sub < nsub; sub += stride, ++it) {  // uniform
    const int64_t e0 = sub * kSub;
    const int64_t nxt = sub + stride;
    const int cur = (int)(it % 3), n1 = (int)((it + 1) % 3), n2 = (int)((it + 2) % 3);
    // 1. this lane's 72 raw samples -> registers
    const uint8_t* eb = (const uint8_t*)(win + el * G::ESTR) + (int)(wbB[cur][el] & 15) + 2 * col;
    const int16_t* own = (const int16_t*)(eb + 16 * G::SEGQ * s);
    const int16_t* nx = (const int16_t*)(eb + 16 * G::SEGQ * ((s + 1) & 7));
    int16_t xr[kIn];
#pragma unroll
    for (int k = 0; k < kSegLen; ++k) xr[k] = own[k * CT];
#pragma unroll
    for (int k = 0; k < 8; ++k) xr[kSegLen + k] = nx[k * CT];
    const float b = bcur;
    // 2. positions two sub-tiles ahead into the ring (loaded an iteration ago), the next load
    if (w == 0) {
      if (lane < kSub) wbB[n2][lane] = pq;
      pq = wbyte(sub + 3 * stride);
    }
    __syncthreads();  // (A) the window is free; positions of sub-tiles it+1, it+2 are published
    // 3. the next window streams in while the filter bank runs
    const bool more = nxt < nsub;
    bool need_fix = false;
    if (more) {
      bcur = (nxt * kSub + el < n) ? base[(nxt * kSub + el) * C + w] : 0.0f;
      if (!(EEGFX_FUSED_ABLATION & 1)) need_fix = dma_issue_b<CT, C>(raw, nbytes, wbB[n1], win, w, lane);
    }
    double x[kIn];
    decode_pairs(xr, r, b, x);
    double a6, d6;
    dwt8_cascade<FAST, true>(x, nullptr, lane & ~7, s, a6, d6);
    feat[el * F + w * 16 + s] = a6;
    feat[el * F + w * 16 + 8 + s] = d6;
    if (need_fix) dma_fixup_b<CT, C>(raw, nbytes, wbB[n1], win, w, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (B) features(it) and window(it+1) complete
    if (w == (int)(it % C))
      normalise_store<F, FAST>(feat, norm, out + e0 * F, (n - e0) < kSub ? (int)(n - e0) : kSub, lane);
  }
}

// ================================================================================================
// engine_kernel -- the same sub-tile computation, decoupled from HBM by a loader wave.
//
// Persistent: one workgroup per CU = L loader waves + G groups of C consumer waves (wave c of a
// group = channel c).  Every group owns one LDS window slot (8 epochs, ESTR_E dwords per epoch).
// The workgroup's tiles i = 0, 1, 2, ... (tile = 8 epochs, global tile blockIdx.x + i*gridDim.x)
// go to group i % G in round i / G and are fetched by loader i % L:
//   loader:   wait until the group released its slot for the round (free[g] >= C*round) ->
//             8 positions + 24 baselines by scalar loads -> misalignments + baselines into the
//             slot header -> 32 unconditional LDS-DMA instructions (dummy lanes read the first
//             quad of the recording into the slot's padding) -> wait for the PREVIOUS tile to
//             land (s_waitcnt vmcnt(32): exactly one tile newer), patch its past-the-end quads,
//             publish it (full[g] = round + 1).  Two tiles in flight per loader.
//   consumer: wait full[g] > round -> copy its 72 samples to VGPRs -> release (free[g] += 1)
//             -> decode + filter bank -> features into the group's LDS feature block ->
//             progress word fdone[g][c] = round + 1; wave round % C waits for the group's
//             words, normalises, stores.
// Compute waves never issue or wait on HBM traffic, so loads overlap the filter bank across the
// whole CU.  Flags live in LDS; every spin is bounded (a broken hand-off ends the kernel with
// wrong rows -- caught by the parity tests -- instead of hanging the GPU).
template <int CT>
struct EngineGeo {
  using G = Geometry<CT>;
  static constexpr int PER_E = (G::EPQ + 63) / 64;         // 4 DMA instructions per epoch
  static constexpr int NI = kSub * PER_E;                    // 32 per tile
  static constexpr int ESTR_E = round_up_res(PER_E * 256, 32, 1);  // 1025 dwords: no DMA clobber
  static constexpr int SLOT_DW = kSub * ESTR_E;
};

__device__ __forceinline__ uint32_t lds_addr32(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Publishes an LDS-DMA'd slot to the other waves: after the loader's covering vmcnt wait, one
// read of the slot's last-written dword drains this CU's LDS write path before the flag store.
__device__ __forceinline__ void publish_slot(uint32_t* flag, uint32_t v, const uint32_t* last) {
  uint32_t t;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(lds_addr32(last)) : "memory");
  (void)t;
  lds_st(flag, v);
}
__device__ __forceinline__ void lds_inc(uint32_t* p) {
  __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Bounded spin (~2^24 polls with s_sleep): false if the flag never reached v.
__device__ __forceinline__ bool spin_ge(const uint32_t* p, uint32_t v) {
  for (int k = 0; k < (1 << 24); ++k) {
    if (lds_ld(p) >= v) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

template <int CT, int C>
__device__ __forceinline__ void engine_fix(const uint8_t* __restrict__ raw, int64_t nbytes,
                                           const int64_t (&B)[kSub], int64_t e0, int64_t n,
                                           uint32_t* win, int lane) {
  using G = Geometry<CT>;
  using E = EngineGeo<CT>;
  for (int e = 0; e < kSub; ++e) {
    if (e0 + e >= n) break;
    for (int i = lane; i < G::EPQ; i += 64) {
      const int sg = i / G::SEGQ, q = i - sg * G::SEGQ;
      const int64_t A = (B[e] & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * q;
      if (A + 16 > nbytes) lds_store4(win + e * E::ESTR_E + 4 * i, load16(raw, nbytes, A));
    }
  }
}

// Meta ring: per batch of kMetaT consecutive tiles of the workgroup, the 8 positions (4 quads) and
// 8*C baselines (2*C quads) of each tile, fetched by one LDS-DMA instruction (lane = quad).
// Ring depth: batch b + kMetaR reuses batch b's slot; it is fetched at tile kMetaT*(b + kMetaR - 2),
// by which time the loader has seen every tile of batch b released (each group releases a tile
// right after reading its meta, and the loader is at most G tiles ahead of the releases):
// kMetaT*(kMetaR - 2) >= G + kMetaT - 1.
constexpr int kMetaT = 4;
constexpr int kMetaR = 4;
constexpr int kMetaQ = 64;  // quads per batch slot (one DMA instruction)
__device__ __forceinline__ const int64_t* meta_pos(const uint32_t* mring, int64_t i) {
  return (const int64_t*)(mring + ((i / kMetaT) % kMetaR) * kMetaQ * 4 + (i % kMetaT) * 16);
}
__device__ __forceinline__ const float* meta_base(const uint32_t* mring, int64_t i) {
  return (const float*)(mring + ((i / kMetaT) % kMetaR) * kMetaQ * 4 + kMetaT * 16) +
         (i % kMetaT) * kSub * 3;
}
// Lanes 0..4*kMetaT-1: positions (quad q of tile t = lane/4); lanes 16..16+2*C*kMetaT-1:
// baselines.  Out-of-range quads read the first quad of the recording (discarded).
template <int C>
__device__ __forceinline__ void dma_meta_batch(const uint8_t* __restrict__ safe,
                                               const int64_t* __restrict__ pos,
                                               const float* __restrict__ base, int64_t n,
                                               int64_t ntl, int64_t batch, uint32_t* dst, int lane) {
  static_assert(C == 3, "meta layout assumes 3 channels");
  const uint8_t* src = safe;
  if (lane < 4 * kMetaT) {
    const int64_t i = batch * kMetaT + lane / 4;
    const int64_t e = ((int64_t)blockIdx.x + i * gridDim.x) * kSub + 2 * (lane % 4);
    if (i < ntl && e + 1 < n) src = (const uint8_t*)(pos + e);
  } else if (lane < 4 * kMetaT + 2 * C * kMetaT) {
    const int k = lane - 4 * kMetaT;
    const int64_t i = batch * kMetaT + k / (2 * C);
    const int64_t f = ((int64_t)blockIdx.x + i * gridDim.x) * kSub * C + 4 * (k % (2 * C));
    if (i < ntl && f + 3 < n * C) src = (const uint8_t*)(base + f);
  }
  dma16(src, dst);
}

// Some window quad of the tile reaches past the recording (its DMA lane read a dummy quad).
template <int CT>
__device__ __forceinline__ bool tile_late(const int64_t (&B)[kSub], int64_t nbytes) {
  bool late = false;
#pragma unroll
  for (int e = 0; e < kSub; ++e) late |= (B[e] & ~(int64_t)15) + 16 * 8 * Geometry<CT>::SEGQ > nbytes;
  return late;
}

template <int CT, int C, bool FAST, int G_, int L>
__global__ __launch_bounds__(64 * (L + G_ * C), 1) void engine_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using G = Geometry<CT>;
  using E = EngineGeo<CT>;
  constexpr int F = C * 16;
  __shared__ __attribute__((aligned(16))) uint32_t win[G_][E::SLOT_DW];
  __shared__ __attribute__((aligned(16))) double feat[G_][2][kSub * F];
  __shared__ double norm[G_][kSub];
  __shared__ __attribute__((aligned(16))) uint32_t mring[kMetaR * kMetaQ * 4];
  static_assert(kMetaT * (kMetaR - 2) >= G_ + kMetaT - 1, "meta ring too shallow");
  __shared__ uint32_t full[G_], freed[G_], fdone[G_][C];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < G_) {
    full[tid] = 0;
    freed[tid] = 0;
  }
  if (tid < G_ * C) fdone[tid / C][tid % C] = 0;
  __syncthreads();  // the only workgroup barrier
  const int64_t nbytes = n_frames * G::FB;
  const int64_t ntiles = (n + kSub - 1) / kSub;
  const int64_t ntl = ntiles > blockIdx.x ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  auto tile_e0 = [&](int64_t i) { return ((int64_t)blockIdx.x + i * gridDim.x) * kSub; };

  if (w >= G_ * C) {  // ---------------------------------------------------------------- loader
    // Every vector-memory op of this wave is an LDS-DMA with a known count, so `s_waitcnt
    // vmcnt(N)` waits for exactly one earlier tile; nothing in the loop waits on SMEM.
    bool pending = false, ok = true;
    int pg = 0, pround = 0;
    int64_t pe0 = 0;
    int64_t pB[kSub];
    int32_t qoff[E::PER_E];  // byte offset of this lane's quad in DMA instruction j of an epoch
#pragma unroll
    for (int j = 0; j < E::PER_E; ++j) {
      const int i2 = 64 * j + lane, sg = i2 / G::SEGQ, q = i2 - sg * G::SEGQ;
      qoff[j] = i2 < G::EPQ ? kSegLen * G::FB * sg + 16 * q : 0;
    }
    for (int b0 = 0; b0 < 2; ++b0)  // meta of the first two batches
      dma_meta_batch<C>(safe_quad(raw, nbytes), pos, base, n, ntl, b0, mring + b0 * kMetaQ * 4, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int64_t i = 0; i < ntl && ok; ++i) {
      const int g = (int)(i % G_);
      const int round = (int)(i / G_);
      const int64_t e0 = tile_e0(i);
      const bool batch_start = (i % kMetaT) == 0;
      ok = spin_ge(&freed[g], (uint32_t)(C * round));
      if (e0 + kSub > n) {  // the last tile: quads straddling the end of pos[]/base[] were dummies
        int64_t* wp = (int64_t*)meta_pos(mring, i);
        float* wb = (float*)meta_base(mring, i);
        if (lane < kSub && e0 + lane < n) wp[lane] = pos[e0 + lane];
        if (lane < kSub * C && e0 * C + lane < n * C) wb[lane] = base[e0 * C + lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        wave_sync();
      }
      const int64_t* mp = meta_pos(mring, i);
      int64_t B[kSub];
#pragma unroll
      for (int e = 0; e < kSub; ++e) B[e] = e0 + e < n ? (mp[e] + 175) * G::FB : 0;
      if (batch_start)  // meta of batch i/kMetaT + 2
        dma_meta_batch<C>(safe_quad(raw, nbytes), pos, base, n, ntl, i / kMetaT + 2,
                          mring + ((i / kMetaT + 2) % kMetaR) * kMetaQ * 4, lane);
      uint32_t* wn = win[g];
      if (e0 + kSub <= n && !tile_late<CT>(B, nbytes)) {
        // fast path: per-lane quad offsets are loop invariants; padding lanes re-read the
        // epoch's first quad (no select, no bounds test)
#pragma unroll
        for (int m = 0; m < E::NI; ++m) {
          const int e = m / E::PER_E, j = m - e * E::PER_E;
          const uint8_t* eb = raw + (B[e] & ~(int64_t)15);
          if constexpr (!(EEGFX_FUSED_ABLATION & 8)) dma16(eb + qoff[j], wn + e * E::ESTR_E + 256 * j);
        }
      } else {
#pragma unroll
        for (int m = 0; m < E::NI; ++m) {
          const int e = m / E::PER_E, j = m - e * E::PER_E;
          const int i2 = 64 * j + lane;
          const int sg = i2 / G::SEGQ, q = i2 - sg * G::SEGQ;
          const int64_t A = (B[e] & ~(int64_t)15) + kSegLen * G::FB * sg + 16 * q;
          const bool okq = e0 + e < n && i2 < G::EPQ && A + 16 <= nbytes;
          if constexpr (!(EEGFX_FUSED_ABLATION & 8)) dma16(okq ? raw + A : safe_quad(raw, nbytes), wn + e * E::ESTR_E + 256 * j);
        }
      }
      if (pending) {  // the previous tile: exactly its successor's DMAs (+ one meta DMA) are newer
        if (batch_start) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(E::NI + 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(E::NI) : "memory");
        if (tile_late<CT>(pB, nbytes)) engine_fix<CT, C>(raw, nbytes, pB, pe0, n, win[pg], lane);
        publish_slot(&full[pg], (uint32_t)(pround + 1), win[pg] + E::SLOT_DW - 1);
      }
      pending = true;
      pg = g;
      pround = round;
      pe0 = e0;
#pragma unroll
      for (int e = 0; e < kSub; ++e) pB[e] = B[e];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (pending) {
      if (tile_late<CT>(pB, nbytes)) engine_fix<CT, C>(raw, nbytes, pB, pe0, n, win[pg], lane);
      publish_slot(&full[pg], (uint32_t)(pround + 1), win[pg] + E::SLOT_DW - 1);
    }
    return;
  }

  // ----------------------------------------------------------------------------------- consumer
  const int g = w / C, c = w - g * C;
  const int el = lane >> 3, s = lane & 7;
  const int col = sel.col[c];
  const float r = sel.res[c];
  for (int64_t i = g, round = 0; i < ntl; i += G_, ++round) {
    const int64_t e0 = (blockIdx.x + i * gridDim.x) * kSub;
    if (!spin_ge(&full[g], (uint32_t)(round + 1))) return;
    const int64_t* mp = meta_pos(mring, i);
    const int dl = e0 + el < n ? (int)(((mp[el] + 175) * G::FB) & 15) : 0;
    const uint8_t* eb = (const uint8_t*)(win[g] + el * E::ESTR_E) + dl + 2 * col;
    const int16_t* own = (const int16_t*)(eb + 16 * G::SEGQ * s);
    const int16_t* nxt = (const int16_t*)(eb + 16 * G::SEGQ * ((s + 1) & 7));
    int16_t xr[kIn];
#pragma unroll
    for (int k = 0; k < kSegLen; ++k) xr[k] = own[k * CT];
#pragma unroll
    for (int k = 0; k < 8; ++k) xr[kSegLen + k] = nxt[k * CT];
    const float b = meta_base(mring, i)[el * C + c];
    lds_inc(&freed[g]);  // DS ops of a wave complete in order: the reads above are done
    double a6, d6;
    if constexpr (EEGFX_FUSED_ABLATION & 16) {
      a6 = (double)xr[0] + b;
      d6 = (double)xr[kIn - 1];
    } else {
      double x[kIn];
      decode_pairs(xr, r, b, x);
      dwt8_cascade<FAST, true>(x, nullptr, lane & ~7, s, a6, d6);
    }
    double* fb = feat[g][round & 1];
    fb[el * F + c * 16 + s] = a6;
    fb[el * F + c * 16 + 8 + s] = d6;
    lds_st(&fdone[g][c], (uint32_t)(round + 1));
    if (!(EEGFX_FUSED_ABLATION & 32) && c == (int)(round % C)) {
      // per-wave progress words: a wave may already be one round ahead, so a shared counter
      // could be satisfied before this round's features are all written
      bool ok = true;
#pragma unroll
      for (int k = 0; k < C; ++k) ok = ok && spin_ge(&fdone[g][k], (uint32_t)(round + 1));
      if (!ok) return;
      normalise_store<F, FAST>(fb, norm[g], out + e0 * F, (n - e0) < kSub ? (int)(n - e0) : kSub, lane);
    }
  }
}
}  // namespace dev

// Baselines folded inside window_kernel (FUSEB, one launch per batch) instead of by the
// baseline_kernel pass before it.  EEGFX_FUSE_BASELINE=0/1 overrides the default.
bool fused_baseline_in_window() {
  static const bool v = [] {
    const char* e = getenv("EEGFX_FUSE_BASELINE");
    return e ? e[0] == '1' : false;
  }();
  return v;
}

// Non-temporal (streaming) reads when the average marker spacing n_frames / n leaves the regions
// a kernel reads (min_spacing frames per epoch) disjoint, so no other epoch would reuse the bytes
// through L2.  EEGFX_DMA_NT=0/1 overrides.
static bool streaming_reads(int64_t n_frames, int64_t n, int64_t min_spacing) {
  static const int env = [] {
    const char* e = getenv("EEGFX_DMA_NT");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  return env >= 0 ? env == 1 : (n > 0 && n_frames / n >= min_spacing);
}

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
  if (fused_baseline_in_window()) {
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, 4, 1, true, true>), dim3((unsigned)nsub),
                       dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel, pos, nullptr, n, out);
    return;
  }
  // Non-temporal window reads when the 512-frame windows of neighbouring markers do not overlap
  // (lds_dma.h has the measurements).
  const bool nt = streaming_reads(n_frames, n, dev::kWin + 8);
  if (nt && im.minw == 4 && im.k == 1 && im.shfl) {
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, 4, 1, true, false, true>),
                       dim3((unsigned)nsub), dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel,
                       pos, base, n, out);
    return;
  }
  const dim3 g((unsigned)((nsub + im.k - 1) / im.k));
  bool launched = false;
#define EEGFX_D(MW, KK, SH)                                                                     \
  if (!launched && im.minw == MW && im.k == KK && im.shfl == SH) {                                \
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, MW, KK, SH>), g, dim3(192), 0, st,          \
                       (const uint8_t*)raw, n_frames, sel, pos, base, n, out);                    \
    launched = true;                                                                              \
  }
  EEGFX_D(4, 1, true) EEGFX_D(5, 1, true) EEGFX_D(3, 1, true) EEGFX_D(2, 2, true) EEGFX_D(3, 2, true)
  EEGFX_D(4, 2, true) EEGFX_D(4, 4, true) EEGFX_D(4, 8, true) EEGFX_D(3, 4, true)
  EEGFX_D(3, 1, false) EEGFX_D(3, 2, false)
#undef EEGFX_D
  if (!launched)
    hipLaunchKernelGGL((dev::window_kernel<3, 3, FAST, 4, 1, true>), dim3((unsigned)nsub),
                       dim3(192), 0, st, (const uint8_t*)raw, n_frames, sel, pos, base, n, out);
}
}  // namespace

template <bool FAST, int G_, int L>
hipError_t launch_engine3(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                          const int64_t* pos, const float* base, int64_t n, double* out) {
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const int64_t ntiles = (n + dev::kSub - 1) / dev::kSub;
  const int64_t grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL((dev::engine_kernel<3, 3, FAST, G_, L>), dim3((unsigned)grid),
                     dim3(64 * (L + G_ * 3)), 0, st, (const uint8_t*)raw, n_frames, sel, pos, base,
                     n, out);
  return hipGetLastError();
}

// The loader/consumer engine is opt-in (EEGFX_ENGINE=1): parity-green, but slower than
// window_kernel on MI355X so far (DESIGN.md "Alternatives measured").
bool engine_enabled() {
  static const bool v = [] {
    const char* e = getenv("EEGFX_ENGINE");
    return e && e[0] == '1';
  }();
  return v;
}

// Persistent window kernel (EEGFX_WINDOW=p) vs the one-shot per-sub-tile one.
bool window_p_enabled() {
  static const bool v = [] {
    const char* e = getenv("EEGFX_WINDOW");
    return e && e[0] == 'p';
  }();
  return v;
}

bool fused_supported(int fmt, int ct, int C, const double* out) {
  return fmt == 0 && ct == 3 && C == 3 && ((uintptr_t)out & 15) == 0;
}

size_t fused_scratch_bytes(int64_t n, int C) { return sizeof(float) * (size_t)n * (size_t)C; }

int64_t fused_window_bytes_per_epoch(int ct, int C) {
  // window + (12 B of baselines | the 100 pre-stimulus frames when folded in the kernel) +
  // position + feature row
  const int64_t b = fused_baseline_in_window() ? (int64_t)dev::kPre * ct * 2 : (int64_t)C * 4;
  return (int64_t)dev::kWin * ct * 2 + b + 8 + (int64_t)C * 16 * 8;
}

hipError_t launch_fused_baseline(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 void* scratch) {
  if (ct != 3 || C != 3) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  // 64 epochs per workgroup; 16/32/128 measured the same or slower.  Streaming
  // reads unless another epoch's window or baseline may share the pre-stimulus frames.
  const dim3 g((unsigned)((n + 63) / 64));
  if (streaming_reads(n_frames, n, dev::kPre + 687))
    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 64, true>), g, dim3(192), 0, st,
                       (const uint8_t*)raw, n_frames, sel, pos, n, (float*)scratch);
  else
    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 64>), g, dim3(192), 0, st, (const uint8_t*)raw,
                       n_frames, sel, pos, n, (float*)scratch);
  return hipGetLastError();
}

hipError_t launch_fused_window(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n, bool fast,
                               const void* scratch, double* out) {
  if (ct != 3 || C != 3) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  const float* bs = (const float*)scratch;
  if (engine_enabled() && n_frames * ct * 2 >= 16) {
    const char* gv = getenv("EEGFX_ENGINE_G");
    const int gsel = gv ? atoi(gv) : 3;
    if (fast)
      return gsel == 4 ? launch_engine3<true, 4, 1>(st, raw, n_frames, sel, pos, bs, n, out)
                       : launch_engine3<true, 3, 1>(st, raw, n_frames, sel, pos, bs, n, out);
    return gsel == 4 ? launch_engine3<false, 4, 1>(st, raw, n_frames, sel, pos, bs, n, out)
                     : launch_engine3<false, 3, 1>(st, raw, n_frames, sel, pos, bs, n, out);
  }
  if (window_p_enabled()) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const int64_t nsub = (n + dev::kSub - 1) / dev::kSub;
    const char* wv = getenv("EEGFX_WINDOW_WG");  // workgroups per CU (default 5: LDS-bound)
    const int64_t per = wv ? atoi(wv) : 5;
    const int64_t grid = nsub < per * (int64_t)cus ? nsub : per * (int64_t)cus;
    const bool m3 = per <= 4;  // 4 WGs/CU fit 3 waves/SIMD: no spills at 168 VGPRs
#define EEGFX_P(FA, MW)                                                                          \
  hipLaunchKernelGGL((dev::window_p_kernel<3, 3, FA, MW>), dim3((unsigned)grid), dim3(192), 0, st, \
                     (const uint8_t*)raw, n_frames, sel, pos, bs, n, out)
    if (fast) { if (m3) EEGFX_P(true, 3); else EEGFX_P(true, 4); }
    else { if (m3) EEGFX_P(false, 3); else EEGFX_P(false, 4); }
#undef EEGFX_P
    return hipGetLastError();
  }
  if (fast) launch_window3<true>(st, raw, n_frames, sel, pos, (const float*)scratch, n, out);
  else launch_window3<false>(st, raw, n_frames, sel, pos, (const float*)scratch, n, out);
  return hipGetLastError();
}

}  // namespace eegfx
