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
//                   b[n][C] (12 B per epoch) and each epoch's window word (byte offset of the
//                   window + an out-of-range bit) for window_kernel.  It also validates every
//                   marker position (OffLineDataProvider.java:220-225: pos-100 in [0, n_frames]).
//
//  window_kernel    workgroup = C waves (wave c = channel c), sub-tile = 8 epochs x 8 lanes per
//                   signal (dwt8.h).  The 512-frame windows arrive by LDS-DMA
//                   (global_load_lds_dwordx4: 16-byte aligned per-lane sources, no VGPRs) into a
//                   per-epoch LDS layout whose strides keep every half-wave of ds_read_u16 on
//                   distinct banks; each lane folds the window's sub-16-byte misalignment into
//                   its read base.  Lanes decode (float)raw*res - b two samples at a time just in
//                   time inside level 1 and run the cascade (fma numerics: partial-sum halos,
//                   dwt8_fast_cascade; EXACT: value halos in the reference's order), and one wave
//                   normalises the 8 x 48 features (EXACT: sequential sum of squares,
//                   SignalProcessing.java:38-52) and stores them as contiguous wave stores.
//
// The alternatives measured against this pair (persistent, work-queue, two-sub-tile and
// loader/consumer variants, the baselines folded into the window kernel, the collapsed operator
// on the FP64 matrix cores, the register-direct window) are kept as patches under
// tools/probes/history/ with their numbers in
// DESIGN.md §6; none of them ships.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "dwt8.h"
#include "guard.h"
#include "launch.h"
#include "lds_dma.h"
#include "rows.h"

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
  // bytes a window DMA spans from floor16(B): 7 segments + the last segment's 25 quads
  static constexpr int64_t SPANB = (int64_t)kSegLen * FB * 7 + 16 * (SEGQ - 1) + 16;
};

// Window word of an epoch, written by baseline_kernel for window_kernel: the byte offset of its
// 512-frame window, B = (pos + 175) * FB (even), with bit 0 set when the DMA span from floor16(B)
// does not lie wholly inside the recording (the guarded path).  The window kernel then needs no
// 64-bit compares on its fast path (SALU has no 64-bit ordered compare on gfx950: every such
// test was a VALU instruction pair per epoch).

__device__ __forceinline__ void lds_store4(uint32_t* dst, const u32x4_a4& v) {
  dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
}

// One 16-byte quad at byte offset A (16-aligned; may lie outside the recording): the bytes of the
// recording it covers, zero elsewhere (Arrays.copyOfRange's zero padding).
__device__ __forceinline__ u32x4_a4 load16(const uint8_t* __restrict__ raw, int64_t nbytes,
                                           int64_t A) {
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
// lane reads a placeholder quad and discards it), so the compiler batches every load of a thread
// before the first wait; the rare quad that straddles the end of the recording is patched
// afterwards by load16.  NT: non-temporal read, for pre-stimulus frames no other epoch's window
// or baseline shares (baseline_kernel 0.136 -> 0.124 ms with markers 1,000 frames apart).
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

// Marker positions the reference cuts (OffLineDataProvider.java:220-225): copyOfRange(ch, pos-100,
// pos+750) throws unless 0 <= pos-100 <= len.  Device-resident positions are checked here, where
// the kernels read them anyway; a violation raises the context's error word (vector store to
// host-mapped memory), reported as EEGFX_ERANGE by the next eegfx_ctx_synchronize.  The kernels
// stay memory-safe for any position: an invalid one is replaced by kPre (a valid cut) before any
// address is formed from it, so no offset arithmetic can overflow, and every read is still
// bounds-tested or zero-filled.
__device__ __forceinline__ bool position_ok(int64_t p, int64_t n_frames) {
  return p >= kPre && p - kPre <= n_frames;
}
__device__ __forceinline__ int64_t safe_position(int64_t p, int64_t n_frames) {
  return position_ok(p, n_frames) ? p : kPre;
}
__device__ __forceinline__ void flag_position(int* err) {
  if (err) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int CT, int C, int TILE, bool STREAM = false>
__global__ __launch_bounds__((TILE * C + 63) / 64 * 64) void baseline_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    int64_t n, float* __restrict__ bout, int64_t* __restrict__ wout, int* __restrict__ err,
    int* __restrict__ guard_count, const unsigned long long* __restrict__ rechecked,
    unsigned long long* __restrict__ adapt, unsigned int* __restrict__ track_out) {
  using G = Geometry<CT>;
  constexpr int NT = (TILE * C + 63) / 64 * 64;
  __shared__ __attribute__((aligned(16))) uint32_t stage[TILE * G::BSTR];
  __shared__ int64_t tB[TILE];
  const int tid = threadIdx.x;
  const int64_t nbytes = n_frames * G::FB;
  const int64_t t0 = (int64_t)blockIdx.x * TILE;
  const int nt = (n - t0) < TILE ? (int)(n - t0) : TILE;
  // a window kernel that follows may append to the guard list (fma numerics)
  if (guard_count && blockIdx.x == 0 && tid == 0) *guard_count = 0;
  // the window kernel's guard strategy for this launch (guard.h guard_adapt_update)
  if (adapt && rechecked && blockIdx.x == 0 && tid < 64)
    guard_adapt_update(rechecked, adapt, track_out, n, tid);
  if (tid < TILE) {
    const int64_t p = tid < nt ? pos[t0 + tid] : kPre;
    if (!position_ok(p, n_frames)) flag_position(err);
    const int64_t sp = safe_position(p, n_frames);
    tB[tid] = (sp - kPre) * G::FB;
    if (tid < nt) {
      const int64_t B = (sp + 175) * G::FB;
      const int64_t Bq = B & ~(int64_t)15;
      wout[t0 + tid] = B | ((Bq >= 0 && Bq + G::SPANB <= nbytes) ? 0 : 1);
    }
  }
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
#pragma unroll 20
  for (int i = 0; i < kPre; ++i) b = b + (float)src[i * CT] * r;
  if (e < nt) bout[(t0 + e) * C + c] = b / (float)kPre;
}


// a3 + a6 + a7 fused into level 1 (dwt8.h level1_jit): (double)((float)raw * res - b), the
// multiply and the subtraction each one correctly rounded fp32 operation
// (DataProviderUtils.java:49-59, Baseline.java:39-41), two samples at a time with packed fp32
// math, read straight from the staged window: own[k*CT] for k < 64, then the 8 halo samples
// nxt[k*CT] of the next segment.
// FMA numerics: dwt8_fast_cascade (own samples only; partial-sum halos); EXACT: level1_exact
// (own samples; the 8 level-1 halo samples as decoded doubles from lane s+1) and value halos.
template <int CT, bool FAST, bool TRACK = false>
__device__ __forceinline__ void cascade_lds(const int16_t* own, const int16_t* nxt, float r,
                                            float b, int gbase, int s, double& a6, double& d6,
                                            float* ymax = nullptr) {
  if constexpr (FAST) {
#if EEGFX_COLLAPSED
    if constexpr (TRACK) {
      dwt8_collapsed_cascade<true>([&](int k) { return (float)own[k * CT]; }, r, b, gbase, s, a6,
                                   d6, ymax);
    } else if constexpr (EEGFX_LDS_B64 && CT == 3) {
      typedef uint64_t u64_a2 __attribute__((aligned(2)));
      dwt8_collapsed_cascade_b64([&](int k) { return *(const u64_a2*)(own + k * CT); }, r, b,
                                 gbase, s, a6, d6);
    } else {
      dwt8_collapsed_cascade([&](int k) { return (float)own[k * CT]; }, r, b, gbase, s, a6, d6);
    }
#else
    dwt8_fast_cascade([&](int k) { return (float)own[k * CT]; }, r, b, gbase, s, a6, d6);
#endif
  } else {
    double a1[40];
    (void)nxt;
    level1_exact([&](int k) { return (float)own[k * CT]; }, r, b, gbase, s, a1);
    halo<32, true>(a1, nullptr, gbase, s);
    dwt8_levels2to6<FAST, true>(a1, nullptr, gbase, s, a6, d6);
  }
}

// DMA rows of an epoch window: each row (one global_load_lds_dwordx4, lanes < SPR * SEGQ active)
// carries SPR whole segments, so the lane's source offset is the same for every row:
// lane l lands in segment SPR j + l / SEGQ, quad l % SEGQ, i.e. from byte
// 64 FB (SPR j + l / SEGQ) + 16 (l % SEGQ) = (64 FB SPR) j + 16 l - (16 SEGQ - 64 FB) (l / SEGQ)
// of floor16(B): a scalar row base plus one per-lane constant.
template <int CT>
struct DmaRows {
  using G = Geometry<CT>;
  static constexpr int SPR = 64 / G::SEGQ;                 // segments per row (2 for CT = 3)
  static constexpr int PER_E = (8 + SPR - 1) / SPR;        // rows per epoch window (4)
  static constexpr int LANES = SPR * G::SEGQ;              // active lanes per row (50)
  static constexpr int ROWB = kSegLen * G::FB * SPR;       // source bytes per row (768)
  static constexpr int ROWDW = G::SEGQ * SPR * 4;          // LDS dwords per row (200)
  static_assert(SPR >= 1 && 8 % SPR == 0, "whole segments per row");
  uint32_t off;
  bool active;
  __device__ __forceinline__ explicit DmaRows(int lane) {
    const int sg = lane / G::SEGQ;
    off = (uint32_t)(16 * lane - (16 * G::SEGQ - kSegLen * G::FB) * sg);
    active = lane < LANES;
  }
};

// Issues the LDS-DMA of one sub-tile's windows: wave w stages epochs w, w+C, w+2C, ... (every
// DMA row of each).  The window words of those epochs are loaded (scalar: e0 and e are
// wave-uniform, so these are lgkmcnt loads and every vector-memory counter slot stays with the
// DMAs) before the first DMA, so the DMAs leave back to back; an epoch whose window lies wholly
// inside the recording (bit 0 of its word clear) takes the unguarded path.  Returns whether some
// quad of this lane could not be DMA'd (the window reaches past either end of the recording).
template <int CT, int C, bool NT, int SUB = kSub>
__device__ __forceinline__ bool dma_issue(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const int64_t* __restrict__ wb, int64_t e0, int ne,
                                          uint32_t* win, int w, int lane, const DmaRows<CT>& rows) {
  using G = Geometry<CT>;
  constexpr int PER_E = DmaRows<CT>::PER_E;
  constexpr int NE = (SUB + C - 1) / C;
  int64_t W[NE];
#pragma unroll
  for (int t = 0; t < NE; ++t) {  // unconditional (clamped) loads: one scalar round trip
    const int e = w + t * C < SUB ? w + t * C : SUB - 1;
    W[t] = wb[e0 + (e < ne ? e : ne - 1)];
  }
  bool need_fix = false;
#pragma unroll
  for (int t = 0; t < NE; ++t) {
    const int e = w + t * C;
    if (e >= SUB || e >= ne) continue;  // uniform
    const int64_t Bq = W[t] & ~(int64_t)15;
    const uint8_t* sb = raw + Bq;
    uint32_t* dst = win + e * G::ESTR;
    if (((uint32_t)W[t] & 1u) == 0) {
      if (rows.active) {
#pragma unroll
        for (int j = 0; j < PER_E; ++j)
          dma16_s<NT>(sb + DmaRows<CT>::ROWB * j, rows.off, dst + DmaRows<CT>::ROWDW * j);
      }
    } else if (rows.active) {
#pragma unroll
      for (int j = 0; j < PER_E; ++j) {
        const int64_t A = Bq + DmaRows<CT>::ROWB * j + rows.off;
        if (A >= 0 && A + 16 <= nbytes)
          dma16_s<NT>(sb + DmaRows<CT>::ROWB * j, rows.off, dst + DmaRows<CT>::ROWDW * j);
        else need_fix = true;
      }
    }
  }
  return need_fix;
}

// Direct (non-DMA) fill of the quads dma_issue skipped (same wave -> epoch mapping): zero or
// partial quads at either end of the recording.
template <int CT, int C, int SUB = kSub>
__device__ __forceinline__ void dma_fixup(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const int64_t* __restrict__ wb, int64_t e0, int ne,
                                          uint32_t* win, int w, int lane, const DmaRows<CT>& rows) {
  using G = Geometry<CT>;
  constexpr int PER_E = DmaRows<CT>::PER_E;
  for (int e = w; e < SUB; e += C) {
    if (e >= ne) break;
    const int64_t Bq = wb[e0 + e] & ~(int64_t)15;
#pragma unroll
    for (int j = 0; j < PER_E; ++j) {
      const int64_t A = Bq + DmaRows<CT>::ROWB * j + rows.off;
      if (rows.active && (A < 0 || A + 16 > nbytes))
        lds_store4(win + e * G::ESTR + DmaRows<CT>::ROWDW * j + 4 * lane, load16(raw, nbytes, A));
    }
  }
}

// SUBS sub-tiles (8 epochs x C channels each) per workgroup of C * SUBS waves: wave w works on
// channel w % C of sub-tile w / C.  The windows land by LDS-DMA (NT: non-temporal, when
// neighbouring windows do not overlap); after the barrier that publishes them each lane decodes
// its 64 + 8 samples straight from LDS inside level 1, the cascade runs in registers with
// cross-lane halos (ds_bpermute), the a6/d6 rows overwrite the start of their sub-tile's window
// buffer once every wave has read its samples (26 KB of LDS per sub-tile: 6 sub-tiles, 18 waves
// per CU), and one wave per sub-tile normalises and stores its 8 rows.  Each sub-tile's LDS is
// laid out as a one-sub-tile workgroup's; the sub-tiles of a workgroup share only its barriers
// and its dispatch.
#ifndef EEGFX_WIN_SUBS
#define EEGFX_WIN_SUBS 1
#endif
// the guard's second stage in the 3-channel window kernel: every flagged row of a sub-tile in one
// pass (recheck_c3_rows), or (0, A/B builds) one row at a time (recheck_c3)
#ifndef EEGFX_RECHECK_ROWS
#define EEGFX_RECHECK_ROWS 1
#endif
// fma numerics: each channel wave normalises and stores its own 16 features of every row from
// registers (the row's sum of squares combined through LDS), and the guard's second stage runs on
// all channel waves against the windows still staged (window_rows_fast); 0 (A/B builds): the rows
// go through LDS and one wave normalises, guards and stores them (normalise_store)
#ifndef EEGFX_REG_ROWS
#define EEGFX_REG_ROWS 1
#endif
// Newton steps after v_rsq_f64 in the register-rows normalisation (1; 2 in A/B builds)
#ifndef EEGFX_RSQ_STEPS
#define EEGFX_RSQ_STEPS 1
#endif
// EEGFX_TRACK_X (guard.h): the guard's second-stage strategy of the fma window kernel.

// The guard's second stage for channel `col` of the flagged rows of a sub-tile, by one channel
// wave: the flagged rows (bit LPS e of `flagged` = epoch e, LPS lanes per signal)
// share the wave, L = 64, 32, 16, 8 or 4 lanes per row for 1, 2, 3-4, 5-8 or 9-16 rows; each lane
// reads 512 / L consecutive frames of its row's window as staged in LDS (segment s at 16 SEGQ s
// bytes past the epoch's misalignment) and keeps the column's min and max raw sample; those two
// are decoded exactly as the kernel decodes every sample (x = fl(fl(raw * r) - b) is monotone in
// raw), and X_c = max |x| is reduced over the row's lanes.  Returns X_c^2 on the lane sub == 0 of
// each row's slot (0 elsewhere) and the epoch of the lane's slot in *row (-1 for lanes without
// one).  delta, b: the misalignment and baseline of the lane's epoch (lane / LPS), shuffled to the
// slot's epoch.
template <int FB, int SEGQ, int EBYTES, int SUB = kSub, int LPS = 8>
__device__ __forceinline__ double channel_x2_rows(uint64_t flagged, const uint8_t* win, int col,
                                                  float r, float b, int delta, int lane,
                                                  int* row) {
  static_assert(SUB * LPS == 64 && SUB <= 16, "one wave per channel, 4-bit epoch slots");
  uint64_t T = 0;
  int k = 0;
#pragma unroll
  for (int e = 0; e < SUB; ++e)
    if ((flagged >> (LPS * e)) & 1ull) { T |= (uint64_t)e << (4 * k); ++k; }
  const int sh = k <= 1 ? 6 : k <= 2 ? 5 : k <= 4 ? 4 : k <= 8 ? 3 : 2;  // log2(L)
  const int j = lane >> sh, sub = lane & ((1 << sh) - 1);
  const bool valid = j < k;
  const int e = valid ? (int)((T >> (4 * j)) & 15u) : (int)(T & 15u);
  const int de = __shfl(delta, LPS * e, 64);
  const float be = __shfl(b, LPS * e, 64);
  const uint8_t* p0 = win + e * EBYTES + de + 2 * col;
  int mn = 32767, mx = -32768;
  // FPL = 512 / L frames per lane (a multiple of 8: runs never cross a segment), one fully unrolled
  // scan per row count so that every read of a lane is in flight before the first min / max
  auto scan = [&](auto fplc) {
    constexpr int FPL = decltype(fplc)::value;
    const int f0 = sub * FPL;
#pragma unroll
    for (int t = 0; t < FPL; t += 8) {
      const int f = f0 + t;
      const uint8_t* p = p0 + 16 * SEGQ * (f >> 6) + FB * (f & 63);
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const int v0 = *(const int16_t*)(p + FB * i), v1 = *(const int16_t*)(p + FB * (i + 1));
        mn = min(mn, min(v0, v1));
        mx = max(mx, max(v0, v1));
      }
    }
  };
  switch (sh) {  // uniform
    case 6: scan(std::integral_constant<int, 8>()); break;
    case 5: scan(std::integral_constant<int, 16>()); break;
    case 4: scan(std::integral_constant<int, 32>()); break;
    case 3: scan(std::integral_constant<int, 64>()); break;
    default: scan(std::integral_constant<int, 128>()); break;
  }
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  // (min, max) decoded as one pair: packed fp32 multiply and add, each lane rounded as the scalar
  // fl(fl(raw * r) - b)
  f32x2 x = f32x2{(float)mn, (float)mx} * f32x2{r, r};
  x = x + f32x2{-be, -be};
  // maximum over the row's L lanes (|x| >= 0: its bit pattern orders like the value)
  uint32_t u = __float_as_uint(fmaxf(fabsf(x.x), fabsf(x.y)));
  u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0xB1, 0xF, 0xF, true));
  u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x4E, 0xF, 0xF, true));
  if (sh >= 3) u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x141, 0xF, 0xF, true));
  if (sh >= 4) u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x140, 0xF, 0xF, true));
  if (sh >= 5) u = max(u, (uint32_t)__shfl_xor((int)u, 16, 64));
  if (sh >= 6) u = max(u, (uint32_t)__shfl_xor((int)u, 32, 64));
  const double X = (double)__uint_as_float(u);
  *row = valid && sub == 0 ? e : -1;
  return X * X;
}
template <int CT, int C, bool FAST, bool NT, int SUBS = EEGFX_WIN_SUBS, bool TRK = false>
__global__ __launch_bounds__(64 * C * SUBS, (5 + SUBS - 1) / SUBS) void window_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ wb,
    const float* __restrict__ base, int64_t n, double* __restrict__ out, Guard guard) {
  using G = Geometry<CT>;
  constexpr int F = C * 16;
  static_assert(kSub * F * 8 <= kSub * G::ESTR * 4, "feature rows alias the window buffer");
  __shared__ __attribute__((aligned(16))) uint32_t win_all[SUBS * kSub * G::ESTR];
  __shared__ double norm_all[SUBS * kSub];
  __shared__ double gx_all[FAST ? SUBS * kSub * C : 1];  // the guard's X^2 per signal (fma)
  // the REG guard paths synchronise the whole workgroup: one sub-tile only
  constexpr bool REG = FAST && EEGFX_REG_ROWS && SUBS == 1;
  __shared__ double part_all[REG ? SUBS * kSub * C : 1];  // per-signal sums of squares (REG)
  __shared__ double xs_all[REG ? SUBS * kSub * C : 1];    // measured X_c^2 of flagged rows (REG)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = SUBS > 1 ? wid / C : 0, w = SUBS > 1 ? wid - h * C : wid;  // sub-tile, channel
  uint32_t* win = win_all + h * kSub * G::ESTR;
  double* norm = norm_all + h * kSub;
  double* gx = gx_all + (FAST ? h * kSub * C : 0);
  const int el = lane >> 3, s = lane & 7;
  const int64_t nbytes = n_frames * G::FB;
  const int col = sel.col[w];
  const float r = sel.res[w];
  const int64_t e0 = ((int64_t)xcd_tile(blockIdx.x, gridDim.x) * SUBS + h) * kSub;
  const int64_t rest = n - e0;  // >= 1 for the first sub-tile; a later one may be empty
  const int ne = rest <= 0 ? 0 : (rest >> 31) != 0 ? kSub : ((int)rest < kSub ? (int)rest : kSub);

  const bool mine = el < ne;
  // This lane's baseline and window word: loaded unconditionally (clamped to a valid epoch) and
  // used only once the window DMAs are in flight, so the prologue waits on one round trip (the
  // window words' scalar loads) before the DMAs leave instead of three.
  const int64_t ec = SUBS > 1 && ne == 0 ? n - 1 : e0 + (mine ? el : ne - 1);
  const float b_ld = base[ec * C + w];
  const uint32_t w_ld = (uint32_t)wb[ec];
  const DmaRows<CT> rows(lane);
  if (SUBS == 1 || ne > 0) {  // wave-uniform
    if (dma_issue<CT, C, NT>(raw, nbytes, wb, e0, ne, win, w, lane, rows))
      dma_fixup<CT, C>(raw, nbytes, wb, e0, ne, win, w, lane, rows);
  }
  const float b = mine ? b_ld : 0.0f;
  const int delta = mine ? (int)(w_ld & 14u) : 0;
  if (FAST && EEGFX_GUARD && (lane & 7) == 0) gx[el * C + w] = guard_x2_int16(r, b);  // read after the barriers
  dma_drain();
  __syncthreads();

  // this lane's 64 samples + 8 halo samples of signal (epoch el, channel w), decoded in level 1
  double a6 = 0.0, d6 = 0.0;
  // TRK: this launch tracks max |x| (EEGFX_TRACK_X, guard.h) -- a variant of its own, so the
  // scanning launches carry no second filter loop
  constexpr bool TRACKABLE = REG && TRK && EEGFX_GUARD;
  constexpr bool track = TRACKABLE;  // (no flag is raised without guard.total either way)
  float ymax = 0.0f;
  if (SUBS == 1 || ne > 0) {
    const uint8_t* eb = (const uint8_t*)(win + el * G::ESTR) + delta + 2 * col;
    const int16_t* own = (const int16_t*)(eb + 16 * G::SEGQ * s);
    const int16_t* nxt = (const int16_t*)(eb + 16 * G::SEGQ * ((s + 1) & 7));
    cascade_lds<CT, FAST, TRACKABLE>(own, nxt, r, b, lane & ~7, s, a6, d6, &ymax);
  }

  if constexpr (REG) {
    // Each channel wave keeps its 16 features of each row in registers: the row's sum of squares
    // is the three channels' shares, combined through LDS in channel order (the same value in
    // every wave), and every wave normalises and stores its own part -- 8 lines of 128 B, a6 then
    // d6 of its channel -- so the staged windows stay intact for the guard's second stage, which
    // then runs on all channel waves at once.
    double* part = part_all + h * kSub * C;
    double* xs = xs_all + h * kSub * C;
    const double q = group8_sum(__builtin_fma(a6, a6, d6 * d6));
    if constexpr (track) {
      // the signal's measured X_c = max |x| over its 8 lanes (|x| >= 0 orders like its bits)
      uint32_t u = __float_as_uint(ymax);
      u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0xB1, 0xF, 0xF, true));
      u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x4E, 0xF, 0xF, true));
      u = max(u, (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x141, 0xF, 0xF, true));
      const double X = (double)__uint_as_float(u);
      if (s == 0) xs[el * C + w] = X * X;
    }
    if (s == 0) part[el * C + w] = q;
    __syncthreads();
    double acc = part[el * C];
#pragma unroll
    for (int c = 1; c < C; ++c) acc += part[el * C + c];
    bool fails = false;
    if (EEGFX_GUARD && guard.total && s == 0 && mine) {
      double sx = gx[el * C];
#pragma unroll
      for (int c = 1; c < C; ++c) sx += gx[el * C + c];
      fails = guard_fails(acc, kGuardK2Collapsed, sx);
    }
    const uint64_t flagged = __ballot(fails);  // bit 8e; the same mask in every channel wave
    uint64_t left = 0;
    if (track && flagged) {  // the measured X_c of every row is already in LDS
      bool f2 = false;
      if (s == 0 && ((flagged >> (8 * el)) & 1ull)) {
        double sx = xs[el * C];
#pragma unroll
        for (int c = 1; c < C; ++c) sx += xs[el * C + c];
        f2 = guard_fails(acc, kGuardK2Collapsed, sx * (1.0 + 0x1p-20));
      }
      left = __ballot(f2);
      if (w == 0 && lane == 0) {
        guard_count_rechecked(guard, __popcll(flagged));
        if (left) guard_count_recomputed(guard, (unsigned long long)__popcll(left));
      }
    } else if (flagged) {  // uniform over the workgroup, rare
      int row;
      const double x2 = channel_x2_rows<G::FB, G::SEGQ, G::ESTR * 4>(
          flagged, (const uint8_t*)win, col, r, b, delta, lane, &row);
      if (row >= 0) xs[row * C + w] = x2;
      __syncthreads();
      bool f2 = false;
      if (s == 0 && ((flagged >> (8 * el)) & 1ull)) {
        double sx = xs[el * C];
#pragma unroll
        for (int c = 1; c < C; ++c) sx += xs[el * C + c];
        f2 = guard_fails(acc, kGuardK2Collapsed, sx * (1.0 + 0x1p-20));
      }
      left = __ballot(f2);
      if (w == 0 && lane == 0) {
        guard_count_rechecked(guard, __popcll(flagged));
        if (left) guard_count_recomputed(guard, (unsigned long long)__popcll(left));
      }
    }
    const double inv = EEGFX_RSQ_STEPS == 1 ? rsqrt_nr1(acc) : rsqrt_nr(acc);
    if (mine && !((left >> (8 * el)) & 1ull)) {
      double* o = out + (e0 + el) * F + w * 16 + s;
      __builtin_nontemporal_store(a6 * inv, o);
      __builtin_nontemporal_store(d6 * inv, o + 8);
    }
    if (left) {  // uniform
      // the guard's rarest path: each such row recomputed under EXACT from the recording, channel
      // w by wave w (the staged windows as scratch, 768 doubles per wave: every wave is done with
      // them, the barrier above), then normalised and stored by wave 0
      double* scratch = (double*)win + w * 768;
      double* rowbuf = (double*)win + C * 768;
      for (uint64_t f = left; f; f &= f - 1) {
        const int e = (__ffsll((unsigned long long)f) - 1) >> 3;
        const int64_t B = wb[e0 + e] & ~(int64_t)1;  // byte offset of the window
        const int64_t f0 = B / G::FB;
        dwt8_exact_channel_wave(
            [&](int k) {
              const float bc = base[(e0 + e) * C + w];
              const float v = f0 + k < n_frames
                                  ? (float)*(const int16_t*)(raw + B + (int64_t)k * G::FB + 2 * col)
                                  : 0.0f;
              float y = v * r;
              y = y - bc;
              return (double)y;
            },
            16, scratch, rowbuf + w * 16, lane);
        __syncthreads();
        if (w == 0) {
          dwt8_normalise_row_wave(rowbuf, F, scratch, lane);
          for (int i = lane; i < F; i += 64) out[(e0 + e) * F + i] = rowbuf[i];
        }
        __syncthreads();
      }
    }
    return;
  }
  double* fb = (double*)win;
  __syncthreads();  // every wave has read its samples: the rows may overwrite the window
  // the row slot is recomputed here from an opaque copy of the lane id, so its address is not
  // kept live across the filter bank (it was the one spilled VGPR)
  int l2 = lane;
  asm volatile("" : "+v"(l2));
  const int slot = (l2 >> 3) * F + w * 16 + (l2 & 7);
  fb[slot] = a6;
  fb[slot + 8] = d6;
  __syncthreads();
  if (w == 0 && (SUBS == 1 || ne > 0)) {
    // the guard's rare path: the row recomputed under EXACT from the recording by this wave, with
    // the LDS past the 8 feature rows of its sub-tile as scratch (every other wave is done with
    // this sub-tile's window)
    auto redo = [&](int e, double* row) {
      const int64_t B = wb[e0 + e] & ~(int64_t)1;  // byte offset of the window (frame pos + 175)
      const int64_t f0 = B / G::FB;
      dwt8_exact_row_wave(
          [&](int c, int k) {
            const float rc = sel.res[c], bc = base[(e0 + e) * C + c];
            const float v = f0 + k < n_frames
                                ? (float)*(const int16_t*)(raw + B + (int64_t)k * G::FB + 2 * sel.col[c])
                                : 0.0f;
            float y = v * rc;
            y = y - bc;
            return (double)y;
          },
          C, 16, fb + kSub * F, row, lane);
    };
    // the guard's second stage: the rows' measured max |x|, from the staged windows (epochs
    // 1-7, recheck_c3_rows: every flagged row of the sub-tile in one pass; epoch 0's window lies
    // under the rows: from the recording, recheck_c3)
#if EEGFX_RECHECK_ROWS
    auto recheck = [&](uint64_t flagged, double acc) {
      return recheck_c3_rows<G::SEGQ, G::ESTR * 4>(
          flagged, acc, sel, base + e0 * C, (const uint8_t*)win, delta, lane, [&] {
            return recheck_c3<G::FB, G::SEGQ>(raw, n_frames, sel, wb[e0], base + e0 * C,
                                              nullptr, true, lane);
          });
    };
    normalise_store<F, FAST, C>(fb, norm, out + e0 * F, ne, lane, gx, guard, redo, recheck);
#else
    auto recheck = [&](int e) {
      return recheck_c3<G::FB, G::SEGQ>(raw, n_frames, sel, wb[e0 + e], base + (e0 + e) * C,
                            (const uint8_t*)(win + e * G::ESTR), e == 0, lane);
    };
    normalise_store<F, FAST, C>(fb, norm, out + e0 * F, ne, lane, gx, guard, redo,
                                per_row_recheck(recheck));
#endif
  }
}

// fma numerics, 3-channel int16 recordings, A/B builds (-DEEGFX_WIN4=1): the six-point form with
// 4 lanes per signal (dwt8.h dwt8_toom6_core).  A channel wave holds 16 epochs and a workgroup
// (3 waves, wave w = channel w) a 16-epoch sub-tile: 51 KB of staged windows in window_kernel's
// per-epoch layout, three workgroups per CU.  Each lane reads its 128 samples (two segments)
// straight from LDS; the rows are normalised and stored from registers by every channel wave
// (a6[2 s], a6[2 s + 1], d6[2 s], d6[2 s + 1] of its channel: two 16-byte stores per lane), and the
// guard's second stage scans the staged windows on all channel waves.  8.9 % fewer VALU
// instructions than window_kernel (SQ_INSTS_VALU) but 2.5 % slower per step: with half the waves
// per CU the window DMA is no longer covered by other workgroups' work (the kernel without its DMA
// runs in 0.56 ms); persistent forms that overlap the next sub-tile's DMA themselves measured
// slower still (DESIGN_LOG.md §R6).
#ifndef EEGFX_WIN4
#define EEGFX_WIN4 0
#endif
constexpr int kSub4 = 16;  // epochs per sub-tile of window4_kernel (16 epochs x 4 lanes = 64 lanes)

template <bool NT>
__global__ __launch_bounds__(192, 3) void window4_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ wb,
    const float* __restrict__ base, int64_t n, double* __restrict__ out, Guard guard) {
  using G = Geometry<3>;
  constexpr int C = 3, F = C * 16, SUB = kSub4, LPS = kLanesPerSignal4;
  static_assert(SUB * LPS == 64, "one wave per channel");
  __shared__ __attribute__((aligned(16))) uint32_t win[SUB * G::ESTR];
  __shared__ double gx[SUB * C];    // the guard's a-priori X^2 per signal
  __shared__ double part[SUB * C];  // per-signal sums of squares
  __shared__ double xs[SUB * C];    // measured X_c^2 of flagged rows
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // channel
  const int el = lane >> 2, s = lane & 3;
  const int64_t nbytes = n_frames * G::FB;
  const int col = sel.col[w];
  const float r = sel.res[w];
  const int64_t e0 = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * SUB;
  const int64_t rest = n - e0;  // >= 1
  const int ne = rest >= SUB ? SUB : (int)rest;
  const bool mine = el < ne;
  const int64_t ec = e0 + (mine ? el : ne - 1);
  const float b_ld = base[ec * C + w];
  const uint32_t w_ld = (uint32_t)wb[ec];
  const DmaRows<3> rows(lane);
  if (dma_issue<3, C, NT, SUB>(raw, nbytes, wb, e0, ne, win, w, lane, rows))
    dma_fixup<3, C, SUB>(raw, nbytes, wb, e0, ne, win, w, lane, rows);
  const float b = mine ? b_ld : 0.0f;
  const int delta = mine ? (int)(w_ld & 14u) : 0;
  if (EEGFX_GUARD && s == 0) gx[el * C + w] = guard_x2_int16(r, b);  // read after the barriers
  dma_drain();
  __syncthreads();

  // samples 128 s + k of signal (epoch el, channel w): segment 2 s + k / 64, frame k % 64
  const uint8_t* own = (const uint8_t*)(win + el * G::ESTR) + delta + 2 * col + 32 * G::SEGQ * s;
  double a6[2], d6[2];
  dwt8_toom6_cascade(
      [&](int k) { return (int)*(const int16_t*)(own + 16 * G::SEGQ * (k >> 6) + G::FB * (k & 63)); },
      r, b, lane & ~(LPS - 1), s, a6, d6);

  const double q = group4_sum(__builtin_fma(
      a6[0], a6[0], __builtin_fma(a6[1], a6[1], __builtin_fma(d6[0], d6[0], d6[1] * d6[1]))));
  if (s == 0) part[el * C + w] = q;
  __syncthreads();
  const double acc = (part[el * C] + part[el * C + 1]) + part[el * C + 2];
  bool fails = false;
  if (EEGFX_GUARD && guard.total && s == 0 && mine)
    fails = guard_fails(acc, kGuardK2Toom6, (gx[el * C] + gx[el * C + 1]) + gx[el * C + 2]);
  const uint64_t flagged = __ballot(fails);  // bit 4e; the same mask in every channel wave
  uint64_t left = 0;
  if (flagged) {  // uniform over the workgroup, rare
    int row;
    const double x2 = channel_x2_rows<G::FB, G::SEGQ, G::ESTR * 4, SUB, LPS>(
        flagged, (const uint8_t*)win, col, r, b, delta, lane, &row);
    if (row >= 0) xs[row * C + w] = x2;
    __syncthreads();
    bool f2 = false;
    if (s == 0 && ((flagged >> (LPS * el)) & 1ull))
      f2 = guard_fails(acc, kGuardK2Toom6,
                       ((xs[el * C] + xs[el * C + 1]) + xs[el * C + 2]) * (1.0 + 0x1p-20));
    left = __ballot(f2);
    if (w == 0 && lane == 0) {
      guard_count_rechecked(guard, __popcll(flagged));
      if (left) guard_count_recomputed(guard, (unsigned long long)__popcll(left));
    }
  }
  const double inv = rsqrt_nr1(acc);
  if (mine && !((left >> (LPS * el)) & 1ull)) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    f64x2* o = (f64x2*)(out + (e0 + el) * F + w * 16 + 2 * s);
    __builtin_nontemporal_store(f64x2{a6[0] * inv, a6[1] * inv}, o);
    __builtin_nontemporal_store(f64x2{d6[0] * inv, d6[1] * inv}, o + 4);
  }
  if (left && w == 0) {
    // the guard's rare path: each such row recomputed under EXACT from the recording by wave 0,
    // the staged windows as scratch (every wave is done with them: the barrier above)
    double* scratch = (double*)win;
    double* rowbuf = scratch + 768;
    for (uint64_t f = left; f; f &= f - 1) {
      const int e = (__ffsll((unsigned long long)f) - 1) / LPS;
      const int64_t B = wb[e0 + e] & ~(int64_t)1;  // byte offset of the window
      const int64_t f0 = B / G::FB;
      dwt8_exact_row_wave(
          [&](int c, int k) {
            const float rc = sel.res[c], bc = base[(e0 + e) * C + c];
            const float v = f0 + k < n_frames
                                ? (float)*(const int16_t*)(raw + B + (int64_t)k * G::FB + 2 * sel.col[c])
                                : 0.0f;
            float y = v * rc;
            y = y - bc;
            return (double)y;
          },
          C, 16, scratch, rowbuf, lane);
      for (int i = lane; i < F; i += 64) out[(e0 + e) * F + i] = rowbuf[i];
      wave_sync();
    }
  }
}

}  // namespace dev

// Non-temporal (streaming) reads when the average marker spacing n_frames / n leaves the regions
// a kernel reads (min_spacing frames per epoch) disjoint, so no other epoch would reuse the bytes
// through L2 (markers 1,000 frames apart: window_kernel 0.918 -> 0.910 ms; 100 frames apart, where
// each frame sits in ~6 windows: 0.777 -> 0.802 ms -- hence the test).
bool streaming_reads(int64_t n_frames, int64_t n, int64_t min_spacing) {
  return n > 0 && n_frames / n >= min_spacing;
}

bool fused_supported(int fmt, int ct, int C, const double* out) {
  return fmt == 0 && ct == 3 && C == 3 && ((uintptr_t)out & 15) == 0;
}

// Scratch of the fused path: [n][C] float baselines, then (16-byte aligned) the n int64 window
// words of baseline_kernel.
static size_t window_words_offset(int64_t n, int C) {
  return (sizeof(float) * (size_t)n * (size_t)C + 15) & ~(size_t)15;
}
size_t fused_scratch_bytes(int64_t n, int C) {
  return window_words_offset(n, C) + sizeof(int64_t) * (size_t)n;
}

int64_t fused_window_bytes_per_epoch(int ct, int C) {
  // window + 12 B of baselines + position + feature row
  return (int64_t)dev::kWin * ct * 2 + (int64_t)C * 4 + 8 + (int64_t)C * 16 * 8;
}

hipError_t launch_fused_baseline(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 void* scratch, int* err, int* guard_count, const Guard* guard) {
  const unsigned long long* rechecked = guard ? guard->rechecked : nullptr;
  unsigned long long* adapt = guard && guard->total ? guard->adapt : nullptr;
  unsigned int* track_out = adapt ? guard->track_out : nullptr;
  if (ct != 3 || C != 3) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  // 64 epochs per workgroup; 16/32/128 measured the same or slower.  Streaming
  // reads unless another epoch's window or baseline may share the pre-stimulus frames.
  const dim3 g((unsigned)((n + 63) / 64));
  int64_t* words = (int64_t*)((uint8_t*)scratch + window_words_offset(n, C));
  if (streaming_reads(n_frames, n, dev::kPre + 687))
    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 64, true>), g, dim3(192), 0, st,
                       (const uint8_t*)raw, n_frames, sel, pos, n, (float*)scratch, words, err,
                       guard_count, rechecked, adapt, track_out);
  else
    hipLaunchKernelGGL((dev::baseline_kernel<3, 3, 64>), g, dim3(192), 0, st, (const uint8_t*)raw,
                       n_frames, sel, pos, n, (float*)scratch, words, err, guard_count, rechecked,
                       adapt, track_out);
  return hipGetLastError();
}

hipError_t launch_fused_window(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n, bool fast,
                               const void* scratch, double* out, const Guard& guard, bool track) {
  if (ct != 3 || C != 3) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  const float* bs = (const float*)scratch;
  const int64_t* words = (const int64_t*)((const uint8_t*)scratch + window_words_offset(n, C));
  (void)pos;  // read by launch_fused_baseline, which wrote the window words
  const bool nt = streaming_reads(n_frames, n, dev::kWin + 8);
  if (fast && EEGFX_WIN4) {
    const dim3 g4((unsigned)((n + dev::kSub4 - 1) / dev::kSub4));
    if (nt)
      hipLaunchKernelGGL((dev::window4_kernel<true>), g4, dim3(192), 0, st, (const uint8_t*)raw,
                         n_frames, sel, words, bs, n, out, guard);
    else
      hipLaunchKernelGGL((dev::window4_kernel<false>), g4, dim3(192), 0, st, (const uint8_t*)raw,
                         n_frames, sel, words, bs, n, out, guard);
    return hipGetLastError();
  }
  constexpr int subs = EEGFX_WIN_SUBS;
  const dim3 g((unsigned)((n + dev::kSub * subs - 1) / (dev::kSub * subs)));
#define EEGFX_WIN(FA, NTV, TK)                                                               \
  hipLaunchKernelGGL((dev::window_kernel<3, 3, FA, NTV, subs, TK>), g, dim3(192 * subs), 0, st, \
                     (const uint8_t*)raw, n_frames, sel, words, bs, n, out, guard)
  const bool trk = EEGFX_TRACK_X != 0 && (EEGFX_TRACK_X == 2 || track) && guard.total;
  if (fast && trk) { if (nt) EEGFX_WIN(true, true, true); else EEGFX_WIN(true, false, true); }
  else if (fast) { if (nt) EEGFX_WIN(true, true, false); else EEGFX_WIN(true, false, false); }
  else { if (nt) EEGFX_WIN(false, true, false); else EEGFX_WIN(false, false, false); }
#undef EEGFX_WIN
  return hipGetLastError();
}

}  // namespace eegfx
