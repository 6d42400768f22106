// mfma.hip -- the dwt-8 window as a collapsed 16x512 linear operator on the FP64 matrix cores.
//
// Reference: WaveletTransform.java:126-137 keeps the first 16 coefficients (a6 ++ d6) of the
// eegdsp 1.0 periodic db5 pyramid of x = epoch[c][175..686].  The pyramid
// is linear in x, so those 16 coefficients are M x for a fixed 16 x 512 matrix M (dwt8_operator.cpp
// builds it once per context).  This kernel evaluates M X for X = [512 samples x 16 epochs] with
// v_mfma_f64_16x16x4_f64 (8,192 fp64 MAC per signal against the cascade's 5,120, on the matrix
// pipe, which measured 77 TF/s fp64 against 56 TF/s for VALU v_fma_f64 on MI355X --
// tools/probes/fp64_probe.hip) and leaves the VALU free for the a3/a6/a7 decode
// (double)((float)raw * res - b), which it performs per sample between the MFMAs.
// Numerics: fp64 products and sums in a different order than the reference -> the FMA contract
// (<= 1e-9 of the reference per normalised feature); EXACT stays on the cascade.
//
// Engine (one workgroup of 4 waves per CU, every wave independent -- no workgroup barrier):
//   * M is block-circulant (shifting the window by 64 samples shifts a6/d6 by one), so rows a6[0]
//     and d6[0] define it: the workgroup keeps them (each stored twice, to unroll the periodic
//     wrap) as a 16 KB LDS table; the A fragment of K-step t, lane l is
//     M[l&15][4t + (l>>4)] = T[(l>>3)&1][4t + (l>>4) - 64 (l&7) + 512], one ds_read_b64.
//   * A tile is 16 consecutive epochs (MFMA N = epoch n = l&15) x C channels (C accumulators).
//     Its 512-frame windows stream through a wave-private LDS ring of 4 slots, one 64-frame chunk
//     (16 epochs x 25 aligned quads) per slot, fetched by LDS-DMA (global_load_lds_dwordx4) three
//     chunks ahead -- across tile boundaries -- so every wave keeps ~20 KB of HBM reads in flight
//     while its MFMAs run.  Marker positions and baselines of the next tile are DMA'd into a
//     per-wave meta block the same way.  All DMA is issued through inline asm and drained with
//     counted `s_waitcnt vmcnt(N)`; the compiler's own vector-memory ops in the loop are stores and
//     the rare end-of-recording fixup loads, which can only make those waits conservative.
//   * Epilogue per tile: the 4 lanes holding an epoch's 48 coefficients reduce the sum of squares
//     (SignalProcessing.java:38-52), divide and store.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dwt8.h"
#include "launch.h"

// Perf-study builds only (tools/probes/mfma_probe.hip): bit 0 drops the DMA waits, bit 1 the
// decode (B operand = a constant); the library is always built with 0.
#ifndef EEGFX_MFMA_ABLATION
#define EEGFX_MFMA_ABLATION 0
#endif

namespace eegfx {
namespace dev {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a16 __attribute__((ext_vector_type(4), aligned(16)));

constexpr int kTileE = 16;           // epochs per tile (MFMA N)
constexpr int kChunkF = 64;          // window frames per DMA chunk
constexpr int kChunks = kWin / kChunkF;  // 8
constexpr int kRing = 4;             // LDS ring slots per wave
constexpr int kAhead = 3;            // chunks in flight ahead of the one being consumed
constexpr int kWaves = 4;            // waves per workgroup (one per SIMD)
constexpr int kMetaB = 1024;         // one meta block: a whole DMA instruction (pos[16] + base[16][C])

template <int CT>
struct MGeo {
  static constexpr int FB = 2 * CT;                  // bytes per frame
  static constexpr int CHB = kChunkF * FB;           // bytes of one epoch's chunk (16-B multiple)
  static constexpr int EQ = CHB / 16 + 1;            // quads per epoch chunk (+1: misalignment)
  static constexpr int QUADS = kTileE * EQ;          // quads per slot
  static constexpr int NI = (QUADS + 63) / 64;       // DMA instructions per chunk
  static constexpr int SLOT = NI * 64 * 16;          // bytes per slot (tail = DMA padding)
  static constexpr int WAVE_LDS = kRing * SLOT + 2 * kMetaB;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(lds_ptr_t)p;
}

// One LDS-DMA wave instruction: lane l's 16 bytes at `src` land at LDS byte lds + 16*l.
__device__ __forceinline__ void dma16(const uint8_t* src, uint32_t lds) {
  uint32_t saved;
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

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  if constexpr ((EEGFX_MFMA_ABLATION & 1) && N > 0) return;
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Per-tile addressing state of one lane.
struct TileAddr {
  int64_t src[8];   // byte offset of the first quad of DMA instruction i (chunk 0), or -1
  int32_t dlt;      // byte misalignment of this lane's epoch window (even, 0..14)
};

// Meta DMA: pos[e0 .. e0+16) (8 quads) then base[e0*C .. (e0+16)*C) (C*4 quads) into meta.
// Lanes past the arrays read `raw` = the recording's safe_quad (value discarded).
template <int C>
__device__ __forceinline__ void dma_meta(const uint8_t* __restrict__ raw, const int64_t* __restrict__ pos,
                                         const float* __restrict__ base, int64_t n, int64_t e0,
                                         uint32_t meta, int lane) {
  const uint8_t* src;
  if (lane < 8) {
    const int64_t i = e0 + 2 * lane;  // quad = 2 positions
    src = i + 1 < n ? (const uint8_t*)(pos + i) : raw;  // raw: the caller's safe_quad
  } else if (lane < 8 + 4 * C) {
    const int64_t f = e0 * C + 4 * (lane - 8);  // quad = 4 floats
    src = f + 3 < n * C ? (const uint8_t*)(base + f) : raw;
  } else {
    src = raw;
  }
  dma16(src, meta);
}

// Positions and baselines that straddle the end of pos[]/base[] (n not a multiple of 2 or 4):
// the DMA above read a dummy quad for them; patch the few valid values after the DMA landed.
template <int C>
__device__ __forceinline__ void meta_fixup(const int64_t* __restrict__ pos,
                                           const float* __restrict__ base, int64_t n, int64_t e0,
                                           uint8_t* meta, int lane) {
  if (e0 + kTileE <= n) return;  // uniform: only the last tile can straddle
  if (lane < kTileE && e0 + lane < n) ((int64_t*)meta)[lane] = pos[e0 + lane];
  for (int i = lane; i < kTileE * C; i += 64)
    if (e0 * C + i < n * C) ((float*)(meta + 128))[i] = base[e0 * C + i];
}

template <int CT>
__device__ __forceinline__ void tile_addr(const uint8_t* meta, int64_t e0, int64_t n,
                                          int64_t n_frames, int lane, TileAddr& ta) {
  using G = MGeo<CT>;
  const int64_t* mpos = (const int64_t*)meta;
#pragma unroll
  for (int i = 0; i < G::NI; ++i) {
    const int qd = 64 * i + lane;
    const int m = qd / G::EQ, r = qd - m * G::EQ;
    if (qd < G::QUADS && e0 + m < n) {
      const int64_t B = (mpos[m] + 175) * G::FB;
      ta.src[i] = (B & ~(int64_t)15) + 16 * r;
    } else {
      ta.src[i] = -1;
    }
  }
  const int nn = lane & 15;
  ta.dlt = e0 + nn < n ? (int)(((mpos[nn] + 175) * G::FB) & 15) : 0;
  (void)n_frames;
}

// Issues chunk j of a tile into LDS slot `slot`; returns whether some lane's quad lies (partly)
// past the recording end or belongs to no epoch (those lanes DMA a dummy quad; see fixup).
template <int CT>
__device__ __forceinline__ bool dma_chunk(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const TileAddr& ta, int j, uint32_t slot) {
  using G = MGeo<CT>;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < G::NI; ++i) {
    const int64_t a = ta.src[i] < 0 ? -1 : ta.src[i] + (int64_t)G::CHB * j;
    const bool ok = a >= 0 && a + 16 <= nbytes;
    bad |= a >= 0 && !ok;
    dma16(ok ? raw + a : safe_quad(raw, nbytes), slot + 1024 * i);
  }
  return bad;
}

// Rewrites the quads of chunk j that dma_chunk could not fetch: zero past the recording end
// (Arrays.copyOfRange zero-pads, OffLineDataProvider.java:220-225), partial at the boundary.
template <int CT>
__device__ __attribute__((noinline)) void fix_chunk(const uint8_t* __restrict__ raw, int64_t nbytes,
                                          const TileAddr& ta, int j, uint8_t* slot) {
  using G = MGeo<CT>;
#pragma unroll
  for (int i = 0; i < G::NI; ++i) {
    const int64_t a = ta.src[i] < 0 ? -1 : ta.src[i] + (int64_t)G::CHB * j;
    if (a >= 0 && a + 16 > nbytes) {
      uint32_t t[4] = {0u, 0u, 0u, 0u};
      for (int k = 0; k < 4; ++k) {
        const int64_t b = a + 4 * k;
        if (b + 4 <= nbytes) t[k] = *(const uint32_t*)(raw + b);
        else if (b + 2 <= nbytes) t[k] = *(const uint16_t*)(raw + b);
      }
      uint32_t* d = (uint32_t*)(slot + 1024 * i + 16 * (threadIdx.x & 63));
      d[0] = t[0]; d[1] = t[1]; d[2] = t[2]; d[3] = t[3];
    }
  }
}

// The 16 K-steps of chunk j: lane (n, q) decodes frame 64j + 4t' + q of epoch n, channel c, and
// feeds it as the B operand; acc[c][t&1] alternate so consecutive MFMAs are independent.
template <int CT, int C>
__device__ __forceinline__ void mfma_chunk(const uint8_t* slot, const double* arow,
                                           const int32_t (&boff)[C], const float (&res)[C],
                                           const float (&b)[C], d4 (&acc)[C][2]) {
  using G = MGeo<CT>;
#pragma unroll
  for (int tt = 0; tt < kChunkF / 4; ++tt) {
    const double a = arow[4 * tt];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double x;
      if constexpr (EEGFX_MFMA_ABLATION & 2) {
        x = (double)b[c] + tt;
      } else {
        const int16_t r16 = *(const int16_t*)(slot + boff[c] + 4 * G::FB * tt);
        const float v = (float)r16 * res[c];
        x = (double)(v - b[c]);
      }
      acc[c][tt & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, x, acc[c][tt & 1], 0, 0, 0);
    }
  }
}

template <int CT, int C>
__global__ __launch_bounds__(64 * kWaves, 1) void mfma_window_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ pos,
    const float* __restrict__ base, int64_t n, const double* __restrict__ mrows,
    double* __restrict__ out) {
  using G = MGeo<CT>;
  static_assert(8 + 4 * C <= 64, "meta DMA: one instruction");
  static_assert(G::NI <= 8, "TileAddr holds 8 DMA instructions");
  constexpr int F = 16 * C;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[kWaves * G::WAVE_LDS];
  __shared__ __attribute__((aligned(16))) double mtab[2][2 * kWin];
  for (int i = threadIdx.x; i < 2 * 2 * kWin; i += blockDim.x)
    mtab[i / (2 * kWin)][i % (2 * kWin)] = mrows[(i / (2 * kWin)) * kWin + (i % kWin)];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nn = lane & 15, q = lane >> 4;
  uint8_t* ring = lds + w * G::WAVE_LDS;
  uint8_t* meta0 = ring + kRing * G::SLOT;
  const uint32_t ring_a = lds_addr(ring), meta_a = lds_addr(meta0);
  const int64_t nbytes = n_frames * G::FB;
  const int64_t ntiles = (n + kTileE - 1) / kTileE;
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  int64_t tile = (int64_t)blockIdx.x * kWaves + w;
  if (tile >= ntiles) return;  // uniform per wave; nothing issued yet

  // this lane's A-fragment column: M[r][k] = T[r >> 3][k - 64 (r & 7) + 512], k = 4t + q
  const double* arow0 = &mtab[(nn >> 3) & 1][q - 64 * (nn & 7) + kWin];
  float res[C];
  int32_t col2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    res[c] = sel.res[c];
    col2[c] = 2 * sel.col[c];
  }

  // prologue: meta of the first tile, then its first kAhead chunks
  int mb = 0;
  dma_meta<C>(safe_quad(raw, nbytes), pos, base, n, tile * kTileE, meta_a, lane);
  wait_vm<0>();
  meta_fixup<C>(pos, base, n, tile * kTileE, meta0, lane);
  TileAddr cur, nxt;
  tile_addr<CT>(meta0, tile * kTileE, n, n_frames, lane, cur);
  uint32_t fix = 0, fix_next = 0;  // bit j: chunk j of the current / next tile needs a fixup
#pragma unroll
  for (int j = 0; j < kAhead; ++j)
    fix |= (__builtin_amdgcn_ballot_w64(dma_chunk<CT>(raw, nbytes, cur, j, ring_a + j * G::SLOT)) != 0) << j;

  while (true) {
    const int64_t e0 = tile * kTileE;
    const int64_t next = tile + nwaves;
    const bool has_next = next < ntiles;
    // where the chunks fetched ahead for "the next tile" come from on the last tile: the current
    // tile again (valid addresses, results unused) -- keeps the vmcnt bookkeeping uniform
    const int64_t e0n = has_next ? next * kTileE : e0;
    uint8_t* meta_cur = meta0 + mb * kMetaB;
    uint8_t* meta_nxt = meta0 + (mb ^ 1) * kMetaB;
    float b[C];
    int32_t boff[C];
    {
      const float* mbase = (const float*)(meta_cur + 128);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        b[c] = mbase[nn * C + c];
        boff[c] = nn * G::EQ * 16 + cur.dlt + q * G::FB + col2[c];
      }
    }
    d4 acc[C][2];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c][0] = acc[c][1] = (d4){0.0, 0.0, 0.0, 0.0};

    for (int j = 0; j < kChunks; ++j) {  // uniform
      // outstanding after chunk j's DMAs: chunks j+1, j+2 (+ the meta DMA issued at step 2)
      if (j == 3 || j == 4) wait_vm<2 * G::NI + 1>();
      else wait_vm<2 * G::NI>();
      uint8_t* slot = ring + (j % kRing) * G::SLOT;
      if (fix & (1u << j)) fix_chunk<CT>(raw, nbytes, cur, j, slot);
      if (j == 2) dma_meta<C>(safe_quad(raw, nbytes), pos, base, n, e0n, meta_a + (mb ^ 1) * kMetaB, lane);
      if (j == 5) {
        meta_fixup<C>(pos, base, n, e0n, meta_nxt, lane);
        tile_addr<CT>(meta_nxt, e0n, n, n_frames, lane, nxt);
      }
      const int ja = j + kAhead;
      const uint32_t dst = ring_a + (ja % kRing) * G::SLOT;
      if (ja < kChunks) {
        fix |= (__builtin_amdgcn_ballot_w64(dma_chunk<CT>(raw, nbytes, cur, ja, dst)) != 0) << ja;
      } else {
        fix_next |= (__builtin_amdgcn_ballot_w64(dma_chunk<CT>(raw, nbytes, nxt, ja - kChunks, dst))
                     != 0) << (ja - kChunks);
      }
      mfma_chunk<CT, C>(slot, arow0 + 64 * j, boff, res, b, acc);
    }

    // epilogue: lanes (n, q) hold rows q + 4r of epoch n for every channel
    double s = 0.0;
    double a[C][4];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[c][r] = acc[c][0][r] + acc[c][1][r];
        s += a[c][r] * a[c][r];
      }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const double nrm = sqrt(s);
    if (e0 + nn < n) {
      double* o = out + (e0 + nn) * F + q;
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[16 * c + 4 * r] = a[c][r] / nrm;
    }
    if (!has_next) break;
    tile = next;
    cur = nxt;
    fix = fix_next;
    fix_next = 0;
    mb ^= 1;
  }
  wait_vm<0>();  // no LDS-DMA may land after the workgroup's LDS is released
}

}  // namespace dev

namespace {
template <int CT, int C>
hipError_t launch_mfma_t(hipStream_t st, const void* raw, int64_t n_frames, const ChanSel& sel,
                         const int64_t* pos, const float* base, int64_t n, const double* mrows,
                         double* out) {
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const int64_t ntiles = (n + dev::kTileE - 1) / dev::kTileE;
  int64_t grid = (ntiles + dev::kWaves - 1) / dev::kWaves;
  if (grid > cus) grid = cus;
  hipLaunchKernelGGL((dev::mfma_window_kernel<CT, C>), dim3((unsigned)grid), dim3(64 * dev::kWaves),
                     0, st, (const uint8_t*)raw, n_frames, sel, pos, base, n, mrows, out);
  return hipGetLastError();
}
}  // namespace

bool mfma_supported(int fmt, int ct, int C) { return fmt == 0 && ct == 3 && C == 3; }

hipError_t launch_mfma_window(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                              const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                              const void* scratch, const double* mrows, double* out) {
  if (!mfma_supported(0, ct, C)) return hipErrorNotSupported;
  if (n == 0) return hipSuccess;
  return launch_mfma_t<3, 3>(st, raw, n_frames, sel, pos, (const float*)scratch, n, mrows, out);
}

}  // namespace eegfx
