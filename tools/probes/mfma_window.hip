// Probe: the collapsed fma filter of window_kernel on the matrix pipe (v_mfma_f64_4x4x4f64), timed
// against the product kernel on the bench workload, with the feature difference.  DESIGN.md §6
// costs it from the measured energy per MAC; this settles it.
//
// Per sub-tile of 8 epochs (wave = channel, as window_kernel), two groups of 4 signals.  Each group
// computes the block products G[b][j] = sum_{p < 32} x[32 b + p] H5[32 j + p] (16 data blocks x 9
// tap blocks, padded to 12) as 4x4x4 blocks: instruction block = signal, rows = 4 data blocks,
// columns = 4 tap blocks, K = 4 samples (4 x 3 x 8 = 96 instructions per group).  Operand layouts
// (tools/probes/mfma44_probe.hip): A[blk][row][k] at lane 16k + 4blk + row, B[blk][k][col] at lane
// 16k + 4blk + col, D[blk][row][col] at lane 16row + 4blk + col.  a5[k] = sum_j G[k + j][j]: the
// 12 accumulators of a lane fall into 4 classes (b0 - j0) mod 16 that each target one output,
// then the 4 partials of an output are summed through LDS (the window buffer, after a barrier), and
// level 6, normalisation and the row store are the product's.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I../../include \
//     -I../../eeg_dataanalysispackage_amd/csrc mfma_window.hip -o mfma_window
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../eeg_dataanalysispackage_amd/csrc/fused.hip"
#include "../../eeg_dataanalysispackage_amd/csrc/wide.hip"
#include "../../eeg_dataanalysispackage_amd/csrc/kernels.hip"

namespace eegfx {
namespace dev {

// B operand per lane pattern q = 4k + c (k = lane / 16, c = lane % 4): [q][p0i][j0i] =
// H5[32 (4 j0i + c) + 4 p0i + k], zero for tap blocks past 8 or taps past 279
__constant__ double kB44[16 * 8 * 3];

#ifndef MW_WAVES
#define MW_WAVES 5
#endif

template <bool NT>
__global__ __launch_bounds__(192, MW_WAVES) void window_mfma_kernel(
    const uint8_t* __restrict__ raw, int64_t n_frames, ChanSel sel, const int64_t* __restrict__ wb,
    const float* __restrict__ base, int64_t n, double* __restrict__ out) {
  using G = Geometry<3>;
  constexpr int C = 3, F = C * 16;
  __shared__ __attribute__((aligned(16))) uint32_t win[kSub * G::ESTR];
  __shared__ double norm[kSub];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t nbytes = n_frames * G::FB;
  const int col = sel.col[w];
  const float r = sel.res[w];
  const int64_t e0 = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * kSub;
  const int64_t rest = n - e0;
  const int ne = (rest >> 31) != 0 ? kSub : ((int)rest < kSub ? (int)rest : kSub);

  const DmaRows<3> rows(lane);
  if (dma_issue<3, C, NT>(raw, nbytes, wb, e0, ne, win, w, lane, rows))
    dma_fixup<3, C>(raw, nbytes, wb, e0, ne, win, w, lane, rows);
  // this lane's B operands (taps), loaded while the windows land
  double Bc[8][3];
  {
    const int q = 4 * (lane >> 4) + (lane & 3);
    const double* bt = kB44 + q * 24;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Bc[i][j] = bt[i * 3 + j];
  }
  dma_drain();
  __syncthreads();

  // A operand coordinates: row (data block within the b0 tile) = lane & 3, signal = (lane >> 2) & 3,
  // k (sample within the p0 step) = lane >> 4
  const int ra = lane & 3, sa = (lane >> 2) & 3, ka = lane >> 4;
  const dwt8_f32x2 rr = {r, r};
  double Q[2][4];
#ifndef MW_INTERLEAVE
#define MW_INTERLEAVE 0
#endif
#if MW_INTERLEAVE
  // both groups in one p loop: 24 independent accumulator chains per p step
  const uint8_t* lbg[2];
  dwt8_f32x2 bbg[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int el = 4 * g + sa;
    const bool mine = el < ne;
    const float b = mine ? base[(e0 + el) * C + w] : 0.0f;
    bbg[g] = (dwt8_f32x2){b, b};
    const int delta = mine ? (int)((uint32_t)wb[e0 + el] & 14u) : 0;
    lbg[g] = (const uint8_t*)(win + el * G::ESTR) + delta + 2 * col + 16 * G::SEGQ * (ra >> 1) +
             G::FB * (32 * (ra & 1) + ka);
  }
  double acc[2][4][3];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      float s[4];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
        s[bi] = (float)*(const int16_t*)(lbg[g] + 16 * G::SEGQ * 2 * bi + G::FB * 4 * p);
      const dwt8_f32x2 v0 = {s[0], s[1]}, v1 = {s[2], s[3]};
      const dwt8_f32x2 y0 = v0 * rr - bbg[g], y1 = v1 * rr - bbg[g];
      const double xa[4] = {(double)y0.x, (double)y0.y, (double)y1.x, (double)y1.y};
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int ji = 0; ji < 3; ++ji)
          acc[g][bi][ji] = __builtin_amdgcn_mfma_f64_4x4x4f64(
              xa[bi], Bc[p][ji], p == 0 ? 0.0 : acc[g][bi][ji], 0, 0, 0);
    }
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      double q = 0.0;
      bool first = true;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int ji = 0; ji < 3; ++ji)
          if (((bi - ji) & 3) == d) {
            q = first ? acc[g][bi][ji] : q + acc[g][bi][ji];
            first = false;
          }
      Q[g][d] = q;
    }
#else
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int el = 4 * g + sa;
    const bool mine = el < ne;
    const float b = mine ? base[(e0 + el) * C + w] : 0.0f;
    const dwt8_f32x2 bb = {b, b};
    const int delta = mine ? (int)((uint32_t)wb[e0 + el] & 14u) : 0;
    // sample m = 32 (b0 + ra) + p0 + ka of the window: segment (b0 + ra) / 2, frame
    // 32 ((b0 + ra) % 2) + p0 + ka; b0 even, so the lane part is (ra / 2) segments and
    // 32 (ra % 2) + ka frames, and (b0 / 2) segments + p0 frames are immediates
    const uint8_t* lb = (const uint8_t*)(win + el * G::ESTR) + delta + 2 * col +
                        16 * G::SEGQ * (ra >> 1) + G::FB * (32 * (ra & 1) + ka);
    double acc[4][3];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      float s[4];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
        s[bi] = (float)*(const int16_t*)(lb + 16 * G::SEGQ * 2 * bi + G::FB * 4 * p);
      const dwt8_f32x2 v0 = {s[0], s[1]}, v1 = {s[2], s[3]};
      const dwt8_f32x2 y0 = v0 * rr - bb, y1 = v1 * rr - bb;
      const double xa[4] = {(double)y0.x, (double)y0.y, (double)y1.x, (double)y1.y};
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int ji = 0; ji < 3; ++ji)
          acc[bi][ji] = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[bi], Bc[p][ji],
                                                            p == 0 ? 0.0 : acc[bi][ji], 0, 0, 0);
    }
    // D lane = 16 row + 4 sig + c holds G[4 bi + row][4 ji + c]: class (bi - ji) mod 4 targets
    // output 4 ((bi - ji) mod 4) + row - c (mod 16)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      double q = 0.0;
      bool first = true;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int ji = 0; ji < 3; ++ji)
          if (((bi - ji) & 3) == d) {
            q = first ? acc[bi][ji] : q + acc[bi][ji];
            first = false;
          }
      Q[g][d] = q;
    }
  }
#endif
  __syncthreads();  // every wave has read its samples: the window buffer becomes scratch
  // partials: after the 3 KB of feature rows, 512 doubles per wave, slot
  // ((g * 64 + sig * 16 + row * 4 + c) * 4 + class)
  double* fb = (double*)win;
  double* qs = fb + kSub * F + w * 512;
  {
    const int rd = lane >> 4, sd = (lane >> 2) & 3, cd = lane & 3;
    typedef double f64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      double* dst = qs + (g * 64 + sd * 16 + rd * 4 + cd) * 4;
      *(f64x2*)dst = (f64x2){Q[g][0], Q[g][1]};
      *(f64x2*)(dst + 2) = (f64x2){Q[g][2], Q[g][3]};
    }
  }
  wave_sync();
  // the product's owner layout: lane 8 el + s holds a5[2s], a5[2s + 1] of epoch el
  const int el = lane >> 3, s = lane & 7, g = el >> 2, sig = el & 3;
  double a5[2 + 8];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = 2 * s + t;
    double v = 0.0;
#pragma unroll
    for (int row = 0; row < 4; ++row) {
      const int c = (row - k) & 3;
      const int cls = ((k - row + c) & 15) >> 2;
      v += qs[(g * 64 + sig * 16 + row * 4 + c) * 4 + cls];
    }
    a5[t] = v;
  }
  halo<2, true>(a5, nullptr, lane & ~7, s);
  const double a6 = fir10<true, false>(a5);
  const double d6 = fir10<true, true>(a5);
  int l2 = lane;
  asm volatile("" : "+v"(l2));
  const int slot = (l2 >> 3) * F + w * 16 + (l2 & 7);
  fb[slot] = a6;
  fb[slot + 8] = d6;
  __syncthreads();
  if (w == 0) normalise_store<F, true>(fb, norm, out + e0 * F, ne, lane);
}

}  // namespace dev
}  // namespace eegfx

int main() {
  using namespace eegfx;
  // B table from the generated taps
  const double tab[] = EEGFX_H5_TABLE;
  auto H5 = [&](int m) { return m < 256 ? tab[(m % 32) * 8 + m / 32] : (m < 280 ? tab[256 + m - 256] : 0.0); };
  std::vector<double> b44(16 * 8 * 3);
  for (int q = 0; q < 16; ++q) {
    const int k = q / 4, c = q % 4;
    for (int p = 0; p < 8; ++p)
      for (int ji = 0; ji < 3; ++ji) {
        const int j = 4 * ji + c, m = 32 * j + 4 * p + k;
        b44[(q * 8 + p) * 3 + ji] = (j <= 8 && m < 280) ? H5(m) : 0.0;
      }
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(dev::kB44), b44.data(), b44.size() * 8);

  const int64_t n = 1000000, nf = 1000 * n + 2000;
  int16_t* raw;
  int64_t* pos;
  float* base;
  double *out0, *out1;
  (void)hipMalloc(&raw, nf * 3 * 2);
  (void)hipMalloc(&pos, n * 8);
  (void)hipMalloc(&base, fused_scratch_bytes(n, 3));
  (void)hipMalloc(&out0, n * 48 * 8);
  (void)hipMalloc(&out1, n * 48 * 8);
  (void)launch_synth(0, raw, nf, 3, 0x5EED);
  std::vector<int64_t> hp(n);
  for (int64_t i = 0; i < n; ++i) hp[i] = 1000 + 1000 * i;
  (void)hipMemcpy(pos, hp.data(), n * 8, hipMemcpyHostToDevice);
  ChanSel sel{};
  for (int c = 0; c < 3; ++c) { sel.col[c] = c; sel.res[c] = 0.1f; }
  (void)launch_fused_baseline(0, raw, nf, 3, sel, 3, pos, n, base, nullptr);
  const int64_t* words = (const int64_t*)((const uint8_t*)base + ((sizeof(float) * n * 3 + 15) & ~(size_t)15));
  const dim3 g((unsigned)((n + 7) / 8));
  auto product = [&] { (void)launch_fused_window(0, raw, nf, 3, sel, 3, pos, n, true, base, out0); };
  auto mfma = [&] {
    hipLaunchKernelGGL((dev::window_mfma_kernel<true>), g, dim3(192), 0, 0, (const uint8_t*)raw, nf,
                       sel, words, (const float*)base, n, out1);
  };
  product();
  mfma();
  (void)hipDeviceSynchronize();
  std::vector<double> h0(n * 48), h1(n * 48);
  (void)hipMemcpy(h0.data(), out0, h0.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(h1.data(), out1, h1.size() * 8, hipMemcpyDeviceToHost);
  double md = 0;
  for (size_t i = 0; i < h0.size(); ++i) md = fmax(md, fabs(h0[i] - h1[i]));
  printf("max |mfma - product| over %lld x 48 features: %.3e (%s)\n", (long long)n, md,
         hipGetErrorString(hipGetLastError()));
  const int iters = getenv("PROBE_ITERS") ? atoi(getenv("PROBE_ITERS")) : 2000;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* only = getenv("PROBE_ONLY");  // "mfma" / "product": one kernel, for power sampling
  for (int rep = 0; rep < 2; ++rep) {
    for (int which = 0; which < 2; ++which) {
      if (only && (which == 1) != (only[0] == 'm')) continue;
      for (int i = 0; i < 200; ++i) which ? mfma() : product();
      (void)hipEventRecord(a);
      for (int i = 0; i < iters; ++i) which ? mfma() : product();
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("%s: %.4f ms per launch\n", which ? "mfma   " : "product", ms / iters);
    }
  }
  return md <= 1e-9 ? 0 : 1;
}
